#!/bin/bash
# GPU box: the drop-in leg (one ByteTrack stream through create_tracker + update) under
# rocprofv3 --kernel-trace --memory-copy-trace, and the kernel / copy timeline of its frames.
TAG=${1:-dropin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/bench_dropin.py --trackers bytetrack --frames 200 > $O/plain.json 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/bench_dropin.py --trackers bytetrack --frames 200 > $O/kt.log 2>&1 || exit $?
cat $O/plain.json | tail -2
python3 - $O/kt/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{r["Name"][:56]:56s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1000:9.2f} us')
PY
