#!/bin/bash
# GPU box: C3 (BoT-SORT 1024 x 1024, 512-d embeddings, one stream) under rocprofv3 --kernel-trace
# --stats, plus the plain timing; -> gpurun_out/TAG/
TAG=${1:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--tracker botsort --n 1024 --dim 512 --streams 1 --steps 30"
timeout -k 10 200 python3 $R/tools/bench_tracker.py $ARGS > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/bench_tracker.py $ARGS > $O/kt.log 2>&1 || exit $?
tail -c 300 $O/bench.json
python3 - $O/kt/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1000:9.2f} us {float(r["Percentage"]):6.2f} %')
PY
