#!/bin/bash
# GPU box: the pipelined path under runtime settings, one process each.  Usage:
#   tools/pipe_env_ab.sh TAG "ENV=VAL ..." ...   -> gpurun_out/TAG/<n>.jsonl (+ trace of the last)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
n=0
for cfg in "$@"; do
  n=$((n+1))
  env $cfg timeout -k 10 200 python3 $R/tools/pipe_probe.py --first 6 --frames 16 \
      --legs pipe_pinned,pipe_pinned_f32 > $O/$n.jsonl 2>&1 || exit $?
  python3 - "$cfg" $O/$n.jsonl <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{"probe": "pipe'):
        d = json.loads(l)
        print(f"{sys.argv[1]:>44s} {d['probe']:>16s} {round(d['value']):>8d} {d['ms_per_step']:.3f} ms")
PY
done
env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d $O/trace -o run -- python3 $R/tools/pipe_probe.py --first 6 --frames 12 --legs pipe_pinned \
    > $O/trace.log 2>&1 || exit $?
python3 $R/tools/trace_dump.py $O/trace 10 4.5 | tee $O/dump.txt
