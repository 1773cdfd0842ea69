#!/bin/bash
# GPU box: A/B of the pipelined path's host / dependency switches in separate processes (the
# switches are read once per process), then a kernel + copy trace of the default.
# Usage: tools/pipe_ab.sh TAG  -> gpurun_out/TAG/
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-"1 1 1 1" "1 0 1 1" "1 0 0 1" "0 0 0 1" "0 0 0 0"}; do
  set -- $cfg
  tag=spin$1_fence$2_devrel$3_flush$4
  YTA_PIPE_SPIN=$1 YTA_PIPE_IN_FENCE=$2 YTA_PIPE_IN_DEVREL=$3 YTA_PIPE_FLUSH=$4 timeout -k 10 200 python3 \
      $R/tools/pipe_probe.py --first 6 --frames 16 --legs pipe_pinned,pipe_pinned_f32,pipe \
      > $O/$tag.jsonl 2>&1 || exit $?
  python3 - $O/$tag.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"probe": "pipe'):
        d = json.loads(l)
        print(sys.argv[1].split('/')[-1], d["probe"], round(d["value"]), round(d["ms_per_step"], 3))
PY
done
YTA_PIPE_KERNEL_D2H=0 timeout -k 10 200 python3 $R/tools/pipe_probe.py --first 6 --frames 16 \
    --legs pipe_pinned,pipe_pinned_f32 > $O/sdma_d2h.jsonl 2>&1 || exit $?
grep -o '"probe": "pipe[a-z_0-9]*", "wall_s": [0-9.]*, "value": [0-9.]*' $O/sdma_d2h.jsonl || true
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace \
    -o run -- python3 $R/tools/pipe_probe.py --first 6 --frames 12 --legs pipe_pinned \
    > $O/trace.log 2>&1 || exit $?
python3 $R/tools/pipe_timeline.py $O/trace --last 12 | tee $O/timeline.txt
