#!/bin/bash
# GPU box: the pipelined legs at several (untimed, timed) frame counts, one process each:
#   tools/pipe_frames_ab.sh TAG "FIRST FRAMES" ...   -> gpurun_out/TAG/<first>_<frames>.jsonl
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 240 python3 $R/tools/pipe_probe.py --first $1 --frames $2 \
      --legs ${LEGS:-pipe_pinned,pipe_pinned_f32} > $O/$1_$2.jsonl 2>&1 || exit $?
  grep '"probe": "pipe' $O/$1_$2.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('first $1 frames $2', d['probe'], round(d['value']), round(d['ms_per_step'], 3))"
done
