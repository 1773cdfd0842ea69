#!/bin/bash
# Engines-per-GPU sweep of the DeepOCSORT / HybridSORT configs (GPU box): Q engines of S/Q streams
# on Q HIP streams (tools/bench_tracker.py --queues).  Usage: TAG=r03zf bash tools/queues_sweep.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-queues}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for spec in "hybridsort 8 1" "hybridsort 8 2" "hybridsort 8 4" "hybridsort 8 8" "deepocsort 8 1" "deepocsort 8 2" "deepocsort 8 4"; do
  set -- $spec
  timeout -k 10 240 python3 $R/tools/bench_tracker.py --tracker $1 --streams $2 --queues $3 --steps 6 --warmup 2 --cpu-frames 0 > $O/$1_s$2_q$3.json 2> $O/$1_s$2_q$3.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$O/$1_s$2_q$3.json')); print('$1 streams $2 queues $3', round(d['value'],1), 'calls/s', round(d['ms_per_step'],3), 'ms/step')"
done
echo done
