#!/bin/bash
# GPU box: headline calls/s vs streams per GPU and engines (bench.py --streams S --queues Q).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stream_sweep.txt
: > $O
for SQ in "2048 2" "3072 3" "4096 2" "4096 4" "3072 2"; do
  set -- $SQ
  timeout -k 10 300 python3 $R/bench.py --streams $1 --queues $2 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-isolated > $R/gpurun_out/ss.json 2>$R/gpurun_out/ss.err || { echo "fail $1 $2"; tail -3 $R/gpurun_out/ss.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/ss.json').read().strip().splitlines()[-1])
print('streams $1 queues $2', round(d['value']), 'step %.3f' % d['ms_per_step'])" | tee -a $O
done
