#!/bin/bash
# GPU box: A/B of two libraries on the OCSORT-family configs (tools/bench_tracker.py, no CPU leg),
# interleaved twice.  Usage: A=<lib> B=<lib> bash tools/ab_configs.sh -> gpurun_out/ab_configs.txt
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_configs.txt
: > $O
for rep in 1 2; do
  for L in "$A" "$B"; do
    for T in "ocsort --steps 30" "deepocsort --steps 20" "hybridsort --steps 12"; do
      set -- $T
      YTA_LIBRARY=$L timeout -k 10 300 python3 $R/tools/bench_tracker.py --tracker $1 $2 $3 --warmup 3 --cpu-frames 0 > $R/gpurun_out/abc.json 2>$R/gpurun_out/abc.err || { tail -3 $R/gpurun_out/abc.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$R/gpurun_out/abc.json').read().strip().splitlines()[-1])
print('$(basename $L)', '$1', round(d['value'], 1), 'ms %.3f' % d['ms_per_step'])" | tee -a $O
    done
  done
done
