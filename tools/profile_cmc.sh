#!/bin/bash
# GPU box: SparseOptFlow bench at 1 / 64 / 256 streams + rocprofv3 kernel stats at 64 streams.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
: > gpurun_out/cmc_bench.jsonl
for S in 1 64 256; do
  OMP_NUM_THREADS=1 timeout -k 10 300 python tools/bench_cmc.py --streams $S $([ $S = 1 ] || echo --no-cpu) >> gpurun_out/cmc_bench.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cmc_prof -o run -- python3 $R/tools/bench_cmc.py --streams 64 --no-cpu > $R/gpurun_out/cmc_prof.log 2>&1
cat $R/gpurun_out/cmc_bench.jsonl
