#!/bin/bash
# GPU box: ECC bench at 1 / 64 / 256 streams (euclidean), 64 streams translation / affine, and a
# rocprofv3 kernel trace at 64 streams -> gpurun_out/ecc_*.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
: > gpurun_out/ecc_bench.jsonl
for S in 1 64 256; do
  OMP_NUM_THREADS=1 timeout -k 10 300 python tools/bench_cmc.py --estimator ecc --streams $S $([ $S = 1 ] || echo --no-cpu) >> gpurun_out/ecc_bench.jsonl
done
for M in 0 2; do
  timeout -k 10 300 python tools/bench_cmc.py --estimator ecc --warp-mode $M --streams 64 --no-cpu >> gpurun_out/ecc_bench.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ecc_prof -o run -- python3 $R/tools/bench_cmc.py --estimator ecc --streams 64 --no-cpu > $R/gpurun_out/ecc_prof.log 2>&1
cat $R/gpurun_out/ecc_bench.jsonl
