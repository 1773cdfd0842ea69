#!/bin/bash
# L1/L2 request counters on the bench (GPU box) -> gpurun_out/pmc_mem/<pass>/
set -e
S=${1:-256}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_mem
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
run() {
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- python3 $R/bench.py --streams $S --steps 4 --warmup 2 --no-cpu-baseline > $O/$1.log 2>&1
}
run m1 "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum"
run m2 "TCP_TOTAL_CACHE_ACCESSES_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
run m3 "FETCH_SIZE"
run m4 "WRITE_SIZE"
echo done
