#!/bin/bash
# rocprofv3 evidence for the ReID preprocessing kernel (GPU box): bench lines (f32, f16), kernel
# trace + stats, then FETCH_SIZE and WRITE_SIZE in their own passes.  Usage: tools/profile_reid.sh TAG
set -e
TAG=${1:-r01h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/reid_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/bench_reid.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 200 python3 $R/tools/bench_reid.py --half 1 >> $O/bench.jsonl 2>> $O/bench.err
echo bench
CMD="python3 $R/tools/bench_reid.py --steps 10 --cpu-sample 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $CMD > $O/kt.log 2>&1
echo kt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD > $O/write.log 2>&1
echo profiled
