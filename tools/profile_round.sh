#!/bin/bash
# rocprofv3 evidence for profiles/ (GPU box): kernel trace + stats, then FETCH_SIZE and WRITE_SIZE
# in their own passes, all on the same bench.py command.  Usage: tools/profile_round.sh TAG STREAMS
set -e
TAG=$1
S=${2:-1024}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --streams $S --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 400 python3 $R/bench.py --streams $S --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $CMD > $O/kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD > $O/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD > $O/write.log 2>&1
echo profiled
