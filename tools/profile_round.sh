#!/bin/bash
# rocprofv3 evidence for profiles/ (GPU box): the bench line, kernel trace + stats, then FETCH_SIZE
# and WRITE_SIZE in their own passes, all on the same bench.py command (the driver's round-end
# step count, with the isolated leg: the summary splits every kernel's launches into the timed
# window and the isolated one).  Usage: tools/profile_round.sh TAG [STREAMS] [QUEUES]  -> gpurun_out/prof_TAG/
set -e
TAG=$1
S=${2:-2048}
Q=${3:-2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--streams $S --queues $Q --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-dropin --no-configs"
ISO=3; [ "$Q" = "1" ] && ISO=0
timeout -k 10 400 python3 $R/bench.py $ARGS > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py $ARGS > $O/kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py $ARGS > $O/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py $ARGS > $O/write.log 2>&1
cd $R && python3 profiles/summarize.py $TAG $O/kt $O/fetch $O/write --streams $S --queues $Q --pre 40 --steps 20 --iso $ISO --bench-json $O/bench.json > $O/summary.txt
echo profiled
