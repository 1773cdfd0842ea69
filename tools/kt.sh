#!/bin/bash
# rocprofv3 kernel-trace stats of one bench.py run (GPU box): tools/kt.sh TAG [bench args...]
# -> gpurun_out/kt_TAG/ and a per-kernel table on stdout.
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-pcie "$@" > $R/gpurun_out/kt_$TAG.json 2> $R/gpurun_out/kt_$TAG.err
cd $R && python3 tools/_kstats.py gpurun_out/kt_$TAG
