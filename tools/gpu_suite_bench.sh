#!/bin/bash
# GPU box: the -m gpu suite (or the tests named after TAG), then the driver's bench command, into
# gpurun_out/TAG/.  A pytest run that ends in a crash, abort or time limit (exit status other than
# 0 = passed / 1 = some test failed) stops the script before anything else touches the GPU.
# Usage: tools/gpu_suite_bench.sh TAG [pytest args...]
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
TESTS=${@:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/suite.txt 2>&1
rc=$?
tail -3 $O/suite.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
brc=$?
tail -c 400 $O/bench.json
exit $(( rc > brc ? rc : brc ))
