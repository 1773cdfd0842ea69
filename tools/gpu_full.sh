#!/bin/bash
# GPU box: the driver's round-end sequence (full -m gpu suite, smoke, default bench.py line).
# Usage (from gpurun): TAG=r03e bash tools/gpu_full.sh   -> gpurun_out/$TAG/
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-full}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
echo done
