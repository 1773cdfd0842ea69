#!/bin/bash
# GPU box: a subset of the -m gpu suite with prints (-s), one process, per-test time limits.
# Usage (from gpurun): TAG=x TESTS="tests/a.py tests/b.py" bash tools/gpu_tests.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-tests}
mkdir -p $O
cd $R
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread --durations=15 > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 $O/pytest.log
exit $rc
