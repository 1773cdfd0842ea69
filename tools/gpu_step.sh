#!/bin/bash
# GPU box: selected GPU tests then (optionally) the default bench line.
# Usage (from gpurun): TAG=r04a TESTS="tests/test_x.py tests/test_y.py" BENCH=1 bash tools/gpu_step.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-step}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 $O/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BENCH" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 python3 $R/bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
echo done
