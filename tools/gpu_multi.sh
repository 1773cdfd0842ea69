#!/bin/bash
# GPU box: several steps, each under its own time limit; a step that fails an assertion (rc 1)
# does not stop the next, a fault / abort / time limit (rc >= 124) does.
# Usage: TAG=x bash tools/gpu_multi.sh "cmd1" "cmd2" ...   (outputs under gpurun_out/$TAG/stepN.log)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-multi}
mkdir -p $O
cd $R
n=0
for c in "$@"; do
  n=$((n+1))
  echo "== step $n: $c"
  bash -c "$c" > $O/step$n.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -8 $O/step$n.log
  if [ $rc -ge 124 ]; then echo "stopping after rc $rc"; exit $rc; fi
done
echo done
