#!/bin/bash
# GPU box: BoT-SORT / ECC parity tests on library B, then a C3 A/B of libraries A and B (twice).
# Usage: A=<lib> B=<lib> bash tools/ab_c3.sh -> gpurun_out/ab_c3/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_c3
mkdir -p $O
cd $R
YTA_LIBRARY=$B timeout -k 10 400 python -u -m pytest tests/test_gpu_ecc.py tests/test_gpu_botsort.py tests/test_gpu_full_deep.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
: > $O/ab.txt
for rep in 1 2; do
  for L in "$A" "$B"; do
    YTA_LIBRARY=$L timeout -k 10 120 python3 tools/bench_tracker.py --tracker botsort --n 1024 --steps 30 --warmup 3 --cpu-frames 0 > $O/c3.json 2> $O/c3.err || { tail -3 $O/c3.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1])
print('$(basename $L)', round(d['value'], 1), 'ms %.4f' % d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
