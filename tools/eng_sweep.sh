set -e
mkdir -p gpurun_out
O=gpurun_out/eng_sweep.txt
: > $O
for L in default l128 l112; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/tools/_diag/libyta_$L.so; fi
  YTA_LIBRARY=$LIB timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/e1.json 2>/dev/null
  python -c "
import json; d=json.loads(open('gpurun_out/e1.json').read().strip().splitlines()[-1]); pk=d['per_kernel']
print('$L E=1 bench', round(d['value']), 'fb', d['frame_counts']['fallback1'], d['frame_counts']['fallback23'], ' '.join(f'{k} {v[\"ms\"]*1000:.0f}' for k,v in pk.items()))" >> $O
  for E in 1 2 4; do
    YTA_LIBRARY=$LIB timeout -k 10 200 python tools/bench_engines.py --engines $E >> $O 2>/dev/null
  done
  echo "done $L"
done
cat $O
