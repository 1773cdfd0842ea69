set -e
O=gpurun_out/blk_sweep.txt
: > $O
for L in default b512_l76 b512_l72 b768_l100; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/tools/_diag/libyta_$L.so; fi
  YTA_LIBRARY=$LIB timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie > gpurun_out/e1.json 2>gpurun_out/e1.err
  python -c "
import json; d=json.loads(open('gpurun_out/e1.json').read().strip().splitlines()[-1]); pk=d['per_kernel']
print('$L', round(d['value']), 'fb', d['frame_counts']['fallback1'], d['frame_counts']['fallback23'], ' '.join(f'{k} {v[\"ms\"]*1000:.0f}' for k,v in pk.items()))" >> $O
done
cat $O
