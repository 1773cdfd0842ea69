#!/bin/bash
# k_stage1 block-size / LDS-arena experiment: default library vs variants, ByteTrack 1024 streams.
O=gpurun_out/exp_blk.txt
: > $O
for L in ${LS:-default b512 b256}; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/tools/variants/libyta_$L.so; fi
  for N in ${NS:-512 1024}; do
    YTA_LIBRARY=$LIB timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --n $N > gpurun_out/e1.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/e1.json').read().strip().splitlines()[-1]); pk=d['per_kernel']
print('$L n=$N', round(d['value']), 'fb', d['frame_counts']['fallback1'], d['frame_counts']['fallback23'], ' '.join(f'{k} {v[\"ms\"]*1000:.0f}' for k,v in pk.items()))" >> $O
  done
done
cat $O
