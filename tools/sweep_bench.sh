#!/bin/bash
# Tuning sweep: bench.py over library variants x streams per GPU (GPU box; writes gpurun_out/sweep.txt)
mkdir -p gpurun_out
out=gpurun_out/sweep.txt
: > $out
for lib in "$@"; do
  for s in ${SWEEP_STREAMS:-256 512 1024}; do
    if [ "$lib" = default ]; then L=""; else L="$lib"; fi
    YTA_LIBRARY=$L timeout -k 10 300 python bench.py --streams $s --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sw.json 2>/dev/null || { echo "FAIL $lib $s" >> $out; exit 1; }
    python - "$lib" "$s" >> $out <<'PY'
import json,sys
d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1])
pk=d['per_kernel']
print(f"{sys.argv[1]:>28s} S={sys.argv[2]:>5s} {d['value']:>10.0f} calls/s  step {d['ms_per_step']:.3f} ms  " + "  ".join(f"{k} {v['ms']*1000:.1f}us" for k,v in pk.items()) + f"  fb {d['frame_counts']['fallback1']}/{d['frame_counts']['fallback23']}")
PY
    echo "done $lib $s"
  done
done
cat $out
