#!/bin/bash
# Streams x engines sweep of bench.py (GPU box; writes gpurun_out/sweep_sq.txt).  Args: "S:Q" pairs.
mkdir -p gpurun_out
out=gpurun_out/sweep_sq.txt
: > $out
for sq in "$@"; do
  s=${sq%%:*}; q=${sq##*:}
  timeout -k 10 300 python bench.py --streams $s --queues $q --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sq.json 2>gpurun_out/sq.err || { echo "FAIL $s $q" >> $out; exit 1; }
  python - "$s" "$q" >> $out <<'PY'
import json,sys
d=json.loads(open('gpurun_out/sq.json').read().strip().splitlines()[-1])
print(f"S={sys.argv[1]:>5s} Q={sys.argv[2]} {d['value']:>10.0f} calls/s  step {d['ms_per_step']:.3f} ms")
PY
  echo "done $s $q"
done
cat $out
