#!/bin/bash
# A/B of library variants on the headline bench (GPU box), interleaved so that both see the same
# box state: for each round, each library at --queues 1 and 2.  Usage:
#   TAG=x ROUNDS=2 bash tools/ab_bench.sh default tools/variants/libyta_base.so
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
out=$O/ab.txt
: > $out
cd /tmp && export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
  for lib in "$@"; do
    for q in ${QUEUES:-1 2}; do
      if [ "$lib" = default ]; then L=""; else L="$R/$lib"; fi
      YTA_LIBRARY=$L timeout -k 10 300 python3 $R/bench.py --queues $q --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-isolated > $O/b.json 2> $O/b.err || { echo "FAIL $lib q$q" >> $out; cat $O/b.err | tail -5; exit 1; }
      python3 - "$lib" "$q" "$O/b.json" >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
pk = d["per_kernel"]
print(f"{sys.argv[1]:>32s} q{sys.argv[2]} {d['value']:>10.0f} calls/s  step {d['ms_per_step']:.3f} ms  "
      + "  ".join(f"{k} {v['ms']*1000:.1f}" for k, v in pk.items()))
PY
    done
  done
done
cat $out
