#!/bin/bash
# GPU box: bench.py's PCIe legs (headline engines alive, as in the default run) under runtime
# settings, one process each:  tools/bench_pcie_ab.sh TAG "ENV=VAL ..." ...
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
n=0
for cfg in "$@"; do
  n=$((n+1))
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-configs --no-dropin \
      --no-cpu-baseline > $O/$n.json 2> $O/$n.err || exit $?
  python3 - "$cfg" $O/$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
p = d["pcie_inclusive"]["pipelined"]
print(f"{sys.argv[1]:>32s} value {round(d['value'])} pipelined pageable {round(p['value'])} "
      f"pinned {round(p['pinned']['value'])} f32 {round(p['pinned_f32']['value'])}")
PY
done
