#!/bin/bash
# Kernel time of one kernel across library variants (GPU box): rocprofv3 --kernel-trace --stats of
# the same command with YTA_LIBRARY set per variant.  Usage:
#   tools/kstat_variants.sh <kernel-substring> "<command>" default lib1.so lib2.so ...
set -e
K=$1; CMD=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kstat
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then L=""; else L="$R/$lib"; fi
  YTA_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- $CMD > $O/$n.log 2>&1
  f=$(ls $O/$n/*/run_kernel_stats.csv 2>/dev/null | head -1 || true)
  [ -z "$f" ] && f=$(find $O/$n -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$K" "$n" <<'PY'
import csv, sys
f, k, n = sys.argv[1:]
for r in csv.DictReader(open(f)):
    if k in r["Name"]:
        print(f"{n:>28s} {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
