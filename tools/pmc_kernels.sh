#!/bin/bash
# FETCH_SIZE and WRITE_SIZE per kernel of one short bench.py run, each counter in its own rocprofv3
# pass (GPU box): tools/pmc_kernels.sh TAG [bench args...] -> gpurun_out/pmc_TAG_{fetch,write}/
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${TAG}_$C -o run -- python3 $R/bench.py --no-cpu-baseline --no-pcie --steps 6 --warmup 2 "$@" > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1
done
cd $R && python3 - "$TAG" <<'PY'
import collections, csv, glob, re, sys
tag = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_{tag}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            agg[m.group(1) if m else r["Kernel_Name"][:20]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{c:<11s} {k:<14s} launches {len(v):3d}  avg {sum(v)/len(v)/1024:10.1f} MB (KB units)  last {v[-1]/1024:10.1f}")
PY
