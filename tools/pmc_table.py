#!/usr/bin/env python3
"""Per-kernel averages of every counter under gpurun_out/pmc_sq/*/ (rocprofv3 counter CSVs)."""
import collections, csv, glob, os, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("yta::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not k.startswith("k_"):
        continue
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:<24s} {sum(v) / len(v):16.0f}")
