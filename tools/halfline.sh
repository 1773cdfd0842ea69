#!/bin/bash
# GPU box: the half-line gather microbenchmark, plain and under FETCH_SIZE.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-halfline}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/_diag/halfline > $O/halfline.txt 2>&1 || exit $?
cat $O/halfline.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $R/tools/_diag/halfline > $O/fetch.log 2>&1 || exit $?
python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/fetch/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, "launches", len(v), "FETCH_SIZE KB/launch (median)", sorted(v)[len(v)//2])
PY
