#!/bin/bash
# GPU box: one vs two engines on the 8-stream family configs, same frames (frame_counts summed over
# the engines must match), then the kernel stats + roofline line of the two-engine C5 run.
# Usage: TAG=r03zg bash tools/queues_check.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-qcheck}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for t in hybridsort deepocsort; do
  for q in 1 2; do
    timeout -k 10 240 python3 $R/tools/bench_tracker.py --tracker $t --streams 8 --queues $q --steps 6 --warmup 2 --cpu-frames 0 > $O/${t}_q$q.json 2> $O/${t}_q$q.err || exit $?
  done
  python3 - $O/${t}_q1.json $O/${t}_q2.json <<'PY' || exit $?
import json, sys
a, b = (json.load(open(f)) for f in sys.argv[1:])
print(a["config"]["workload"], "q1", round(a["value"], 1), "q2", round(b["value"], 1), "calls/s;",
      "frame_counts equal:", a["frame_counts"] == b["frame_counts"], a["frame_counts"], b["frame_counts"])
PY
done
n=hybridsort_s8_q2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/tools/bench_tracker.py --tracker hybridsort --streams 8 --queues 2 --steps 6 --warmup 2 --cpu-frames 0 > $O/$n.json 2> $O/$n.err || exit $?
ks=$(find $O/$n -name '*kernel_stats.csv' | head -1)
python3 $R/tools/config_roofline.py $O/hybridsort_q2.json $ks > $O/${n}_roofline.json || exit $?
echo done
