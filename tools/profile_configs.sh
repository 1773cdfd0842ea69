set -e
# Per-config evidence for profiles/ (GPU box): bench line with the CPU leg, then rocprofv3 kernel stats,
# for BASELINE.json configs 2-5 (tools/bench_tracker.py).  Usage: bash tools/profile_configs.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for t in ocsort botsort deepocsort hybridsort; do
  st=30; [ $t = hybridsort ] && st=10; [ $t = deepocsort ] && st=20
  timeout -k 10 300 python3 $R/tools/bench_tracker.py --tracker $t --steps $st --warmup 3 > $O/${t}_bench.json 2> $O/${t}_bench.err
  echo bench $t
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t -o run -- python3 $R/tools/bench_tracker.py --tracker $t --steps $st --warmup 3 --cpu-frames 0 > $O/$t.json 2> $O/$t.err
  echo prof $t
done
timeout -k 10 300 python3 $R/tools/bench_tracker.py --tracker hybridsort --streams 8 --steps 5 --warmup 2 --cpu-frames 0 > $O/hybridsort_s8.json 2> $O/hybridsort_s8.err
echo s8
