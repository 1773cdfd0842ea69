#!/bin/bash
# Per-config evidence for profiles/ (GPU box): bench line with the CPU leg, then rocprofv3 kernel
# stats of the same command, then the roofline line (tools/config_roofline.py), for BASELINE.json
# configs 2-5 (tools/bench_tracker.py).  Usage: TAG=r03h bash tools/profile_configs.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-configs}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {   # name, bench_tracker args
  local n=$1; shift
  timeout -k 10 300 python3 $R/tools/bench_tracker.py "$@" > $O/${n}_bench.json 2> $O/${n}_bench.err || return $?
  echo bench $n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/tools/bench_tracker.py "$@" --cpu-frames 0 > $O/$n.json 2> $O/$n.err || return $?
  # measured HBM bytes: FETCH_SIZE and WRITE_SIZE, each in its own pass
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${n}_fetch -o run -- python3 $R/tools/bench_tracker.py "$@" --cpu-frames 0 > $O/${n}_fetch.log 2>&1 || return $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${n}_write -o run -- python3 $R/tools/bench_tracker.py "$@" --cpu-frames 0 > $O/${n}_write.log 2>&1 || return $?
  local ks=$(find $O/$n -name '*kernel_stats.csv' | head -1)
  python3 $R/tools/config_roofline.py $O/${n}_bench.json $ks $O/${n}_fetch $O/${n}_write > $O/${n}_roofline.json || return $?
  echo prof $n
}
run ocsort --tracker ocsort --steps 30 --warmup 3 || exit $?
run botsort --tracker botsort --steps 30 --warmup 3 || exit $?
run deepocsort --tracker deepocsort --steps 20 --warmup 3 || exit $?
run hybridsort --tracker hybridsort --steps 10 --warmup 3 || exit $?
run hybridsort_s8 --tracker hybridsort --streams 8 --steps 5 --warmup 2 --cpu-frames 1 || exit $?
echo done
