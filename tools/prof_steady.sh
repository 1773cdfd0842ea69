set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --queues 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/bench_q1.json 2> $O/bench_q1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --queues 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/kt.log 2>&1
echo done
