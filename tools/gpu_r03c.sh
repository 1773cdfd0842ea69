# GPU box: bytetrack-family tests, then (unless a test crashed / hung) benches + a kernel trace
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r03c}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_bytetrack.py tests/test_gpu_full_configs.py tests/test_gpu_botsort.py} -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --queues 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/bench_q1.json 2> $O/bench_q1.err || exit $?
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/bench_q2.json 2> $O/bench_q2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --queues 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/kt.log 2>&1 || exit $?
echo done
