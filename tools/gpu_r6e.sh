set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
tools/gpu_suite_bench.sh r6e || exit $?
tools/pipe_trace.sh r6e_pipe || exit $?
cd /tmp && YTA_PIPE_IN_FENCE=0 timeout -k 10 200 python3 $R/tools/pipe_probe.py --first 6 --frames 12 --legs pipe_pinned,pipe_pinned_f32 > $R/gpurun_out/r6e_pipe/probe_nofence.jsonl 2>&1
cut -c1-300 $R/gpurun_out/r6e_pipe/probe_nofence.jsonl
