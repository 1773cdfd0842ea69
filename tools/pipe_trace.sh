#!/bin/bash
# GPU box: the pipelined host-buffer path under a kernel + memory-copy trace (no counters), plus the
# probe's own accounting at two capacities.  Usage: tools/pipe_trace.sh TAG [probe args...]
#   -> gpurun_out/TAG/{probe.jsonl, probe_cap5.jsonl, trace/, timeline.txt}
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python3 $R/tools/pipe_probe.py --first 6 --frames 12 \
    --legs pipe_pinned,pipe_pinned_f32,pipe "$@" > $O/probe.jsonl 2> $O/probe.err || exit $?
timeout -k 10 240 python3 $R/tools/pipe_probe.py --first 6 --frames 12 --cap-mult 5 \
    --legs pipe_pinned "$@" > $O/probe_cap5.jsonl 2> $O/probe_cap5.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace \
    -o run -- python3 $R/tools/pipe_probe.py --first 6 --frames 12 --legs pipe_pinned "$@" \
    > $O/trace.log 2>&1 || exit $?
python3 $R/tools/pipe_timeline.py $O/trace --last 14 > $O/timeline.txt 2>&1
cat $O/probe.jsonl $O/probe_cap5.jsonl | cut -c1-400
cat $O/timeline.txt
