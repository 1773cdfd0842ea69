#!/bin/bash
# round 6: pipelined-path dependency A/B, k_s1_edges SQ counters (default vs -DYTA_S1_P1=0), and
# the single-engine headline A/B of the same two libraries.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
tools/pipe_env_ab.sh r6l_pipe "YTA_PIPE_FLAGS=0" "YTA_PIPE_FLAGS=2" "YTA_PIPE_FLAGS=3" "YTA_PIPE_FLAGS=1" || exit $?
PMC_TAG=r6l_sq_p1 bash tools/pmc_sq.sh 1024 || exit $?
YTA_LIBRARY=$R/tools/variants/libyta_p0.so PMC_TAG=r6l_sq_p0 bash tools/pmc_sq.sh 1024 || exit $?
python3 tools/pmc_table.py gpurun_out/r6l_sq_p1 > gpurun_out/r6l_sq_p1/table.txt
python3 tools/pmc_table.py gpurun_out/r6l_sq_p0 > gpurun_out/r6l_sq_p0/table.txt
grep -A26 "^k_s1_edges" gpurun_out/r6l_sq_p1/table.txt | head -27
grep -A26 "^k_s1_edges" gpurun_out/r6l_sq_p0/table.txt | head -27
TAG=r6l_ab ROUNDS=2 QUEUES=1 bash tools/ab_bench.sh default tools/variants/libyta_p0.so
