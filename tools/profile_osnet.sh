#!/bin/bash
# GPU box: rocprofv3 kernel stats of the OSNet forward (1024 crops, x0_25), f16 and f32, HIP
# block kernels.  CSV output in /tmp; only the kernel_stats summaries are kept.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/osnet_prof
cd /tmp && export TMPDIR=/tmp
for M in half f32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/osp_$M -o run -- python3 $R/tools/prof_osnet.py $([ $M = half ] && echo --half) > $R/gpurun_out/osnet_prof/$M.log 2>&1
  cp $(find /tmp/osp_$M -name '*kernel_stats.csv') $R/gpurun_out/osnet_prof/${M}_kernel_stats.csv
done
