#!/bin/bash
# SQ counter passes on the ECC bench (GPU box, one stream by default): where k_ecc's cycles go.
# Usage: tools/pmc_ecc.sh [streams] [warp_mode]  -> gpurun_out/pmc_ecc/<pass>/
set -e
S=${1:-1}
MODE=${2:-1}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PMC_TAG:-pmc_ecc}
mkdir -p $O
run() {
  timeout -k 10 120 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- python3 $R/tools/bench_cmc.py --estimator ecc --warp-mode $MODE --streams $S --steps 2 --no-cpu > $O/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
run p2 "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
run p3 "SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_INSTS_SENDMSG"
echo done
