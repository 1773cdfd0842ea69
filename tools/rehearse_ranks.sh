#!/bin/bash
# GPU box: the N-rank paths of bench.py on one card (--shared-gpu: both ranks on device 0, gloo):
# the headline and the C4 / C5 configs at two ranks.  Not a scaling measurement.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ranks}
mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --shared-gpu "$@" \
      > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -20 $O/$tag.err; return 1; }
  tail -c 600 $O/$tag.json; echo
}
run headline --streams 512 --steps 5 --warmup 2 --no-configs --no-dropin --no-cpu-baseline --no-pcie && \
run c4 --tracker deepocsort && \
run c5 --tracker hybridsort
