#!/bin/bash
# A/B variant of libyta.so with extra defines (CPU container; the .so travels to the GPU box):
#   tools/variants/build_variant.sh NAME "-DYTA_X=0 ..."  -> tools/variants/libyta_NAME.so
# Select it with YTA_LIBRARY=tools/variants/libyta_NAME.so (tools/kstat_variants.sh).
set -e
NAME=$1; DEFS=$2
HERE=$(cd $(dirname $0) && pwd)
SRC=$HERE/../../yolo_tracking_amd/csrc
B=$HERE/build_$NAME
mkdir -p $B
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -munsafe-fp-atomics"
for s in util kat bytetrack ocsort deepocsort hybridsort gsi reid cmc ecc osnet; do
  echo "/opt/rocm/bin/hipcc $FLAGS $DEFS -c $SRC/$s.hip -o $B/$s.o"
done | xargs -P 8 -I{} bash -c '{}'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $HERE/libyta_$NAME.so $B/*.o
echo built $HERE/libyta_$NAME.so
