#!/bin/bash
# Build a variant of libyta.so with extra -D flags into tools/variants/libyta_<name>.so
# (git-ignored, travels to the GPU box; select it with YTA_LIBRARY=<path>).
# usage: tools/build_variant.sh <name> -DYTA_BLK1=512 -DYTA_LDS1_KB=75 ...
set -e
name=$1; shift
cd "$(dirname "$0")/../yolo_tracking_amd/csrc"
out=../../tools/variants/build_$name
mkdir -p $out
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -munsafe-fp-atomics $*"
objs=""
for s in util kat bytetrack ocsort deepocsort hybridsort gsi reid cmc ecc osnet; do
  /opt/rocm/bin/hipcc $FLAGS -c $s.hip -o $out/$s.o 2>/dev/null &
  objs="$objs $out/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/variants/libyta_$name.so $objs
echo built tools/variants/libyta_$name.so
