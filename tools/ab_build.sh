#!/bin/bash
# A/B builds of the tracker engine: compile bytetrack.hip from a variant source directory (a copy of
# csrc with the variant's bytetrack.hip / bytetrack.hpp) and link it with the main build's other
# objects into tools/variants/libyta_<name>.so (select with YTA_LIBRARY=...).
# usage: tools/ab_build.sh <name> <variant_csrc_dir> [extra hipcc flags, e.g. -DYTA_LDSL_KB=39]
set -e
name=$1; src=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/yolo_tracking_amd/csrc/build
mkdir -p $R/tools/variants
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -munsafe-fp-atomics $*"
/opt/rocm/bin/hipcc $FLAGS -I$R/yolo_tracking_amd/csrc -c $src/bytetrack.hip -o $src/bytetrack_$name.o
objs=$(ls $B/*.o | grep -v '/bytetrack.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/tools/variants/libyta_$name.so $objs $src/bytetrack_$name.o
echo built tools/variants/libyta_$name.so
