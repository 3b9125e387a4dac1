#!/bin/bash
# Build an A/B variant of librtx.so with extra compile definitions into abl/librtx_<name>.so
# (run here, on the CPU; scripts/gpu_ab_libs.sh times it against the in-tree build on the GPU).
#   scripts/build_ab.sh <name> "-DRTX_ASM_STEP=0 ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1
DEFS=$2
B=abl/build_$NAME
mkdir -p "$B"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result $DEFS"
cd raytracer-go_amd
$HIPCC $FLAGS -Xclang -target-feature -Xclang -packed-fp32-ops -c csrc/rtx_kernel.hip -o ../$B/rtx_kernel.o 2>&1 |
    grep -v "packed-fp32-ops' is not a recognized feature" || true
for f in rtx_capi rtx_ppm rtx_bvh rtx_topology rtx_collapse; do
    $HIPCC $FLAGS -c csrc/$f.hip -o ../$B/$f.o &
done
wait
$HIPCC $FLAGS -shared -o ../abl/librtx_$NAME.so ../$B/*.o -Wl,-rpath,/opt/rocm/lib
echo "built abl/librtx_$NAME.so"
