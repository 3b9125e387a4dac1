#!/bin/bash
# An A/B build of librtx.so with extra defines on the megakernel: abl/librtx_<name>.so, the other objects
# shared with the in-tree build.   bash scripts/build_ab_lib.sh nocoop -DRTX_COOP_CAMERA=0
set -eo pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
make -C raytracer-go_amd -s librtx.so
mkdir -p abl/build_$NAME
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -Xclang -target-feature -Xclang -packed-fp32-ops -c raytracer-go_amd/csrc/rtx_kernel.hip \
    -o abl/build_$NAME/rtx_kernel.o 2>&1 | { grep -v "packed-fp32-ops' is not a recognized feature" || true; }
B=raytracer-go_amd/build
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o abl/librtx_$NAME.so abl/build_$NAME/rtx_kernel.o $B/rtx_capi.o $B/rtx_ppm.o \
    $B/rtx_bvh.o $B/rtx_topology.o $B/rtx_collapse.o -Wl,-rpath,/opt/rocm/lib
echo "abl/librtx_$NAME.so"
