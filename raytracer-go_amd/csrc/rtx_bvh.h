// rtx_bvh.h — GPU build of the reference's BVH over a World of spheres (rtx_bvh.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_layout.h"

namespace rtxd {
// NewBVHFromWorld (bvh.go:138-185) of spheres[0..n) in World.Add order, the k-th NewBVH
// call drawing Intn(3) from word draw0 + k of the global host stream of
// `seed`, written as the threaded pre-order entries rtx_scene_create would emit for the
// flattened tree.  Runs on the current device; build_ms = host wall time of the build.
hipError_t build_sphere_bvh(const rtx_sphere* spheres, uint32_t n, uint64_t seed, uint64_t draw0,
                            std::vector<rtx_entry>& out, double* build_ms);
}  // namespace rtxd
