// rtx_kernel.h — launch interface between the C-ABI layer and the megakernel.
#pragma once
#include <hip/hip_runtime.h>

namespace rtxd {
struct Params;
// Enqueue a render of p's region on `stream` (render_items + reduce_samples per sample
// chunk; the caller provides p.scratch / p.kn / p.sub).  flags: RTX_FLAG_COUNTERS selects
// the instantiation that accumulates the work counters into p.counters; RTX_FLAG_NO_LDS
// reads the scene from global memory (A/B, identical output).
// far != nullptr: a tiered walk: p is the near pass (p.tier = 1), *far the far
// pass over the same region (tier 2), per chunk: near pass, far pass, redo pass (the far layout
// over the samples whose records did not fit the near pass's queue, if any), then the reduction.
hipError_t launch_render(const Params& p, uint32_t flags, hipStream_t stream, const Params* far = nullptr);
// Where a launch reads the scene (RTX_SCENE_IN_LDS / LDS_CACHE / IN_HBM, rtx.h).
uint32_t scene_placement(const Params& p, uint32_t flags);
// Where a tiered walk reads both layouts: their common placement, or RTX_SCENE_IN_HBM when they differ.
uint32_t tier_placement(const Params& near, const Params& far, uint32_t flags);
}  // namespace rtxd
