// rtx_kernel.h — launch interface between the C-ABI layer and the megakernel.
#pragma once
#include <hip/hip_runtime.h>

namespace rtxd {
struct Params;
// True when the render runs v3 (render_items + reduce_samples): the default unless a
// flag selects another schedule.  The caller then provides p.scratch / p.kn / p.sub.
bool uses_items(const Params& p, uint32_t flags);
// Enqueue a render of p's region on `stream`.  flags: RTX_FLAG_COUNTERS selects the
// instantiation that accumulates the work counters into p.counters; RTX_FLAG_KERNEL_*,
// RTX_FLAG_WAVE_GEOM and RTX_FLAG_NO_LDS select A/B variants (identical output).
hipError_t launch_render(const Params& p, uint32_t flags, hipStream_t stream);
}  // namespace rtxd
