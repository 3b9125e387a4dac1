// rtx_kernel.h — launch interface between the C-ABI layer and the megakernel.
#pragma once
#include <hip/hip_runtime.h>

namespace rtxd {
struct Params;
// Enqueue a render of p's region on `stream`; `count` selects the instantiation that
// accumulates the work counters into p.counters.
hipError_t launch_render(const Params& p, bool count, hipStream_t stream);
}  // namespace rtxd
