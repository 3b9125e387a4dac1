// rtx_kernel.hip — the path-tracing megakernel for gfx950 (MI355X).
//
// Replaces the per-pixel goroutine body of Camera.Render (camera.go:208-217):
// GetPixelColor (camera.go:254-263) = for k < spp { sum += GetColor(GetRay()) },
// then sum * (1/spp).  One work-item owns one pixel of a 16x16 tile (a 64-lane
// wave = 16x4 pixels) and walks its samples in order k = 0..spp-1, so the float32
// sum is accumulated in exactly the reference's order.  Each sample is independent
// (counter-based RNG keyed by global pixel index and k), so the value of a pixel
// does not depend on the tile, the region or the number of GPUs.
#include <hip/hip_runtime.h>

#include "rtx_device.h"
#include "rtx_kernel.h"

namespace rtxd {

constexpr int TILE_W = 16;
constexpr int TILE_H = 16;
constexpr int BLOCK = TILE_W * TILE_H;

template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void render_pixels(Params p) {
    const uint32_t lx = blockIdx.x * TILE_W + (threadIdx.x % TILE_W);
    const uint32_t lr = blockIdx.y * TILE_H + (threadIdx.x / TILE_W);
    if (lx >= p.width || lr >= p.rows) return;
    const uint32_t x = p.x0 + lx;
    const uint32_t y = p.y0 + p.rank + lr * p.world;
    const rtx_camera& c = p.cam;

    // camera.go:266-274: (pixel00 + du*i) + dv*j — the same for every sample.
    const V3 base = add(add(v3(c.pixel00[0], c.pixel00[1], c.pixel00[2]),
                            scale(v3(c.pixel_du[0], c.pixel_du[1], c.pixel_du[2]), (float)x)),
                        scale(v3(c.pixel_dv[0], c.pixel_dv[1], c.pixel_dv[2]), (float)y));
    const uint32_t pixel = y * c.image_width + x;

    Counters cnt{0, 0, 0, 0, 0};
    uint64_t draws = 0;
    V3 sum = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t k = 0; k < c.samples_per_pixel; ++k) {
        Rng rng;
        rng.init(p.seed, pixel, k);
        const Ray r = camera_ray(c, base, rng);
        const V3 col = trace_path<COUNT>(p, r, rng, cnt);
        sum = add(sum, col);  // camera.go:259
        if (COUNT) draws += rng.n;
    }
    const V3 avg = scale(sum, 1.0f / (float)c.samples_per_pixel);  // camera.go:261
    float* o = p.out + ((size_t)lr * p.width + lx) * 3;
    o[0] = avg.x;
    o[1] = avg.y;
    o[2] = avg.z;

    if (COUNT) {
        atomicAdd(&p.counters[0], (unsigned long long)c.samples_per_pixel);
        atomicAdd(&p.counters[1], (unsigned long long)cnt.segments);
        atomicAdd(&p.counters[2], (unsigned long long)cnt.node_visits);
        atomicAdd(&p.counters[3], (unsigned long long)cnt.prim_tests);
        atomicAdd(&p.counters[4], (unsigned long long)cnt.hits);
        atomicAdd(&p.counters[5], (unsigned long long)cnt.texel_fetches);
        atomicAdd(&p.counters[6], (unsigned long long)draws);
    }
}

hipError_t launch_render(const Params& p, bool count, hipStream_t stream) {
    if (p.width == 0 || p.rows == 0) return hipSuccess;
    const dim3 grid((p.width + TILE_W - 1) / TILE_W, (p.rows + TILE_H - 1) / TILE_H);
    if (count)
        hipLaunchKernelGGL(render_pixels<true>, grid, dim3(BLOCK), 0, stream, p);
    else
        hipLaunchKernelGGL(render_pixels<false>, grid, dim3(BLOCK), 0, stream, p);
    return hipGetLastError();
}

}  // namespace rtxd
