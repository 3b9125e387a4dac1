// rtx_kernel.hip — the path-tracing megakernel for gfx950 (MI355X).
//
// Replaces the per-pixel goroutine body of Camera.Render (camera.go:208-217):
// GetPixelColor (camera.go:254-263) = for k < spp { sum += GetColor(GetRay()) },
// then sum * (1/spp).  Every pixel's samples are added in order k = 0..spp-1, so the
// float32 sum is the reference's.  Every sample is independent (counter-based RNG
// keyed by global pixel index and k), so a pixel's value does not depend on the tile,
// the region, the scheduling or the number of GPUs.
//
// Four schedules of the same per-sample code (rtx_device.h), identical output:
//  v3 render_items  (default) persistent waves over (pixel, sample) items; colours go
//                   to an HBM scratch and reduce_samples sums them in sample order.
//  v1 render_wave   one 8x8 tile per wave, one pixel per lane, path regeneration
//                   (RTX_FLAG_KERNEL_V1; RTX_FLAG_WAVE_GEOM variants).
//  v2 render_pool   persistent waves over a pool of pixels fed by a global tile queue;
//                   lanes take any idle pixel of the pool (RTX_FLAG_KERNEL_POOL).
//  v0 render_pixels thread per pixel, samples in a plain loop (the first version).
// v1-v3 step every traversing lane through BVH entries (three per wave vote) and shade
// in batches: once `shade_thresh` lanes of the wave wait (or none traverses), all
// waiting lanes shade together, so shading and its Philox blocks run in lockstep.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "rtx_device.h"
#include "rtx_kernel.h"

namespace rtxd {

__device__ __forceinline__ void flush_counters(const Params& p, uint64_t samples, const Counters& cnt) {
    atomicAdd(&p.counters[0], (unsigned long long)samples);
    atomicAdd(&p.counters[1], (unsigned long long)cnt.segments);
    atomicAdd(&p.counters[2], (unsigned long long)cnt.node_visits);
    atomicAdd(&p.counters[3], (unsigned long long)cnt.prim_tests);
    atomicAdd(&p.counters[4], (unsigned long long)cnt.hits);
    atomicAdd(&p.counters[5], (unsigned long long)cnt.texel_fetches);
    atomicAdd(&p.counters[6], (unsigned long long)cnt.draws);
    if (cnt.cache_hits) atomicAdd(&p.counters[15], (unsigned long long)cnt.cache_hits);
}

__device__ __forceinline__ void flush_sched(const Params& p, uint64_t wi, uint64_t ls, uint64_t sp, uint64_t sl) {
    atomicAdd(&p.counters[8], (unsigned long long)wi);
    atomicAdd(&p.counters[9], (unsigned long long)ls);
    atomicAdd(&p.counters[10], (unsigned long long)sp);
    atomicAdd(&p.counters[11], (unsigned long long)sl);
}

// ------------------------------------------------------------------------------------
// v0: thread per pixel, samples in a loop, traversal from global memory.
// ------------------------------------------------------------------------------------
constexpr int TILE_W = 16;
constexpr int TILE_H = 16;
constexpr int BLOCK = TILE_W * TILE_H;

template <bool COUNT, bool QUADS>
__global__ __launch_bounds__(BLOCK) void render_pixels(Params p) {
    const uint32_t lx = blockIdx.x * TILE_W + (threadIdx.x % TILE_W);
    const uint32_t lr = blockIdx.y * TILE_H + (threadIdx.x / TILE_W);
    if (lx >= p.width || lr >= p.rows) return;
    const uint32_t x = p.x0 + lx;
    const uint32_t y = p.y0 + p.rank + lr * p.world;
    const rtx_camera& c = p.cam;
    const V3 base = pixel_base(c, x, y);
    PathRng rng{(uint32_t)p.seed, (uint32_t)(p.seed >> 32), y * c.image_width + x, 0};
    Counters cnt{0, 0, 0, 0, 0, 0};
    const SceneRef E = scene_ref(p.entries, p.n_entries, p.materials);
    V3 sum = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t k = 0; k < c.samples_per_pixel; ++k) {
        rng.sample = k;
        Ray r = camera_ray(c, base, rng, cnt.draws);
        V3 thr = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f), col = acc;
        for (uint32_t seg = 0; seg < c.max_depth; ++seg) {  // ray.go:33 depth limit
            if (COUNT) ++cnt.segments;
            Trav t;
            trav_begin(t, r);
            while (t.i < 16 * p.n_entries) trav_step<COUNT, QUADS>(t, r, E, cnt);
            if (shade<COUNT, QUADS>(p, E, t, seg, r, thr, acc, rng, cnt, col)) break;
        }
        sum = add(sum, col);  // camera.go:259 (col = 0 when the depth ran out)
    }
    const V3 avg = scale(sum, 1.0f / (float)c.samples_per_pixel);  // camera.go:261
    float* o = p.out + ((size_t)lr * p.width + lx) * 3;
    o[0] = avg.x;
    o[1] = avg.y;
    o[2] = avg.z;
    if (COUNT) flush_counters(p, c.samples_per_pixel, cnt);
}

// ------------------------------------------------------------------------------------
// Traversal phase shared by v1 and v2.  Lane modes: 0 = traversing, 1 and 2 = waiting
// for the shading phase, 3 = neither.  Runs BVH steps until at least `thresh` lanes
// wait or none traverses.  Each traversing lane takes one entry (box or sphere, by its
// tag) per iteration.  (Separate box and sphere batches, steered by link-type bits in
// the entries, were measured: the extra decode per step cost more than the reduced
// divergence saved, DESIGN.md.)
// ------------------------------------------------------------------------------------
// STEPS > 1 takes up to STEPS entries per lane between two wave votes.  (A branch-free
// step that evaluates the box and the sphere test on every lane measured 8 % slower:
// most waves hold only box entries at a step, and the branch skips the sphere test.)
template <bool COUNT, int STEPS = 1, bool QUADS = false, bool FIXED = false, bool HYB = false, bool BATCH = false>
__device__ __forceinline__ void traverse_phase(uint32_t& mode, Trav& t, const Ray& r, const SceneRef E,
                                               uint32_t n_entries, uint32_t thresh, Counters& cnt,
                                               uint64_t& wave_iters, uint64_t& lane_steps, uint64_t& shade_phases,
                                               uint64_t& shade_lanes, uint64_t& idle_lanes, uint32_t prim_batch = 0) {
    for (;;) {
        // Every lane steps: one that is not traversing (or finishes early) waits on the
        // sentinel, t.i = 16 * n_entries, where a step changes nothing — cheaper than masking
        // the wave per step.
        uint32_t done = 0;  // COUNT: lane-steps that tested an entry (a lane on the sentinel idles)
        if constexpr (BATCH) {
#pragma unroll
            for (int s = 0; s < STEPS; ++s)
                done += trav_step_batched<COUNT, QUADS, FIXED, HYB>(t, r, E, cnt, 16 * n_entries, prim_batch);
        } else {
#pragma unroll
            for (int s = 0; s < STEPS; ++s) {
                if (COUNT) done += (uint32_t)__popcll(ballot(t.i < 16 * n_entries));
                trav_step<COUNT, QUADS, FIXED, HYB>(t, r, E, cnt);
            }
        }
        // votes on single compares, combined with SALU (a vote on a combined condition was
        // materialised with two extra VALU)
        const uint64_t walking = ballot(mode == 0), at_end = ballot(t.i >= 16 * n_entries);
        if (mode == 0 && t.i >= 16 * n_entries) mode = 1;
        const uint64_t trav = walking & ~at_end;
        const uint64_t pend = ballot(mode - 1u < 2u);  // mode 1 or 2
        if (COUNT) {
            ++wave_iters;
            lane_steps += done;
            idle_lanes += (uint64_t)__popcll(ballot(mode == 3));
        }
        if (trav == 0 || (uint32_t)__popcll(pend) >= thresh) {
            if (COUNT) {
                ++shade_phases;
                shade_lanes += (uint64_t)__popcll(pend);
            }
            return;
        }
    }
}

// ------------------------------------------------------------------------------------
// v1: wave loop, one pixel per lane, path regeneration, batched shading.
//
// PERSIST = false (default): one wave per 8x8 tile; a lane idles once its pixel is finished
// until the wave's slowest pixel is (measured: 26 % of lane slots at the headline
// config).  PERSIST = true: the grid is the device's resident capacity; a wave claims
// 8x8 tiles from a global counter and hands their pixels, in order, to its lanes as
// they finish, so its lanes stay on one or two neighbouring tiles (per-lane claims from
// the global counter scattered a wave over the whole claim frontier and lost 24 % per
// iteration to incoherence).  A pixel is still traced by one lane, samples
// k = 0..spp-1 in order, so its float32 sum is the reference's whatever the schedule.
// Measured at 100 spp: PERSIST raises traversal lane use from 0.50 to 0.62 but costs
// 15 % more cycles per iteration (divergence grows with the active lanes), a net loss.
// ------------------------------------------------------------------------------------
enum : uint32_t { M_TRAV = 0, M_SHADE = 1, M_START = 2, M_DONE = 3, M_CLAIM = 4 };

// BLOCK = 64 * WX * WY threads: a WX x WY grid of waves, each an 8x8 pixel tile; one LDS
// copy of the scene per block.  MINW = minimum waves per SIMD requested from the
// register allocator (0 = compiler's choice).  STEPS: entries per lane between votes.
template <bool COUNT, bool USE_LDS, int WX, int WY, int MINW, int STEPS, bool PERSIST, bool QUADS>
__global__ __launch_bounds__(64 * WX * WY, MINW) void render_wave(Params p) {
    constexpr uint32_t WAVE_BLOCK = 64 * WX * WY;
    extern __shared__ float4 lds_entries[];
    SceneRef E;
    if constexpr (USE_LDS) {
        const uint32_t n4 = scene_float4s(p.n_entries, p.n_quads);  // entries, then the quad table
        for (uint32_t t = threadIdx.x; t < n4; t += WAVE_BLOCK) lds_entries[t] = p.entries[t];
        __syncthreads();
        E = scene_ref(lds_entries, p.n_entries, p.materials);
    } else {
        E = scene_ref(p.entries, p.n_entries, p.materials);
    }
    const uint32_t n_entries = p.n_entries;
    const uint32_t thresh = p.shade_thresh;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const rtx_camera& c = p.cam;
    const uint32_t spp = c.samples_per_pixel;
    const uint32_t tiles_x = (p.width + 7u) / 8u;
    const uint32_t n_tiles = tiles_x * ((p.rows + 7u) / 8u);
    uint32_t cur_tile = 0, cursor = 64u;  // PERSIST: the wave's tile and its next pixel (uniform)
    bool exhausted = false;

    uint32_t lx = blockIdx.x * (8u * WX) + (wave % WX) * 8u + (lane & 7u);
    uint32_t lr = blockIdx.y * (8u * WY) + (wave / WX) * 8u + (lane >> 3);
    const bool active = !PERSIST && lx < p.width && lr < p.rows;
    V3 base = pixel_base(c, p.x0 + lx, p.y0 + p.rank + lr * p.world);
    uint32_t mode = PERSIST ? M_CLAIM : (active ? M_START : M_DONE);
    uint32_t seg = 0, pixels_done = 0;
    V3 sum = v3(0.0f, 0.0f, 0.0f);
    V3 thr = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f);
    Ray r{v3(0, 0, 0), v3(0, 0, 0)};
    PathRng rng{(uint32_t)p.seed, (uint32_t)(p.seed >> 32),
                (p.y0 + p.rank + lr * p.world) * c.image_width + p.x0 + lx, 0};
    Trav t{};
    t.i = 16 * p.n_entries;  // on the sentinel until its first ray
    Counters cnt{0, 0, 0, 0, 0, 0};
    uint64_t wave_iters = 0, lane_steps = 0, shade_phases = 0, shade_lanes = 0;
    uint64_t trav_cycles = 0, shade_cycles = 0, clk = 0, idle_lanes = 0;  // COUNT only

    for (;;) {
        if (COUNT) clk = __builtin_amdgcn_s_memtime();
        traverse_phase<COUNT, STEPS, QUADS>(mode, t, r, E, n_entries, thresh, cnt, wave_iters, lane_steps, shade_phases,
                                     shade_lanes, idle_lanes);
        if (COUNT) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            trav_cycles += now - clk;
            clk = now;
        }
        if (ballot(mode != M_DONE) == 0) break;

        // ---- shading phase ----------------------------------------------------------
        // The scatter samples of this phase, drawn by the whole wave together.
        const Scatter sc = coop_scatter<QUADS>(p, E, rng, seg + 1, mode == M_SHADE ? t.hit : -1);
        bool ready = false;                // a ray to trace (continued path or new sample)
        bool fresh = mode == M_START;      // the lane needs its pixel's next sample
        if (mode == M_SHADE) {
            V3 color;
            bool done = shade<COUNT, QUADS>(p, E, t, seg, r, thr, acc, rng, cnt, color, &sc);
            ++seg;
            if (!done && seg == c.max_depth) {  // depth exhausted: GetColor(0) = 0 (ray.go:33)
                done = true;
                color = acc;
            }
            if (done) {
                sum = add(sum, color);  // camera.go:259
                ++rng.sample;
                fresh = true;
            } else {
                ready = true;
            }
        }
        // New samples, at one program point for the whole wave (camera_ray's Philox runs
        // in lockstep).  Loops only for max depth 0 (every sample black) and ragged claims.
        for (;;) {
            if (fresh && rng.sample >= spp) {  // pixel finished (camera.go:261)
                const V3 avg = scale(sum, 1.0f / (float)spp);
                float* o = p.out + ((size_t)lr * p.width + lx) * 3;
                o[0] = avg.x;
                o[1] = avg.y;
                o[2] = avg.z;
                ++pixels_done;
                fresh = false;
                mode = PERSIST ? M_CLAIM : M_DONE;
            }
            if constexpr (PERSIST) {  // lanes without a pixel take the next ones of the wave's tile
                for (;;) {
                    const uint64_t wm = ballot(mode == M_CLAIM);
                    if (wm == 0) break;
                    if (cursor >= 64u && !exhausted) {  // claim the next 8x8 tile (wave-uniform)
                        uint32_t tl = 0;
                        if (lane == 0) tl = atomicAdd(p.tile_counter, 1u);
                        cur_tile = (uint32_t)__shfl((int)tl, 0);
                        cursor = 0;
                        exhausted = cur_tile >= n_tiles;
                    }
                    if (exhausted) {
                        if (mode == M_CLAIM) mode = M_DONE;
                        break;
                    }
                    const uint32_t rank = (uint32_t)__popcll(wm & ((1ull << lane) - 1ull));
                    if (mode == M_CLAIM && rank < 64u - cursor) {
                        const uint32_t l = cursor + rank;
                        lx = (cur_tile % tiles_x) * 8u + (l & 7u);
                        lr = (cur_tile / tiles_x) * 8u + (l >> 3);
                        if (lx < p.width && lr < p.rows) {  // else: outside a ragged tile, claim again
                            const uint32_t x = p.x0 + lx, y = p.y0 + p.rank + lr * p.world;
                            base = pixel_base(c, x, y);
                            rng.pixel = y * c.image_width + x;
                            rng.sample = 0;
                            sum = v3(0.0f, 0.0f, 0.0f);
                            fresh = true;
                            mode = M_START;
                        }
                    }
                    const uint32_t taken = (uint32_t)__popcll(wm);
                    cursor = cursor + taken > 64u ? 64u : cursor + taken;
                }
            }
            if (fresh && rng.sample < spp) {
                r = camera_ray(c, base, rng, cnt.draws);  // GetRay, camera.go:257
                thr = v3(1.0f, 1.0f, 1.0f);
                acc = v3(0.0f, 0.0f, 0.0f);
                seg = 0;
                if (c.max_depth > 0) {
                    fresh = false;
                    ready = true;
                } else {
                    sum = add(sum, acc);  // max depth 0: GetColor returns black
                    ++rng.sample;
                }
            }
            if (ballot(fresh) == 0) break;
        }
        if (ready) {  // begin a segment: world.Hit (ray.go:36)
            if (COUNT) ++cnt.segments;
            trav_begin(t, r);
            mode = n_entries > 0 ? M_TRAV : M_SHADE;
        }
        if (COUNT) shade_cycles += __builtin_amdgcn_s_memtime() - clk;
    }
    if (COUNT) {
        flush_counters(p, (uint64_t)pixels_done * spp, cnt);
        if (lane == 0) {
            flush_sched(p, wave_iters, lane_steps / STEPS, shade_phases, shade_lanes);
            atomicAdd(&p.counters[12], (unsigned long long)trav_cycles);
            atomicAdd(&p.counters[13], (unsigned long long)shade_cycles);
            atomicAdd(&p.counters[14], (unsigned long long)idle_lanes);
        }
    }
}

// ------------------------------------------------------------------------------------
// v3: persistent waves over (pixel, sample) items; the sum is formed afterwards.
//
// GetPixelColor's float32 sum (camera.go:256-261) must add a pixel's samples in order
// k = 0..spp-1, which ties v1 to one lane per pixel: a wave lasts as long as its slowest
// pixel, and an image with fewer 8x8 tiles than the device has wave slots (the Cornell
// box: 5625 tiles, 4096 slots) leaves the GPU part-idle.  v3 spends HBM instead: every
// sample's colour is stored (12 B; 12.4 GB for 1920x1080x500 of the 288 GB), and
// reduce_samples adds each pixel's colours in k order afterwards — the same float32
// operations in the same order, so the same bits.  The work is then a pool of
// independent items: a wave claims units of (8x8 tile, `sub` consecutive samples) from a
// global counter and hands the unit's items to its lanes in sample-major order as they
// finish, so a wave stays on one tile (coherent rays) and no lane waits for another.
// Samples beyond the scratch budget run in chunks [k0, k0 + kn); the running sum of a
// pixel is carried in the output between chunks.
// ------------------------------------------------------------------------------------
template <bool COUNT, bool USE_LDS, bool QUADS, bool NOISE, int WAVES = 8, int MINW = 0, bool HYB = false>
__global__ __launch_bounds__(64 * WAVES, MINW) void render_items(Params p) {
    constexpr uint32_t WAVE_BLOCK = 64 * WAVES, STEPS = 6;  // walk steps between two wave votes (A/B with primitive batching: 4 +0.7 %, 8 +0.8 %, 12 +1.3 %)
    extern __shared__ float4 lds_entries[];
    SceneRef E;
    if constexpr (USE_LDS) {
        // scene_ref_fixed: the walk addresses LDS directly, so the copy must start at 0
        if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)lds_entries != 0u) __builtin_trap();
        const uint32_t m = p.n_entries + 1, nq4 = 4 * p.n_quads;
        for (uint32_t t = threadIdx.x; t < m; t += WAVE_BLOCK) {
            lds_entries[t] = p.entries[t];
            lds_entries[LDS_B / 16 + t] = p.entries[m + t];
        }
        for (uint32_t t = threadIdx.x; t < nq4; t += WAVE_BLOCK) lds_entries[LDS_B / 16 + m + t] = p.entries[2 * m + t];
        const uint32_t mo = lds_mat_offset(p.n_entries, p.n_quads, p.n_materials) / 16;
        const float4* mg = reinterpret_cast<const float4*>(p.materials);
        for (uint32_t t = threadIdx.x; t < 2 * p.n_materials; t += WAVE_BLOCK) lds_entries[mo + t] = mg[t];
        __syncthreads();
        E = scene_ref_fixed(lds_entries, p.n_entries, p.n_quads, p.n_materials);
    } else {
        E = scene_ref(p.entries, p.n_entries, p.materials);
        if constexpr (HYB) {  // the scene's top levels, stored first, cached in LDS (fixed layout)
            if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)lds_entries != 0u) __builtin_trap();
            const uint32_t m = p.n_entries + 1;
            for (uint32_t t = threadIdx.x; t < p.n_hot; t += WAVE_BLOCK) {
                lds_entries[t] = p.entries[t];
                lds_entries[LDS_B / 16 + t] = p.entries[m + t];
            }
            __syncthreads();
            E.la = lds_entries;
            E.lb = lds_entries + LDS_B / 16;
            E.hot = 16 * p.n_hot;
        }
    }
    const uint32_t n_entries = p.n_entries;
    const uint32_t thresh = p.shade_thresh;
    const uint32_t lane = threadIdx.x & 63u;
    const rtx_camera& c = p.cam;
    const uint32_t tiles_x = (p.width + 7u) / 8u;
    const uint32_t n_tiles = tiles_x * ((p.rows + 7u) / 8u);
    const uint32_t nsub = (p.kn + p.sub - 1u) / p.sub;
    const uint64_t n_units = (uint64_t)n_tiles * nsub;
    const size_t npix = (size_t)p.width * p.rows;

    // the wave's unit (uniform): tile, first sample, items, next item
    uint32_t u_tile = 0, u_k0 = 0, u_items = 0, cursor = 0;
    bool exhausted = false;

    uint32_t mode = M_CLAIM, seg = 0, items_done = 0;
    size_t pix = 0;  // region-linear pixel of the lane's item
    V3 base = v3(0.0f, 0.0f, 0.0f);
    V3 thr = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f);
    Ray r{v3(0, 0, 0), v3(0, 0, 0)};
    PathRng rng{(uint32_t)p.seed, (uint32_t)(p.seed >> 32), 0u, 0u};
    Trav t{};
    t.i = 16 * p.n_entries;  // on the sentinel until its first ray
    Counters cnt{0, 0, 0, 0, 0, 0};
    uint64_t wave_iters = 0, lane_steps = 0, shade_phases = 0, shade_lanes = 0;
    uint64_t trav_cycles = 0, shade_cycles = 0, clk = 0, idle_lanes = 0;  // COUNT only

    auto store = [&](V3 col) {  // the item's colour, GetColor's result for sample k
        float* o = p.scratch + ((size_t)(rng.sample - p.k0) * npix + pix) * 3;
        o[0] = col.x;
        o[1] = col.y;
        o[2] = col.z;
        ++items_done;
    };

    for (;;) {
        if (COUNT) clk = __builtin_amdgcn_s_memtime();
        // primitive batching only for a scene in LDS: a lane that waits re-reads its entry, which
        // from HBM cost config 4 +34 %
        traverse_phase<COUNT, STEPS, QUADS, USE_LDS, HYB, USE_LDS>(mode, t, r, E, n_entries, thresh, cnt, wave_iters,
                                                              lane_steps, shade_phases, shade_lanes, idle_lanes,
                                                              p.prim_batch);
        if (COUNT) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            trav_cycles += now - clk;
            clk = now;
        }
        if (ballot(mode != M_DONE) == 0) break;

        // ---- shading phase ----------------------------------------------------------
        const Scatter sc = coop_scatter<QUADS>(p, E, rng, seg + 1, mode == M_SHADE ? t.hit : -1);
        bool ready = false;
        if (mode == M_SHADE) {
            V3 color;
            bool done = shade<COUNT, QUADS, NOISE>(p, E, t, seg, r, thr, acc, rng, cnt, color, &sc);
            ++seg;
            if (!done && seg == c.max_depth) {  // depth exhausted: GetColor(0) = 0 (ray.go:33)
                done = true;
                color = acc;
            }
            if (done) {
                store(color);
                mode = M_CLAIM;
            } else {
                ready = true;
            }
        }
        // Lanes without an item take the next ones of the wave's unit; new camera rays
        // at one program point.  Loops only for max depth 0 and ragged tiles.
        for (;;) {
            const uint64_t wm = ballot(mode == M_CLAIM);
            if (wm == 0) break;
            if (cursor >= u_items && !exhausted) {  // claim the next unit (wave-uniform)
                uint32_t un = 0;
                if (lane == 0) un = atomicAdd(p.tile_counter, 1u);
                const uint64_t uu = (uint32_t)__shfl((int)un, 0);
                exhausted = uu >= n_units;
                if (!exhausted) {
                    u_tile = (uint32_t)(uu / nsub);
                    u_k0 = p.k0 + (uint32_t)(uu % nsub) * p.sub;
                    const uint32_t cnt_k = min(p.sub, p.k0 + p.kn - u_k0);
                    u_items = 64u * cnt_k;
                    cursor = 0;
                }
            }
            if (exhausted) {
                if (mode == M_CLAIM) mode = M_DONE;
                break;
            }
            const uint32_t rank = (uint32_t)__popcll(wm & ((1ull << lane) - 1ull));
            bool got = false;
            if (mode == M_CLAIM && rank < u_items - cursor) {
                const uint32_t j = cursor + rank, l = j & 63u;  // sample-major within the unit
                const uint32_t lx = (u_tile % tiles_x) * 8u + (l & 7u);
                const uint32_t lr = (u_tile / tiles_x) * 8u + (l >> 3);
                if (lx < p.width && lr < p.rows) {  // else: outside a ragged tile, claim again
                    const uint32_t x = p.x0 + lx, y = p.y0 + p.rank + lr * p.world;
                    base = pixel_base(c, x, y);
                    rng.pixel = y * c.image_width + x;
                    rng.sample = u_k0 + (j >> 6);
                    pix = (size_t)lr * p.width + lx;
                    got = true;
                }
            }
            const uint32_t taken = (uint32_t)__popcll(wm);
            cursor = cursor + taken > u_items ? u_items : cursor + taken;
            if (got) {
                r = camera_ray<!COUNT>(c, base, rng, cnt.draws);  // GetRay, camera.go:257
                thr = v3(1.0f, 1.0f, 1.0f);
                acc = v3(0.0f, 0.0f, 0.0f);
                seg = 0;
                if (c.max_depth > 0) {
                    mode = M_START;
                    ready = true;
                } else {
                    store(acc);  // max depth 0: GetColor returns black
                }
            }
        }
        if (ready) {  // begin a segment: world.Hit (ray.go:36)
            if (COUNT) ++cnt.segments;
            trav_begin(t, r);
            mode = n_entries > 0 ? M_TRAV : M_SHADE;
        }
        if (COUNT) shade_cycles += __builtin_amdgcn_s_memtime() - clk;
    }
    if (COUNT) {
        flush_counters(p, items_done, cnt);
        if (lane == 0) {
            flush_sched(p, wave_iters, lane_steps / STEPS, shade_phases, shade_lanes);
            atomicAdd(&p.counters[12], (unsigned long long)trav_cycles);
            atomicAdd(&p.counters[13], (unsigned long long)shade_cycles);
            atomicAdd(&p.counters[14], (unsigned long long)idle_lanes);
        }
    }
}

// GetPixelColor's sum over the stored colours of samples [k0, k0 + kn), in k order
// (camera.go:256-259), continued from the running sum in `out` when k0 > 0; the last
// chunk applies Scale(1/spp) (camera.go:261).  One thread per pixel, coalesced reads.
__global__ __launch_bounds__(256) void reduce_samples(Params p, uint32_t last) {
    const size_t npix = (size_t)p.width * p.rows;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= npix) return;
    float* o = p.out + i * 3;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    if (p.k0 > 0) {
        sx = o[0];
        sy = o[1];
        sz = o[2];
    }
    const float* src = p.scratch + i * 3;
    for (uint32_t k = 0; k < p.kn; ++k, src += npix * 3) {
        sx = sx + src[0];
        sy = sy + src[1];
        sz = sz + src[2];
    }
    if (last) {
        const float inv = 1.0f / (float)p.cam.samples_per_pixel;
        sx = sx * inv;
        sy = sy * inv;
        sz = sz * inv;
    }
    o[0] = sx;
    o[1] = sy;
    o[2] = sz;
}

// ------------------------------------------------------------------------------------
// v2: persistent waves over a pool of pixels fed by a global tile queue.
//
// v1 keeps one pixel per lane, so a wave lasts as long as its most expensive pixel
// (a sky pixel needs ~1 segment per sample, a glass one ~8).  v2 decouples lanes from
// pixels: each wave owns CH chunks of 64 pixels (8x8 tiles of the region, taken from
// a global atomic queue) = a pool of POOL_SLOTS pixels in LDS, each with its running
// float32 sum and next sample index.  A free lane claims any idle pixel of the pool
// and traces its next sample; a pixel has at most ONE sample in flight, so samples
// still complete — and are summed — in order k = 0..spp-1 (camera.go:256-261).  When
// all pixels of a chunk are done, the chunk is refilled from the queue.  The grid is
// sized to the device's resident capacity; every wave exits once the queue is empty
// and its chunks are finished, or when its watchdog fires.
// ------------------------------------------------------------------------------------
constexpr int POOL_BLOCK = 512;  // 8 waves share one LDS copy of the scene
constexpr int POOL_WAVES = POOL_BLOCK / 64;
enum : uint32_t { Q_TRAV = 0, Q_SHADE = 1, Q_FREE = 2, Q_IDLE = 3 };
constexpr uint32_t ST_INFLIGHT = 0x80000000u, ST_INVALID = 0x40000000u, ST_K = 0x00FFFFFFu;

template <int NCH>  // chunks (8x8 tiles) per wave
struct WavePool {
    static constexpr int SLOTS = NCH * 64;
    float sx[SLOTS], sy[SLOTS], sz[SLOTS];
    uint32_t st[SLOTS];        // next sample index | INFLIGHT | INVALID
    int32_t tile[NCH];         // tile of the region held by chunk c, -1 = empty
    uint32_t remaining[NCH];   // pixels of chunk c not finished yet
    uint32_t origin[NCH];      // region x0 | y0 << 16 of the tile
    uint32_t pad[NCH];
};
static_assert(sizeof(WavePool<2>) % 16 == 0 && sizeof(WavePool<4>) % 16 == 0, "keep the scene copy 16-B aligned");

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool COUNT, bool USE_LDS, int NCH>
__global__ __launch_bounds__(POOL_BLOCK) void render_pool(Params p) {
    using Pool = WavePool<NCH>;
    constexpr uint32_t CH = NCH, POOL_SLOTS = Pool::SLOTS;
    extern __shared__ float4 lds_dyn[];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    Pool* wp = reinterpret_cast<Pool*>(lds_dyn) + wave;
    SceneRef E;
    if constexpr (USE_LDS) {
        float4* scene = lds_dyn + (POOL_WAVES * sizeof(Pool)) / 16;
        const uint32_t n4 = scene_float4s(p.n_entries, 0);
        for (uint32_t t = threadIdx.x; t < n4; t += POOL_BLOCK) scene[t] = p.entries[t];
        E = scene_ref(scene, p.n_entries, p.materials);
    } else {
        E = scene_ref(p.entries, p.n_entries, p.materials);
    }
    const uint32_t n_entries = p.n_entries;
    const uint32_t thresh = p.shade_thresh;
    const rtx_camera& c = p.cam;
    const uint32_t spp = c.samples_per_pixel;
    const uint32_t tiles_x = (p.width + 7) / 8;
    const uint32_t n_tiles = tiles_x * ((p.rows + 7) / 8);

    // Take the next 8x8 tile of the region into chunk ch (wave-uniform call).
    auto load_chunk = [&](uint32_t ch) {
        uint32_t tl = 0;
        if (lane == 0) tl = atomicAdd(p.tile_counter, 1u);
        tl = __shfl(tl, 0);
        const bool has = tl < n_tiles;
        const uint32_t ox = (tl % tiles_x) * 8, oy = (tl / tiles_x) * 8;
        const uint32_t lx = ox + (lane & 7u), lr = oy + (lane >> 3);
        const bool valid = has && lx < p.width && lr < p.rows;
        const uint32_t s = ch * 64 + lane;
        wp->sx[s] = 0.0f;
        wp->sy[s] = 0.0f;
        wp->sz[s] = 0.0f;
        wp->st[s] = valid ? 0u : ST_INVALID;
        const uint32_t nvalid = (uint32_t)__popcll(ballot(valid));
        if (lane == 0) {
            wp->tile[ch] = has ? (int32_t)tl : -1;
            wp->remaining[ch] = nvalid;
            wp->origin[ch] = ox | (oy << 16);
        }
    };
    for (uint32_t ch = 0; ch < CH; ++ch) load_chunk(ch);
    __syncthreads();  // scene copy + pool init visible

    uint32_t mode = Q_FREE;
    bool begin = false;  // set up a new segment at the end of this shading phase
    uint32_t slot = 0, px = 0, py = 0, seg = 0;
    uint32_t cursor = 0;  // wave-uniform claim cursor over the pool
    V3 thr = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f);
    Ray r{v3(0, 0, 0), v3(0, 0, 0)};
    PathRng rng{(uint32_t)p.seed, (uint32_t)(p.seed >> 32), 0, 0};
    Trav t{};
    t.i = 16 * p.n_entries;  // on the sentinel until its first ray
    Counters cnt{0, 0, 0, 0, 0, 0};
    uint64_t samples = 0;
    uint64_t wave_iters = 0, lane_steps = 0, shade_phases = 0, shade_lanes = 0;
    uint64_t idle_lanes = 0;  // (v2: Q_IDLE lanes; not reported)
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint32_t iter = 0;

    for (;;) {
        // Watchdog: a wave never outlives p.watchdog_ticks (the grid always drains).
        if ((++iter & 255u) == 0 && __builtin_amdgcn_s_memrealtime() - t_start > p.watchdog_ticks) {
            if (lane == 0) atomicOr(p.error_flag, 1u);
            break;
        }
        traverse_phase<COUNT, 3>(mode, t, r, E, n_entries, thresh, cnt, wave_iters, lane_steps, shade_phases,
                                 shade_lanes, idle_lanes);

        // ---- shading phase: finish or continue paths ---------------------------------------
        if (mode == Q_SHADE) {
            V3 color = acc;
            bool done = c.max_depth == 0;  // GetColor(0) returns black (ray.go:33-35)
            if (!done) {
                done = shade<COUNT>(p, E, t, seg, r, thr, acc, rng, cnt, color);
                ++seg;
                if (!done && seg == c.max_depth) {  // depth exhausted
                    done = true;
                    color = acc;
                }
            }
            if (done) {  // sum += sample, in sample order (camera.go:259)
                wp->sx[slot] = wp->sx[slot] + color.x;
                wp->sy[slot] = wp->sy[slot] + color.y;
                wp->sz[slot] = wp->sz[slot] + color.z;
                const uint32_t kn = (wp->st[slot] & ST_K) + 1;
                wp->st[slot] = kn;  // clears INFLIGHT
                if (COUNT) ++samples;
                if (kn == spp) {  // pixel complete: sum * (1/spp), camera.go:261
                    const float inv = 1.0f / (float)spp;
                    float* o = p.out + ((size_t)py * p.width + px) * 3;
                    o[0] = wp->sx[slot] * inv;
                    o[1] = wp->sy[slot] * inv;
                    o[2] = wp->sz[slot] * inv;
                    atomicSub(&wp->remaining[slot >> 6], 1u);
                }
                mode = Q_FREE;
            } else {
                mode = Q_TRAV;
                begin = true;
            }
        }
        wave_sync();

        // ---- refill finished chunks from the global queue (wave-uniform) -------------------
        bool any_chunk = false;
        for (uint32_t ch = 0; ch < CH; ++ch) {
            if (wp->tile[ch] >= 0 && wp->remaining[ch] == 0) {
                load_chunk(ch);
                wave_sync();
            }
            any_chunk |= wp->tile[ch] >= 0;
        }
        if (!any_chunk && ballot(mode == Q_TRAV || mode == Q_SHADE) == 0) break;

        // ---- claim idle pixels for free lanes ------------------------------------------------
        const uint64_t freem = ballot(mode == Q_FREE || mode == Q_IDLE);
        if (mode == Q_FREE || mode == Q_IDLE) {
            const uint32_t rank = (uint32_t)__popcll(freem & ((1ull << lane) - 1ull));
            const uint32_t cand = (cursor + rank) % POOL_SLOTS;
            const uint32_t st = wp->st[cand];
            if ((st & (ST_INFLIGHT | ST_INVALID)) == 0 && (st & ST_K) < spp) {
                wp->st[cand] = st | ST_INFLIGHT;
                slot = cand;
                const uint32_t org = wp->origin[cand >> 6];
                const uint32_t j = cand & 63u;
                px = (org & 0xFFFFu) + (j & 7u);
                py = (org >> 16) + (j >> 3);
                const uint32_t x = p.x0 + px, y = p.y0 + p.rank + py * p.world;
                rng.pixel = y * c.image_width + x;
                rng.sample = st & ST_K;
                r = camera_ray(c, pixel_base(c, x, y), rng, cnt.draws);
                thr = v3(1.0f, 1.0f, 1.0f);
                acc = v3(0.0f, 0.0f, 0.0f);
                seg = 0;
                mode = Q_TRAV;
                begin = true;
                if (c.max_depth == 0) {
                    mode = Q_SHADE;  // finishes black at the next shading phase
                    begin = false;
                }
            } else {
                mode = Q_IDLE;
            }
        }
        cursor = (cursor + (uint32_t)__popcll(freem)) % POOL_SLOTS;

        // ---- begin the next segment (world.Hit, ray.go:36) for lanes that just scattered
        // or claimed a sample; lanes still mid-traversal keep their state ----------------------
        if (begin) {
            begin = false;
            if (COUNT) ++cnt.segments;
            trav_begin(t, r);
            if (n_entries == 0) mode = Q_SHADE;
        }
    }

    if (COUNT) {
        flush_counters(p, samples, cnt);
        if (lane == 0) flush_sched(p, wave_iters, lane_steps / 3, shade_phases, shade_lanes);
    }
}

// ------------------------------------------------------------------------------------
// launches
// ------------------------------------------------------------------------------------
constexpr uint32_t LDS_MAX_BYTES = 64 * 1024;

// LDS bytes of the scene copy: entries and the quad table.
inline size_t scene_lds_bytes(const Params& p) { return (size_t)scene_float4s(p.n_entries, p.n_quads) * 16; }

template <bool COUNT, int NCH>
hipError_t launch_pool(const Params& p, bool use_lds, hipStream_t stream) {
    const size_t shmem = POOL_WAVES * sizeof(WavePool<NCH>) + (use_lds ? scene_lds_bytes(p) : 0);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    e = use_lds
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, render_pool<COUNT, true, NCH>, POOL_BLOCK, shmem)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, render_pool<COUNT, false, NCH>, POOL_BLOCK, shmem);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const uint32_t tiles = ((p.width + 7) / 8) * ((p.rows + 7) / 8);
    uint32_t blocks = (uint32_t)(per_cu * cus);
    const uint32_t need = (tiles + POOL_WAVES * NCH - 1) / (POOL_WAVES * NCH);  // no wave starts empty-handed
    if (blocks > need) blocks = need;
    if (blocks == 0) blocks = 1;
    e = hipMemsetAsync(p.tile_counter, 0, 2 * sizeof(uint32_t), stream);  // queue head + watchdog flag
    if (e != hipSuccess) return e;
    if (use_lds)
        hipLaunchKernelGGL((render_pool<COUNT, true, NCH>), dim3(blocks), dim3(POOL_BLOCK), shmem, stream, p);
    else
        hipLaunchKernelGGL((render_pool<COUNT, false, NCH>), dim3(blocks), dim3(POOL_BLOCK), shmem, stream, p);
    return hipGetLastError();
}

template <bool COUNT, int WX, int WY, int MINW, int STEPS = 1, bool PERSIST = false, bool QUADS = false>
hipError_t launch_wave_geom(const Params& p, bool use_lds, hipStream_t stream) {
    const size_t shmem = use_lds ? scene_lds_bytes(p) : 0;
    const auto kern = use_lds ? render_wave<COUNT, true, WX, WY, MINW, STEPS, PERSIST, QUADS>
                              : render_wave<COUNT, false, WX, WY, MINW, STEPS, PERSIST, QUADS>;
    constexpr int block = 64 * WX * WY;
    if constexpr (PERSIST) {
        int dev = 0, cus = 0, per_cu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, shmem);
        if (e != hipSuccess) return e;
        if (per_cu < 1) per_cu = 1;
        const uint64_t tiles = (uint64_t)((p.width + 7) / 8) * ((p.rows + 7) / 8);
        uint64_t blocks = (uint64_t)per_cu * cus;
        if (p.grid_pct > 0 && p.grid_pct < 100) blocks = (blocks * p.grid_pct + 99) / 100;
        const uint64_t need = (tiles + WX * WY - 1) / (WX * WY);  // no wave starts without a tile
        if (blocks > need) blocks = need;
        if (blocks == 0) blocks = 1;
        e = hipMemsetAsync(p.tile_counter, 0, 2 * sizeof(uint32_t), stream);  // claim counter + flag
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(block), shmem, stream, p);
    } else {
        const dim3 grid((p.width + 8 * WX - 1) / (8 * WX), (p.rows + 8 * WY - 1) / (8 * WY));
        hipLaunchKernelGGL(kern, grid, dim3(block), shmem, stream, p);
    }
    return hipGetLastError();
}

// Block geometry of v1 (RTX_FLAG_WAVE_GEOM): waves per block and the register budget.
template <bool COUNT>
hipError_t launch_wave(const Params& p, uint32_t geom, bool use_lds, hipStream_t stream) {
    switch (geom) {
    case 1: return launch_wave_geom<COUNT, 2, 2, 0, 3, true>(p, use_lds, stream);   // persistent, claims tiles
    case 2: return launch_wave_geom<COUNT, 2, 2, 0, 1, true>(p, use_lds, stream);   // 1 step per vote
    case 3: return launch_wave_geom<COUNT, 2, 2, 0, 4, true>(p, use_lds, stream);   // 4 steps per vote
    case 4: return launch_wave_geom<COUNT, 4, 2, 0, 3, true>(p, use_lds, stream);   // 8 waves per block
    case 5: return launch_wave_geom<COUNT, 4, 2, 8, 3, true>(p, use_lds, stream);   // 8 waves, >= 8/SIMD
    case 6: return launch_wave_geom<COUNT, 1, 1, 0, 3, true>(p, use_lds, stream);   // 1 wave per block
    default: return launch_wave_geom<COUNT, 2, 2, 0, 3, false>(p, use_lds, stream); // one tile per wave
    }
}

// v3: chunks of p.kn samples (the scratch holds one chunk), each rendered by a
// resident-capacity grid of render_items and summed into p.out by reduce_samples.
template <bool COUNT, bool QUADS, bool NOISE, int WAVES = 8, int MINW = 0>
hipError_t launch_items(Params p, bool use_lds, hipStream_t stream) {
    // a scene too big for LDS: its top levels (p.n_hot entries) cached in LDS when the
    // device layout stored them first (RTX_HOT_ENTRIES=0 turns that off)
    const bool hyb = !use_lds && p.n_hot > 0 && !NOISE;
    const size_t shmem = use_lds ? lds_fixed_bytes(p.n_entries, p.n_quads, p.n_materials)
                                 : (hyb ? lds_hot_bytes(p.n_hot) : 0);
    const auto kern = use_lds ? render_items<COUNT, true, QUADS, NOISE, WAVES, MINW>
                              : (hyb ? render_items<COUNT, false, QUADS, NOISE, WAVES, MINW, !NOISE>
                                     : render_items<COUNT, false, QUADS, NOISE, WAVES, MINW>);
    constexpr int block = 64 * WAVES;
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, shmem);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const uint32_t spp = p.cam.samples_per_pixel, chunk = p.kn, sub = p.sub;
    const uint64_t tiles = (uint64_t)((p.width + 7) / 8) * ((p.rows + 7) / 8);
    const uint64_t npix = (uint64_t)p.width * p.rows;
    for (uint32_t k0 = 0; k0 < spp; k0 += chunk) {
        p.k0 = k0;
        p.kn = spp - k0 < chunk ? spp - k0 : chunk;
        if (sub == 0) {
            // Samples per unit: 8, or fewer when that leaves under 8 units per resident wave
            // (a small image's last units would run on a near-empty GPU).  Measured at 100 spp:
            // 1920x1080 8 -1.6 % vs 16; 400x225 2 -42 % vs 16; Cornell 600x600 8 -3 % vs 16.
            const uint64_t per_wave = tiles * p.kn / (8ull * WAVES * (uint64_t)per_cu * cus);
            p.sub = per_wave >= 8 ? 8u : (per_wave >= 4 ? 4u : (per_wave >= 2 ? 2u : 1u));
        }
        const uint64_t units = tiles * ((p.kn + p.sub - 1) / p.sub);
        uint64_t blocks = (uint64_t)per_cu * cus;
        if (blocks > (units + WAVES - 1) / WAVES) blocks = (units + WAVES - 1) / WAVES;  // no wave starts idle
        if (p.debug_launch)
            fprintf(stderr, "rtx v3: waves/wg %d, wgs/CU %d, CUs %d, grid %llu, sub %u, units %llu, lds %zu B\n", WAVES,
                    per_cu, cus, (unsigned long long)blocks, p.sub, (unsigned long long)units, shmem);
        e = hipMemsetAsync(p.tile_counter, 0, 2 * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(block), shmem, stream, p);
        hipLaunchKernelGGL(reduce_samples, dim3((uint32_t)((npix + 255) / 256)), dim3(256), 0, stream, p,
                           (uint32_t)(k0 + p.kn >= spp));
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

bool uses_items(const Params& p, uint32_t flags) {
    const bool work = p.width > 0 && p.rows > 0 && p.cam.samples_per_pixel > 0 && p.cam.max_depth > 0;
    if (p.has_noise) return work;  // Perlin scenes run v3 only (the NOISE instantiations)
    if (flags & (RTX_FLAG_KERNEL_V0 | RTX_FLAG_KERNEL_V1 | RTX_FLAG_KERNEL_POOL)) return false;
    if (((flags >> 24) & 7u) != 0) return false;  // RTX_FLAG_WAVE_GEOM tunes v1
    return work;
}

#ifndef RTX_HYB_WAVES  // the same for scenes in HBM with a 64 KB LDS cache of their top levels
#define RTX_HYB_WAVES 12
#define RTX_HYB_MINW 6
#endif
#ifndef RTX_V3_WAVES  // workgroup size and waves per SIMD of the default v3 kernel (A/B builds override)
#define RTX_V3_WAVES 8
#define RTX_V3_MINW 6
#endif

template <bool COUNT>
hipError_t launch_items_for(const Params& p, bool use_lds, hipStream_t stream) {
    if (p.has_noise) return p.n_quads ? launch_items<COUNT, true, true>(p, use_lds, stream)
                                      : launch_items<COUNT, false, true>(p, use_lds, stream);
    if (p.item_waves == 4)  // A/B: 4 waves per LDS copy of the scene
        return p.n_quads ? launch_items<COUNT, true, false, 4>(p, use_lds, stream)
                         : launch_items<COUNT, false, false, 4>(p, use_lds, stream);
    // 6 waves per SIMD: at most 80 VGPRs (the allocation granule is 8)
    if (!use_lds && p.n_hot > HOT_ENTRIES_8W)  // a 64 KB LDS cache: 12-wave workgroups, two per CU
        return p.n_quads ? launch_items<COUNT, true, false, RTX_HYB_WAVES, COUNT ? 0 : RTX_HYB_MINW>(p, use_lds, stream)
                         : launch_items<COUNT, false, false, RTX_HYB_WAVES, COUNT ? 0 : RTX_HYB_MINW>(p, use_lds, stream);
    return p.n_quads ? launch_items<COUNT, true, false, RTX_V3_WAVES, COUNT ? 0 : RTX_V3_MINW>(p, use_lds, stream)
                     : launch_items<COUNT, false, false, RTX_V3_WAVES, COUNT ? 0 : RTX_V3_MINW>(p, use_lds, stream);
}

hipError_t launch_render(const Params& p, uint32_t flags, hipStream_t stream) {
    if (p.width == 0 || p.rows == 0) return hipSuccess;
    const bool count = (flags & RTX_FLAG_COUNTERS) != 0;
    const bool quads = p.n_quads > 0;
    const bool use_lds = !(flags & RTX_FLAG_NO_LDS) && scene_lds_bytes(p) <= LDS_MAX_BYTES;
    if (uses_items(p, flags)) {
        if (!p.scratch) return hipErrorInvalidValue;  // the caller sizes the v3 scratch
        const bool use_lds = !(flags & RTX_FLAG_NO_LDS) && (p.n_entries + 1) * 16 <= LDS_B &&
                             lds_fixed_bytes(p.n_entries, p.n_quads, p.n_materials) <= LDS_MAX_BYTES;
        return count ? launch_items_for<true>(p, use_lds, stream) : launch_items_for<false>(p, use_lds, stream);
    }
    if (flags & RTX_FLAG_KERNEL_V0) {
        const dim3 grid((p.width + TILE_W - 1) / TILE_W, (p.rows + TILE_H - 1) / TILE_H);
        const auto kern = count ? (quads ? render_pixels<true, true> : render_pixels<true, false>)
                                : (quads ? render_pixels<false, true> : render_pixels<false, false>);
        hipLaunchKernelGGL(kern, grid, dim3(BLOCK), 0, stream, p);
        return hipGetLastError();
    }
    // Scenes with quads (hittables.go:138-216) run the default v1 schedule built with the
    // three-kind step; the scheduling variants below are sphere-only.
    if (quads)
        return count ? launch_wave_geom<true, 2, 2, 0, 3, false, true>(p, use_lds, stream)
                     : launch_wave_geom<false, 2, 2, 0, 3, false, true>(p, use_lds, stream);
    // v2 keeps tile origins in 16 bits: regions wider or taller than 65535 use v1.
    if ((flags & RTX_FLAG_KERNEL_POOL) && p.width <= 0xFFFFu && p.rows <= 0xFFFFu) {
        if (flags & RTX_FLAG_POOL4)
            return count ? launch_pool<true, 4>(p, use_lds, stream) : launch_pool<false, 4>(p, use_lds, stream);
        return count ? launch_pool<true, 2>(p, use_lds, stream) : launch_pool<false, 2>(p, use_lds, stream);
    }
    uint32_t geom = (flags >> 24) & 7u;
    // The persistent kernels claim 8x8 tiles by a 32-bit index.
    if (geom != 0 && (uint64_t)((p.width + 7) / 8) * ((p.rows + 7) / 8) > 0xFFFF0000ull) geom = 0;
    return count ? launch_wave<true>(p, geom, use_lds, stream) : launch_wave<false>(p, geom, use_lds, stream);
}

}  // namespace rtxd
