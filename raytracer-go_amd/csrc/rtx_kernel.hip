// rtx_kernel.hip — the path-tracing megakernel for gfx950 (MI355X).
//
// Replaces the per-pixel goroutine body of Camera.Render (camera.go:208-217):
// GetPixelColor (camera.go:254-263) = for k < spp { sum += GetColor(GetRay()) },
// then sum * (1/spp).  Every pixel's samples are added in order k = 0..spp-1, so the
// float32 sum is the reference's.  Every sample is independent (counter-based RNG
// keyed by global pixel index and k), so a pixel's value does not depend on the tile,
// the region, the scheduling or the number of GPUs.
//
// Schedule (v3): persistent waves over (pixel, sample) items; every item's colour goes to
// an HBM scratch and reduce_samples sums them in sample order afterwards.  Waves step
// every traversing lane through BVH entries (six per wave vote) and shade in batches:
// once `shade_thresh` lanes of the wave wait (or none traverses), all waiting lanes shade
// together, so shading and its Philox blocks run in lockstep.  (The earlier schedules
// v0 thread-per-pixel, v1 wave-per-tile and v2 pixel pool were measured slower and
// removed in ABI 4; DESIGN.md §5 keeps their numbers.)
#include <hip/hip_runtime.h>

#include <cstdio>

#include "rtx_device.h"
#include "rtx_kernel.h"

#ifndef RTX_WALK_STEPS  // walk steps per lane between two wave votes
#define RTX_WALK_STEPS 6
#endif
#ifndef RTX_SUB_MAX  // samples per unit of a render with >= 128 units of 8 samples per resident wave
#define RTX_SUB_MAX 16
#endif
#ifndef RTX_HYB_BATCH  // 1: primitive batching also for a scene in HBM with an LDS cache (A/B)
#define RTX_HYB_BATCH 0
#endif
#ifndef RTX_ASM_STEP  // 1: the timed kernel's walk step in assembly (trav_step_asm); 0 for A/B
#define RTX_ASM_STEP 1
#endif
#ifndef RTX_NEAR_FMA  // 1: the near pass's slab tests in the FMA form (box_step FMA); 0 for A/B
#define RTX_NEAR_FMA 1
#endif

#ifndef RTX_DEBUG_PARTIAL  // 1: the debug library (librtx_dbgclaim.so) that enters a claim with half the wave
#define RTX_DEBUG_PARTIAL 0
#endif

namespace rtxd {

// The wave-level claims (the unit queue, the defer queue, the redo list) take ONE atomic, issued by
// lane 0, and broadcast its result with readfirstlane.  That is only right with the whole wave
// active: without lane 0 no atomic is issued and every lane reads the first active lane's stale
// value (slot 0, unit 0: colliding records and a unit rendered again and again — the hang of the
// round-4 early-claim refactor), and with lane 0 the absent lanes would claim on
// their own later.  Each site therefore checks EXEC first, on SALU only (s_cmp on a copy of exec, a
// bit of the loop counter as the flag, no VGPR in the hot loop): a partial wave claims nothing (a unit
// claim leaves the wave exhausted, a queue claim drops its paths), the wave flags the render when it
// ends (KERR_PARTIAL_WAVE -> RTX_ERR_HIP), and the render fails loudly instead of hanging or returning
// a corrupt frame.  (The first version set the flag with an atomic at each site: one more spilled VGPR
// in the near pass and +2.4 % at C2.)
#ifndef RTX_CLAIM_GUARD  // 0: the guard compiled out (A/B of its cost only)
#define RTX_CLAIM_GUARD 1
#endif
#ifndef RTX_KARG_RELOAD  // 1: uniform values of the shading phase re-read from the kernel arguments at their use (0: A/B)
#define RTX_KARG_RELOAD 1
#endif
#ifndef RTX_KARG_CAM  // the pool's camera / the near region's bounds re-read from the kernel arguments (A/B)
#define RTX_KARG_CAM RTX_KARG_RELOAD
#endif
#ifndef RTX_KARG_NEAR
#define RTX_KARG_NEAR RTX_KARG_RELOAD
#endif
#ifndef RTX_HYB_DRAIN  // 1: the drain also for scenes in HBM with an LDS cache (A/B; round 5: +2.3 % at config 4)
#define RTX_HYB_DRAIN 0
#endif
#ifndef RTX_NT_COLOR  // 1: the sample colours stored non-temporally (A/B of the scratch's write amplification)
#define RTX_NT_COLOR 0
#endif
#ifndef RTX_NEAR_AND  // 1: the near region's test reads its bounds at once (0: short-circuit form, A/B)
#define RTX_NEAR_AND 1
#endif
#ifndef RTX_PRIO_WALK  // >= 0: the wave's issue priority (s_setprio) in the walk / the shading phase (A/B; -1: unset)
#define RTX_PRIO_WALK 1
#endif
#ifndef RTX_PRIO_SHADE
#define RTX_PRIO_SHADE 0
#endif
#ifndef RTX_PRIO_CLAIM  // >= 0: the priority from the claims on (new items, camera rays, the segment's begin; A/B)
#define RTX_PRIO_CLAIM -1
#endif
#ifndef RTX_DRAIN_LDS  // 1: the drain's per-workgroup record count and far unit cursor in LDS (0: in HBM, A/B)
#define RTX_DRAIN_LDS 1
#endif
#ifndef RTX_STATIC_FIRST  // 1: a wave's first unit from its grid index, no atomic (0: every unit claimed; 2: wave-major, A/B)
#define RTX_STATIC_FIRST 1
#endif
#ifndef RTX_CAM_DEFER  // 1: the near pass also tests each new camera ray against the near region (the host's gate,
#define RTX_CAM_DEFER 0  // camera_in_near, already admits only cameras whose defocus disk lies inside it)
#endif
// The kernel's Params as its kernel arguments hold them, behind an opaque copy of their address: a field read
// through it is loaded (s_load) at its use instead of being kept live through the main loop, where the kernel
// is at the SGPR limit and a live value is spilled to a VGPR lane (a v_readlane per use).  Only
// for fields whose kernel-argument value is the one in use: render_items' Params, render_drain's near Params
// (its first member), whose camera and near region its far phase shares.
__device__ __forceinline__ const Params& karg_params() {
    typedef const __attribute__((address_space(4))) Params* KP;
    KP q = (KP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return *(const Params*)q;
}

__device__ __forceinline__ bool partial_wave() { return RTX_CLAIM_GUARD && __builtin_amdgcn_read_exec() != ~0ull; }
// The debug library only: the odd lanes stay out of claim site `site` (tests/test_claim_guard.py).
__device__ __forceinline__ bool dbg_skip(const Params& p, uint32_t site, uint32_t lane) {
    return RTX_DEBUG_PARTIAL && p.debug_partial == site && (lane & 1u);
}

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
// Traversal phase.  Lane modes: 0 = traversing, 1 and 2 = waiting for the shading
// phase, 3 = neither.  Runs BVH steps until at least `thresh` lanes
// wait or none traverses.  Each traversing lane takes one entry (box or sphere, by its
// tag) per iteration.  (Separate box and sphere batches, steered by link-type bits in
// the entries, were measured: the extra decode per step cost more than the reduced
// divergence saved, DESIGN.md.)
// ------------------------------------------------------------------------------------
// STEPS > 1 takes up to STEPS entries per lane between two wave votes.  (A branch-free
// step that evaluates the box and the sphere test on every lane measured 8 % slower:
// most waves hold only box entries at a step, and the branch skips the sphere test.)
template <bool COUNT, int STEPS, bool QUADS, bool FIXED, bool HYB, bool BATCH, bool MED3, bool FMA = false>
__device__ __forceinline__ void traverse_loop(uint32_t& mode, Trav& t, const Ray& r, const SceneRef E,
                                              uint32_t n_entries, uint32_t thresh, Counters& cnt,
                                              uint64_t& wave_iters, uint64_t& lane_steps, uint64_t& shade_phases,
                                              uint64_t& shade_lanes, uint64_t& idle_lanes, uint64_t& parked,
                                              uint64_t& deferred, uint32_t prim_batch, bool w2) {
    // The lane modes are fixed during the phase except walking -> waiting (mode 0 -> 1) on
    // reaching the sentinel, so the votes are SALU on masks taken once: walking lanes W, waiting
    // lanes P0, lanes without an item D; per iteration only `at_end` is voted.
    const uint64_t W = ballot(mode == 0), P0 = ballot(mode - 1u < 2u);
    const uint64_t D = COUNT ? ballot(mode == 3) : 0ull;
    // FMA (the near pass): the slab form's -(o / d) per axis, once per phase (box_step FMA)
    const V3 no = FMA ? v3(-(r.o.x * t.ix), -(r.o.y * t.iy), -(r.o.z * t.iz)) : v3(0.0f, 0.0f, 0.0f);
    // The asm walk (walk_phase_asm) for scenes in LDS (spheres, and quads).  (For config 4's scene in HBM with
    // its top levels in LDS an asm walk lost to this C++ one: +9 % batched, +23 % running both
    // kinds per step)
    if constexpr (RTX_ASM_STEP && BATCH && !COUNT && FIXED && !HYB && MED3) {
        const uint64_t at_end = walk_phase_asm<QUADS, FMA>(t, r, 16 * n_entries, prim_batch, 0.001f, W, P0, thresh,
                                                           E.prim_end, LDS_B + 16 * (n_entries + 1), no);  // quad table
        if (__builtin_amdgcn_inverse_ballot_w64(W & at_end)) mode = 1;  // walked to the end
        return;
    }
    for (;;) {
        // Every lane steps: one that is not traversing (or finishes early) waits on the
        // sentinel, t.i = 16 * n_entries, where a step changes nothing — cheaper than masking
        // the wave per step.
        uint32_t done = 0;  // COUNT: lane-steps that tested an entry (a lane on the sentinel idles)
        uint32_t idle = 0;  // COUNT: parked (low 16 bits) and deferred (high 16 bits) lane-steps
        if (HYB && w2) {  // the paired walk's records
#pragma unroll
            for (int s = 0; s < STEPS; ++s) {
                if (COUNT) {
                    const uint32_t w = (uint32_t)__popcll(ballot(t.i < 16 * n_entries));
                    done += w;
                    idle += 64u - w;
                }
                trav_step_w2<COUNT, QUADS, MED3, FMA>(t, r, E, cnt, 16 * n_entries, no);
            }
        } else if constexpr (BATCH) {
#pragma unroll
            for (int s = 0; s < STEPS; ++s)
                done += trav_step_batched<COUNT, QUADS, FIXED, HYB, MED3, FMA>(t, r, E, cnt, 16 * n_entries,
                                                                              prim_batch, idle, no);
        } else {
#pragma unroll
            for (int s = 0; s < STEPS; ++s) {
                if (COUNT) {
                    const uint32_t w = (uint32_t)__popcll(ballot(t.i < 16 * n_entries));
                    done += w;
                    idle += 64u - w;
                }
                trav_step<COUNT, QUADS, FIXED, HYB, MED3, FMA>(t, r, E, cnt, no);
            }
        }
        const uint64_t at_end = ballot(t.i >= 16 * n_entries);
        const uint64_t trav = W & ~at_end;
        const uint64_t pend = P0 | (W & at_end);  // mode 1 or 2 after this iteration
        if (COUNT) {
            ++wave_iters;
            lane_steps += done;
            parked += idle & 0xFFFFu;
            deferred += idle >> 16;
            idle_lanes += (uint64_t)__popcll(D);
        }
        if (trav == 0 || (uint32_t)__popcll(pend) >= thresh) {
            if (COUNT) {
                ++shade_phases;
                shade_lanes += (uint64_t)__popcll(pend);
            }
            if (__builtin_amdgcn_inverse_ballot_w64(W & at_end)) mode = 1;  // walked to the end
            return;
        }
    }
}

// The traversal phase: the med3 box test (box_step) when every walking lane's ray has finite
// 1/dir and origin — all but a handful of rays per frame —, else the select form for the whole
// phase.  (A lane's ray is fixed for the phase; lanes parked on the sentinel do not matter: a
// step there changes nothing either way.)
template <bool COUNT, int STEPS = 1, bool QUADS = false, bool FIXED = false, bool HYB = false, bool BATCH = false,
          bool FMA = false>
__device__ __forceinline__ void traverse_phase(uint32_t& mode, Trav& t, const Ray& r, const SceneRef E,
                                               uint32_t n_entries, uint32_t thresh, Counters& cnt,
                                               uint64_t& wave_iters, uint64_t& lane_steps, uint64_t& shade_phases,
                                               uint64_t& shade_lanes, uint64_t& idle_lanes, uint64_t& parked,
                                               uint64_t& deferred, uint32_t prim_batch = 0, bool w2 = false) {
    if (ballot(!t.safe && t.i < 16 * n_entries) == 0)
        traverse_loop<COUNT, STEPS, QUADS, FIXED, HYB, BATCH, true, FMA>(mode, t, r, E, n_entries, thresh, cnt,
                                                                       wave_iters, lane_steps, shade_phases,
                                                                       shade_lanes, idle_lanes, parked, deferred,
                                                                       prim_batch, w2);
    else
        traverse_loop<COUNT, STEPS, QUADS, FIXED, HYB, BATCH, false, FMA>(mode, t, r, E, n_entries, thresh, cnt,
                                                                        wave_iters, lane_steps, shade_phases,
                                                                        shade_lanes, idle_lanes, parked, deferred,
                                                                        prim_batch, w2);
}

enum : uint32_t { M_TRAV = 0, M_SHADE = 1, M_START = 2, M_DONE = 3, M_CLAIM = 4 };

// COUNT: add the shader cycles since `clk` to `acc` and restart the clock.
__device__ __forceinline__ void split_clk(uint64_t& acc, uint64_t& clk) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    acc += now - clk;
    clk = now;
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
// CLK (RTX_FLAG_TIMING, diagnostics): the timed kernel (asm walk, no work counters) with the
// counting kernel's s_memtime split of wave cycles into walk and shading phases.
//
// TIER: 1 = the near pass of a tiered walk: a path whose next segment starts
// outside the near region is written to the defer queue (its segment start: ray, throughput,
// colour so far, pixel, sample, segment, scratch slot) and its lane takes a new item; 2 = the far
// pass: the items are the queue's records, each resumed at its segment start on the far tree;
// 3 = the redo pass: the samples whose record did not fit the queue (flagged in p.redo_bits)
// rendered again from their camera rays on the far tree — it returns at once when none did.
// Every sample's Philox blocks are keyed by (pixel, sample, event), so a path resumed in another
// launch draws exactly what it would have drawn.
//
// POOL (the timed kernel's near pass, scene in the LDS copy): new items take their camera
// rays from a per-wave pool in LDS after the scene copy, which holds the rays of one 64-item block of
// the unit — one sample of the tile's 64 pixels, sample-major as the items are handed out — drawn by
// the whole wave at once when the first item of the block is claimed.  The rays (GetRay, camera.go:
// 265-299: Philox block (0, 0) of (pixel, sample), the defocus disk's rejection loop) are the same
// bits; only who evaluates them changes: 64 lanes per evaluation instead of the few lanes a shading
// phase claims for (about a third of the wave).
//
// ST: the region's shard is in stripes of 2^stripe_log2 > 1 rows; the image row of a tile row comes from
// a per-unit base.  Single-row shards (every one-GPU render) run the ST = false instantiation, whose row arithmetic is
// the one before stripes existed (its code unchanged: the headline kernel).
//
// DRAIN (render_drain): TIER 1 writes the records to the workgroup's own region of the queue
// (Params::drain_count, drain_region); TIER 2 resumes that region's records only, its units claimed by the
// workgroup's waves.
template <bool COUNT, bool USE_LDS, bool QUADS, bool NOISE, int WAVES, bool HYB, bool CLK, int TIER, bool POOL, bool ST,
          bool DRAIN>
__device__ __forceinline__ void render_body(const Params& p, const uint64_t t0 = 0) {
    constexpr bool TIME = COUNT || CLK;
    static_assert(!DRAIN || (!COUNT && !CLK && (TIER == 1 || TIER == 2)), "the drain: the timed near and far passes");
    static_assert(!POOL || (USE_LDS && (TIER == 0 || TIER == 1)), "the camera-ray pool: LDS scenes, near pass or one walk");
    if constexpr (TIER == 3) {
        if (__builtin_amdgcn_readfirstlane(*(volatile uint32_t*)p.redo_count) == 0u) return;
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&p.counters[24], 1ull);  // chunks with a redo
    }
    // walk steps between two wave votes (A/B with primitive batching: 4 +0.7 %, 8 +0.8 %, 12 +1.3 %)
    constexpr uint32_t WAVE_BLOCK = 64 * WAVES, STEPS = RTX_WALK_STEPS;
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
        const uint32_t mo = lds_mat_offset(p.n_entries, p.n_quads, p.n_materials, p.n_textures) / 16;
        const float4* mg = reinterpret_cast<const float4*>(p.materials);
        for (uint32_t t = threadIdx.x; t < 2 * p.n_materials; t += WAVE_BLOCK) lds_entries[mo + t] = mg[t];
        const float4* tg = reinterpret_cast<const float4*>(p.textures);  // 48 B = 3 float4 each
        for (uint32_t t = threadIdx.x; t < 3 * p.n_textures; t += WAVE_BLOCK)
            lds_entries[mo + 2 * p.n_materials + t] = tg[t];
        __syncthreads();
        E = scene_ref_fixed(lds_entries, p.n_entries, p.n_quads, p.n_materials, p.n_textures);
        E.prim_end = p.prim_end;
    } else {
        E = scene_ref(p.entries, p.n_entries, p.materials);
        E.tx = p.textures;
        if constexpr (HYB) {  // the scene's top levels, stored first, cached in LDS (fixed layout)
            if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)lds_entries != 0u) __builtin_trap();
            const uint32_t m = p.n_entries + 1;
            for (uint32_t t = threadIdx.x; t < p.n_hot; t += WAVE_BLOCK) {
                lds_entries[t] = p.entries[t];
                lds_entries[HOT_B / 16 + t] = p.entries[m + t];
            }
            __syncthreads();
            E.la = lds_entries;
            E.lb = lds_entries + HOT_B / 16;
            E.hot = 16 * p.n_hot;
        }
    }
    const uint32_t n_entries = p.n_entries;
    const uint32_t thresh = p.shade_thresh;
    const uint32_t lane = threadIdx.x & 63u;
    const rtx_camera& c = p.cam;
    const uint32_t twl = p.tile_w_log2, tw_mask = (1u << twl) - 1u, th = 64u >> twl;  // tile: (1 << twl) x th
    const uint32_t tiles_x = tiles_x_of(p.width, twl);
    const uint32_t n_tiles = tiles_x * tiles_y_of(p.rows, twl);
    const uint32_t nsub = (p.kn + p.sub - 1u) / p.sub;
    // far pass: units of 64 queue records
    // (DRAIN: this workgroup's records, written by its own waves before the barrier that ended its near phase)
    // DRAIN: the workgroup's record count and far unit cursor: two LDS words at float4 index p.drain_lds, past both
    // phases' layouts (RTX_DRAIN_LDS), else drain_count's HBM words (a compile-time choice: a pointer that may be
    // either would make every claim a flat atomic)
    uint32_t* const rec_count = !DRAIN           ? p.defer_count
                                : RTX_DRAIN_LDS ? reinterpret_cast<uint32_t*>(lds_entries + p.drain_lds)
                                                : p.drain_count + blockIdx.x;
    uint32_t* const far_cursor = !DRAIN           ? p.tile_counter
                                 : RTX_DRAIN_LDS ? reinterpret_cast<uint32_t*>(lds_entries + p.drain_lds) + 1
                                                 : p.drain_count + gridDim.x + blockIdx.x;
    const uint32_t n_rec =
        TIER == 2 ? (DRAIN ? min(__builtin_amdgcn_readfirstlane(*(volatile uint32_t*)rec_count), p.drain_region)
                           : min(__builtin_amdgcn_readfirstlane(*(volatile uint32_t*)p.defer_count), p.defer_cap))
                  : 0u;
    // redo pass: the compacted list of flagged samples when it held them all (else the bits, unit by unit)
    const uint32_t n_ids = TIER == 3 ? __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)p.redo_count) : 0u;
    const bool listed = TIER == 3 && n_ids <= p.redo_cap;
    const uint64_t n_units = TIER == 2 ? (uint64_t)((n_rec + 63u) / 64u)
                                       : (listed ? (uint64_t)((n_ids + 63u) / 64u) : (uint64_t)n_tiles * nsub);
    if (TIER == 2 && (DRAIN || blockIdx.x == 0) && threadIdx.x == 0 && n_rec)
        atomicAdd(&p.counters[23], (unsigned long long)n_rec);  // deferred paths, all chunks
    const size_t tile_floats = (size_t)n_tiles * 64 * 3;  // one sample of every tile (tile-major scratch)
    const uint64_t* const redo64 = reinterpret_cast<const uint64_t*>(p.redo_bits);  // redo pass: 64 slots a word

    // the wave's unit (uniform, kept in SGPRs: every value below is derived from readfirstlane):
    // tile (index, origin u_x, u_r), first sample, items, next item
    uint32_t u_tile = 0, u_x = 0, u_r = 0, u_k0 = 0, u_items = 0, cursor = 0;
    // ST: the image row of the unit's first tile row; a tile's rows lie in one stripe (make_params: its height divides
    // the stripe), so row i of the tile is image row u_y + i
    uint32_t u_y = 0;
    bool exhausted = false;
    // POOL: the wave's 64 camera rays (2 float4 each) after the scene copy, and the unit's block they hold
    float4* const pool = POOL ? lds_entries + pool_f4_offset(p) + (threadIdx.x >> 6) * 128 : nullptr;
    uint32_t pool_blk = 0xFFFFFFFFu;
    // main-loop iterations (the watchdog's clock); bit 31: a claim site found a partial wave (partial_wave),
    // flagged once the wave ends.  (A bool of its own cost 0.6 % at C2, this bit 0.2 %: one SGPR fewer
    // live through the walk; profiles/r05_guard_ab.jsonl.)
    uint32_t iter = 0;
#define RTX_SET_KERR() (iter |= 0x80000000u)
#define RTX_KERR() ((iter & 0x80000000u) != 0u)

    uint32_t mode = M_CLAIM, seg = 0, items_done = 0;
    uint32_t pix = 0;  // the lane's item in the tile-major scratch: 64 * tile + pixel within the tile (< 2^32: rtx_capi)
    V3 base = v3(0.0f, 0.0f, 0.0f);
    V3 thr = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f);
    Ray r{v3(0, 0, 0), v3(0, 0, 0)};
    PathRng rng{(uint32_t)p.seed, (uint32_t)(p.seed >> 32), 0u, 0u};
    Trav t{};
    t.i = 16 * p.n_entries;  // on the sentinel until its first ray
    Counters cnt{0, 0, 0, 0, 0, 0};
    Counters path0 = cnt;  // COUNT, near pass: the counters when the lane's sample began
    uint64_t wave_iters = 0, lane_steps = 0, shade_phases = 0, shade_lanes = 0;
    uint64_t trav_cycles = 0, shade_cycles = 0, clk = 0, idle_lanes = 0, parked = 0, deferred = 0;  // COUNT only
    uint64_t split[4] = {0, 0, 0, 0};  // COUNT: shading-phase cycles: scatter, shade, claims + camera rays, trav_begin

    auto store = [&](V3 col) {  // the item's colour, GetColor's result for sample k
        float* o = p.scratch + (size_t)(rng.sample - p.k0) * tile_floats + (size_t)pix * 3;
        if (RTX_NT_COLOR) {
            __builtin_nontemporal_store(col.x, o);
            __builtin_nontemporal_store(col.y, o + 1);
            __builtin_nontemporal_store(col.z, o + 2);
        } else {
            o[0] = col.x;
            o[1] = col.y;
            o[2] = col.z;
        }
        ++items_done;
    };

    // near pass: hand the lanes with `far` set (their segment starts at r) to the far pass (the whole
    // wave is here; one queue atomic per wave)
    auto defer = [&](const bool far) {
        const uint64_t fm = ballot(far);
        if (fm == 0) return;
        if (dbg_skip(p, 1u, lane)) return;  // (debug library: the even lanes reach the claim alone)
        if (partial_wave()) {  // no claim without the whole wave: the paths are dropped, the render fails
            RTX_SET_KERR();
            if (far) mode = M_CLAIM;
            return;
        }
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(rec_count, (uint32_t)__popcll(fm));
        b = __builtin_amdgcn_readfirstlane(b);
        bool full = false;
        if (far) {
            const uint32_t slot = b + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
            if (slot < (DRAIN ? p.drain_region : p.defer_cap)) {
                float4* q = p.defer + 4 * ((DRAIN ? (size_t)blockIdx.x * p.drain_region : 0) + slot);
                q[0] = make_float4(r.o.x, r.o.y, r.o.z, __uint_as_float(rng.pixel));
                q[1] = make_float4(r.d.x, r.d.y, r.d.z, __uint_as_float(rng.sample));
                q[2] = make_float4(thr.x, thr.y, thr.z, __uint_as_float(seg));
                q[3] = make_float4(acc.x, acc.y, acc.z, __uint_as_float(pix));
            } else {
                full = true;
            }
            mode = M_CLAIM;
        }
        // No room: the redo pass renders the sample again from its camera ray on the far tree (the same
        // path: its Philox blocks are keyed by (pixel, sample, event)), and counts it.  Its id goes to the
        // redo list (one reservation per wave, coalesced stores); past the list's end, to the redo bits.
        const uint64_t om = ballot(full);
        if (om == 0) return;
        if (dbg_skip(p, 2u, lane)) return;
        if (partial_wave()) {
            RTX_SET_KERR();
            return;
        }
        uint32_t b2 = 0;
        if (lane == 0) b2 = atomicAdd(p.redo_count, (uint32_t)__popcll(om));
        b2 = __builtin_amdgcn_readfirstlane(b2);
        if (full) {
            const uint32_t at = b2 + (uint32_t)__popcll(om & ((1ull << lane) - 1ull));
            const uint32_t id = (rng.sample - p.k0) * n_tiles * 64u + pix;
            if (at < p.redo_cap) p.redo_ids[at] = id;
            else atomicOr(p.redo_bits + (id >> 5), 1u << (id & 31u));
            if (COUNT) cnt = path0;
        }
    };
    auto defer_far = [&](bool& ready) {  // segments that would start outside the near region
        const Params& q = RTX_KARG_NEAR && !HYB ? karg_params() : p;  // (the cache kernels: kept live)
        // all six bounds read unconditionally and combined with `&`: through the opaque kernel-argument pointer the
        // compiler cannot speculate a load, so `&&` became six scalar loads, each behind its own wait and branch
        // (C2 +2.6 % with two such tests per phase)
        const float x0 = q.near_min[0], y0 = q.near_min[1], z0 = q.near_min[2];
        const float x1 = q.near_max[0], y1 = q.near_max[1], z1 = q.near_max[2];
        const bool inside = RTX_NEAR_AND ? ((r.o.x >= x0) & (r.o.x <= x1) & (r.o.y >= y0) & (r.o.y <= y1) &
                                            (r.o.z >= z0) & (r.o.z <= z1))
                                         : (r.o.x >= x0 && r.o.x <= x1 && r.o.y >= y0 && r.o.y <= y1 &&
                                            r.o.z >= z0 && r.o.z <= z1);
        const bool far = ready && !inside;
        defer(far);
        if (far) ready = false;
    };

    // the watchdog's start: the launch's (render_drain hands its near phase's start to its far phase, so the
    // limit holds for the whole launch), or now
    const uint64_t t_start = t0 ? t0 : __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // Watchdog (RTX_WATCHDOG_S): a wave never outlives p.watchdog_ticks, so a bug cannot
        // keep the GPU busy forever; the render then fails with RTX_ERR_HIP (collect_on).
        // The loop is wave-uniform, so is this test.
        if ((++iter & 255u) == 0) {
            // the count wrapped into the flag bit (2^31 iterations: only with RTX_WATCHDOG_S raised): flip it
            // back, which restores the flag as it was whether it was set (0xFFFFFFFF + 1 = 0) or not
            if ((iter & 0x7FFFFFFFu) == 0u) iter ^= 0x80000000u;
            if (__builtin_amdgcn_s_memrealtime() - t_start > p.watchdog_ticks) {
                if (lane == 0) atomicAdd(p.error_flag + KERR_WATCHDOG, 1u);
                break;
            }
        }
        if (TIME) clk = __builtin_amdgcn_s_memtime();
        if (RTX_PRIO_WALK >= 0) __builtin_amdgcn_s_setprio(RTX_PRIO_WALK);
        // primitive batching only for a scene in LDS: a lane that waits re-reads its entry, which
        // from HBM cost config 4 +34 %
        traverse_phase<COUNT, STEPS, QUADS, USE_LDS, HYB, USE_LDS || (RTX_HYB_BATCH && HYB), TIER == 1 && RTX_NEAR_FMA && !QUADS>(
            mode, t, r, E, n_entries, thresh, cnt, wave_iters,
                                                              lane_steps, shade_phases, shade_lanes, idle_lanes,
                                                              parked, deferred, p.prim_batch, HYB && p.w2);
        if (TIME) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            trav_cycles += now - clk;
            clk = now;
        }
        if (ballot(mode != M_DONE) == 0) break;
        if (RTX_PRIO_SHADE >= 0) __builtin_amdgcn_s_setprio(RTX_PRIO_SHADE);

        // ---- shading phase ----------------------------------------------------------
        // POOL: a MISS PHASE instead when fewer than p.refill_hits of the waiting lanes hit something: only
        // the paths that ended on the background finish (ray.go:52: their colour stored) and take new items,
        // whose camera rays the pool already holds; the lanes waiting on a hit stay parked and the walk goes
        // on.  The full phase then shades more hits at once (its Philox evaluations and scatter are paid per
        // phase).  The same operations per path, so the same bits.
        // (The lanes a miss phase leaves parked on a hit wait as M_START, which the walk treats as waiting and
        // the phase's shading skips; they are M_SHADE again at the next phase.)
        bool mini = false;
        if constexpr (POOL) {
            if (mode == M_START) mode = M_SHADE;
            // (ballots of single compares, combined on SALU: a ballot of `a && b` costs a lane-mask materialisation)
            const uint64_t wait = ballot(mode == M_SHADE), miss = wait & ballot(t.hit < 0);
            mini = miss != 0 && (uint32_t)__popcll(wait & ~miss) < p.refill_hits;
            if (mini && mode == M_SHADE && t.hit >= 0) mode = M_START;
        }
        bool ready = false;
        if constexpr (TIER == 1) {
            // The near walk's closest hit is the guarded walk's when the hit sphere's own box (inside
            // its reference leaf's) passes with the bound just past the hit; else the
            // segment is walked again on the guarded tree by the far pass.
            const bool check = mode == M_SHADE && t.hit >= 0;
            float lo = 0.0f, hi = 1.0f;  // the test's interval (a lane without a hit passes); bad = !(lo < hi), one compare
            if (check) {
                if (QUADS && __float_as_int(E.b[t.hit].w) == RTX_E_QUAD) {  // a quad's own box
                    const uint32_t qi = 4u * (uint32_t)__float_as_int(E.b[t.hit].x);
                    if (!quad_own_box_pass(t, r, E.q[qi], E.q[qi + 1], E.q[qi + 2])) lo = 1.0f;
                } else {
                    own_box_interval(t, r, E.a[t.hit], lo, hi);
                }
            }
            const bool bad = !(lo < hi);
            if (COUNT && bad) --cnt.segments;  // the far pass walks the segment again and counts it
            defer(bad);
        }
        Scatter sc{v3(0.0f, 0.0f, 0.0f), 0u, 0u};
        if (!mini) {  // (a miss phase draws nothing)
            U4 b0{0u, 0u, 0u, 0u};
            if (mode == M_SHADE && t.hit >= 0) b0 = rng.block(seg + 1, 0u);
            sc = coop_scatter<QUADS>(p, E, rng, seg + 1, mode == M_SHADE ? t.hit : -1, b0);
        }
        if (TIME) split_clk(split[0], clk);
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
        if constexpr (TIER == 1) defer_far(ready);  // before the claims: the lane takes a new item now
        if (TIME) split_clk(split[1], clk);
        if (RTX_PRIO_CLAIM >= 0) __builtin_amdgcn_s_setprio(RTX_PRIO_CLAIM);
        // Lanes without an item take the next ones of the wave's unit; new camera rays
        // at one program point.  Loops only for max depth 0 and ragged tiles.
        for (;;) {
            const uint64_t wm = ballot(mode == M_CLAIM);
            if (wm == 0) break;
            if (cursor >= u_items && !exhausted && dbg_skip(p, 3u, lane)) {
                exhausted = true;  // (debug library: the even lanes reach the claim alone)
            } else if (cursor >= u_items && !exhausted) {  // claim the next unit (wave-uniform)
                // RTX_STATIC_FIRST (units on a global counter: TIER 0 / 1, a far launch): a wave's first unit is its grid index, the
                // counter hands out the rest from there, so the launch does not start with every wave's atomic queued
                // on one address (u_items is 0 only before the first claim: a claimed unit holds >= 64 items)
                constexpr bool STATIC_FIRST = RTX_STATIC_FIRST && (TIER <= 1 || (TIER == 2 && !DRAIN));
                const uint32_t n_waves = gridDim.x * WAVES;
                uint32_t uu;
                if (STATIC_FIRST && u_items == 0u) {
                    uu = __builtin_amdgcn_readfirstlane(RTX_STATIC_FIRST == 2 ? (threadIdx.x >> 6) * gridDim.x + blockIdx.x
                                                                              : blockIdx.x * WAVES + (threadIdx.x >> 6));
                } else {
                    uint32_t un = 0;
                    if (lane == 0) un = atomicAdd(DRAIN && TIER == 2 ? far_cursor : p.tile_counter, 1u);
                    uu = __builtin_amdgcn_readfirstlane(un) + (STATIC_FIRST ? n_waves : 0u);  // the whole wave is here: lane 0's
                }
                if (partial_wave()) {  // else: the wave stops (exhausted) and the render fails
                    RTX_SET_KERR();
                    uu = 0xFFFFFFFFu;
                }
                exhausted = uu >= n_units;
                if (!exhausted && (TIER == 2 || listed)) {
                    u_k0 = 64u * uu;  // the unit's first record / listed sample
                    u_items = min(64u, (TIER == 2 ? n_rec : n_ids) - u_k0);
                    cursor = 0;
                } else if (!exhausted) {
                    u_tile = uu / nsub;
                    u_x = (u_tile % tiles_x) << twl;
                    u_r = (u_tile / tiles_x) * th;
                    if constexpr (ST) u_y = p.y0 + region_row(u_r, p.rank, p.world, p.stripe_log2);
                    u_k0 = p.k0 + (uu - u_tile * nsub) * p.sub;
                    const uint32_t cnt_k = min(p.sub, p.k0 + p.kn - u_k0);
                    u_items = 64u * cnt_k;
                    cursor = 0;
                    pool_blk = 0xFFFFFFFFu;
                    if (TIER == 3 && !listed) {  // a unit without a flagged sample: the next unit
                        const bool any = lane < cnt_k && redo64[(size_t)(u_k0 + lane - p.k0) * n_tiles + u_tile] != 0;
                        if (ballot(any) == 0) cursor = u_items;
                    }
                }
            }
            if (exhausted) {
                if (mode == M_CLAIM) mode = M_DONE;
                break;
            }
            uint32_t avail = u_items - cursor;  // items this round can hand out
            if constexpr (POOL) {
                const uint32_t blk = cursor >> 6;
                if (blk != pool_blk) {  // the block's 64 camera rays, one per lane (sample u_k0 + blk, pixel lane)
                    pool_blk = blk;
                    const rtx_camera& c = RTX_KARG_CAM ? karg_params().cam : p.cam;
                    const uint32_t lx = u_x + (lane & tw_mask), lr = u_r + (lane >> twl);
                    if (lx < p.width && lr < p.rows) {
                        const uint32_t x = p.x0 + lx, y = ST ? u_y + (lane >> twl) : p.y0 + p.rank + lr * p.world;
                        const PathRng cr{rng.k0, rng.k1, y * c.image_width + x, u_k0 + blk};
                        uint32_t dr = 0;
                        const Ray cray = camera_ray<!COUNT>(c, pixel_base(c, x, y), cr, cr.block(0u, 0u), dr);
                        pool[2 * lane] = make_float4(cray.o.x, cray.o.y, cray.o.z, __uint_as_float(dr));  // (COUNT: draws)
                        pool[2 * lane + 1] = make_float4(cray.d.x, cray.d.y, cray.d.z, 0.0f);
                    }
                    __builtin_amdgcn_wave_barrier();  // (LDS is in order within the wave)
                }
                avail = min(u_items, 64u * blk + 64u) - cursor;
            }
            const uint32_t rank = (uint32_t)__popcll(wm & ((1ull << lane) - 1ull));
            bool got = false;
            uint32_t pool_draws = 0;  // COUNT, POOL: the draws of the ray the lane takes
            if (TIER == 2 && mode == M_CLAIM && rank < avail) {  // resume a record
                const float4* q = p.defer + 4 * ((DRAIN ? (size_t)blockIdx.x * p.drain_region : 0) + u_k0 + cursor + rank);
                const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
                r = Ray{v3(q0.x, q0.y, q0.z), v3(q1.x, q1.y, q1.z)};
                rng.pixel = __float_as_uint(q0.w);
                rng.sample = __float_as_uint(q1.w);
                thr = v3(q2.x, q2.y, q2.z);
                seg = __float_as_uint(q2.w);
                acc = v3(q3.x, q3.y, q3.z);
                pix = __float_as_uint(q3.w);
                mode = M_START;
                ready = true;
            } else if (TIER != 2 && mode == M_CLAIM && rank < avail) {
                uint32_t j = cursor + rank, l = j & 63u;  // sample-major within the unit
                uint32_t lx = u_x + (l & tw_mask);
                uint32_t lr = u_r + (l >> twl);
                size_t slot = (size_t)u_tile * 64 + l;
                uint32_t k = u_k0 + (j >> 6);
                if (TIER == 3 && listed) {  // a listed sample: its bit index in the chunk
                    const uint32_t id = p.redo_ids[u_k0 + j];
                    const uint32_t per_k = n_tiles * 64u;
                    k = p.k0 + id / per_k;
                    slot = id - (k - p.k0) * per_k;
                    l = (uint32_t)slot & 63u;
                    const uint32_t tile = (uint32_t)(slot >> 6);
                    lx = ((tile % tiles_x) << twl) + (l & tw_mask);
                    lr = (tile / tiles_x) * th + (l >> twl);
                }
                // else: outside a ragged tile (or, redo pass, not flagged), claim again
                if (lx < p.width && lr < p.rows &&
                    (TIER != 3 || listed || ((redo64[((size_t)(k - p.k0) * n_tiles * 64 + slot) >> 6] >> l) & 1ull))) {
                    const uint32_t x = p.x0 + lx,
                                   y = !ST ? p.y0 + p.rank + lr * p.world
                                           : (TIER == 3 && listed ? p.y0 + region_row(lr, p.rank, p.world, p.stripe_log2)
                                                                  : u_y + (l >> twl));
                    if constexpr (POOL) {  // the ray the wave drew for this item (l: the pixel of the block)
                        const float4 po = pool[2 * l], pd = pool[2 * l + 1];
                        r = Ray{v3(po.x, po.y, po.z), v3(pd.x, pd.y, pd.z)};
                        if (COUNT) pool_draws = __float_as_uint(po.w);
                    } else {
                        base = pixel_base(c, x, y);
                    }
                    rng.pixel = y * c.image_width + x;
                    rng.sample = k;
                    pix = (uint32_t)slot;
                    got = true;
                }
            }
            const uint32_t taken = (uint32_t)__popcll(wm);
            cursor += taken < avail ? taken : avail;
            if (got) {
                if (COUNT && TIER == 1) path0 = cnt;
                if constexpr (!POOL) r = camera_ray<!COUNT>(c, base, rng, rng.block(0u, 0u), cnt.draws);  // GetRay, camera.go:257
                else if (COUNT) cnt.draws += pool_draws;  // the camera ray's draws, counted by its own lane
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
        // a camera ray outside the region: none, by the host's gate (rtx_capi camera_in_near: the defocus disk's box,
        // with room for rounding, inside the region), so the test is compiled only for A/B
        if constexpr (TIER == 1 && RTX_CAM_DEFER) defer_far(ready);
        if (TIME) split_clk(split[2], clk);
        if (ready) {  // begin a segment: world.Hit (ray.go:36)
            if (COUNT) ++cnt.segments;
            trav_begin<TIER == 1 && RTX_NEAR_FMA && !QUADS>(t, r, p.start);
            mode = n_entries > 0 ? M_TRAV : M_SHADE;
        }
        if (TIME) split_clk(split[3], clk);
    }
    if (RTX_KERR()) atomicAdd(p.error_flag + KERR_PARTIAL_WAVE, 1u);
#undef RTX_SET_KERR
#undef RTX_KERR
    if (COUNT) {
        flush_counters(p, items_done, cnt);
        if (lane == 0) {
            flush_sched(p, wave_iters, lane_steps / STEPS, shade_phases, shade_lanes);
            atomicAdd(&p.counters[14], (unsigned long long)idle_lanes);
            atomicAdd(&p.counters[16], (unsigned long long)(parked / STEPS));
            atomicAdd(&p.counters[17], (unsigned long long)(deferred / STEPS));
        }
    }
    if (TIME && lane == 0) {
        atomicAdd(&p.counters[12], (unsigned long long)trav_cycles);
        for (int q = 0; q < 4; ++q) {
            shade_cycles += split[q];
            atomicAdd(&p.counters[18 + q], (unsigned long long)split[q]);
        }
        atomicAdd(&p.counters[13], (unsigned long long)shade_cycles);
    }
}

template <bool COUNT, bool USE_LDS, bool QUADS, bool NOISE, int WAVES = 8, int MINW = 0, bool HYB = false,
          bool CLK = false, int TIER = 0, bool POOL = false, bool ST = false>
__global__ __launch_bounds__(64 * WAVES, MINW) void render_items(Params p) {
    render_body<COUNT, USE_LDS, QUADS, NOISE, WAVES, HYB, CLK, TIER, POOL, ST, false>(p);
}

// The timed tiered render's near pass with its drain: the near phase (pn, the near tree, records to the
// workgroup's region), then — once all the workgroup's waves are out of near work — its far phase over those records
// (pf, the far tree, copied into the same LDS).  A workgroup whose near work ends early walks its far paths while
// others still render, so the far tree's long paths no longer wait for the last near wave, nor for a second launch.
// The far phase's own settings (the rest of its Params are the near pass's): its layout and walk knobs.
struct FarLayout {
    const float4* entries;
    uint32_t n_entries, n_hot, start, prim_end, shade_thresh, refill_hits, prim_batch, w2;
};
inline FarLayout far_layout(const Params& pf) {
    return FarLayout{pf.entries, pf.n_entries, pf.n_hot, pf.start, pf.prim_end, pf.shade_thresh, pf.refill_hits, pf.prim_batch,
                     pf.w2};
}

struct DrainArgs {
    Params pn;
    FarLayout fl;
};

template <bool USE_LDS, int WAVES, int MINW, bool HYB, bool POOL, bool ST, bool QUADS = false>
__global__ __launch_bounds__(64 * WAVES, MINW) void render_drain(DrainArgs a) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime() | 1ull;  // the watchdog's start for both phases (nonzero)
    if constexpr (RTX_DRAIN_LDS) {  // the workgroup's two drain words in LDS (past both phases' layouts): zero first
        extern __shared__ float4 lds_words[];
        if (threadIdx.x < 2) reinterpret_cast<uint32_t*>(lds_words + a.pn.drain_lds)[threadIdx.x] = 0u;
        __syncthreads();
    }
    render_body<false, USE_LDS, QUADS, false, WAVES, HYB, false, 1, POOL, ST, true>(a.pn, t0);
    __syncthreads();  // every wave's near work and records done: the far phase overwrites the scene copy
    // The far phase reads its settings from the kernel arguments afresh, through an opaque copy of their address:
    // values it shares with the near phase are then not kept live through the near phase (which spilled 4 more VGPRs).
    typedef const __attribute__((address_space(4))) DrainArgs* KArgs;
    KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const DrainArgs& k = *(const DrainArgs*)ka;
    Params pf = k.pn;
    pf.entries = k.fl.entries;
    pf.n_entries = k.fl.n_entries;
    pf.n_hot = k.fl.n_hot;
    pf.start = k.fl.start;
    pf.prim_end = k.fl.prim_end;
    pf.shade_thresh = k.fl.shade_thresh;
    pf.refill_hits = k.fl.refill_hits;
    pf.prim_batch = k.fl.prim_batch;
    pf.w2 = k.fl.w2;
    pf.tier = 2;
    render_body<false, USE_LDS, QUADS, false, WAVES, HYB, false, 2, false, false, true>(pf, t0);
}

// The redo list overflowed (more samples than p.redo_cap): its ids join the ones the near pass set in
// p.redo_bits, and the redo pass scans the bits.  A return when it did not.
__global__ __launch_bounds__(256) void spill_redo_list(Params p) {
    if (__builtin_amdgcn_readfirstlane(*(volatile uint32_t*)p.redo_count) <= p.redo_cap) return;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < p.redo_cap; i += (uint64_t)gridDim.x * 256) {
        const uint32_t id = p.redo_ids[i];
        atomicOr(p.redo_bits + (id >> 5), 1u << (id & 31u));
    }
}

// A tiered chunk's counters, zeroed by one launch before its near pass (four memsets cost C1 ~20 us of launch gaps):
// the unit queue head, the record count, the redo list count, the drain's per-workgroup words [0, n_drain), and the
// far and redo passes' own unit queue heads (DRAIN_WORDS - 2, - 1); for the render's first chunk (first != 0) every
// stats slot too (rtx_capi's enqueue_on leaves them to this launch for a tiered render).
__global__ __launch_bounds__(256) void chunk_start(Params p, uint32_t n_drain, uint32_t first) {
    if (first)
        for (uint32_t i = threadIdx.x; i < COUNTER_SLOTS; i += 256) p.counters[i] = 0ull;
    __syncthreads();  // (the unit queue head and the record count share the slots)
    if (threadIdx.x == 0) {
        *p.tile_counter = 0u;
        *p.defer_count = 0u;
        *p.redo_count = 0u;
        p.drain_count[DRAIN_WORDS - 2] = 0u;
        p.drain_count[DRAIN_WORDS - 1] = 0u;
    }
    for (uint32_t i = threadIdx.x; i < n_drain; i += 256) p.drain_count[i] = 0u;
}

// GetPixelColor's sum over the stored colours of samples [k0, k0 + kn), in k order
// (camera.go:256-259), continued from the running sum in `out` when k0 > 0; the last
// chunk applies Scale(1/spp) (camera.go:261).  The scratch is tile-major — sample k of tile t
// is one 768-B block of its 64 pixels' colours, so a wave's colour stores fill whole lines
// (pixel-major rows of 96 B wrote 1.26x the colour bytes to HBM as partial lines).  Thread i
// sums pixel i % 64 of tile i / 64: consecutive threads read consecutive colours.
//
// Tiered renders: the redo bits are set only when the redo list overflowed (redo_count > redo_cap: by the near pass
// past the list's end, and by spill_redo_list); the redo pass has read them by now, and this clears the chunk's bits
// again, so they are zero at every chunk's start without a memset of the whole bitmap per chunk (130 MB at C2,
// ~180 MB at C5).  Nothing to do when the list held every id.
__global__ __launch_bounds__(256) void reduce_samples(Params p, uint32_t last) {
    const uint32_t twl = p.tile_w_log2;
    const uint32_t tiles_x = tiles_x_of(p.width, twl);
    const size_t n_tiles = (size_t)tiles_x * tiles_y_of(p.rows, twl);
    if (p.redo_count && __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)p.redo_count) > p.redo_cap) {
        const uint64_t words = (uint64_t)p.kn * n_tiles * 2;  // 64 bits a tile
        for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < words; w += (uint64_t)gridDim.x * 256)
            p.redo_bits[w] = 0u;
    }
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_tiles * 64) return;
    const uint32_t t = (uint32_t)(i >> 6), l = (uint32_t)(i & 63u);
    const uint32_t lx = ((t % tiles_x) << twl) + (l & ((1u << twl) - 1u)), lr = (t / tiles_x) * (64u >> twl) + (l >> twl);
    if (lx >= p.width || lr >= p.rows) return;  // outside a ragged tile
    float* o = p.out + ((size_t)lr * p.width + lx) * 3;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    if (p.k0 > 0) {
        sx = o[0];
        sy = o[1];
        sz = o[2];
    }
    // 8 samples' colours in flight per thread, then added in k order; the scratch is read once (non-temporal loads)
    const float* src = p.scratch + i * 3;
    const size_t stride = n_tiles * 64 * 3;
    uint32_t k = 0;
    for (; k + 8 <= p.kn; k += 8, src += 8 * stride) {
        float c[8][3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // (read once: non-temporal)
            c[j][0] = __builtin_nontemporal_load(src + j * stride);
            c[j][1] = __builtin_nontemporal_load(src + j * stride + 1);
            c[j][2] = __builtin_nontemporal_load(src + j * stride + 2);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sx = sx + c[j][0];
            sy = sy + c[j][1];
            sz = sz + c[j][2];
        }
    }
    for (; k < p.kn; ++k, src += stride) {
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
// launches
// ------------------------------------------------------------------------------------
constexpr uint32_t LDS_MAX_BYTES = 64 * 1024;

// v3: chunks of p.kn samples (the scratch holds one chunk), each rendered by a
// resident-capacity grid of render_items and summed into p.out by reduce_samples.
// Samples per unit: 8, or fewer when that leaves under 8 units per resident wave (a small
// image's last units would run on a near-empty GPU).  Measured at 100 spp: 1920x1080 8 -1.6 % vs
// 16; 400x225 2 -42 % vs 16; Cornell 600x600 8 -3 % vs 16.  16 when that still leaves >= 64
// units per wave (the drain stays short): 1920x1080x500 -0.9 % vs 8 (142.5 vs 143.8 ms).
// 4 instead of 2 below 8 units of 8 samples per resident wave: the tiered walk (C1 400x225x100: 1.68 ms against 1.77 at
// 2 and 1.77 at 8; profiles/r05_unit_sweep.jsonl), and since round 6 every render (quadDemo 400x225x100: 0.60 ms
// against 0.99 at 2, perlinDemo 3.31 against 3.33; profiles/r06_demo_knobs.jsonl).
inline uint32_t unit_samples(uint64_t tiles, uint32_t kn, int waves, int per_cu, int cus, bool tiered = false) {
    const uint64_t per_wave = tiles * kn / (8ull * waves * (uint64_t)per_cu * cus);
    (void)tiered;
    if (per_wave >= 2 && per_wave < 8) return 4u;
    return per_wave >= 128 ? RTX_SUB_MAX : (per_wave >= 8 ? 8u : (per_wave >= 4 ? 4u : (per_wave >= 2 ? 2u : 1u)));
}

hipError_t resident_grid(const void* kern, int block, size_t shmem, int* per_cu, int* cus) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kern, block, shmem);
    if (*per_cu < 1) *per_cu = 1;
    return e;
}

// v3: chunks of p.kn samples (the scratch holds one chunk), each rendered by a
// resident-capacity grid of render_items and summed into p.out by reduce_samples.
// POOL (a scene in the LDS copy, the timed kernel): the camera-ray pool after the scene copy (render_items<POOL>).
template <bool COUNT, bool QUADS, bool NOISE, int WAVES = 8, int MINW = 0, bool CLK = false, bool POOL = false,
          bool ST = false>
hipError_t launch_items(Params p, bool use_lds, hipStream_t stream) {
    // a scene too big for LDS: its top levels (p.n_hot entries) cached in LDS when the
    // device layout stored them first (RTX_HOT_ENTRIES=0 turns that off)
    const bool hyb = !use_lds && p.n_hot > 0 && !NOISE;
    const size_t shmem = POOL ? (size_t)pool_f4_offset(p) * 16 + WAVES * POOL_BYTES_PER_WAVE
                              : use_lds ? lds_fixed_bytes(p.n_entries, p.n_quads, p.n_materials, p.n_textures)
                                        : (hyb ? lds_hot_bytes(p.n_hot) : 0);
    const auto kern = POOL      ? render_items<COUNT, true, QUADS, NOISE, WAVES, MINW, false, CLK, 0, POOL, ST>
                      : use_lds ? render_items<COUNT, true, QUADS, NOISE, WAVES, MINW, false, CLK, 0, false, ST>
                                : (hyb ? render_items<COUNT, false, QUADS, NOISE, WAVES, MINW, !NOISE, CLK, 0, false, ST>
                                       : render_items<COUNT, false, QUADS, NOISE, WAVES, MINW, false, CLK, 0, false, ST>);
    constexpr int block = 64 * WAVES;
    int cus = 0, per_cu = 0;
    hipError_t e = resident_grid((const void*)kern, block, shmem, &per_cu, &cus);
    if (e != hipSuccess) return e;
    const uint32_t spp = p.cam.samples_per_pixel, chunk = p.kn, sub = p.sub;
    const uint64_t tiles = (uint64_t)tiles_x_of(p.width, p.tile_w_log2) * tiles_y_of(p.rows, p.tile_w_log2);
    const uint64_t slots = tiles * 64;  // pixels of the tile-major scratch (ragged tiles padded)
    for (uint32_t k0 = 0; k0 < spp; k0 += chunk) {
        p.k0 = k0;
        p.kn = spp - k0 < chunk ? spp - k0 : chunk;
        if (sub == 0) p.sub = unit_samples(tiles, p.kn, WAVES, per_cu, cus);
        const uint64_t units = tiles * ((p.kn + p.sub - 1) / p.sub);
        uint64_t blocks = (uint64_t)per_cu * cus;
        if (blocks > (units + WAVES - 1) / WAVES) blocks = (units + WAVES - 1) / WAVES;  // no wave starts idle
        if (p.debug_launch)
            fprintf(stderr, "rtx v3: waves/wg %d, wgs/CU %d, CUs %d, grid %llu, sub %u, units %llu, lds %zu B\n", WAVES,
                    per_cu, cus, (unsigned long long)blocks, p.sub, (unsigned long long)units, shmem);
        e = hipMemsetAsync(p.tile_counter, 0, sizeof(uint32_t), stream);  // (the watchdog flag: once per render)
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(block), shmem, stream, p);
        hipLaunchKernelGGL(reduce_samples, dim3((uint32_t)((slots + 255) / 256)), dim3(256), 0, stream, p,
                           (uint32_t)(k0 + p.kn >= spp));
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// LDS bytes of a render_items launch: the fixed layout's whole scene (USE_LDS), the hot entries of a
// scene in HBM (HYB), or none.
inline size_t items_shmem(const Params& p, bool use_lds, bool hyb) {
    return use_lds ? lds_fixed_bytes(p.n_entries, p.n_quads, p.n_materials, p.n_textures)
                   : (hyb ? lds_hot_bytes(p.n_hot) : 0);
}

// The tiered walk of a sphere scene whose near and far layouts are placed alike —
// both in the LDS copy (USE_LDS), both in HBM with an LDS cache of their hot entries (HYB), or both
// in HBM: per chunk the near pass (pn), the far pass over its queue (pf), the redo pass over the
// samples whose records did not fit (its waves return at once when none), the reduction.
// POOL: the near pass takes its camera rays from the waves' LDS pools (render_items<POOL>), in
// workgroups of WN waves (12: two per CU, each with its scene copy and 12 pools); the far and redo
// passes keep WAVES.
template <bool COUNT, int WAVES, int MINW, bool CLK = false, bool USE_LDS = true, bool HYB = false, bool POOL = false,
          bool ST = false, bool QUADS = false, int WN = POOL ? RTX_POOL_WAVES : WAVES>
hipError_t launch_tiered(Params pn, Params pf, hipStream_t stream) {
    constexpr int MN = POOL && MINW ? RTX_POOL_MINW : MINW;  // the near (and drain) kernel's waves per SIMD
    const auto kn = render_items<COUNT, USE_LDS, QUADS, false, WN, MN, HYB, CLK, 1, POOL, ST>;
    const auto kf = render_items<COUNT, USE_LDS, QUADS, false, WAVES, MINW, HYB, CLK, 2>;  // (rows from the records)
    const auto kr = render_items<COUNT, USE_LDS, QUADS, false, WAVES, MINW, HYB, false, 3, false, ST>;
    const size_t sn = POOL ? (size_t)pool_f4_offset(pn) * 16 + WN * POOL_BYTES_PER_WAVE : items_shmem(pn, USE_LDS, HYB),
                 sf = items_shmem(pf, USE_LDS, HYB);
    constexpr int block = 64 * WAVES, block_n = 64 * WN;
    int cus = 0, per_n = 0, per_f = 0, per_r = 0;
    hipError_t e = resident_grid((const void*)kn, block_n, sn, &per_n, &cus);
    if (e == hipSuccess) e = resident_grid((const void*)kf, block, sf, &per_f, &cus);
    if (e == hipSuccess) e = resident_grid((const void*)kr, block, sf, &per_r, &cus);
    if (e != hipSuccess) return e;
    // The drain (render_drain, the timed kernels): the near grid's workgroups resume their own records in the
    // same LDS (the larger of the two layouts), when that keeps the near pass's occupancy.
    // (Not for a scene in HBM with LDS caches: the combined kernel spilled 24 VGPRs there, and config 4 took +2.3 %.)
    constexpr bool CAN_DRAIN = !COUNT && !CLK && (!HYB || RTX_HYB_DRAIN);
    const void* kd = nullptr;
    if constexpr (CAN_DRAIN) kd = (const void*)render_drain<USE_LDS, WN, MN, HYB, POOL, ST, QUADS>;
    // (RTX_DRAIN_LDS: the drain's two per-workgroup words in LDS after the larger layout)
    const size_t sl = ((sn > sf ? sn : sf) + 15) / 16 * 16, sd = RTX_DRAIN_LDS ? sl + 16 : sl;
    pn.drain_lds = RTX_DRAIN_LDS ? (uint32_t)(sl / 16) : 0u;
    int per_d = 0;
    bool drain = CAN_DRAIN && pn.drain && pn.drain_count;
    if (drain && (e = resident_grid(kd, block_n, sd, &per_d, &cus)) != hipSuccess) return e;
    drain = drain && per_d >= per_n;
    const uint32_t spp = pn.cam.samples_per_pixel, chunk = pn.kn, sub = pn.sub;
    const uint64_t tiles = (uint64_t)tiles_x_of(pn.width, pn.tile_w_log2) * tiles_y_of(pn.rows, pn.tile_w_log2);
    const uint64_t slots = tiles * 64;
    Params pr = pf;  // the redo pass: the far layout over the chunk's units, flagged samples only
    pr.tier = 0;
    // the far and redo passes' unit queue heads: words of their own, zeroed with the chunk's others (chunk_start)
    pf.tile_counter = pn.drain_count + DRAIN_WORDS - 2;
    pr.tile_counter = pn.drain_count + DRAIN_WORDS - 1;
    for (uint32_t k0 = 0; k0 < spp; k0 += chunk) {
        pn.k0 = pf.k0 = pr.k0 = k0;
        pn.kn = pf.kn = pr.kn = spp - k0 < chunk ? spp - k0 : chunk;
        pn.sub = sub ? sub : unit_samples(tiles, pn.kn, WN, per_n, cus, true);
        pf.sub = pr.sub = pn.sub;
        const uint64_t units = tiles * ((pn.kn + pn.sub - 1) / pn.sub);
        uint64_t bn = (uint64_t)per_n * cus, br = (uint64_t)per_r * cus;
        if (bn > (units + WN - 1) / WN) bn = (units + WN - 1) / WN;
        if (br > (units + WAVES - 1) / WAVES) br = (units + WAVES - 1) / WAVES;
        if (pn.debug_launch)
            fprintf(stderr, "rtx tiered: waves/wg %d / %d, wgs/CU %d / %d / %d, grid %llu, sub %u, units %llu, lds %zu / %zu B, "
                    "cap %u, camera-ray pool %d, drain %d\n", WN, WAVES, per_n, per_f, per_r, (unsigned long long)bn, pn.sub,
                    (unsigned long long)units, sn, sf, pn.defer_cap, (int)POOL, (int)drain);
        // the chunk's counters (the redo bits are zero: the caller zeroes them once, reduce_samples after every chunk
        // that set any); with the drain each workgroup's region is the queue over the near grid (a region that fills
        // sends the rest to the redo pass)
        const bool drain_now = drain && 2 * bn + 2 <= DRAIN_WORDS;
        hipLaunchKernelGGL(chunk_start, dim3(1), dim3(256), 0, stream, pn, drain_now ? (uint32_t)(2 * bn) : 0u,
                           (uint32_t)(k0 == 0));
        if (drain_now) {
            pn.drain_region = pf.drain_region = pn.defer_cap / (uint32_t)bn;
            if constexpr (CAN_DRAIN)
                hipLaunchKernelGGL((render_drain<USE_LDS, WN, MN, HYB, POOL, ST, QUADS>), dim3((uint32_t)bn), dim3(block_n), sd,
                                   stream, DrainArgs{pn, far_layout(pf)});
        } else {
            hipLaunchKernelGGL(kn, dim3((uint32_t)bn), dim3(block_n), sn, stream, pn);
            hipLaunchKernelGGL(kf, dim3((uint32_t)per_f * cus), dim3(block), sf, stream, pf);
        }
        hipLaunchKernelGGL(spill_redo_list, dim3((uint32_t)cus * 4), dim3(256), 0, stream, pn);
        hipLaunchKernelGGL(kr, dim3((uint32_t)br), dim3(block), sf, stream, pr);
        hipLaunchKernelGGL(reduce_samples, dim3((uint32_t)((slots + 255) / 256)), dim3(256), 0, stream, pn,
                           (uint32_t)(k0 + pn.kn >= spp));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

#ifndef RTX_HYB_WAVES  // the same for scenes in HBM with an 80 KB LDS cache of their most-read entries
#define RTX_HYB_WAVES 12
#define RTX_HYB_MINW 6
#endif
#ifndef RTX_V3_WAVES  // workgroup size and waves per SIMD of the default v3 kernel (A/B builds override)
#define RTX_V3_WAVES 8
#define RTX_V3_MINW 6
#endif

template <bool COUNT, bool ST>
hipError_t launch_items_for(const Params& p, bool use_lds, hipStream_t stream) {
    if (p.has_noise) return p.n_quads ? launch_items<COUNT, true, true, 8, 0, false, false, ST>(p, use_lds, stream)
                                      : launch_items<COUNT, false, true, 8, 0, false, false, ST>(p, use_lds, stream);
    if (p.item_waves == 4)  // A/B: 4 waves per LDS copy of the scene
        return p.n_quads ? launch_items<COUNT, true, false, 4, 0, false, false, ST>(p, use_lds, stream)
                         : launch_items<COUNT, false, false, 4, 0, false, false, ST>(p, use_lds, stream);
    // 6 waves per SIMD: at most 80 VGPRs (the allocation granule is 8)
    constexpr int MV = COUNT ? 0 : RTX_V3_MINW, MH = COUNT ? 0 : RTX_HYB_MINW, MP = COUNT ? 0 : RTX_POOL_MINW;
    if (!use_lds && p.n_hot > HOT_ENTRIES_8W)  // an LDS cache past a third of the CU: 12-wave workgroups, two per CU
        return p.n_quads ? launch_items<COUNT, true, false, RTX_HYB_WAVES, MH, false, false, ST>(p, use_lds, stream)
                         : launch_items<COUNT, false, false, RTX_HYB_WAVES, MH, false, false, ST>(p, use_lds, stream);
    if (use_lds && pool_fits(p))  // the camera-ray pool (12-wave workgroups, two per CU) when the scene copy leaves room
        return p.n_quads ? launch_items<COUNT, true, false, RTX_POOL_WAVES, MP, false, true, ST>(p, use_lds, stream)
                         : launch_items<COUNT, false, false, RTX_POOL_WAVES, MP, false, true, ST>(p, use_lds, stream);
    return p.n_quads ? launch_items<COUNT, true, false, RTX_V3_WAVES, MV, false, false, ST>(p, use_lds, stream)
                     : launch_items<COUNT, false, false, RTX_V3_WAVES, MV, false, false, ST>(p, use_lds, stream);
}

uint32_t scene_placement(const Params& p, uint32_t flags) {
    // the whole scene in LDS (fixed layout) when its 'a' halves fit below LDS_B and all of it
    // in 64 KB; else from HBM, with the top levels cached in LDS when stored first (n_hot)
    if (!(flags & RTX_FLAG_NO_LDS) && (p.n_entries + 1) * 16 <= LDS_B &&
        lds_fixed_bytes(p.n_entries, p.n_quads, p.n_materials, p.n_textures) <= LDS_MAX_BYTES)
        return RTX_SCENE_IN_LDS;
    return p.n_hot > 0 && !p.has_noise ? RTX_SCENE_LDS_CACHE : RTX_SCENE_IN_HBM;
}

uint32_t tier_placement(const Params& near, const Params& far, uint32_t flags) {
    const uint32_t a = scene_placement(near, flags), b = scene_placement(far, flags);
    return a == b ? a : RTX_SCENE_IN_HBM;  // placed unalike: both passes read their layouts from HBM
}

// ST: the render's shard is striped (Params::stripe_log2 > 0): every kernel's ST instantiation (render_items).
template <bool ST>
hipError_t launch_render_t(const Params& p, uint32_t flags, hipStream_t stream, const Params* far) {
    const bool count = (flags & RTX_FLAG_COUNTERS) != 0;
    if (far) {  // the caller checked: spheres only, both layouts placed alike (tier_placement), no noise
        const uint32_t place = tier_placement(p, *far, flags);
        if ((p.w2 || far->w2) && place != RTX_SCENE_LDS_CACHE) return hipErrorInvalidValue;  // (records: cache kernels)
        if (p.tier != 1 || far->tier != 2 || !p.defer || !far->defer || !p.redo_bits || p.has_noise)
            return hipErrorInvalidValue;
        if (p.n_quads) {  // quads: single-row shards, the timed and counting kernels (rtx_capi's enqueue_on)
            if (ST || (!count && (flags & RTX_FLAG_TIMING))) return hipErrorInvalidValue;
            if constexpr (!ST) {
                constexpr int V = RTX_V3_WAVES, MV = RTX_V3_MINW, H = RTX_HYB_WAVES, MH = RTX_HYB_MINW;
                if (place == RTX_SCENE_IN_LDS) {
                    const bool pool = pool_fits(p);
                    if (count) return pool ? launch_tiered<true, V, 0, false, true, false, true, false, true>(p, *far, stream)
                                           : launch_tiered<true, V, 0, false, true, false, false, false, true>(p, *far, stream);
                    return pool ? launch_tiered<false, V, MV, false, true, false, true, false, true>(p, *far, stream)
                                : launch_tiered<false, V, MV, false, true, false, false, false, true>(p, *far, stream);
                }
                if (place == RTX_SCENE_LDS_CACHE)
                    return count ? launch_tiered<true, H, 0, false, false, true, false, false, true>(p, *far, stream)
                                 : launch_tiered<false, H, MH, false, false, true, false, false, true>(p, *far, stream);
                return count ? launch_tiered<true, V, 0, false, false, false, false, false, true>(p, *far, stream)
                             : launch_tiered<false, V, MV, false, false, false, false, false, true>(p, *far, stream);
            }
        }
        const bool clk = !count && (flags & RTX_FLAG_TIMING);  // diagnostics: the wave-cycle split of the passes
        constexpr int V = RTX_V3_WAVES, MV = RTX_V3_MINW, H = RTX_HYB_WAVES, MH = RTX_HYB_MINW;
        if (place == RTX_SCENE_IN_LDS) {
            const bool pool = pool_fits(p);  // (the counting kernel too: its schedule counters are the timed kernel's)
            if (clk) return pool ? launch_tiered<false, V, MV, true, true, false, true, ST>(p, *far, stream)
                                 : launch_tiered<false, V, MV, true, true, false, false, ST>(p, *far, stream);
            if (count) return pool ? launch_tiered<true, V, 0, false, true, false, true, ST>(p, *far, stream)
                                   : launch_tiered<true, V, 0, false, true, false, false, ST>(p, *far, stream);
            return pool ? launch_tiered<false, V, MV, false, true, false, true, ST>(p, *far, stream)
                        : launch_tiered<false, V, MV, false, true, false, false, ST>(p, *far, stream);
        }
        if (place == RTX_SCENE_LDS_CACHE)  // both cached in LDS (tier_placement): 12-wave workgroups, two per CU
            return count ? launch_tiered<true, H, 0, false, false, true, false, ST>(p, *far, stream)
                         : launch_tiered<false, H, MH, false, false, true, false, ST>(p, *far, stream);
        return count ? launch_tiered<true, V, 0, false, false, false, false, ST>(p, *far, stream)
                     : launch_tiered<false, V, MV, false, false, false, false, ST>(p, *far, stream);
    }
    const bool use_lds = scene_placement(p, flags) == RTX_SCENE_IN_LDS;
    if (p.w2 && scene_placement(p, flags) != RTX_SCENE_LDS_CACHE) return hipErrorInvalidValue;  // (records: cache kernels)
    if (!count && (flags & RTX_FLAG_TIMING) && !p.has_noise && p.item_waves != 4)  // diagnostics: sphere scenes
        return p.n_quads ? launch_items<false, true, false, RTX_V3_WAVES, RTX_V3_MINW, true, false, ST>(p, use_lds, stream)
                         : launch_items<false, false, false, RTX_V3_WAVES, RTX_V3_MINW, true, false, ST>(p, use_lds, stream);
    return count ? launch_items_for<true, ST>(p, use_lds, stream) : launch_items_for<false, ST>(p, use_lds, stream);
}

hipError_t launch_render(const Params& p, uint32_t flags, hipStream_t stream, const Params* far) {
    if (p.width == 0 || p.rows == 0) return hipSuccess;
    if (!p.scratch) return hipErrorInvalidValue;  // the caller sizes the sample scratch
    return p.stripe_log2 ? launch_render_t<true>(p, flags, stream, far) : launch_render_t<false>(p, flags, stream, far);
}

}  // namespace rtxd
