/*
 * oracle.h — CPU restatement of TwFlem/raytracer-go's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / CPU baseline,
 * never as the product path.
 *
 * Parity status: PARITY UNPINNED against the reference binary.  The reference is Go
 * (no Go toolchain in this image or on the GPU box), it ships no tests, no fixtures
 * and no golden image (its one PPM is stripped, .MISSING_LARGE_BLOBS:1), and it is
 * nondeterministic by construction (time-seeded RNGs, camera.go:170, main.go:246;
 * global rand in materials.go:103 and bvh.go:147).  The oracle is therefore a
 * line-by-line restatement of the cited Go source with the reference's RNG replaced
 * by the counter-based RNG contract of SURVEY.md §8c (Philox4x32-10, pinned by the
 * published Random123 known-answer vectors), plus known-answer tests derived from the
 * source text (tests/test_oracle_kat.py).
 *
 * Every function cites the reference file:line it restates.  Float semantics: IEEE
 * float32, no contraction (built with -ffp-contract=off), float64 exactly where the Go
 * code widens to float64.
 */
#ifndef RTX_ORACLE_H
#define RTX_ORACLE_H

#include <stdint.h>

#include "../include/rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Colour evaluation order of Ray.GetColor.
 *  REFERENCE: the recursion of ray.go:32-54, emit + att * GetColor(depth-1).
 *  ITERATIVE: L += T*emit; T *= att (front to back) — same path decisions, the colour
 *  product is rounded in the other order.  The HIP kernel uses this order, so it must
 *  match the ITERATIVE oracle bit for bit and the REFERENCE oracle to ~1 ulp.       */
enum { ORACLE_ORDER_REFERENCE = 0, ORACLE_ORDER_ITERATIVE = 1 };

typedef struct oracle_counters {
    uint64_t samples;
    uint64_t segments;        /* world.Hit calls, ray.go:36                         */
    uint64_t node_visits;     /* Aabb.Hit calls, bvh.go:221                         */
    uint64_t prim_tests_ref;  /* Sphere.Hit calls as the reference makes them        */
    uint64_t prim_tests;      /* ... minus the redundant second test of left==right  */
    uint64_t hits;
    uint64_t texel_fetches;
    uint64_t rng_draws;
    uint64_t texel_border;    /* image fetches outside the bounds (the border texel)   */
} oracle_counters;

/* Philox4x32-10 (Salmon et al., SC'11; Random123). */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* The per-sample RNG contract: Philox block of (global pixel, sample, event, attempt). */
void oracle_pixel_block(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t event, uint32_t attempt,
                        uint32_t out[4]);

/* Host streams (scene generation / BVH axis): word n of stream s. */
uint32_t oracle_stream_u32(uint64_t seed, uint32_t stream, uint64_t n);

/* Camera options as the reference's functional options leave them (camera.go:56-117). */
typedef struct oracle_camera_opts {
    int32_t samples_per_pixel;
    int32_t max_depth;
    float fov_radians;     /* default float32(PiO2)                     camera.go:108 */
    float look_from[3];
    float look_at[3];
    float vup[3];
    float defocus_radians;
    float focus_dist;
    float background[3];
} oracle_camera_opts;

void oracle_camera_defaults(oracle_camera_opts* o);               /* camera.go:105-117 */
float oracle_to_radians(float degrees);                           /* math.go:50-52      */
/* Camera.init restated (camera.go:128-165). */
void oracle_camera_init(float aspect_ratio, int32_t image_width, const oracle_camera_opts* o, rtx_camera* out);

/* Render a region (rtx.h semantics).  threads <= 0 -> 1.  out holds
 * rtx_region_rows(region) * region->width * 3 floats.  counters may be NULL.
 * Returns 0, or -1 on bad arguments / unsupported scene features.                */
/* Walk hooks for probes and collapsed-walk parity (NULL = off): per-node box tests and passes
 * (indexed like desc->nodes, counted atomically), and nodes whose box test is left out. */
void oracle_node_hooks(uint64_t* tested, uint64_t* passed, const uint8_t* skip);

/* Tiered-walk hook (NULL far = off): a segment whose origin lies outside near_box (min xyz, max
 * xyz; NaN is outside) walks `far` (same spheres and materials, its own node table and roots)
 * with far_skip instead of the rendered description. */
void oracle_tier(const float near_box[6], const rtx_scene_desc* far, const uint8_t* far_skip);

/* Tie-rule hook (NULL = off): rank[i] = sphere i's place in the reference walk.  A root equal to
 * the running bound then wins when its sphere ranks before the bound's hit, as it would in the
 * reference's order (the device's walks over rebuilt trees do the same). */
void oracle_sphere_rank(const uint32_t* rank);

int oracle_render(const rtx_scene_desc* scene, const rtx_camera* cam, uint64_t seed, const rtx_region* region,
                  int order, int threads, float* out, oracle_counters* counters);

/* One sample of one pixel (GetRay + GetColor), for tracing individual paths. */
int oracle_sample(const rtx_scene_desc* scene, const rtx_camera* cam, uint64_t seed, uint32_t px, uint32_t py,
                  uint32_t k, int order, float rgb[3], oracle_counters* counters);

/* Output path: ToGamma2 -> ToRGB -> String (vec3.go:141-166), into buf (>= 64 B).
 * Returns the string length. */
int oracle_ppm_pixel(const float rgb[3], char* buf);

/* ---- scene builders (main.go restated with the seeded streams) ---------------- */
typedef struct oracle_scene oracle_scene;
/* randSpheres, main.go:227-289 (scene + NewBVHFromWorld, bvh.go:138-185). */
oracle_scene* oracle_build_random_spheres(uint64_t seed);
const rtx_scene_desc* oracle_scene_desc(const oracle_scene* s);
void oracle_scene_free(oracle_scene* s);

/* Go's math.Atan2 / math.Acos algorithms (the UV of hittables.go:122-123). */
double oracle_go_atan2(double y, double x);
double oracle_go_acos(double x);
double oracle_go_sin(double x); /* Go 1.21 math.Sin (sin.go + trig_reduce.go) */
/* NoiseTexture.GetTexture (materials.go:280-288) over an RTX_NOISE_TEXELS table. */
float oracle_noise_texture(const uint32_t* tab, float scale, const float p[3]);

/* color.YCbCr{y, cb, cr}.RGBA() (Go image/color/ycbcr.go): out = r, g, b (16-bit). */
void oracle_ycbcr_rgba(uint8_t y, uint8_t cb, uint8_t cr, uint32_t out[3]);
/* ... for every (y, cb, cr), k = y << 16 | cb << 8 | cr: out[3 * k + c] (3 * 2^24 words). */
void oracle_ycbcr_rgba_all(uint32_t* out);
/* The RTX_TEX_IMAGE texels (RGBA16 raster + border) of an *image.YCbCr with Bounds
 * (0,0)-(w,h): At(x, y).RGBA() via YCbCrAt / COffset (image/ycbcr.go); ratio 0..5 =
 * 4:4:4, 4:2:2, 4:2:0, 4:4:0, 4:1:1, 4:1:0.  out: 2 * (w * h + 1) words. */
int oracle_ycbcr_texels(const uint8_t* Y, const uint8_t* Cb, const uint8_t* Cr, int64_t w, int64_t h,
                        int64_t ystride, int64_t cstride, int ratio, uint32_t* out);

/* Test hook: the tiered walk's near-tree slab test (its FMA form) of ray i
 * (origin o[3i..], direction d[3i..]) against box i (mn, mx) with the interval (lo[i], hi[i]):
 * out[i] = 1 when it passes. */
void oracle_near_slab_pass(const float* o, const float* d, const float* mn, const float* mx, const float* lo,
                           const float* hi, uint8_t* out, uint64_t n);

/* Independent recompute of rtx_region_rows. */
uint32_t oracle_region_rows(const rtx_region* r);

#ifdef __cplusplus
}
#endif
#endif
