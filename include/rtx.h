/*
 * rtx.h — C-ABI of the MI355X path-tracing megakernel (librtx.so).
 *
 * This is the drop-in boundary for the hot path of TwFlem/raytracer-go:
 *
 *   func (c *Camera) Render(world Hittable, writer io.Writer) error      internal/camera.go:180
 *
 * The reference runs the per-pixel / per-sample loop on the CPU
 * (internal/camera.go:254-299 -> internal/ray.go:32-54 -> internal/bvh.go:220-249 ->
 * internal/hittables.go:96-132 -> internal/materials.go:33-193).  A drop-in host
 * (the Go package via cgo, or the C++ mirror in raytracer-go_amd/host/) walks its
 * Hittable tree once, flattens it into the POD tables below, and calls
 * rtx_scene_create() + rtx_render() instead of spawning one goroutine per pixel.
 * PPM formatting (camera.go:183-188, 212-215) stays on the host.
 *
 * Rules of the ABI
 *  - POD structs only, fixed-width types, little-endian; every array is 16-B aligned.
 *  - The caller owns every input table and the output buffer for the duration of a
 *    call.  The library copies what it needs into device memory and never retains a
 *    caller pointer (cgo rule: C must not keep Go memory).
 *  - Functions return 0 on success and a negative RTX_ERR_* code on failure; the
 *    message is available from rtx_last_error() (thread-local).  No exception or
 *    abort crosses the ABI.  This is what Render's `error` return maps to
 *    (camera.go:180, 230).
 *  - rtx_render* are blocking and not re-entrant for one rtx_scene (internal mutex).
 */
#ifndef RTX_H
#define RTX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 10

/* ---- status codes ------------------------------------------------------------ */
enum {
    RTX_OK = 0,
    RTX_ERR_INVALID_ARG = -1, /* null pointer, out-of-range index, bad size          */
    RTX_ERR_HIP = -2,         /* a HIP runtime call failed                            */
    RTX_ERR_RCCL = -3,        /* an RCCL call failed (multi-GPU gather)               */
    RTX_ERR_UNSUPPORTED = -4, /* a feature outside the GPU path (e.g. Perlin noise)   */
    RTX_ERR_NO_DEVICE = -5,   /* no gfx950 device visible                             */
    RTX_ERR_OOM = -6          /* device allocation failed                             */
};

/* ---- scene tables ------------------------------------------------------------ */

/* Child / root reference.  ref >= 0: index into rtx_scene_desc.nodes.
 * ref < 0: a primitive, p = ~ref, type = p >> 28 (RTX_PRIM_*), index = p & 0x0FFFFFFF.
 * RTX_PRIM_LIST (ABI 5): a World nested in the tree (a World handed to NewBVH as a child,
 * hittables.go:39-76): index into rtx_scene_desc.lists; its items are hit in order with a
 * running closest bound, (*World).Hit hittables.go:55-72. */
#define RTX_PRIM_SPHERE 0u
#define RTX_PRIM_QUAD 1u
#define RTX_PRIM_LIST 2u
#define RTX_REF_PRIM(type, index) ((int32_t) ~((int32_t)(((uint32_t)(type) << 28) | ((uint32_t)(index)&0x0FFFFFFFu))))

/* A BVH interior node exactly as internal/bvh.go:132-185 builds it: an AABB
 * (bvh.go:36-50, from NewAabbFromBoxes) and two children.  A one-element split
 * produces left == right (bvh.go:162-165); that is kept as-is in the table.   32 B */
typedef struct rtx_bvh_node {
    float bmin[3];
    int32_t left;
    float bmax[3];
    int32_t right;
} rtx_bvh_node;

/* internal/hittables.go:78-94 (NewSphere).                                       32 B */
typedef struct rtx_sphere {
    float center[3];
    float radius;
    uint32_t material;
    uint32_t pad[3];
} rtx_sphere;

/* internal/hittables.go:138-165 (NewQuad) — derived fields as the constructor
 * computes them (w = n / dot(n, n), normal = Unit(n), d = dot(normal, q)).      80 B */
typedef struct rtx_quad {
    float q[3];
    uint32_t material;
    float u[3];
    float d;
    float v[3];
    float pad0;
    float w[3];
    float pad1;
    float normal[3];
    float pad2;
} rtx_quad;

/* Materials, internal/materials.go:9-119, 297-313.                               */
enum {
    RTX_MAT_LAMBERTIAN = 0,    /* albedo = textures[texture]       materials.go:23-42   */
    RTX_MAT_METAL = 1,         /* albedo[3], fuzz                  materials.go:44-75   */
    RTX_MAT_DIELECTRIC = 2,    /* ior                              materials.go:77-119  */
    RTX_MAT_DIFFUSE_LIGHT = 3  /* emit = textures[texture]         materials.go:297-313 */
};
typedef struct rtx_material { /* 32 B */
    uint32_t type;
    uint32_t texture;
    float fuzz;
    float ior;
    float albedo[3];
    float pad;
} rtx_material;

/* Textures, internal/materials.go:121-193, 280-295.                              */
enum {
    RTX_TEX_SOLID = 0,     /* even[3] = colour                       materials.go:151-163 */
    RTX_TEX_CHECKERED = 1, /* scale, even[3], odd[3]                 materials.go:121-145 */
    RTX_TEX_IMAGE = 2,     /* width x height RGBA16 texels at texel_offset (row-major,
                              y down), then ONE border texel: see below materials.go:165-193 */
    RTX_TEX_NOISE = 3      /* Perlin: scale, and RTX_NOISE_TEXELS words at texel_offset:
                              256 gradient vectors (x, y, z float32 bits), then permX,
                              permY, permZ (256 indices each)        materials.go:195-295 */
};
#define RTX_NOISE_TEXELS 1536u
/* RTX_TEX_IMAGE texels are Go's `img.At(x, y).RGBA()` (materials.go:188), 16 bits per
 * channel, two uint32 words per texel: word 0 = r | g << 16, word 1 = b | a << 16.
 * The texel at index width*height (after the raster) is the colour At() returns OUTSIDE
 * the image's bounds, which GetTexture reads when int(u*Dx) == Dx or int(v*Dy) == Dy
 * (u == 1, v == 0) or a NaN coordinate (int(NaN) = MinInt64 on amd64): for the
 * *image.YCbCr that jpeg.Decode returns that is color.YCbCr{} = (0, 34678, 0)
 * (image/ycbcr.go YCbCrAt, image/color/ycbcr.go RGBA), for *image.RGBA it is 0.
 * The host fills it with At(Bounds().Max.X, Bounds().Min.Y).RGBA().  Exact for every
 * image whose Bounds().Min is (0, 0) (jpeg.Decode, image.New*); texel_offset is even
 * and n_texels counts uint32 words.  Texels are fetched as
 * float32(r16) * float32(1/65535) (materials.go:187-191).                        */
#define RTX_IMAGE_TEXEL_WORDS 2u
typedef struct rtx_texture { /* 48 B */
    uint32_t type;
    float scale;
    uint32_t width;
    uint32_t height;
    float even[3];
    uint32_t texel_offset;
    float odd[3];
    float pad;
} rtx_texture;

/* A World nested in the tree: the refs list_refs[first .. first + count), in Add order.  8 B */
typedef struct rtx_list {
    uint32_t first;
    uint32_t count;
} rtx_list;

typedef struct rtx_scene_desc {
    const rtx_bvh_node* nodes;
    uint32_t n_nodes;
    uint32_t n_roots;
    /* The world handed to Render: a BVH gives one root ref (the tree); a plain World
     * (hittables.go:39-76, linear closest-hit scan in insertion order) gives its items. */
    const int32_t* roots;
    const rtx_sphere* spheres;
    uint32_t n_spheres;
    uint32_t n_quads;
    const rtx_quad* quads;
    const rtx_material* materials;
    uint32_t n_materials;
    uint32_t n_textures;
    const rtx_texture* textures;
    const uint32_t* texels; /* image RGBA16 texels and Perlin tables (uint32 words) */
    uint64_t n_texels;
    /* ABI 5: Worlds nested in the tree (RTX_PRIM_LIST refs); zero / NULL when there are none. */
    const rtx_list* lists;
    uint32_t n_lists;
    uint32_t n_list_refs;
    const int32_t* list_refs;
} rtx_scene_desc;

/* ---- camera ------------------------------------------------------------------ */
/* The derived state of Camera.init (internal/camera.go:128-165), computed by the
 * host exactly as the reference does and uploaded as kernel constants.           */
typedef struct rtx_camera {
    uint32_t image_width;       /* int(c.imageWidth)                     camera.go:181 */
    uint32_t image_height;      /* int(c.imageHeight)                    camera.go:182 */
    uint32_t samples_per_pixel; /* c.samplesPerPixel                     camera.go:256 */
    uint32_t max_depth;         /* c.bounceDepth                         camera.go:258 */
    float center[3];
    float defocus_angle; /* radians; > 0 enables the thin lens          camera.go:279 */
    float pixel00[3];
    float pad0;
    float pixel_du[3];
    float pad1;
    float pixel_dv[3];
    float pad2;
    float defocus_disk_u[3];
    float pad3;
    float defocus_disk_v[3];
    float pad4;
    float background[3];
    float pad5;
} rtx_camera;

/* ---- render region / shard ---------------------------------------------------- */
/* Pixels x in [x0, x0+width), rows y = y0 + r for r in [0, height) whose STRIPE
 * (r / stripe, stripes of `stripe` rows; 0 or 1: single rows) is rank modulo world:
 * stripes dealt round-robin to the shards, so sky and ground are balanced across GPUs.
 * Output rows are stored compacted in shard order: shard row i is image row
 * y0 + rtx_region_row(region, i).  The RNG is keyed by the GLOBAL pixel index
 * y*image_width + x, so every pixel's value is independent of the region, the stripe
 * and the shard count.  ABI 9 added `stripe` (a power of two, at most 4096): 8-row
 * stripes keep a shard's 8x8 work tiles compact in the image (rtx_render with
 * n_gpus > 1 uses them).                                          */
typedef struct rtx_region {
    uint32_t x0, y0, width, height;
    uint32_t rank, world;
    uint32_t stripe;
} rtx_region;



/* Work counters of one render (filled when RTX_FLAG_COUNTERS is set).  These are
 * the units of SURVEY.md §8(d): segments = world.Hit calls (ray.go:36).          */
typedef struct rtx_stats {
    uint64_t samples;
    uint64_t segments;
    uint64_t node_visits;  /* AABB slab tests   (bvh.go:221)                        */
    uint64_t prim_tests;   /* ray-primitive tests (hittables.go:96), duplicates of
                              a one-element split skipped (bit-identical, §8a a5)   */
    uint64_t hits;         /* segments that hit a primitive                          */
    uint64_t texel_fetches;
    uint64_t rng_draws;
    double kernel_ms;      /* device time of the render kernels, HIP events on the render
                              stream (n_gpus > 1: the slowest device)                */
    double gather_ms;      /* rtx_render with n_gpus > 1: the RCCL gather of the bands to
                              device 0 plus the de-interleave, HIP events on device 0  */
    /* scheduling counters of the persistent kernel (RTX_FLAG_COUNTERS):             */
    uint64_t wave_iters;   /* traversal-loop iterations, summed over waves           */
    uint64_t lane_steps;   /* lanes stepping a BVH entry, summed over iterations     */
    uint64_t shade_phases; /* shading phases, summed over waves                      */
    uint64_t shade_lanes;  /* lanes shaded or claiming, summed over shading phases   */
    uint64_t trav_cycles;  /* shader cycles (s_memtime) in traversal, summed over waves */
    uint64_t shade_cycles; /* shader cycles in shading phases, summed over waves      */
    uint64_t idle_lanes;   /* lanes with no item left, summed over iterations         */
    uint64_t cache_hits;   /* scenes too big for LDS: entries (of node_visits + prim_tests and
                              the steps on the end sentinel) read from the LDS cache of the top
                              levels */
    uint64_t sample_chunks; /* launches of the render kernel: the samples of every pixel run in
                               chunks that fit the per-device colour scratch (always filled) */
    uint64_t parked_lanes;   /* lanes parked on the end sentinel (waiting to shade, or without
                                an item) per walk step, summed over steps / steps per vote   */
    uint64_t deferred_lanes; /* lanes whose entry kind (node / primitive) a batched walk step
                                did not run, likewise                                        */
    uint64_t shade_split_cycles[4]; /* shade_cycles split: scatter sampling, shading, item claims +
                                       camera rays, segment starts (1/dir)                    */
    uint64_t walk_layout;   /* ABI 6: the layout walked: 0-7 = the camera octant of a rebuilt tree
                               (rtx_scene_topology), RTX_LAYOUT_REFERENCE = the caller's tree  */
    uint64_t gather_kind;   /* ABI 6, rtx_render: how the bands were assembled (RTX_GATHER_*)    */
    uint64_t scene_placement; /* ABI 6: where the walk read the scene (RTX_SCENE_IN_LDS / ...)    */
    uint64_t deferred_paths;  /* ABI 8, tiered walk: paths the near pass handed to the far pass  */
    uint64_t redo_chunks;     /* ABI 8, tiered walk: sample chunks whose queue of deferred paths
                                 overflowed: the samples that did not fit were rendered again from
                                 their camera rays on the far tree (the rest of the chunk is not) */
} rtx_stats;
#define RTX_SCENE_IN_HBM 0u    /* entries from HBM (through L2)                                   */
#define RTX_SCENE_IN_LDS 1u    /* the whole scene and its materials copied into LDS per workgroup */
#define RTX_SCENE_LDS_CACHE 2u /* top levels cached in LDS, the rest from HBM                     */
#define RTX_LAYOUT_REFERENCE 8u
#define RTX_LAYOUT_TIERED 16u  /* ABI 8: walk_layout bit: the render walked in two tiers (RTX_SCENE_NO_TIER) */
#define RTX_GATHER_NONE 0u   /* one band: it is the image                                        */
#define RTX_GATHER_RCCL 1u   /* ncclGather of the padded bands to device 0, de-interleave kernel  */
#define RTX_GATHER_DEVICE 2u /* RTX_SIM_BANDS (tests): bands on device 0, device copies, kernel   */
#define RTX_GATHER_HOST 3u   /* RCCL unavailable or failed (or RTX_NO_RCCL=1): each band's rows
                                copied into the caller's buffer                                 */

#define RTX_FLAG_COUNTERS 1u /* count work units (separate kernel instantiation) */
#define RTX_FLAG_NO_LDS 4u   /* A/B: read the scene from global memory even if it fits LDS */
#define RTX_FLAG_TIMING (1u << 20) /* diagnostics: the timed kernel with the wave-cycle split of
                                      rtx_stats (trav_cycles, shade_cycles, shade_split_cycles) */
/* Bits 2u, 8u, 16u, 32u, 64u and RTX_FLAG_WAVE_GEOM (bits 24-26) selected the A/B schedules
 * v0/v1/v2 of ABI 3; they were removed in ABI 4 and are ignored. */
/* Tuning: lanes of a wave that must wait before it shades (1..64; 0 = default, or the
 * RTX_SHADE_THRESH environment variable). */
#define RTX_FLAG_SHADE_THRESH(n) (((uint32_t)(n)&0x7Fu) << 8)

typedef struct rtx_scene rtx_scene;

/* ---- entry points ------------------------------------------------------------- */

/* ABI version (RTX_ABI_VERSION) and a static build string. */
int rtx_version(void);
const char* rtx_build_info(void);

/* Last error message of this thread ("" if none). */
const char* rtx_last_error(void);

/* Number of visible GPUs (0 if none). */
int rtx_device_count(void);

/* Validate the tables, convert them to the device layout and upload them once to
 * the current HIP device (replicated to further devices lazily by rtx_render).
 * Replaces the tree walk the reference does on every ray (bvh.go:220).           */
int rtx_scene_create(const rtx_scene_desc* desc, rtx_scene** out);

/* ABI 6.  rtx_scene_create with build flags.  By default a scene whose world is one BVH over
 * spheres (NewBVHFromWorld of a World of spheres, main.go:287) is walked over the library's
 * own tree of the same spheres: a binned surface-area-heuristic split, each node's near child
 * (along the camera's viewing direction) first.  The closest hit bvh.go:220-249 returns is
 * the nearest sphere root among the spheres whose boxes the ray passes, whichever tree the
 * boxes come from; the reference's tree (median splits on a random axis, bvh.go:142-185)
 * costs 1.8x the box tests and 4x the sphere tests on randSpheres (DESIGN.md §12 states the
 * floating-point caveat and how the tests check it).  RTX_SCENE_REFERENCE_BVH keeps the
 * caller's tree and the reference's visit order (left, then right) as they are; so do the
 * environment variable RTX_BVH=reference and every scene with quads, nested Worlds or a
 * World root.  rtx_scene_create(d, out) = rtx_scene_create_ex(d, 0, out).              */
#define RTX_SCENE_REFERENCE_BVH 1u
/* ABI 7.  The collapsed walk: a walk leaves out the box tests of tree nodes
 * whose children are all nodes where that saves tests on sample paths from the first camera
 * rendered with each layout.  A child's box lies inside its parent's and the slab test is
 * monotone in the box, so no primitive test, hit, path or image bit changes — only
 * rtx_stats.node_visits.  RTX_SCENE_EVERY_BOX (or RTX_COLLAPSE=0 in the environment) keeps
 * every box test, as bvh.go:220-249 makes them. */
#define RTX_SCENE_EVERY_BOX 2u
/* ABI 8.  The tiered walk.  A scene of spheres under one tree whose node
 * boxes contain the boxes of the spheres below them (every NewBVH tree) also gets a NEAR tree:
 * the spheres themselves as leaves, each behind its own box grown by the float32 sphere test's
 * derived error bound for ray origins inside a NEAR REGION (the box of the scene's non-huge
 * spheres, grown by 1.5 times its largest extent — by 1 % of it for scenes the rebuild's precision
 * gate refuses, config 4).  A render whose camera lies in the region walks every segment that starts
 * there on the near tree, and accepts a near hit only when the sphere's own box passes with the
 * bound just past it; a path whose segment starts outside the region, or whose near hit fails
 * that check, is handed, once, to a second pass that continues it on the FAR tree: the guarded
 * rebuild (the reference's leaves) when the scene has one, else the caller's own tree.  The
 * closest hit of every segment is the one bvh.go:220-249 returns, ties included (DESIGN.md §15
 * states why and what the tests check).  RTX_SCENE_NO_TIER (or RTX_TIER=0 in the environment)
 * walks the far tree alone; RTX_SCENE_REFERENCE_BVH keeps the caller's tree alone. */
#define RTX_SCENE_NO_TIER 4u
int rtx_scene_create_ex(const rtx_scene_desc* desc, uint32_t flags, rtx_scene** out);

/* The tree a rebuilt scene walks for camera octant `octant` (rtx_camera_octant): *n_nodes
 * nodes with `left` the child visited first; sphere refs index the caller's sphere table;
 * *root is the root ref.  nodes is filled when cap >= *n_nodes.  A scene that keeps the
 * caller's tree reports *n_nodes = 0, *root = -1.  For tests and tools.                */
int rtx_scene_topology(const rtx_scene* scene, uint32_t octant, rtx_bvh_node* nodes, uint32_t cap, uint32_t* n_nodes,
                       int32_t* root);
/* ABI 8: octant | RTX_TREE_NEAR names the near tree of a tiered scene (rtx_scene_topology,
 * rtx_walk_tree; *n_nodes = 0, *root = -1 when the scene has none). */
#define RTX_TREE_NEAR 0x100u

/* The same without a scene or a device: the tree rtx_scene_create_ex(desc, flags) walks for
 * `octant` (*n_nodes = 0, *root = -1 when it would keep the caller's).  Host only.       */
int rtx_walk_tree(const rtx_scene_desc* desc, uint32_t flags, uint32_t octant, rtx_bvh_node* nodes, uint32_t cap,
                  uint32_t* n_nodes, int32_t* root);

/* ABI 7.  The box tests the walk for `cam` leaves out: skip[k] = 1 for the k-th node entry of
 * the uncollapsed walk (the walked tree — rtx_scene_topology's, or the caller's — in visit
 * order: a node, then its first child's subtree, then its second's).  *n = the number of node
 * entries; skip is filled when cap >= *n.  The walk for a layout is planned on that layout's
 * first render (or on this call); later cameras of the same layout reuse it.  For tests and
 * tools (the oracle walks the same skips: parity of node_visits).                        */
int rtx_scene_walk_skip(rtx_scene* scene, const rtx_camera* cam, uint8_t* skip, uint32_t cap, uint32_t* n);

/* The same without a scene or a device: the skips rtx_scene_create_ex(desc, flags) plans for
 * a first render with `cam`.  Host only.                                                   */
int rtx_walk_skip(const rtx_scene_desc* desc, uint32_t flags, const rtx_camera* cam, uint8_t* skip, uint32_t cap,
                  uint32_t* n);

/* ABI 8.  The near region of a tiered scene (box = min xyz, max xyz; a segment whose origin o
 * has box[k] <= o[k] <= box[3 + k] for every k starts in it, a NaN origin does not; box is left
 * alone when the scene has no near tree), and *active = whether renders with `cam` qualify:
 * the camera's rays start in the region, spheres only, no Perlin texture (rtx_stats.walk_layout
 * & RTX_LAYOUT_TIERED says that a render walked in two tiers).  For tests and tools. */
int rtx_scene_near_region(rtx_scene* scene, const rtx_camera* cam, float box[6], uint32_t* active);
/* ABI 8.  rtx_scene_walk_skip of the near walk for `cam` (over rtx_scene_topology's
 * octant | RTX_TREE_NEAR tree). */
int rtx_scene_near_skip(rtx_scene* scene, const rtx_camera* cam, uint8_t* skip, uint32_t cap, uint32_t* n);
/* ABI 8.  The same without a scene or a device: the near region rtx_scene_create_ex(desc,
 * flags) would walk with and *active for `cam`.  Host only. */
int rtx_walk_near_region(const rtx_scene_desc* desc, uint32_t flags, const rtx_camera* cam, float box[6],
                         uint32_t* active);

/* Octant of the camera's viewing direction (pixel00 + du W/2 + dv H/2 - center): bit k set
 * when it points to negative axis k. */
uint32_t rtx_camera_octant(const rtx_camera* cam);

/* Release device memory owned by the scene (NULL is a no-op). */
void rtx_scene_destroy(rtx_scene* scene);

/* Size of the device layout in bytes (entries + materials + textures + texels). */
uint64_t rtx_scene_device_bytes(const rtx_scene* scene);

/* The whole of Camera.Render's pixel loop (camera.go:198-222): render every pixel
 * of the image, averaged over samples_per_pixel, linear (pre-gamma) float32 RGB,
 * row-major, rows top to bottom, into caller-owned host memory out_rgb[W*H*3].
 * n_gpus > 1 row-interleaves the image over devices 0..n_gpus-1 of this process
 * (rank d renders rows y = d, d + n, ...), gathers the equal-sized bands to device 0
 * with one RCCL ncclGather over xGMI (communicators from ncclCommInitAll, cached per
 * device set; librccl is loaded on first use), de-interleaves them on device 0 and
 * copies the image to the host.  Without RCCL (not loadable, or a failing
 * CommInitAll / Gather) each band's rows are copied into out_rgb instead: slower,
 * same bits (stats->gather_kind says which).  The band, gather and image buffers are
 * kept per device between calls (rtx_release_device_memory frees them).
 * stats (optional) receives the time (kernel_ms, gather_ms), samples, sample_chunks,
 * walk_layout and gather_kind of the call; its work counters stay 0: rtx_render runs the
 * timed kernel.  rtx_render = rtx_render_ex(..., flags = 0, ...).                     */
int rtx_render(rtx_scene* scene, const rtx_camera* cam, uint64_t seed, int n_gpus, float* out_rgb,
               rtx_stats* stats);

/* ABI 6: rtx_render with flags: RTX_FLAG_COUNTERS runs the counting kernel instead (same
 * image; every work counter of stats filled; about twice the kernel time of the timed
 * kernel on the headline config).                                                     */
int rtx_render_ex(rtx_scene* scene, const rtx_camera* cam, uint64_t seed, int n_gpus, uint32_t flags,
                  float* out_rgb, rtx_stats* stats);

/* Free the device memory the library keeps between renders on `device` (-1: every
 * device): the per-device sample-colour scratch (up to RTX_SCRATCH_MB, 12 B per
 * sample of a chunk) and the cached RCCL communicators.  Scenes are not affected;
 * the next render allocates again.  The scratch of a device is also freed when the
 * last scene with a copy on that device is destroyed.  Blocking.                   */
int rtx_release_device_memory(int device);

/* Bytes of the per-device scratch currently held on `device` (for tests and tools). */
uint64_t rtx_device_scratch_bytes(int device);

/* ABI 10.  Wait for every render enqueued on `device` and report whether any of them failed inside the
 * kernel since the last report: RTX_OK, or RTX_ERR_HIP when a wave hit the watchdog (RTX_WATCHDOG_S) or
 * reached a wave-level claim without the whole wave (the output of that render is then invalid).  The
 * kernel's error word is sticky: no later render clears it, so renders enqueued back to back without
 * stats (rtx_render_region_device with stats == NULL) are checked by ONE call after the last of them.
 * A render that returns stats reports (and acknowledges) the same word itself.  The report is
 * acknowledged: a second call without a failed render in between returns RTX_OK.  Blocking.
 * The Go side: the error a pipelined Render loop returns once (camera.go:180, 230). */
int rtx_device_check(int device);

/* Render one region/shard on the CURRENT device into device memory d_out (float32
 * RGB, compacted shard rows, see rtx_region) on the given HIP stream (hipStream_t,
 * NULL = default stream).  Returns after enqueueing unless stats != NULL, in which
 * case it synchronises the stream and fills stats (kernel_ms from HIP events
 * recorded on that same stream).  This is the entry a one-process-per-GPU launcher
 * (torch.distributed / RCCL) uses.                                               */
int rtx_render_region_device(rtx_scene* scene, const rtx_camera* cam, uint64_t seed, const rtx_region* region,
                             float* d_out, void* hip_stream, uint32_t flags, rtx_stats* stats);

/* Number of output rows of a region shard: the rows of the stripes rank, rank + world, ... that
 * lie in [0, height) (ceil((height - rank) / world) for single-row stripes). */
uint32_t rtx_region_rows(const rtx_region* region);
/* ABI 9.  The row (relative to y0) of shard row i of a region: row i % S of stripe (i / S) * world + rank
 * (S = max(stripe, 1)). */
uint32_t rtx_region_row(const rtx_region* region, uint32_t i);

/* ---- BVH build on the GPU ----------------------------------
 * rtx_scene_create for NewBVHFromWorld(world) (bvh.go:138-185) of a World holding only
 * spheres, with the BVH built on the current device instead of by the caller: spheres
 * in World.Add order; the k-th NewBVH call (pre-order) takes Intn(3) from word
 * bvh_draw0 + k of the global host stream of bvh_seed (the RNG contract, DESIGN.md
 * §3), which is the axis the host builder draws.  The scene equals the one
 * rtx_scene_create makes from the host-built tree (same entries, tests).  build_ms
 * (optional) receives the build's wall time.                                        */
int rtx_scene_create_spheres(const rtx_sphere* spheres, uint32_t n_spheres, const rtx_material* materials,
                             uint32_t n_materials, const rtx_texture* textures, uint32_t n_textures,
                             const uint32_t* texels, uint64_t n_texels, uint64_t bvh_seed, uint64_t bvh_draw0,
                             rtx_scene** out, double* build_ms);

/* Copy the scene's threaded BVH entries (32 B each, rtx_layout.h order) to out when
 * cap is large enough; returns their size in bytes.  For tests and tools.            */
uint64_t rtx_scene_export(const rtx_scene* scene, void* out, uint64_t cap);

/* ---- PPM output on the GPU ---------------------------------
 * Render's output tail, camera.go:183-188 and 212-215 with vec3.go:141-166: the P3
 * header "P3\n<W> <H>\n255\n", then per pixel int(Clamp(0,1,float32(sqrt(c)))*255.999)
 * for R, G, B as "%d %d %d\n" (a NaN channel prints Go's int(NaN) = MinInt64).     */

/* Upper bound of the PPM text of a width x height image (header + 63 B per pixel). */
uint64_t rtx_ppm_max_bytes(uint32_t width, uint32_t height);

/* Encode a float32 RGB image in device memory (d_rgb, width*height*3, row-major) into
 * device memory d_text (capacity bytes) on the current device and the given stream;
 * synchronises that stream and stores the text length in *out_len.  Replaces the
 * reference's per-pixel fmt.Sprintf + channel pipeline (camera.go:198-231).          */
int rtx_encode_ppm_device(const float* d_rgb, uint32_t width, uint32_t height, char* d_text, uint64_t capacity,
                          uint64_t* out_len, void* hip_stream);

/* Render + encode on the current device and copy the PPM text to the caller's host
 * buffer: the bytes (*Camera).Render(world, writer) writes (camera.go:180).  Blocking. */
int rtx_render_ppm(rtx_scene* scene, const rtx_camera* cam, uint64_t seed, char* out_text, uint64_t capacity,
                   uint64_t* out_len, rtx_stats* stats);

/* ABI 9.  rtx_render_ppm for n_gpus devices: the bands rendered and gathered to device 0 exactly
 * as rtx_render(n_gpus) does (one RCCL ncclGather over xGMI and the de-interleave kernel, or the
 * per-band copies without RCCL), then the PPM encoded ON device 0 (rtx_encode_ppm_device) and only
 * the text copied to the caller: the multi-GPU (*Camera).Render(world, writer) of camera.go:180-231
 * with no per-pixel formatting on the host.  Devices 0..n_gpus-1 (n_gpus <= 1: device 0, one band;
 * RTX_SIM_BANDS=k simulates k bands on device 0 as rtx_render does).  The bytes equal
 * rtx_render_ppm's for any n_gpus.  stats as rtx_render's.  Blocking. */
int rtx_render_ppm_ex(rtx_scene* scene, const rtx_camera* cam, uint64_t seed, int n_gpus, char* out_text,
                      uint64_t capacity, uint64_t* out_len, rtx_stats* stats);

#ifdef __cplusplus
}
#endif

#endif /* RTX_H */
