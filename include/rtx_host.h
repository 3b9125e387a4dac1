/*
 * rtx_host.h — C entry points of librtxhost.so, the C++ mirror of the reference's Go
 * `internal` package (raytracer-go_amd/host/).  These let test drivers and bench.py
 * (Python, via ctypes) build the reference's scenes exactly as main.go does and run
 * the full Camera.Render drop-in path; a Go host would not need them (it builds its
 * scenes in Go and calls rtx.h directly).
 */
#ifndef RTX_HOST_H
#define RTX_HOST_H

#include <stdint.h>

#include "rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rtxhost_scene rtxhost_scene;

/* Build a scene of main.go by name: "random_spheres" (main.go:227-289),
 * "stress_100k" (config 4), "earth_dielectric" (config 5), "earth" (main.go:80-104; its
 * map as jpeg.Decode's *image.YCbCr), "earth_rgba" (the same map as an *image.RGBA),
 * "earth_far_side" (main.go's earth seen from z = -12), "quad_demo", "cornell_box",
 * "perlin_demo", "simple_light_demo".
 * The BVH is built by the NewBVH restatement (bvh.go:142-185) and flattened. */
int rtxhost_build_scene(const char* name, uint64_t seed, rtxhost_scene** out);
void rtxhost_scene_free(rtxhost_scene* s);

/* The flattened tables (valid until rtxhost_scene_free). */
const rtx_scene_desc* rtxhost_scene_desc(const rtxhost_scene* s);

/* The planes of SyntheticEarth(seed, w, h), the *image.YCbCr 4:2:0 map the earth scenes
 * texture with: y[w*h], cb and cr [((w+1)/2) * ((h+1)/2)] each (strides w and (w+1)/2). */
int rtxhost_synthetic_earth_ycbcr(uint64_t seed, int32_t w, int32_t h, uint8_t* y, uint8_t* cb, uint8_t* cr);

/* color.YCbCr{y, cb, cr}.RGBA() as the mirror computes it: out = r, g, b, a. */
void rtxhost_ycbcr_rgba(uint8_t y, uint8_t cb, uint8_t cr, uint32_t out[4]);

/* The scene's camera (NewCamera with main.go's options), with overrides; a value
 * <= 0 keeps the scene's own setting. */
int rtxhost_scene_camera(const rtxhost_scene* s, int32_t image_width, int32_t samples_per_pixel, int32_t max_depth,
                         rtx_camera* out);

/* The whole drop-in path: NewCamera(...).Render(world, file) -> PPM at `path`. */
int rtxhost_render_ppm(const char* scene_name, uint64_t scene_seed, int32_t image_width, int32_t samples_per_pixel,
                       int32_t max_depth, uint64_t render_seed, int32_t n_gpus, const char* path);

/* PPM body lines for a linear float RGB image (ToGamma2, ToRGB, String per pixel);
 * returns the byte count, writing at most cap bytes (call with cap = 0 to size). */
uint64_t rtxhost_ppm_encode(const float* rgb, uint32_t width, uint32_t height, char* out, uint64_t cap);

/* The World the scene's BVH was built from, in World.Add order: its spheres (material
 * indices into rtxhost_scene_desc's table; at most cap written), the global-rand
 * position at NewBVHFromWorld and the scene seed — the inputs of
 * rtx_scene_create_spheres.  Returns the sphere count, or a negative rtx error code
 * if the World holds other primitives. */
int64_t rtxhost_scene_world_spheres(const rtxhost_scene* s, rtx_sphere* out, uint64_t cap, uint64_t* bvh_draw0,
                                    uint64_t* seed);

/* Last error of this thread from an rtxhost_* call. */
const char* rtxhost_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
