/* trace_walk.c — measurement tool (not product code): every segment of a render traced by the
 * oracle on the caller's tree (the reference's, bvh.go:220-249) and again, on the same ray, on
 * the tree the library walks (rtx_walk_tree; RTX_BVH=sah for the unguarded tree); prints every
 * segment whose closest hit differs (t or material) with its ray.
 *
 *   gcc -O2 -std=c11 -ffp-contract=off -fno-fast-math -D_GNU_SOURCE -o /tmp/trace_walk scripts/trace_walk.c \
 *       -Lraytracer-go_amd -lrtxhost -lrtx -Wl,-rpath,$PWD/raytracer-go_amd -lm -lpthread
 *   /tmp/trace_walk <scene> <width> <spp> <part> <parts> [px py]    (rows part, part + parts, ...)
 */
#include "../oracle/oracle.c"
#include "../include/rtx_host.h"
static const rtx_scene_desc* WD;
static int32_t hit_prim(const ctx_t* cx, const ray_t* r, hit_t* h, int* ok) { *ok = world_hit(cx, r, 0.001f, INFINITY, h); return 0; }
#define SEED 2024
int main(int argc, char** argv) {
    const char* name = argv[1]; int width = atoi(argv[2]); int spp = atoi(argv[3]); int part = atoi(argv[4]), parts = atoi(argv[5]);
    rtxhost_scene* hs = NULL;
    if (rtxhost_build_scene(name, 1, &hs)) return 1;
    const rtx_scene_desc* s = rtxhost_scene_desc(hs);
    rtx_camera cam; rtxhost_scene_camera(hs, width, spp, 0, &cam);
    uint32_t n = 0; int32_t root = -1;
    uint32_t oct = rtx_camera_octant(&cam);
    rtx_walk_tree(s, 0, oct, NULL, 0, &n, &root);
    rtx_bvh_node* nodes = malloc(sizeof(rtx_bvh_node) * n);
    rtx_walk_tree(s, 0, oct, nodes, n, &n, &root);
    rtx_scene_desc wd = *s; wd.nodes = nodes; wd.n_nodes = n; wd.roots = &root; wd.n_roots = 1;
    oracle_counters c1, c2; memset(&c1, 0, sizeof c1); memset(&c2, 0, sizeof c2);
    ctx_t cx = {s, &cam, SEED, ORACLE_ORDER_ITERATIVE, &c1};
    ctx_t cw = {&wd, &cam, SEED, ORACLE_ORDER_ITERATIVE, &c2};
    uint64_t segs = 0, mism = 0;
    int px = argc > 6 ? atoi(argv[6]) : -1, py = argc > 7 ? atoi(argv[7]) : -1;
    for (uint32_t j = part; j < cam.image_height; j += parts)
      for (uint32_t i = 0; i < cam.image_width; ++i)
        if (px < 0 || (i == (uint32_t)px && j == (uint32_t)py))
        for (uint32_t k = 0; k < cam.samples_per_pixel; ++k) {
            rng_t rng; rng.key[0] = SEED; rng.key[1] = 0; rng.pixel = j * cam.image_width + i; rng.sample = k;
            rng.event = rng.attempt = rng.word = 0; rng.draws = &c1.rng_draws;
            ray_t r = get_ray(&cx, &rng, i, j);
            for (int depth = cam.max_depth; depth > 0; --depth) {
                hit_t h, h2; int ok, ok2;
                hit_prim(&cx, &r, &h, &ok); hit_prim(&cw, &r, &h2, &ok2); ++segs;
                if (ok != ok2 || (ok && (h.t != h2.t || h.material != h2.material))) {
                    ++mism;
                    printf("pixel %u,%u k %u seg %d: ref %d t=%.9g mat %u | walk %d t=%.9g mat %u  o=(%.6g %.6g %.6g) d=(%.6g %.6g %.6g)\n", i, j, k, cam.max_depth - depth, ok, ok ? h.t : 0, ok ? h.material : 0, ok2, ok2 ? h2.t : 0, ok2 ? h2.material : 0, r.origin.x, r.origin.y, r.origin.z, r.dir.x, r.dir.y, r.dir.z);
                }
                if (!ok) break;
                vec3 att; ray_t sc; rng_event(&rng, cam.max_depth - (uint32_t)depth + 1u);
                if (!material_scatter(&cx, &r, &h, &rng, &att, &sc)) break;
                r = sc;
            }
        }
    printf("part %d: segments %llu mismatches %llu\n", part, (unsigned long long)segs, (unsigned long long)mism);
    return 0;
}
