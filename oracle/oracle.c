/*
 * oracle.c — CPU restatement of TwFlem/raytracer-go's per-pixel hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for the HIP megakernel and the
 * CPU baseline of bench.py.  Never linked into librtx.so / librtxhost.so.
 * PARITY UNPINNED against the reference binary (Go is absent; the reference has no
 * tests or fixtures) — pinned instead by Random123 KATs for the RNG and by
 * source-derived known-answer tests.
 *
 * Build: gcc -O2 -std=c11 -ffp-contract=off -fno-fast-math (SSE2 scalar float32, the
 * same IEEE single-precision semantics as Go's gc compiler on amd64 at GOAMD64=v1).
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ============================================================================
 * Vec3 — internal/vec3.go:9-139.  Every operation is written in the association
 * order of the Go source (left to right), float32, no fused multiply-add.
 * ========================================================================== */
typedef struct { float x, y, z; } vec3;

static inline vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static inline vec3 v_add(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }   /* vec3.go:43-53 */
static inline vec3 v_sub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }   /* vec3.go:67-77 */
static inline vec3 v_mul(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }   /* vec3.go:55-65 */
static inline vec3 v_scale(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }      /* vec3.go:91-101 */
static inline float v_lensq(vec3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }           /* vec3.go:115-117 */
static inline float v_dot(vec3 l, vec3 r) { return l.x * r.x + l.y * r.y + l.z * r.z; }     /* vec3.go:137-139 */
static inline vec3 v_cross(vec3 l, vec3 r) {                                                 /* vec3.go:129-135 */
    return v3(l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x);
}
/* vec3.go:103-113: l = float32(math.Sqrt(float64(lensq))); v.Scale(1 / l).
 * sqrt in float64 of a float32, rounded back, equals the correctly rounded sqrtf. */
static inline vec3 v_unit(vec3 v) {
    float lensq = v_lensq(v);
    float l = (float)sqrt((double)lensq);
    return v_scale(v, 1.0f / l);
}
/* vec3.go:170-172 */
static inline int v_near_zero(vec3 v) {
    const float eps = 1e-8f;
    return (float)fabs((double)v.x) < eps && (float)fabs((double)v.y) < eps && (float)fabs((double)v.z) < eps;
}
/* vec3.go:212-214 */
static inline vec3 v_reflect(vec3 v, vec3 n) { return v_sub(v, v_scale(n, 2.0f * v_dot(v, n))); }
/* vec3.go:216-221 */
static inline vec3 v_refract(vec3 uv, vec3 n, float eta) {
    float cos_theta = v_dot(v_scale(uv, -1.0f), n);
    vec3 perp = v_scale(v_add(uv, v_scale(n, cos_theta)), eta);
    vec3 par = v_scale(n, -1.0f * (float)sqrt(fabs((double)(1.0f - v_lensq(perp)))));
    return v_add(par, perp);
}

/* Go math.Min / math.Max semantics (NaN wins, -0 < +0): math.go:38-44 via MinF32/MaxF32. */
static inline double go_min(double a, double b) {
    if (isnan(a) || isnan(b)) return NAN;
    if (a == 0 && b == 0) return signbit(a) ? a : b;
    return a < b ? a : b;
}
static inline double go_max(double a, double b) {
    if (isnan(a) || isnan(b)) return NAN;
    if (a == 0 && b == 0) return signbit(a) ? b : a;
    return a > b ? a : b;
}
static inline float min_f32(float a, float b) { return (float)go_min((double)a, (double)b); } /* math.go:38 */
static inline float max_f32(float a, float b) { return (float)go_max((double)a, (double)b); } /* math.go:42 */

/* Go math.Pow(x, 5) for x >= 0 (Go 1.21 src/math/pow.go): y is integral, so Pow
 * multiplies frexp-normalised mantissas by repeated squaring over the bits of 5 and
 * applies Ldexp; scaling by powers of two is exact here, so the result is
 * x * ((x*x) * (x*x)) in float64, with x == 0 -> 0 and x == 1 -> 1 as special cases. */
static double go_pow5(double x) {
    if (x == 1.0) return 1.0;
    if (isnan(x)) return NAN;
    if (x == 0.0) return 0.0;
    int xe;
    double x1 = frexp(x, &xe);
    double a1 = 1.0;
    int ae = 0;
    for (long i = 5; i != 0; i >>= 1) {
        if (i & 1) {
            a1 *= x1;
            ae += xe;
        }
        x1 *= x1;
        xe <<= 1;
        if (x1 < 0.5) {
            x1 += x1;
            xe--;
        }
    }
    return ldexp(a1, ae);
}

/* Go math.Atan2 / math.Acos (Go 1.21 src/math/atan.go, asin.go, atan2.go; pure Go on
 * amd64: Cephes rational approximations, restated operation for operation). */
static double go_xatan(double x) {
    const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
                 P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
                 P4 = -6.485021904942025371773e+01, Q0 = +2.485846490142306297962e+01,
                 Q1 = +1.650270098316988542046e+02, Q2 = +4.328810604912902668951e+02,
                 Q3 = +4.853903996359136964868e+02, Q4 = +1.945506571482613964425e+02;
    double z = x * x;
    z = z * ((((P0 * z + P1) * z + P2) * z + P3) * z + P4) / (((((z + Q0) * z + Q1) * z + Q2) * z + Q3) * z + Q4);
    z = x * z + x;
    return z;
}
static double go_satan(double x) {
    const double Morebits = 6.123233995736765886130e-17; /* pi/2 = PIO2 + Morebits */
    const double Tan3pio8 = 2.41421356237309504880;      /* tan(3*pi/8) */
    if (x <= 0.66) return go_xatan(x);
    if (x > Tan3pio8) return 1.57079632679489661923 - go_xatan(1.0 / x) + Morebits;
    return 0.785398163397448309616 + go_xatan((x - 1.0) / (x + 1.0)) + 0.5 * Morebits;
}
static double go_atan(double x) {
    if (x == 0.0) return x;
    if (x > 0.0) return go_satan(x);
    return -go_satan(-x);
}
double oracle_go_atan2(double y, double x) {
    const double Pi = 3.14159265358979323846;
    if (isnan(y) || isnan(x)) return NAN;
    if (y == 0.0) {
        if (x >= 0.0 && !signbit(x)) return copysign(0.0, y);
        return copysign(Pi, y);
    }
    if (x == 0.0) return copysign(Pi / 2.0, y);
    if (isinf(x)) {
        if (x > 0.0) return isinf(y) ? copysign(Pi / 4.0, y) : copysign(0.0, y);
        return isinf(y) ? copysign(3.0 * Pi / 4.0, y) : copysign(Pi, y);
    }
    if (isinf(y)) return copysign(Pi / 2.0, y);
    double q = go_atan(y / x);
    if (x < 0.0) {
        if (q <= 0.0) return q + Pi;
        return q - Pi;
    }
    return q;
}
static double go_asin(double x) {
    if (x == 0.0) return x;
    int sign = 0;
    if (x < 0.0) {
        x = -x;
        sign = 1;
    }
    if (x > 1.0) return NAN;
    double temp = sqrt(1.0 - x * x);
    if (x > 0.7) temp = 1.57079632679489661923 - go_satan(temp / x);
    else temp = go_satan(x / temp);
    if (sign) temp = -temp;
    return temp;
}
double oracle_go_acos(double x) { return 1.57079632679489661923 - go_asin(x); }

/* ============================================================================
 * RNG contract: Philox4x32-10, key = seed, counter =
 * (global pixel index, sample index, draw block, stream); draw n is word n&3 of
 * block n>>2; u = float32(x >> 8) * 2^-24 in [0, 1) — the range of rand.Float32.
 * ========================================================================== */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline float u32_to_unit(uint32_t x) { return (float)(x >> 8) * 0x1.0p-24f; }

/* The per-sample stream of the contract (GPU-first form): one Philox
 * block per (global pixel, sample, event, attempt).  Event 0 is GetRay; event s+1 the
 * scatter after segment s.  Draws are taken in the reference's order: words of the
 * current attempt's block in sequence; a rejected unit-sphere / unit-disk candidate
 * moves to the next attempt's block (word 0).  GetRay's first block holds dx, dy and
 * the first disk candidate. */
typedef struct {
    uint32_t key[2];
    uint32_t pixel, sample, event, attempt, word;
    uint32_t buf[4];
    uint64_t* draws;
} rng_t;

static void rng_load(rng_t* r) {
    uint32_t ctr[4] = {r->pixel, r->sample, r->event, r->attempt};
    oracle_philox4x32_10(ctr, r->key, r->buf);
    r->word = 0;
}
static void rng_event(rng_t* r, uint32_t event) {
    r->event = event;
    r->attempt = 0;
    rng_load(r);
}
static void rng_next_attempt(rng_t* r) {
    r->attempt++;
    rng_load(r);
}
static inline float rng_float32(rng_t* r) {
    uint32_t w = r->buf[r->word++ & 3u];
    if (r->draws) (*r->draws)++;
    return u32_to_unit(w);
}

void oracle_pixel_block(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t event, uint32_t attempt,
                        uint32_t out[4]) {
    uint32_t ctr[4] = {pixel, sample, event, attempt};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    oracle_philox4x32_10(ctr, key, out);
}

/* Host streams (scene generation, BVH axis): word n of stream s, counter
 * (block lo, block hi, 0, 0x80000000 | s) — disjoint from every pixel counter. */
uint32_t oracle_stream_u32(uint64_t seed, uint32_t stream, uint64_t n) {
    uint64_t blk = n >> 2;
    uint32_t ctr[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0x80000000u | stream};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    oracle_philox4x32_10(ctr, key, out);
    return out[n & 3u];
}

/* RandF32N, math.go:30-32: min + Float32()*(max-min). */
static inline float rand_f32n(rng_t* r, float mn, float mx) { return mn + rng_float32(r) * (mx - mn); }

/* NewVec3UnitRandOnUnitSphere32, vec3.go:182-190 (arguments drawn x, y, z); the
 * caller has opened the event. */
static vec3 rand_unit_on_sphere(rng_t* r) {
    for (;;) {
        float x = rand_f32n(r, -1.0f, 1.0f);
        float y = rand_f32n(r, -1.0f, 1.0f);
        float z = rand_f32n(r, -1.0f, 1.0f);
        vec3 v = v3(x, y, z);
        if (v_lensq(v) < 1.0f) return v_unit(v);
        rng_next_attempt(r);
    }
}

/* NewVec3RandInUnitDisk, vec3.go:203-210 (event 0, after dx and dy). */
static vec3 rand_in_unit_disk(rng_t* r) {
    for (;;) {
        float x = rand_f32n(r, -1.0f, 1.0f);
        float y = rand_f32n(r, -1.0f, 1.0f);
        vec3 v = v3(x, y, 0.0f);
        if (v_lensq(v) < 1.0f) return v;
        rng_next_attempt(r);
    }
}

/* ============================================================================
 * Camera — internal/camera.go:104-178, math.go:48-52.
 * ========================================================================== */
static const float PI_F32 = 3.14159274101257324f;         /* float32(math.Pi)   math.go:48 */
static const float RAD_RATIO = (float)(3.14159265358979323846 / 180.0); /* float32(pi/180), math.go:46;
                                                             single- and double-rounding agree */

float oracle_to_radians(float degrees) { return degrees * RAD_RATIO; }

void oracle_camera_defaults(oracle_camera_opts* o) {
    memset(o, 0, sizeof(*o));
    o->samples_per_pixel = 100;                  /* camera.go:109 */
    o->max_depth = 50;                           /* camera.go:110 */
    o->fov_radians = (float)1.57079632679489662; /* float32(PiO2), camera.go:108 */
    o->focus_dist = 10.0f;                       /* camera.go:111 */
    o->defocus_radians = 0.0f;
    o->look_at[0] = o->look_at[1] = o->look_at[2] = 0.0f;
    o->look_from[0] = 0.0f; o->look_from[1] = 0.0f; o->look_from[2] = -1.0f;
    o->vup[0] = 0.0f; o->vup[1] = 1.0f; o->vup[2] = 0.0f;
    o->background[0] = o->background[1] = o->background[2] = 0.0f;
}

void oracle_camera_init(float aspect_ratio, int32_t image_width, const oracle_camera_opts* o, rtx_camera* out) {
    memset(out, 0, sizeof(*out));
    float image_w = (float)image_width;
    vec3 look_from = v3(o->look_from[0], o->look_from[1], o->look_from[2]);
    vec3 look_at = v3(o->look_at[0], o->look_at[1], o->look_at[2]);
    vec3 vup = v3(o->vup[0], o->vup[1], o->vup[2]);
    vec3 center = look_from;                                                   /* :130 */
    vec3 dist = v_sub(look_from, look_at);                                     /* :132 */
    float h = (float)tan((double)(o->fov_radians / 2.0f));                    /* :134 */
    float viewport_h = 2.0f * h * o->focus_dist;                               /* :135 */
    float image_h = (float)(floor((double)image_w) / (double)aspect_ratio);    /* :137 */
    if (image_h < 1.0f) image_h = 1.0f;                                        /* :138 */
    float viewport_w = viewport_h * (image_w / image_h);                       /* :141 */
    vec3 w = v_unit(dist);                                                     /* :143 */
    vec3 u = v_unit(v_cross(vup, w));                                          /* :144 */
    vec3 v = v_cross(w, u);                                                    /* :145 */
    vec3 viewport_u = v_scale(u, viewport_w);                                  /* :147 */
    vec3 viewport_v = v_scale(v, -viewport_h);                                 /* :148 */
    vec3 pixel_du = v_scale(viewport_u, 1.0f / image_w);                       /* :150-151 */
    vec3 pixel_dv = v_scale(viewport_v, 1.0f / image_h);                       /* :152-153 */
    vec3 ul = center;                                                          /* :155 */
    ul = v_sub(ul, v_scale(w, o->focus_dist));                                 /* :156 */
    ul = v_sub(ul, v_scale(viewport_u, 0.5f));                                 /* :157 */
    ul = v_sub(ul, v_scale(viewport_v, 0.5f));                                 /* :158 */
    vec3 pixel00 = v_add(ul, v_scale(v_add(pixel_du, pixel_dv), 0.5f));        /* :160-161 */
    float defocus_r = o->focus_dist * (float)tan((double)(o->defocus_radians / 2.0f)); /* :163 */
    vec3 disk_u = v_scale(u, defocus_r);                                       /* :164 */
    vec3 disk_v = v_scale(v, defocus_r);                                       /* :165 */

    out->image_width = (uint32_t)(int32_t)image_w;   /* int(c.imageWidth)  camera.go:181 */
    out->image_height = (uint32_t)(int32_t)image_h;  /* int(c.imageHeight) camera.go:182 */
    out->samples_per_pixel = (uint32_t)o->samples_per_pixel;
    out->max_depth = (uint32_t)o->max_depth;
    out->defocus_angle = o->defocus_radians;
#define PUT(dst, src) do { (dst)[0] = (src).x; (dst)[1] = (src).y; (dst)[2] = (src).z; } while (0)
    PUT(out->center, center);
    PUT(out->pixel00, pixel00);
    PUT(out->pixel_du, pixel_du);
    PUT(out->pixel_dv, pixel_dv);
    PUT(out->defocus_disk_u, disk_u);
    PUT(out->defocus_disk_v, disk_v);
#undef PUT
    out->background[0] = o->background[0];
    out->background[1] = o->background[1];
    out->background[2] = o->background[2];
}

/* ============================================================================
 * Ray / HitInfo / scene traversal — ray.go:9-54, hittables.go:7-136, bvh.go:9-253.
 * ========================================================================== */
typedef struct { vec3 origin, dir; } ray_t;

static inline vec3 ray_at(const ray_t* r, float t) { return v_add(v_scale(r->dir, t), r->origin); } /* ray.go:25-30 */

typedef struct {
    vec3 point, normal;
    float t, u, v;
    uint32_t material;
    int front;
    const rtx_sphere* sphere; /* the sphere hit (NULL for a quad): the tiered walk's hit check */
    const rtx_quad* quad;     /* the quad hit (NULL for a sphere): the same check */
} hit_t;

typedef struct {
    const rtx_scene_desc* s;
    const rtx_camera* cam;
    uint64_t seed;
    int order;
    oracle_counters* c; /* per-thread */
} ctx_t;

/* NewHitInfo, hittables.go:22-37. */
static hit_t new_hit_info(float t, float u, float v, vec3 dir, vec3 point, vec3 n, uint32_t mat) {
    hit_t h;
    h.front = v_dot(dir, n) < 0.0f;
    if (!h.front) n = v_scale(n, -1.0f);
    h.point = point;
    h.normal = n;
    h.t = t;
    h.u = u;
    h.v = v;
    h.material = mat;
    h.sphere = NULL;
    h.quad = NULL;
    return h;
}

/* Interval.In, bvh.go:18-20 (padding 0). */
static inline int interval_in(float mn, float mx, float v) { return mn - 0.0f < v && v < mx + 0.0f; }

/* (*Sphere).Hit, hittables.go:96-132. */
/* The tie rule of a walk over another tree than the reference's (oracle_sphere_rank): rank[i] is
 * sphere i's place in the reference walk; a root equal to the bound wins when its sphere comes
 * before the bound's hit (rank trank) — the tie bvh.go:220-249 resolves for the sphere it meets
 * first.  A no-op on the reference's own order. */
static const uint32_t* g_sphere_rank;
void oracle_sphere_rank(const uint32_t* rank) { g_sphere_rank = rank; }
static inline uint32_t hit_rank(const ctx_t* cx, const hit_t* h) {
    return g_sphere_rank && h->sphere ? g_sphere_rank[h->sphere - cx->s->spheres] : 0u;
}

static int sphere_hit(const ctx_t* cx, const rtx_sphere* s, const ray_t* r, float tmin, float tmax, hit_t* out,
                      uint32_t trank) {
    vec3 c = v3(s->center[0], s->center[1], s->center[2]);
    vec3 a_sub_c = v_sub(r->origin, c);                                    /* :97 */
    float a = v_lensq(r->dir);                                             /* :98 */
    float half_b = v_dot(r->dir, a_sub_c);                                 /* :99 */
    float cc = v_lensq(a_sub_c) - s->radius * s->radius;                   /* :100 */
    float disc = half_b * half_b - a * cc;                                 /* :102 */
    if (disc < 0.0f) return 0;                                             /* :104 */
    float sqt = (float)sqrt((double)disc);                                 /* :108 */
    float t;
    float r1 = (-half_b - sqt) / a;                                        /* :110 */
    const int ranked = g_sphere_rank && cx && g_sphere_rank[s - cx->s->spheres] < trank;
    if (interval_in(tmin, tmax, r1) || (ranked && tmin < r1 && r1 == tmax)) {
        t = r1;
    } else {
        float r2 = (-half_b + sqt) / a;                                    /* :112 */
        if (interval_in(tmin, tmax, r2) || (ranked && tmin < r2 && r2 == tmax)) t = r2;
        else return 0;
    }
    vec3 point = ray_at(r, t);                                             /* :118 */
    vec3 norm = v_unit(v_scale(v_sub(point, c), s->radius));               /* :119-120 */
    float theta = (float)oracle_go_acos(-(double)norm.y);                  /* :122 */
    float phi = (float)(oracle_go_atan2(-(double)norm.z, (double)norm.x) + 3.14159265358979323846); /* :123 */
    float u = (phi + 5.0f * PI_F32 / 12.0f) / (2.0f * PI_F32);             /* :125 typed consts fold in float32 */
    float v = theta / PI_F32;                                              /* :126 */
    (void)cx;
    *out = new_hit_info(t, u, v, r->dir, point, norm, s->material);        /* :128 */
    out->sphere = s;
    return 1;
}

/* (Quad).Hit, hittables.go:167-190, with InPlane :192-194.  The derived fields (normal,
 * D, w) are NewQuad's (hittables.go:149-165), computed on the host. */
static int quad_hit(const rtx_quad* q, const ray_t* r, float tmin, float tmax, hit_t* out) {
    vec3 n = v3(q->normal[0], q->normal[1], q->normal[2]);
    float denom = v_dot(r->dir, n);                                        /* :168 */
    if (fabs((double)denom) < 1e-8) return 0;                              /* :170 */
    float t = (q->d - v_dot(n, r->origin)) / denom;                        /* :174 */
    if (!interval_in(tmin, tmax, t)) return 0;                             /* :176 */
    vec3 point = ray_at(r, t);                                             /* :180 */
    vec3 php = v_sub(point, v3(q->q[0], q->q[1], q->q[2]));                /* :181 */
    vec3 w = v3(q->w[0], q->w[1], q->w[2]);
    float alpha = v_dot(w, v_cross(php, v3(q->v[0], q->v[1], q->v[2])));   /* :182 */
    float beta = v_dot(w, v_cross(v3(q->u[0], q->u[1], q->u[2]), php));    /* :183 */
    if (alpha < 0.0f || 1.0f < alpha || beta < 0.0f || 1.0f < beta) return 0; /* :185, :193 */
    *out = new_hit_info(t, alpha, beta, r->dir, point, n, q->material);    /* :189 */
    out->quad = q;
    return 1;
}

/* InBoundary, bvh.go:84-102. */
static inline int in_boundary(float dir, float origin, float amin, float amax, float* rmin, float* rmax) {
    float inv_d = 1.0f / dir;
    float t0 = (amin - origin) * inv_d;
    float t1 = (amax - origin) * inv_d;
    if (inv_d < 0.0f) {
        float t = t0; t0 = t1; t1 = t;
    }
    if (t0 > *rmin) *rmin = t0;
    if (t1 < *rmax) *rmax = t1;
    return *rmin < *rmax;
}

/* (*Aabb).Hit, bvh.go:52-61: rT is passed by value. */
static int aabb_hit(const rtx_bvh_node* n, const ray_t* r, float tmin, float tmax) {
    if (in_boundary(r->dir.x, r->origin.x, n->bmin[0], n->bmax[0], &tmin, &tmax))
        if (in_boundary(r->dir.y, r->origin.y, n->bmin[1], n->bmax[1], &tmin, &tmax))
            if (in_boundary(r->dir.z, r->origin.z, n->bmin[2], n->bmax[2], &tmin, &tmax)) return 1;
    return 0;
}

/* The near walk's slab test (rtx_device.h box_step FMA): the slab distances as
 * fmaf(b, 1/d, -(o * (1/d))) — one rounding instead of two — for a ray whose 1/d components are
 * within 2^64 and whose origin is within 2^32 (near_fma_ok); other rays take the reference's form.
 * The near tree's boxes carry the slack for both forms, and the near walk's result is the
 * reference's by the hit check whichever boxes pass: only the work counts differ. */
static int aabb_hit_near(const rtx_bvh_node* n, const ray_t* r, float tmin, float tmax) {
    const float inv[3] = {1.0f / r->dir.x, 1.0f / r->dir.y, 1.0f / r->dir.z};
    const float o[3] = {r->origin.x, r->origin.y, r->origin.z};
    for (int k = 0; k < 3; ++k)
        if (!(fabsf(inv[k]) <= 0x1p64f && fabsf(o[k]) <= 0x1p32f)) return aabb_hit(n, r, tmin, tmax);
    for (int k = 0; k < 3; ++k) {
        const float no = -(o[k] * inv[k]);
        float t0 = fmaf(n->bmin[k], inv[k], no), t1 = fmaf(n->bmax[k], inv[k], no);
        if (inv[k] < 0.0f) {
            const float t = t0;
            t0 = t1;
            t1 = t;
        }
        if (t0 > tmin) tmin = t0;
        if (t1 < tmax) tmax = t1;
        if (!(tmin < tmax)) return 0;
    }
    return 1;
}

/* Test hook: the near walk's slab test (aabb_hit_near) of n rays against n boxes with intervals. */
void oracle_near_slab_pass(const float* o, const float* d, const float* mn, const float* mx, const float* lo,
                           const float* hi, uint8_t* out, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {
        ray_t r;
        r.origin = v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]);
        r.dir = v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
        rtx_bvh_node b;
        for (int k = 0; k < 3; ++k) {
            b.bmin[k] = mn[3 * i + k];
            b.bmax[k] = mx[3 * i + k];
        }
        out[i] = (uint8_t)aabb_hit_near(&b, &r, lo[i], hi[i]);
    }
}

static int hit_ref(const ctx_t* cx, int32_t ref, const ray_t* r, float tmin, float tmax, hit_t* out, int dup,
                   uint32_t trank);

/* Walk hooks (set between renders, read by every render thread): per-node box tests and
 * passes, and the nodes whose box test a collapsed walk leaves out.  Leaving a node's test
 * out changes no result: a child's box lies inside its parent's (NewAabbFromBoxes' min/max)
 * and InBoundary is monotone in the box, so a child passes only where its parent passes. */
static uint64_t* g_node_tested;
static uint64_t* g_node_passed;
static const uint8_t* g_node_skip;

void oracle_node_hooks(uint64_t* tested, uint64_t* passed, const uint8_t* skip) {
    g_node_tested = tested;
    g_node_passed = passed;
    g_node_skip = skip;
}

/* The tiered walk hook (rtx.h RTX_SCENE_NO_TIER): from the first segment of a
 * path whose origin lies outside the near box on, the path walks the far description (with its
 * own skips) instead of the one being rendered — the device hands such a path to its far pass,
 * which walks the far tree to the path's end.  Both describe trees over the same spheres and
 * materials. */
static const rtx_scene_desc* g_tier_far;
static const uint8_t* g_tier_far_skip;
static float g_tier_box[6];
static __thread int g_tier_path_far; /* this thread's current path has left the near region */

void oracle_tier(const float near_box[6], const rtx_scene_desc* far, const uint8_t* far_skip) {
    g_tier_far = far;
    g_tier_far_skip = far_skip;
    if (near_box) memcpy(g_tier_box, near_box, sizeof(g_tier_box));
}

/* (*BVH).Hit, bvh.go:220-249. */
static int bvh_hit(const ctx_t* cx, const rtx_bvh_node* n, const ray_t* r, float tmin, float tmax, hit_t* out,
                   uint32_t trank) {
    const size_t id = (size_t)(n - cx->s->nodes);
    const int far = g_tier_far && cx->s == g_tier_far;
    const uint8_t* skip = far ? g_tier_far_skip : g_node_skip;
    if (!skip || !skip[id]) {
        cx->c->node_visits++;
        if (g_node_tested && !far) __atomic_fetch_add(&g_node_tested[id], 1, __ATOMIC_RELAXED);
        /* :221; the tiered walk's near tree in its own form (the FMA form in a scene of spheres; with quads the
         * device's near walk keeps the reference's form, rtx_kernel.hip) */
        if (!(g_tier_far && !far && cx->s->n_quads == 0 ? aabb_hit_near(n, r, tmin, tmax) : aabb_hit(n, r, tmin, tmax)))
            return 0;
        if (g_node_passed && !far) __atomic_fetch_add(&g_node_passed[id], 1, __ATOMIC_RELAXED);
    }
    hit_t hl, hr;
    int hit_left = hit_ref(cx, n->left, r, tmin, tmax, &hl, 0, trank);      /* :225 */
    float rmax = tmax;                                                      /* :227 */
    uint32_t rrank = trank;
    if (hit_left) { rmax = hl.t; rrank = hit_rank(cx, &hl); }               /* :228-230 */
    int hit_right = hit_ref(cx, n->right, r, tmin, rmax, &hr, n->right == n->left, rrank); /* :232 */
    if (hit_left && hit_right) {                                            /* :234 */
        *out = (hl.t < hr.t) ? hl : hr;
        return 1;
    }
    if (hit_right) { *out = hr; return 1; }
    if (hit_left) { *out = hl; return 1; }
    return 0;
}

static int list_hit(const ctx_t* cx, const rtx_list* l, const ray_t* r, float tmin, float tmax, hit_t* out,
                    uint32_t trank);

static int hit_ref(const ctx_t* cx, int32_t ref, const ray_t* r, float tmin, float tmax, hit_t* out, int dup,
                   uint32_t trank) {
    if (ref >= 0 || ((uint32_t)(~ref)) >> 28 == RTX_PRIM_LIST) {
        /* A node or a nested World.  As the right child of a one-element split (dup,
         * bvh.go:162-165) its second call runs with the bound clipped to the first one's hit
         * and finds nothing new (every test is monotone in the bound); the device emits it
         * once, so its work is not counted here either. */
        oracle_counters saved;
        if (dup) saved = *cx->c;
        int h = ref >= 0 ? bvh_hit(cx, &cx->s->nodes[ref], r, tmin, tmax, out, trank)
                         : list_hit(cx, &cx->s->lists[((uint32_t)(~ref)) & 0x0FFFFFFFu], r, tmin, tmax, out, trank);
        if (dup) *cx->c = saved;
        return h;
    }
    uint32_t p = (uint32_t)(~ref);
    uint32_t type = p >> 28, idx = p & 0x0FFFFFFFu;
    cx->c->prim_tests_ref++;
    if (!dup) cx->c->prim_tests++;
    if (type == RTX_PRIM_QUAD) return quad_hit(&cx->s->quads[idx], r, tmin, tmax, out);
    return sphere_hit(cx, &cx->s->spheres[idx], r, tmin, tmax, out, trank);
}

/* (*World).Hit, hittables.go:55-72, of a World nested in the tree (RTX_PRIM_LIST). */
static int list_hit(const ctx_t* cx, const rtx_list* l, const ray_t* r, float tmin, float tmax, hit_t* out,
                    uint32_t trank) {
    int hit_any = 0;
    float closest = tmax;
    for (uint32_t i = 0; i < l->count; ++i) {
        hit_t h;
        if (hit_ref(cx, cx->s->list_refs[l->first + i], r, tmin, closest, &h, 0, trank)) {
            hit_any = 1;
            *out = h;
            closest = h.t;
            trank = hit_rank(cx, &h);
        }
    }
    return hit_any;
}

static int world_hit_tree(const ctx_t* cx, const ray_t* r, float tmin, float tmax, hit_t* out);

/* The world passed to Render: a BVH (one root) or a World list, hittables.go:55-72. */
static int world_hit(const ctx_t* cx, const ray_t* r, float tmin, float tmax, hit_t* out) {
    if (g_tier_far && cx->s != g_tier_far) {
        int far = g_tier_path_far ||
                  !(r->origin.x >= g_tier_box[0] && r->origin.x <= g_tier_box[3] && r->origin.y >= g_tier_box[1] &&
                    r->origin.y <= g_tier_box[4] && r->origin.z >= g_tier_box[2] && r->origin.z <= g_tier_box[5]);
        if (!far) {
            /* The near walk, then its hit check: the hit sphere's own box (NewSphere's NewAabb,
             * hittables.go:85-94, inside its reference leaf's box) must pass Aabb.Hit with the
             * bound just past the hit; else the segment is walked again on the far tree. */
            int h = world_hit_tree(cx, r, tmin, tmax, out);
            if (!h || (!out->sphere && !out->quad)) return h;
            rtx_bvh_node own;
            if (out->sphere) {
                const rtx_sphere* sp = out->sphere;
                for (int k = 0; k < 3; ++k) {
                    float p1 = sp->center[k] + sp->radius * -1.0f, p2 = sp->center[k] + sp->radius;
                    own.bmin[k] = p1 < p2 ? p1 : p2;
                    own.bmax[k] = p1 < p2 ? p2 : p1;
                }
            } else {  /* NewQuad's box: NewAabb(Q, Q + u + v).GetPaddedAabb(), hittables.go:162, bvh.go:63-84 */
                const rtx_quad* q = out->quad;
                const float eps = 0.0001f;
                for (int k = 0; k < 3; ++k) {
                    const float c = (q->q[k] + q->u[k]) + q->v[k];
                    float lo = min_f32(q->q[k], c), hi = max_f32(q->q[k], c);
                    if (hi - lo < eps) {
                        lo = lo - eps;
                        hi = hi + eps;
                    }
                    own.bmin[k] = lo;
                    own.bmax[k] = hi;
                }
            }
            if (aabb_hit(&own, r, tmin, nextafterf(out->t, INFINITY))) return h;
        }
        g_tier_path_far = 1;
        ctx_t fx = *cx;  /* from the path's first far segment on: the far tree */
        fx.s = g_tier_far;
        return world_hit(&fx, r, tmin, tmax, out);
    }
    return world_hit_tree(cx, r, tmin, tmax, out);
}

/* The world's roots in order (the walk of one description). */
static int world_hit_tree(const ctx_t* cx, const ray_t* r, float tmin, float tmax, hit_t* out) {
    int hit_any = 0;
    float closest = tmax;
    uint32_t trank = 0;  /* (no hit yet: no tie to win) */
    for (uint32_t i = 0; i < cx->s->n_roots; ++i) {
        hit_t h;
        if (hit_ref(cx, cx->s->roots[i], r, tmin, closest, &h, 0, trank)) {
            hit_any = 1;
            *out = h;
            closest = h.t;
            trank = hit_rank(cx, &h);
        }
    }
    return hit_any;
}

/* Go's math.Sin (Go 1.21 src/math/sin.go, trig_reduce.go; pure Go on amd64, no FMA
 * contraction with the default GOAMD64=v1): Cephes polynomials after Cody-Waite
 * reduction by pi/4 in three parts, Payne-Hanek (trigReduce) from 2^29 up.  Used by
 * NoiseTexture.GetTexture (materials.go:285-287).  The 4/pi words below are the binary
 * expansion of 4/pi (Go's mPi4), computed with integer arithmetic. */
static const uint64_t GO_MPI4[20] = {
    0x0000000000000001ull, 0x45f306dc9c882a53ull, 0xf84eafa3ea69bb81ull, 0xb6c52b3278872083ull,
    0xfca2c757bd778ac3ull, 0x6e48dc74849ba5c0ull, 0x0c925dd413a32439ull, 0xfc3bd63962534e7dull,
    0xd1046bea5d768909ull, 0xd338e04d68befc82ull, 0x7323ac7306a673e9ull, 0x3908bf177bf25076ull,
    0x3ff12fffbc0b301full, 0xde5e2316b414da3eull, 0xda6cfd9e4f96136eull, 0x9e8c7ecd3cbfd45aull,
    0xea4f758fd7cbe2f6ull, 0x7a0e73ef14a525d4ull, 0xd7f6bf623f1aba10ull, 0xac06608df8f6d757ull};

static void go_trig_reduce(double x, uint64_t* j_out, double* z_out) {
    const double PI4 = 3.14159265358979323846 / 4;
    if (x < PI4) {
        *j_out = 0;
        *z_out = x;
        return;
    }
    uint64_t ix;
    memcpy(&ix, &x, 8);
    const int shift = 52, bias = 1023;
    const uint64_t mask = 0x7FF;
    const int exp = (int)((ix >> shift) & mask) - bias - shift;
    ix &= ~(mask << shift);
    ix |= 1ull << shift;
    const unsigned digit = (unsigned)(exp + 61) / 64, bitshift = (unsigned)(exp + 61) % 64;
    #define SHR(v, s) ((s) >= 64 ? 0ull : (v) >> (s))
    const uint64_t z0 = (GO_MPI4[digit] << bitshift) | SHR(GO_MPI4[digit + 1], 64 - bitshift);
    const uint64_t z1 = (GO_MPI4[digit + 1] << bitshift) | SHR(GO_MPI4[digit + 2], 64 - bitshift);
    const uint64_t z2 = (GO_MPI4[digit + 2] << bitshift) | SHR(GO_MPI4[digit + 3], 64 - bitshift);
    const unsigned __int128 p2 = (unsigned __int128)z2 * ix, p1 = (unsigned __int128)z1 * ix;
    const uint64_t z2hi = (uint64_t)(p2 >> 64), z1hi = (uint64_t)(p1 >> 64), z1lo = (uint64_t)p1;
    const uint64_t z0lo = z0 * ix;
    const uint64_t lo = z1lo + z2hi;
    const uint64_t c = lo < z1lo;
    uint64_t hi = z0lo + z1hi + c;
    uint64_t j = hi >> 61;
    hi = hi << 3 | lo >> 61;
    const unsigned lz = (unsigned)__builtin_clzll(hi);
    const uint64_t e = (uint64_t)(bias - (lz + 1));
    hi = (hi << (lz + 1)) | SHR(lo, 64 - (lz + 1));
    hi >>= 64 - shift;
    hi |= e << shift;
    #undef SHR
    double z;
    memcpy(&z, &hi, 8);
    if (j & 1) {
        j++;
        j &= 7;
        z--;
    }
    *j_out = j;
    *z_out = z * PI4;
}

double oracle_go_sin(double x) {
    static const double S[6] = {1.58962301576546568060e-10, -2.50507477628578072866e-8, 2.75573136213857245213e-6,
                                -1.98412698295895385996e-4, 8.33333333332211858878e-3, -1.66666666666666307295e-1};
    static const double C[6] = {-1.13585365213876817300e-11, 2.08757008419747316778e-9, -2.75573141792967388112e-7,
                                2.48015872888517045348e-5, -1.38888888888730564116e-3, 4.16666666666665929218e-2};
    const double PI4A = 7.85398125648498535156e-1, PI4B = 3.77489470793079817668e-8,
                 PI4C = 2.69515142907905952645e-15;
    if (x == 0 || x != x) return x;
    if (isinf(x)) return NAN;
    int sign = 0;
    if (x < 0) {
        x = -x;
        sign = 1;
    }
    uint64_t j;
    double y, z;
    if (x >= (double)(1 << 29)) {
        go_trig_reduce(x, &j, &z);
    } else {
        j = (uint64_t)(x * (4 / 3.14159265358979323846));
        y = (double)j;
        if (j & 1) {
            j++;
            y++;
        }
        j &= 7;
        z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
    }
    if (j > 3) {
        sign = !sign;
        j -= 4;
    }
    const double zz = z * z;
    if (j == 1 || j == 2)
        y = 1.0 - 0.5 * zz + zz * zz * ((((((C[0] * zz) + C[1]) * zz + C[2]) * zz + C[3]) * zz + C[4]) * zz + C[5]);
    else
        y = z + z * zz * ((((((S[0] * zz) + S[1]) * zz + S[2]) * zz + S[3]) * zz + S[4]) * zz + S[5]);
    return sign ? -y : y;
}

/* Perlin noise, materials.go:218-249, with math.go:58-92 (Lerp, BiLinearLerp,
 * TriLinearLerp) as written.  tab = RTX_NOISE_TEXELS words (rtx.h). */
static inline float go_lerp(float t, float x, float y) { return x * (1 - t) + y * t; }
static inline float go_smoothstep(float t) { return t * t * (3 - 2 * t); }
static inline int64_t go_int_f32_trunc(float v) {
    if (v != v || v >= 9.2233720368547758e18f || v < -9.2233720368547758e18f) return INT64_MIN;
    return (int64_t)v;
}
static float perlin_corner(const uint32_t* tab, int ix, int iy, int iz, float x, float y, float z) {
    const uint32_t h = tab[768 + ix] ^ tab[1024 + iy] ^ tab[1280 + iz];
    float g[3];
    memcpy(g, &tab[3 * h], 12);
    return g[0] * x + g[1] * y + g[2] * z; /* Dot(randVec3[h], (x, y, z)) */
}
static float perlin_noise(const uint32_t* tab, vec3 p) {
    const float xi = (float)floor((double)p.x), yi = (float)floor((double)p.y), zi = (float)floor((double)p.z);
    const float tx = p.x - xi, ty = p.y - yi, tz = p.z - zi;
    const int rx0 = (int)(go_int_f32_trunc(xi) & 255), rx1 = (rx0 + 1) & 255;
    const int ry0 = (int)(go_int_f32_trunc(yi) & 255), ry1 = (ry0 + 1) & 255;
    const int rz0 = (int)(go_int_f32_trunc(zi) & 255), rz1 = (rz0 + 1) & 255;
    const float c000 = perlin_corner(tab, rx0, ry0, rz0, tx, ty, tz);
    const float c001 = perlin_corner(tab, rx0, ry0, rz1, tx, ty, tz - 1);
    const float c010 = perlin_corner(tab, rx0, ry1, rz0, tx, ty - 1, tz);
    const float c011 = perlin_corner(tab, rx0, ry1, rz1, tx, ty - 1, tz - 1);
    const float c100 = perlin_corner(tab, rx1, ry0, rz0, tx - 1, ty, tz);
    const float c101 = perlin_corner(tab, rx1, ry0, rz1, tx - 1, ty, tz - 1);
    const float c110 = perlin_corner(tab, rx1, ry1, rz0, tx - 1, ty - 1, tz);
    const float c111 = perlin_corner(tab, rx1, ry1, rz1, tx - 1, ty - 1, tz - 1);
    const float sx = go_smoothstep(tx), sy = go_smoothstep(ty), sz = go_smoothstep(tz);
    const float e = go_lerp(sy, go_lerp(sx, c000, c100), go_lerp(sx, c010, c110));
    const float f = go_lerp(sy, go_lerp(sx, c001, c101), go_lerp(sx, c011, c111));
    return go_lerp(sz, e, f);
}
static float perlin_turb(const uint32_t* tab, vec3 p, int depth) { /* materials.go:238-249 */
    float sum = 0, weight = 1.0f;
    for (int i = 0; i < depth; ++i) {
        sum += weight * perlin_noise(tab, p);
        weight *= 0.5f;
        p = v_scale(p, 2);
    }
    return (float)fabs((double)sum);
}
/* NoiseTexture.GetTexture, materials.go:280-288. */
static float noise_texture(const uint32_t* tab, float scale, vec3 p) {
    p = v_scale(p, scale);
    return 0.5f * (1 + (float)oracle_go_sin((double)(p.z + 10 * perlin_turb(tab, p, 7))));
}
float oracle_noise_texture(const uint32_t* tab, float scale, const float p[3]) {
    return noise_texture(tab, scale, v3(p[0], p[1], p[2]));
}

/* ============================================================================
 * Textures and materials — internal/materials.go:9-193, 297-313.
 * ========================================================================== */
static vec3 texture_value(const ctx_t* cx, uint32_t ti, float u, float v, vec3 p) {
    const rtx_texture* t = &cx->s->textures[ti];
    switch (t->type) {
    case RTX_TEX_SOLID:                                                     /* :151-163 */
        return v3(t->even[0], t->even[1], t->even[2]);
    case RTX_TEX_CHECKERED: {                                               /* :127-137 */
        float inv_scale = 1.0f / t->scale;
        int64_t x = (int64_t)floor((double)(inv_scale * p.x));
        int64_t y = (int64_t)floor((double)(inv_scale * p.y));
        int64_t z = (int64_t)floor((double)(inv_scale * p.z));
        if ((x + y + z) % 2 == 0) return v3(t->even[0], t->even[1], t->even[2]);
        return v3(t->odd[0], t->odd[1], t->odd[2]);
    }
    case RTX_TEX_IMAGE: {                                                   /* :175-193 */
        if ((int32_t)t->height <= 0) return v3(0.0f, 1.0f, 1.0f);          /* Dy() <= 0 */
        /* Clamp(0, 1, x) passes NaN through (math.go:20-28). */
        float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
        float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
        float vv = 1.0f - vc;
        float fi = uu * (float)t->width;
        float fj = vv * (float)t->height;
        cx->c->texel_fetches++;
        /* int(float32): truncation; NaN/out-of-range -> 0x8000000000000000 on amd64. */
        int64_t i = isnan(fi) ? INT64_MIN : (int64_t)fi;
        int64_t j = isnan(fj) ? INT64_MIN : (int64_t)fj;
        /* At(i, j) outside Bounds = [0, Dx) x [0, Dy): the image type's zero colour, held
         * as the border texel after the raster (rtx.h RTX_TEX_IMAGE). */
        uint64_t idx = (uint64_t)t->width * t->height;
        if (i >= 0 && j >= 0 && i < (int64_t)t->width && j < (int64_t)t->height)
            idx = (uint64_t)j * t->width + (uint64_t)i;
        else
            cx->c->texel_border++;
        const uint32_t* px = &cx->s->texels[t->texel_offset + 2 * idx];
        /* r, g, b, _ := pixel.RGBA(); colScale = float32(1.0 / 65535.0). */
        const float col_scale = 1.0f / 65535.0f;
        return v3((float)(px[0] & 0xFFFFu) * col_scale, (float)(px[0] >> 16) * col_scale,
                  (float)(px[1] & 0xFFFFu) * col_scale);
    }
    case RTX_TEX_NOISE: {                                                   /* :267-288 */
        const float g = noise_texture(&cx->s->texels[t->texel_offset], t->scale, p);
        return v3(g, g, g);
    }
    default:
        return v3(0.0f, 0.0f, 0.0f);
    }
}

/* Material.Emit: zero except DiffuseLight (materials.go:25, 51, 83, 311). */
static vec3 material_emit(const ctx_t* cx, const hit_t* h, int* has) {
    const rtx_material* m = &cx->s->materials[h->material];
    if (m->type == RTX_MAT_DIFFUSE_LIGHT) {
        *has = 1;
        return texture_value(cx, m->texture, h->u, h->v, h->point);
    }
    *has = 0;
    return v3(0.0f, 0.0f, 0.0f);
}

/* reflectance, materials.go:115-119. */
static float reflectance(float cos_theta, float eta) {
    float r0 = (1.0f - eta) / (1.0f + eta);
    r0 *= r0;
    return r0 + (1.0f - r0) * (float)go_pow5(1.0 - (double)cos_theta);
}

/* Material.Scatter.  Returns 1 and fills att/out if the ray scatters. */
static int material_scatter(const ctx_t* cx, const ray_t* r, const hit_t* h, rng_t* rng, vec3* att, ray_t* out) {
    const rtx_material* m = &cx->s->materials[h->material];
    switch (m->type) {
    case RTX_MAT_LAMBERTIAN: {                                              /* :33-42 */
        vec3 dir = v_add(h->normal, rand_unit_on_sphere(rng));
        if (v_near_zero(dir)) dir = h->normal;
        out->origin = h->point;
        out->dir = dir;
        *att = texture_value(cx, m->texture, h->u, h->v, h->point);
        return 1;
    }
    case RTX_MAT_METAL: {                                                   /* :60-75 */
        vec3 unit_dir = v_unit(r->dir);
        vec3 reflected = v_reflect(unit_dir, h->normal);
        vec3 fuzz = rand_unit_on_sphere(rng);
        fuzz = v_scale(fuzz, m->fuzz);
        vec3 scattered = v_add(reflected, fuzz);
        if (v_dot(scattered, h->normal) > 0.0f) {
            out->origin = h->point;
            out->dir = scattered;
            *att = v3(m->albedo[0], m->albedo[1], m->albedo[2]);
            return 1;
        }
        return 0;
    }
    case RTX_MAT_DIELECTRIC: {                                              /* :91-113 */
        float eta = m->ior;
        if (h->front) eta = 1.0f / m->ior;
        vec3 unit_dir = v_unit(r->dir);
        float cos_theta = (float)go_min((double)v_dot(v_scale(unit_dir, -1.0f), h->normal), 1.0);
        float sin_theta = (float)sqrt(1.0 - (double)(cos_theta * cos_theta));
        int cannot_refract = sin_theta * eta > 1.0f;
        vec3 direction;
        /* Short-circuit: the uniform is drawn only when refraction is possible.  The
         * reference draws it from the global rand (materials.go:103); the contract
         * moves it onto the per-ray stream. */
        if (cannot_refract || reflectance(cos_theta, eta) > rng_float32(rng))
            direction = v_reflect(unit_dir, h->normal);
        else
            direction = v_refract(unit_dir, h->normal, eta);
        out->origin = h->point;
        out->dir = direction;
        *att = v3(1.0f, 1.0f, 1.0f);
        return 1;
    }
    case RTX_MAT_DIFFUSE_LIGHT:                                             /* :303-305 */
    default:
        return 0;
    }
}

/* (*Ray).GetColor, ray.go:32-54 — the recursion as written. */
static vec3 ray_color_ref(const ctx_t* cx, const ray_t* r, rng_t* rng, int depth) {
    if (depth <= 0) return v3(0.0f, 0.0f, 0.0f);
    hit_t h;
    cx->c->segments++;
    const float inf = INFINITY;
    if (world_hit(cx, r, 0.001f, inf, &h)) {
        cx->c->hits++;
        int has_emit;
        vec3 emit = material_emit(cx, &h, &has_emit);
        vec3 att;
        ray_t scattered;
        rng_event(rng, cx->cam->max_depth - (uint32_t)depth + 1u);  /* scatter after this segment */
        if (!material_scatter(cx, r, &h, rng, &att, &scattered)) return emit;
        vec3 col = v_mul(att, ray_color_ref(cx, &scattered, rng, depth - 1));
        return v_add(emit, col);
    }
    const float* bg = cx->cam->background;
    return v3(bg[0], bg[1], bg[2]);
}

/* The same path, colour accumulated front to back (the kernel's order). */
static vec3 ray_color_iter(const ctx_t* cx, ray_t r, rng_t* rng, int depth) {
    vec3 thr = v3(1.0f, 1.0f, 1.0f);
    vec3 acc = v3(0.0f, 0.0f, 0.0f);
    for (; depth > 0; --depth) {
        hit_t h;
        cx->c->segments++;
        if (!world_hit(cx, &r, 0.001f, INFINITY, &h)) {
            const float* bg = cx->cam->background;
            acc = v_add(acc, v_mul(thr, v3(bg[0], bg[1], bg[2])));
            return acc;
        }
        cx->c->hits++;
        int has_emit;
        vec3 emit = material_emit(cx, &h, &has_emit);
        if (has_emit) acc = v_add(acc, v_mul(thr, emit));
        vec3 att;
        ray_t scattered;
        rng_event(rng, cx->cam->max_depth - (uint32_t)depth + 1u);
        if (!material_scatter(cx, &r, &h, rng, &att, &scattered)) return acc;
        thr = v_mul(thr, att);
        r = scattered;
    }
    return acc;
}

/* GetRay + sampleUnitSquare, camera.go:265-299. */
static ray_t get_ray(const ctx_t* cx, rng_t* rng, uint32_t i, uint32_t j) {
    const rtx_camera* c = cx->cam;
    vec3 du = v3(c->pixel_du[0], c->pixel_du[1], c->pixel_du[2]);
    vec3 dv = v3(c->pixel_dv[0], c->pixel_dv[1], c->pixel_dv[2]);
    vec3 du_off = v_scale(du, (float)i);                                    /* :266-267 */
    vec3 dv_off = v_scale(dv, (float)j);                                    /* :269-270 */
    vec3 pc = v3(c->pixel00[0], c->pixel00[1], c->pixel00[2]);              /* :272 */
    pc = v_add(pc, du_off);                                                 /* :273 */
    pc = v_add(pc, dv_off);                                                 /* :274 */
    rng_event(rng, 0u);
    float dx = -0.5f + rng_float32(rng);                                    /* :290 */
    float dy = -0.5f + rng_float32(rng);                                    /* :291 */
    pc = v_add(pc, v_add(v_scale(du, dx), v_scale(dv, dy)));                /* :275, 293-298 */
    vec3 disc = rand_in_unit_disk(rng);                                     /* :277 (always drawn) */
    vec3 center = v3(c->center[0], c->center[1], c->center[2]);
    vec3 origin = center;                                                   /* :278 */
    if (c->defocus_angle > 0.0f) {                                          /* :279-281 */
        vec3 ddu = v3(c->defocus_disk_u[0], c->defocus_disk_u[1], c->defocus_disk_u[2]);
        vec3 ddv = v3(c->defocus_disk_v[0], c->defocus_disk_v[1], c->defocus_disk_v[2]);
        origin = v_add(center, v_add(v_scale(ddu, disc.x), v_scale(ddv, disc.y)));
    }
    ray_t r;
    r.origin = origin;
    r.dir = v_sub(pc, origin);                                              /* :283-284 */
    return r;
}

static vec3 sample_color(const ctx_t* cx, uint32_t i, uint32_t j, uint32_t k) {
    rng_t rng;
    rng.key[0] = (uint32_t)cx->seed;
    rng.key[1] = (uint32_t)(cx->seed >> 32);
    rng.pixel = j * cx->cam->image_width + i;
    rng.sample = k;
    rng.event = rng.attempt = rng.word = 0;
    rng.draws = &cx->c->rng_draws;
    ray_t r = get_ray(cx, &rng, i, j);
    cx->c->samples++;
    g_tier_path_far = 0;
    if (cx->order == ORACLE_ORDER_ITERATIVE) return ray_color_iter(cx, r, &rng, (int)cx->cam->max_depth);
    return ray_color_ref(cx, &r, &rng, (int)cx->cam->max_depth);
}

/* GetPixelColor, camera.go:254-263. */
static vec3 pixel_color(const ctx_t* cx, uint32_t i, uint32_t j) {
    vec3 sum = v3(0.0f, 0.0f, 0.0f);
    uint32_t spp = cx->cam->samples_per_pixel;
    for (uint32_t k = 0; k < spp; ++k) sum = v_add(sum, sample_color(cx, i, j, k));
    return v_scale(sum, 1.0f / (float)spp);
}

/* ============================================================================
 * Region rendering, threads over rows.
 * ========================================================================== */
/* Rows of a shard (include/rtx.h rtx_region): stripes of S rows dealt round-robin, the last one maybe partial. */
uint32_t oracle_region_rows(const rtx_region* r) {
    if (r->world == 0 || r->rank >= r->world) return 0;
    const uint32_t S = r->stripe > 1u ? r->stripe : 1u;
    const uint32_t nst = (r->height + S - 1) / S;
    if (r->rank >= nst) return 0;
    uint32_t rows = (nst - r->rank + r->world - 1) / r->world * S;
    if ((nst - 1) % r->world == r->rank && r->height % S) rows -= S - r->height % S;
    return rows;
}

static int scene_supported(const rtx_scene_desc* s) {
    if (!s || !s->roots || s->n_roots == 0) return 0;
    for (uint32_t i = 0; i < s->n_materials; ++i)
        if (s->materials[i].type > RTX_MAT_DIFFUSE_LIGHT) return 0;
    for (uint32_t i = 0; i < s->n_textures; ++i) {
        const rtx_texture* t = &s->textures[i];
        if (t->type > RTX_TEX_NOISE) return 0;
        if (t->type == RTX_TEX_IMAGE && (int32_t)t->height > 0 &&
            (uint64_t)t->texel_offset + 2ull * ((uint64_t)t->width * t->height + 1) > s->n_texels)
            return 0; /* RGBA16 raster + border texel (rtx.h) */
    }
    if (s->n_quads && !s->quads) return 0;
    if (s->n_lists && (!s->lists || !s->list_refs)) return 0;
    for (uint32_t i = 0; i < s->n_lists; ++i)
        if ((uint64_t)s->lists[i].first + s->lists[i].count > s->n_list_refs) return 0;
    return 1;
}

typedef struct {
    const rtx_scene_desc* s;
    const rtx_camera* cam;
    uint64_t seed;
    const rtx_region* reg;
    int order;
    float* out;
    uint32_t rows;
    uint32_t next_row;
    pthread_mutex_t mu;
    oracle_counters total;
} job_t;

static void* worker(void* arg) {
    job_t* jb = (job_t*)arg;
    oracle_counters local;
    memset(&local, 0, sizeof(local));
    ctx_t cx = {jb->s, jb->cam, jb->seed, jb->order, &local};
    for (;;) {
        pthread_mutex_lock(&jb->mu);
        uint32_t lr = jb->next_row++;
        pthread_mutex_unlock(&jb->mu);
        if (lr >= jb->rows) break;
        const uint32_t S = jb->reg->stripe > 1u ? jb->reg->stripe : 1u; /* stripes dealt round-robin (rtx.h) */
        uint32_t y = jb->reg->y0 + ((lr / S) * jb->reg->world + jb->reg->rank) * S + lr % S;
        for (uint32_t xx = 0; xx < jb->reg->width; ++xx) {
            vec3 c = pixel_color(&cx, jb->reg->x0 + xx, y);
            float* o = jb->out + ((size_t)lr * jb->reg->width + xx) * 3;
            o[0] = c.x; o[1] = c.y; o[2] = c.z;
        }
    }
    pthread_mutex_lock(&jb->mu);
    jb->total.samples += local.samples;
    jb->total.segments += local.segments;
    jb->total.node_visits += local.node_visits;
    jb->total.prim_tests_ref += local.prim_tests_ref;
    jb->total.prim_tests += local.prim_tests;
    jb->total.hits += local.hits;
    jb->total.texel_fetches += local.texel_fetches;
    jb->total.texel_border += local.texel_border;
    jb->total.rng_draws += local.rng_draws;
    pthread_mutex_unlock(&jb->mu);
    return NULL;
}

int oracle_render(const rtx_scene_desc* s, const rtx_camera* cam, uint64_t seed, const rtx_region* reg, int order,
                  int threads, float* out, oracle_counters* counters) {
    if (!s || !cam || !reg || !out || !scene_supported(s)) return -1;
    if (cam->samples_per_pixel == 0 || reg->world == 0 || reg->rank >= reg->world) return -1;
    if (reg->x0 + reg->width > cam->image_width || reg->y0 + reg->height > cam->image_height) return -1;
    job_t jb;
    memset(&jb, 0, sizeof(jb));
    jb.s = s; jb.cam = cam; jb.seed = seed; jb.reg = reg; jb.order = order; jb.out = out;
    jb.rows = oracle_region_rows(reg);
    pthread_mutex_init(&jb.mu, NULL);
    if (threads <= 1) {
        worker(&jb);
    } else {
        pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
        for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &jb);
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
        free(th);
    }
    pthread_mutex_destroy(&jb.mu);
    if (counters) *counters = jb.total;
    return 0;
}

int oracle_sample(const rtx_scene_desc* s, const rtx_camera* cam, uint64_t seed, uint32_t px, uint32_t py,
                  uint32_t k, int order, float rgb[3], oracle_counters* counters) {
    if (!s || !cam || !rgb || !scene_supported(s)) return -1;
    oracle_counters local;
    memset(&local, 0, sizeof(local));
    ctx_t cx = {s, cam, seed, order, &local};
    vec3 c = sample_color(&cx, px, py, k);
    rgb[0] = c.x; rgb[1] = c.y; rgb[2] = c.z;
    if (counters) *counters = local;
    return 0;
}

/* ToGamma2 -> ToRGB -> String, vec3.go:141-166, math.go:20-28. */
static int64_t go_int_of_f32(float f) {
    /* amd64 CVTTSS2SQ: truncation; NaN and out-of-range give 0x8000000000000000. */
    if (isnan(f) || f >= 9223372036854775808.0f || f < -9223372036854775808.0f) return INT64_MIN;
    return (int64_t)f;
}
int oracle_ppm_pixel(const float rgb[3], char* buf) {
    int64_t q[3];
    for (int c = 0; c < 3; ++c) {
        float v = (float)sqrt((double)rgb[c]);                 /* ToGamma2 */
        if (v < 0.0f) v = 0.0f;                                 /* Clamp(0, 1, v) */
        else if (v > 1.0f) v = 1.0f;
        v *= 255.999f;                                          /* ToRGB */
        q[c] = go_int_of_f32(v);                                /* String: int(v.X) */
    }
    return sprintf(buf, "%lld %lld %lld", (long long)q[0], (long long)q[1], (long long)q[2]);
}

/* ============================================================================
 * Scene builders: main.go:227-289 randSpheres + bvh.go:138-185 NewBVH, with the
 * reference's two RNGs restated as seeded streams: the global math/rand (stream 1;
 * matPer, centres, and the BVH axis, main.go:251-252, bvh.go:147) and randCtx
 * (stream 2; material values, main.go:259-265).
 * ========================================================================== */
enum { STREAM_GLOBAL = 1, STREAM_CTX = 2 };

typedef struct {
    uint64_t seed;
    uint32_t stream;
    uint64_t n;
} host_rng;

static inline uint32_t hr_u32(host_rng* r) { return oracle_stream_u32(r->seed, r->stream, r->n++); }
static inline float hr_float32(host_rng* r) { return u32_to_unit(hr_u32(r)); }
/* rand.Intn(n) of the contract: multiply-shift of one word. */
static inline int hr_intn(host_rng* r, int n) { return (int)(((uint64_t)hr_u32(r) * (uint64_t)n) >> 32); }
/* RandF32N on a host stream, math.go:30-32. */
static inline float rand_f32n_host(host_rng* r, float mn, float mx) { return mn + hr_float32(r) * (mx - mn); }

typedef struct { float mn[3], mx[3]; } aabb_t;

struct oracle_scene {
    rtx_scene_desc desc;
    rtx_bvh_node* nodes;
    uint32_t n_nodes, cap_nodes;
    rtx_sphere* spheres;
    uint32_t n_spheres, cap_spheres;
    rtx_material* materials;
    uint32_t n_materials, cap_materials;
    rtx_texture* textures;
    uint32_t n_textures, cap_textures;
    int32_t root;
    aabb_t* sphere_box;
};

#define GROW(arr, n, cap)                                                        \
    do {                                                                         \
        if ((n) >= (cap)) {                                                      \
            (cap) = (cap) ? (cap)*2 : 64;                                        \
            (arr) = realloc((arr), sizeof(*(arr)) * (size_t)(cap));              \
        }                                                                        \
    } while (0)

static uint32_t add_texture(oracle_scene* s, rtx_texture t) {
    GROW(s->textures, s->n_textures, s->cap_textures);
    s->textures[s->n_textures] = t;
    return s->n_textures++;
}
static uint32_t add_material(oracle_scene* s, rtx_material m) {
    GROW(s->materials, s->n_materials, s->cap_materials);
    s->materials[s->n_materials] = m;
    return s->n_materials++;
}
static uint32_t solid(oracle_scene* s, float r, float g, float b) {        /* NewSolidColor, materials.go:159 */
    rtx_texture t;
    memset(&t, 0, sizeof(t));
    t.type = RTX_TEX_SOLID;
    t.even[0] = r; t.even[1] = g; t.even[2] = b;
    return add_texture(s, t);
}
static uint32_t lambertian(oracle_scene* s, uint32_t tex) {
    rtx_material m;
    memset(&m, 0, sizeof(m));
    m.type = RTX_MAT_LAMBERTIAN;
    m.texture = tex;
    return add_material(s, m);
}
static uint32_t metal(oracle_scene* s, vec3 albedo, float fuzz) {
    rtx_material m;
    memset(&m, 0, sizeof(m));
    m.type = RTX_MAT_METAL;
    m.albedo[0] = albedo.x; m.albedo[1] = albedo.y; m.albedo[2] = albedo.z;
    m.fuzz = fuzz;
    return add_material(s, m);
}
static uint32_t dielectric(oracle_scene* s, float ior) {
    rtx_material m;
    memset(&m, 0, sizeof(m));
    m.type = RTX_MAT_DIELECTRIC;
    m.ior = ior;
    return add_material(s, m);
}
/* NewSphere, hittables.go:85-94: bbox = NewAabb(center + (-r), center + r). */
static void add_sphere(oracle_scene* s, vec3 c, float r, uint32_t mat) {
    GROW(s->spheres, s->n_spheres, s->cap_spheres);
    rtx_sphere* sp = &s->spheres[s->n_spheres++];
    memset(sp, 0, sizeof(*sp));
    sp->center[0] = c.x; sp->center[1] = c.y; sp->center[2] = c.z;
    sp->radius = r;
    sp->material = mat;
}
static aabb_t sphere_bounds(const rtx_sphere* sp) {
    vec3 c = v3(sp->center[0], sp->center[1], sp->center[2]);
    vec3 rv = v3(sp->radius, sp->radius, sp->radius);
    vec3 p1 = v_add(c, v_scale(rv, -1.0f)), p2 = v_add(c, rv);
    aabb_t b;                                                              /* NewAabb, bvh.go:28-34 */
    b.mn[0] = min_f32(p1.x, p2.x); b.mx[0] = max_f32(p1.x, p2.x);
    b.mn[1] = min_f32(p1.y, p2.y); b.mx[1] = max_f32(p1.y, p2.y);
    b.mn[2] = min_f32(p1.z, p2.z); b.mx[2] = max_f32(p1.z, p2.z);
    return b;
}
static aabb_t box_union(aabb_t a, aabb_t b) {                               /* NewAabbFromBoxes, bvh.go:44-50 */
    aabb_t r;
    for (int k = 0; k < 3; ++k) {
        r.mn[k] = min_f32(a.mn[k], b.mn[k]);
        r.mx[k] = max_f32(a.mx[k], b.mx[k]);
    }
    return r;
}

typedef struct { int32_t ref; aabb_t box; } item_t;

static aabb_t ref_box(const oracle_scene* s, int32_t ref) {
    if (ref >= 0) {
        aabb_t b;
        memcpy(b.mn, s->nodes[ref].bmin, sizeof(b.mn));
        memcpy(b.mx, s->nodes[ref].bmax, sizeof(b.mx));
        return b;
    }
    return s->sphere_box[(~ref) & 0x0FFFFFFF];
}

/* HittableCompare{X,Y,Z}, bvh.go:187-218: +1 when h2.min > h1.min (sort descending).
 * The contract's sort is stable (x/exp/slices.SortFunc is pdqsort and unstable; equal
 * keys may land in either order in the reference). */
static int cmp_axis(const item_t* a, const item_t* b, int axis) {
    float diff = b->box.mn[axis] - a->box.mn[axis];
    if (diff > 0.0f) return 1;
    if (diff < 0.0f) return -1;
    return 0;
}
static void stable_sort(item_t* h, size_t n, int axis) {
    /* insertion sort in blocks + merge: n is small (<= a few 1e5); use a simple merge sort */
    if (n < 2) return;
    item_t* tmp = malloc(sizeof(item_t) * n);
    for (size_t width = 1; width < n; width *= 2) {
        for (size_t lo = 0; lo < n; lo += 2 * width) {
            size_t mid = lo + width < n ? lo + width : n;
            size_t hi = lo + 2 * width < n ? lo + 2 * width : n;
            size_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) {
                if (cmp_axis(&h[j], &h[i], axis) < 0) tmp[k++] = h[j++];
                else tmp[k++] = h[i++];
            }
            while (i < mid) tmp[k++] = h[i++];
            while (j < hi) tmp[k++] = h[j++];
        }
        memcpy(h, tmp, sizeof(item_t) * n);
    }
    free(tmp);
}

/* NewBVH, bvh.go:142-185.  Returns the node index.  Nodes are numbered in creation
 * (pre-)order: a node's index is reserved before its children are built. */
static int32_t new_bvh(oracle_scene* s, host_rng* grng, const item_t* in, size_t n) {
    item_t* h = malloc(sizeof(item_t) * n);                                  /* :144-145 */
    memcpy(h, in, sizeof(item_t) * n);
    int axis = hr_intn(grng, 3);                                             /* :147 */
    GROW(s->nodes, s->n_nodes, s->cap_nodes);
    int32_t me = (int32_t)s->n_nodes++;
    int32_t left, right;
    if (n == 1) {                                                            /* :162-165 */
        left = right = h[0].ref;
    } else if (n == 2) {                                                     /* :166-174 */
        if (cmp_axis(&h[0], &h[1], axis) > 0) {
            left = h[1].ref; right = h[0].ref;
        } else {
            left = h[0].ref; right = h[1].ref;
        }
    } else {                                                                 /* :175-180 */
        stable_sort(h, n, axis);
        size_t mid = n / 2;
        left = new_bvh(s, grng, h, mid);
        right = new_bvh(s, grng, h + mid, n - mid);
    }
    aabb_t b = box_union(ref_box(s, left), ref_box(s, right));               /* :182 */
    rtx_bvh_node* node = &s->nodes[me];
    memcpy(node->bmin, b.mn, sizeof(b.mn));
    memcpy(node->bmax, b.mx, sizeof(b.mx));
    node->left = left;
    node->right = right;
    free(h);
    return me;
}

oracle_scene* oracle_build_random_spheres(uint64_t seed) {
    oracle_scene* s = calloc(1, sizeof(oracle_scene));
    host_rng grng = {seed, STREAM_GLOBAL, 0};
    host_rng crng = {seed, STREAM_CTX, 0};
    /* main.go:242-244 */
    rtx_texture chk;
    memset(&chk, 0, sizeof(chk));
    chk.type = RTX_TEX_CHECKERED;
    chk.scale = 0.32f;
    chk.even[0] = 0.2f; chk.even[1] = 0.3f; chk.even[2] = 0.1f;
    chk.odd[0] = 0.9f; chk.odd[1] = 0.9f; chk.odd[2] = 0.9f;
    uint32_t ground = lambertian(s, add_texture(s, chk));
    add_sphere(s, v3(0.0f, -1000.0f, 0.0f), 1000.0f, ground);
    vec3 p = v3(4.0f, 0.2f, 0.0f);                                           /* :248 */
    for (int i = -11; i < 11; ++i) {                                         /* :249 */
        for (int j = -11; j < 11; ++j) {                                     /* :250 */
            float mat_per = hr_float32(&grng);                               /* :251 */
            float cx = (float)i + 0.9f * hr_float32(&grng);                  /* :252 */
            float cz = (float)j + 0.9f * hr_float32(&grng);
            vec3 center = v3(cx, 0.2f, cz);
            vec3 dist = v_sub(center, p);                                    /* :254 */
            float ln = (float)sqrt((double)v_lensq(dist));                   /* :255, vec3.go:119-121 */
            if (ln > 0.9f) {                                                 /* :256 */
                uint32_t m;
                if (mat_per < 0.8f) {                                        /* :258-262 */
                    float a0 = hr_float32(&crng), a1 = hr_float32(&crng), a2 = hr_float32(&crng);
                    float b0 = hr_float32(&crng), b1 = hr_float32(&crng), b2 = hr_float32(&crng);
                    vec3 col = v_mul(v3(a0, a1, a2), v3(b0, b1, b2));
                    m = lambertian(s, solid(s, col.x, col.y, col.z));
                } else if (mat_per < 0.95f) {                                /* :263-267 */
                    float x = rand_f32n_host(&crng, 0.5f, 1.0f);
                    float y = rand_f32n_host(&crng, 0.5f, 1.0f);
                    float z = rand_f32n_host(&crng, 0.5f, 1.0f);
                    float fuzz = rand_f32n_host(&crng, 0.0f, 0.5f);
                    m = metal(s, v3(x, y, z), fuzz);
                } else {                                                     /* :268-271 */
                    m = dielectric(s, 1.5f);
                }
                add_sphere(s, center, 0.2f, m);                              /* :272 */
            }
        }
    }
    add_sphere(s, v3(0.0f, 1.0f, 0.0f), 1.0f, dielectric(s, 1.5f));          /* :278-279 */
    add_sphere(s, v3(-4.0f, 1.0f, 0.0f), 1.0f, lambertian(s, solid(s, 0.4f, 0.2f, 0.1f))); /* :281-282 */
    add_sphere(s, v3(4.0f, 1.0f, 0.0f), 1.0f, metal(s, v3(0.7f, 0.6f, 0.5f), 0.0f));       /* :284-285 */

    /* NewBVHFromWorld, main.go:287 -> bvh.go:138-140 */
    s->sphere_box = malloc(sizeof(aabb_t) * s->n_spheres);
    item_t* items = malloc(sizeof(item_t) * s->n_spheres);
    for (uint32_t k = 0; k < s->n_spheres; ++k) {
        s->sphere_box[k] = sphere_bounds(&s->spheres[k]);
        items[k].ref = RTX_REF_PRIM(RTX_PRIM_SPHERE, k);
        items[k].box = s->sphere_box[k];
    }
    s->root = new_bvh(s, &grng, items, s->n_spheres);
    free(items);

    s->desc.nodes = s->nodes;
    s->desc.n_nodes = s->n_nodes;
    s->desc.n_roots = 1;
    s->desc.roots = &s->root;
    s->desc.spheres = s->spheres;
    s->desc.n_spheres = s->n_spheres;
    s->desc.materials = s->materials;
    s->desc.n_materials = s->n_materials;
    s->desc.textures = s->textures;
    s->desc.n_textures = s->n_textures;
    return s;
}

const rtx_scene_desc* oracle_scene_desc(const oracle_scene* s) { return &s->desc; }

void oracle_scene_free(oracle_scene* s) {
    if (!s) return;
    free(s->nodes);
    free(s->spheres);
    free(s->materials);
    free(s->textures);
    free(s->sphere_box);
    free(s);
}

/* ============================================================================
 * Go's image.YCbCr (image/ycbcr.go) and color.YCbCr.RGBA (image/color/ycbcr.go),
 * Go 1.21 — the *image.YCbCr jpeg.Decode returns for the earth texture (file.go:20-28,
 * main.go:97-100), restated independently of the host mirror.
 * ========================================================================== */
void oracle_ycbcr_rgba(uint8_t y, uint8_t cb, uint8_t cr, uint32_t out[3]) {
    const int32_t yy1 = (int32_t)y * 0x10101;   /* 65536*Y' + adjustment Y'*0x0101 */
    const int32_t cb1 = (int32_t)cb - 128;
    const int32_t cr1 = (int32_t)cr - 128;
    int32_t v[3];
    v[0] = yy1 + 91881 * cr1;
    v[1] = yy1 - 22554 * cb1 - 46802 * cr1;
    v[2] = yy1 + 116130 * cb1;
    for (int k = 0; k < 3; ++k) {
        if (((uint32_t)v[k] & 0xff000000u) == 0)
            out[k] = (uint32_t)(v[k] >> 8);
        else
            out[k] = (uint32_t)(~(v[k] >> 31)) & 0xffffu;
    }
}

void oracle_ycbcr_rgba_all(uint32_t* out) {
    for (uint32_t k = 0; k < (1u << 24); ++k)
        oracle_ycbcr_rgba((uint8_t)(k >> 16), (uint8_t)(k >> 8), (uint8_t)k, &out[3 * (size_t)k]);
}

int oracle_ycbcr_texels(const uint8_t* Y, const uint8_t* Cb, const uint8_t* Cr, int64_t w, int64_t h,
                        int64_t ystride, int64_t cstride, int ratio, uint32_t* out) {
    if (w <= 0 || h <= 0) return -1;
    for (int64_t y = 0; y < h; ++y) {
        for (int64_t x = 0; x < w; ++x) {
            int64_t ci;
            switch (ratio) { /* COffset, Rect.Min = (0, 0) */
            case 1: ci = y * cstride + x / 2; break;           /* 4:2:2 */
            case 2: ci = (y / 2) * cstride + x / 2; break;     /* 4:2:0 */
            case 3: ci = (y / 2) * cstride + x; break;         /* 4:4:0 */
            case 4: ci = y * cstride + x / 4; break;           /* 4:1:1 */
            case 5: ci = (y / 2) * cstride + x / 4; break;     /* 4:1:0 */
            default: ci = y * cstride + x; break;              /* 4:4:4 */
            }
            uint32_t c[3];
            oracle_ycbcr_rgba(Y[y * ystride + x], Cb[ci], Cr[ci], c);
            uint32_t* o = &out[2 * (size_t)(y * w + x)];
            o[0] = c[0] | c[1] << 16;
            o[1] = c[2] | 0xffffu << 16;
        }
    }
    uint32_t c[3]; /* outside Bounds: color.YCbCr{} */
    oracle_ycbcr_rgba(0, 0, 0, c);
    uint32_t* o = &out[2 * (size_t)(w * h)];
    o[0] = c[0] | c[1] << 16;
    o[1] = c[2] | 0xffffu << 16;
    return 0;
}
