// rtx_device.h — device-side building blocks of the megakernel (gfx950).
//
// Float semantics.  Every decision on a path (hit/miss, dot > 0, reflectance > u,
// rejection-sampling acceptance) is chaotic, so the kernel performs exactly the IEEE
// float32 operations of the Go source, in the same association order, with no
// contraction (built with -ffp-contract=off) and with the correctly rounded division
// and square root hipcc emits by default for gfx950.  Where Go widens to float64
// (Dielectric, materials.go:100, 118) the kernel does too.  The cited lines are the
// reference's; the structure (iterative, stackless, branch-light) is the GPU's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtx.h"
#include "rtx_layout.h"

namespace rtxd {

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }       // vec3.go:49
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }       // vec3.go:73
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }       // vec3.go:61
__device__ __forceinline__ V3 scale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }        // vec3.go:97
__device__ __forceinline__ float lensq(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }          // vec3.go:115
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }      // vec3.go:137
__device__ __forceinline__ V3 unit(V3 v) {                                                         // vec3.go:103-113
    float l = __builtin_sqrtf(lensq(v));
    return scale(v, 1.0f / l);
}
__device__ __forceinline__ bool near_zero(V3 v) {                                                  // vec3.go:170-172
    return __builtin_fabsf(v.x) < 1e-8f && __builtin_fabsf(v.y) < 1e-8f && __builtin_fabsf(v.z) < 1e-8f;
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }   // vec3.go:212-214
__device__ __forceinline__ V3 refract(V3 uv, V3 n, float eta) {                                    // vec3.go:216-221
    float cos_t = dot(scale(uv, -1.0f), n);
    V3 perp = scale(add(uv, scale(n, cos_t)), eta);
    float s = __builtin_sqrtf(__builtin_fabsf(1.0f - lensq(perp)));  // f64 sqrt of an f32, rounded back
    V3 par = scale(n, -1.0f * s);
    return add(par, perp);
}

// Go math.Pow(x, 5), x in [0, 2] (see oracle/oracle.c go_pow5): x * ((x*x) * (x*x)) in
// float64 — the frexp/ldexp power-of-two scalings of Go's loop are exact here.
__device__ __forceinline__ double go_pow5(double x) {
    double x2 = x * x;
    double x4 = x2 * x2;
    return x * x4;
}

// ---------------------------------------------------------------------------------
// RNG contract: Philox4x32-10 keyed by the seed; counter =
// (global pixel index, sample index, draw block, stream 0); draw n = word n & 3 of
// block n >> 2; u = float32(x >> 8) * 2^-24.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t& o0, uint32_t& o1, uint32_t& o2, uint32_t& o3) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    o0 = c0;
    o1 = c1;
    o2 = c2;
    o3 = c3;
}

struct Rng {
    uint32_t k0, k1, pixel, sample, n;
    uint32_t w0, w1, w2, w3;
    uint32_t draws;

    __device__ __forceinline__ void init(uint64_t seed, uint32_t px, uint32_t k) {
        k0 = (uint32_t)seed;
        k1 = (uint32_t)(seed >> 32);
        pixel = px;
        sample = k;
        n = 0;
    }
    __device__ __forceinline__ float next() {
        const uint32_t slot = n & 3u;
        if (slot == 0u) philox4x32_10(pixel, sample, n >> 2, 0u, k0, k1, w0, w1, w2, w3);
        const uint32_t w = slot == 0u ? w0 : (slot == 1u ? w1 : (slot == 2u ? w2 : w3));
        ++n;
        return (float)(w >> 8) * 0x1.0p-24f;
    }
    // RandF32N(-1, 1), math.go:30-32: -1 + u * (1 - (-1)).
    __device__ __forceinline__ float signed_unit() { return -1.0f + next() * 2.0f; }
};

// NewVec3UnitRandOnUnitSphere32, vec3.go:182-190.
__device__ __forceinline__ V3 rand_unit_on_sphere(Rng& rng) {
    for (;;) {
        const float x = rng.signed_unit();
        const float y = rng.signed_unit();
        const float z = rng.signed_unit();
        const V3 v = v3(x, y, z);
        if (lensq(v) < 1.0f) return unit(v);
    }
}

// NewVec3RandInUnitDisk, vec3.go:203-210 (LenSq adds the z = 0 term: exact no-op).
__device__ __forceinline__ void rand_in_unit_disk(Rng& rng, float& x, float& y) {
    for (;;) {
        x = rng.signed_unit();
        y = rng.signed_unit();
        if (x * x + y * y < 1.0f) return;
    }
}

// ---------------------------------------------------------------------------------
// Kernel parameters
// ---------------------------------------------------------------------------------
struct Params {
    const float4* entries;   // 2 float4 per rtx_entry
    uint32_t n_entries;
    uint32_t n_materials;
    const rtx_material* materials;
    const rtx_texture* textures;
    const uint32_t* texels;
    rtx_camera cam;
    uint64_t seed;
    uint32_t x0, y0, width, rows, rank, world;
    float* out;
    unsigned long long* counters;  // 7 x u64 (rtx_stats order) when counting
};

struct Ray {
    V3 o, d;
};

struct Counters {
    uint32_t segments, node_visits, prim_tests, hits, texel_fetches;
};

// Closest hit over the threaded pre-order layout (see rtx_layout.h): identical
// sequence of Aabb.Hit (bvh.go:52-61, 84-102) and Sphere.Hit (hittables.go:96-116)
// tests as the reference recursion, running bound = closest hit so far.
template <bool COUNT>
__device__ __forceinline__ int32_t closest_hit(const Params& p, const Ray& r, float& t_hit, Counters& cnt) {
    // InBoundary computes 1/dir per node; hoisting it is bit-identical.
    const float ix = 1.0f / r.d.x, iy = 1.0f / r.d.y, iz = 1.0f / r.d.z;
    const bool nx = ix < 0.0f, ny = iy < 0.0f, nz = iz < 0.0f;
    const float a = lensq(r.d);  // hittables.go:98, loop-invariant
    const float tmin = 0.001f;   // ray.go:37
    float closest = __builtin_inff();
    int32_t hit = -1;
    const float4* __restrict__ E = p.entries;
    const uint32_t n = p.n_entries;
    uint32_t i = 0;
    while (i < n) {
        const float4 ea = E[2 * i];
        const float4 eb = E[2 * i + 1];
        const int32_t tag = __float_as_int(eb.w);
        if (tag == RTX_E_NODE) {
            if (COUNT) ++cnt.node_visits;
            // Per axis: t0 = (min - o) * invD, t1 = (max - o) * invD, swapped if invD < 0
            // (selecting the operands first is the same two operations).
            const float t0x = ((nx ? eb.x : ea.x) - r.o.x) * ix;
            const float t1x = ((nx ? ea.x : eb.x) - r.o.x) * ix;
            const float t0y = ((ny ? eb.y : ea.y) - r.o.y) * iy;
            const float t1y = ((ny ? ea.y : eb.y) - r.o.y) * iy;
            const float t0z = ((nz ? eb.z : ea.z) - r.o.z) * iz;
            const float t1z = ((nz ? ea.z : eb.z) - r.o.z) * iz;
            // `if t0 > min { min = t0 }` keeps min on NaN (0 * inf): fmaxf's NaN rule.
            // The bound only shrinks, so testing min < max once after all three axes
            // equals the reference's per-axis early exit.
            const float lo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tmin, t0x), t0y), t0z);
            const float hi = __builtin_fminf(__builtin_fminf(__builtin_fminf(closest, t1x), t1y), t1z);
            i = (lo < hi) ? i + 1 : (uint32_t)__float_as_int(ea.w);
        } else {
            if (COUNT) ++cnt.prim_tests;
            const float ox = r.o.x - ea.x, oy = r.o.y - ea.y, oz = r.o.z - ea.z;       // :97
            const float hb = r.d.x * ox + r.d.y * oy + r.d.z * oz;                     // :99
            const float c = (ox * ox + oy * oy + oz * oz) - eb.x;                      // :100
            const float disc = hb * hb - a * c;                                        // :102
            if (disc >= 0.0f) {                                                        // :104 (NaN: miss either way)
                const float sq = __builtin_sqrtf(disc);                                // :108
                float t = (-hb - sq) / a;                                              // :110
                bool ok = tmin < t && t < closest;
                if (!ok) {
                    t = (-hb + sq) / a;                                                // :112
                    ok = tmin < t && t < closest;
                }
                if (ok) {
                    closest = t;
                    hit = (int32_t)i;
                }
            }
            ++i;
        }
    }
    t_hit = closest;
    return hit;
}

// Texture.GetTexture, materials.go:127-193.
template <bool COUNT>
__device__ __forceinline__ V3 texture_value(const Params& p, uint32_t ti, float u, float v, V3 pt, Counters& cnt) {
    const rtx_texture& t = p.textures[ti];
    if (t.type == RTX_TEX_SOLID) return v3(t.even[0], t.even[1], t.even[2]);
    if (t.type == RTX_TEX_CHECKERED) {
        const float inv = 1.0f / t.scale;
        const int64_t x = (int64_t)__builtin_floorf(inv * pt.x);
        const int64_t y = (int64_t)__builtin_floorf(inv * pt.y);
        const int64_t z = (int64_t)__builtin_floorf(inv * pt.z);
        return ((x + y + z) & 1) == 0 ? v3(t.even[0], t.even[1], t.even[2]) : v3(t.odd[0], t.odd[1], t.odd[2]);
    }
    // RTX_TEX_IMAGE
    if ((int32_t)t.height <= 0) return v3(0.0f, 1.0f, 1.0f);
    const float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
    const float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    const float vv = 1.0f - vc;
    const float fi = uu * (float)t.width;
    const float fj = vv * (float)t.height;
    if (COUNT) ++cnt.texel_fetches;
    if (!(fi >= 0.0f) || !(fj >= 0.0f)) return v3(0.0f, 0.0f, 0.0f);  // NaN
    const int64_t i = (int64_t)fi, j = (int64_t)fj;
    if (i >= (int64_t)t.width || j >= (int64_t)t.height) return v3(0.0f, 0.0f, 0.0f);
    const uint32_t px = p.texels[t.texel_offset + (uint64_t)j * t.width + (uint64_t)i];
    const float cs = 1.0f / 65535.0f;
    return v3((float)((px & 0xFFu) * 257u) * cs, (float)(((px >> 8) & 0xFFu) * 257u) * cs,
              (float)(((px >> 16) & 0xFFu) * 257u) * cs);
}

__device__ __forceinline__ bool texture_needs_uv(const Params& p, uint32_t ti) {
    return p.textures[ti].type == RTX_TEX_IMAGE;
}

// Spherical UV, hittables.go:122-126 (float64 acos / atan2; typed float32 constants).
__device__ __forceinline__ void sphere_uv(V3 n, float& u, float& v) {
    const float pi32 = 3.14159274101257324f;
    const float theta = (float)acos(-(double)n.y);
    const float phi = (float)(atan2(-(double)n.z, (double)n.x) + 3.14159265358979323846);
    u = (phi + 5.0f * pi32 / 12.0f) / (2.0f * pi32);
    v = theta / pi32;
}

// GetRay + sampleUnitSquare, camera.go:265-299.  base = (pixel00 + du*i) + dv*j.
__device__ __forceinline__ Ray camera_ray(const rtx_camera& c, V3 base, Rng& rng) {
    const V3 du = v3(c.pixel_du[0], c.pixel_du[1], c.pixel_du[2]);
    const V3 dv = v3(c.pixel_dv[0], c.pixel_dv[1], c.pixel_dv[2]);
    const float dx = -0.5f + rng.next();                          // :290
    const float dy = -0.5f + rng.next();                          // :291
    const V3 pc = add(base, add(scale(du, dx), scale(dv, dy)));   // :275
    float x, y;
    rand_in_unit_disk(rng, x, y);                                 // :277, always drawn
    const V3 center = v3(c.center[0], c.center[1], c.center[2]);
    V3 origin = center;
    if (c.defocus_angle > 0.0f) {                                 // :279-281
        const V3 ddu = v3(c.defocus_disk_u[0], c.defocus_disk_u[1], c.defocus_disk_u[2]);
        const V3 ddv = v3(c.defocus_disk_v[0], c.defocus_disk_v[1], c.defocus_disk_v[2]);
        origin = add(center, add(scale(ddu, x), scale(ddv, y)));
    }
    return Ray{origin, sub(pc, origin)};                          // :283-286
}

// One path: GetColor (ray.go:32-54) as a bounded loop, colour accumulated front to
// back (L += T*emit, T *= attenuation).  Path decisions are those of the recursion;
// the colour product differs from it only in rounding (~1 ulp).
template <bool COUNT>
__device__ __forceinline__ V3 trace_path(const Params& p, Ray r, Rng& rng, Counters& cnt) {
    V3 thr = v3(1.0f, 1.0f, 1.0f);
    V3 acc = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t depth = p.cam.max_depth; depth > 0; --depth) {   // ray.go:33
        if (COUNT) ++cnt.segments;
        float t;
        const int32_t e = closest_hit<COUNT>(p, r, t, cnt);
        if (e < 0) {                                                // ray.go:52
            const V3 bg = v3(p.cam.background[0], p.cam.background[1], p.cam.background[2]);
            return add(acc, mul(thr, bg));
        }
        if (COUNT) ++cnt.hits;
        const float4 sa = p.entries[2 * e];
        const float4 sb = p.entries[2 * e + 1];
        const V3 c = v3(sa.x, sa.y, sa.z);
        const float radius = sa.w;
        const uint32_t mi = (uint32_t)__float_as_int(sb.w);
        const V3 pt = add(scale(r.d, t), r.o);                      // ray.go:25-30
        V3 n = unit(scale(sub(pt, c), radius));                     // hittables.go:119-120
        const bool front = dot(r.d, n) < 0.0f;                      // hittables.go:23
        const rtx_material m = p.materials[mi];
        float u = 0.0f, v = 0.0f;
        if ((m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_DIFFUSE_LIGHT) && texture_needs_uv(p, m.texture))
            sphere_uv(n, u, v);                                     // only an image texture reads UV
        if (!front) n = scale(n, -1.0f);                            // hittables.go:24-26

        if (m.type == RTX_MAT_LAMBERTIAN) {                         // materials.go:33-42
            V3 dir = add(n, rand_unit_on_sphere(rng));
            if (near_zero(dir)) dir = n;
            const V3 att = texture_value<COUNT>(p, m.texture, u, v, pt, cnt);
            thr = mul(thr, att);
            r = Ray{pt, dir};
        } else if (m.type == RTX_MAT_METAL) {                       // materials.go:60-75
            const V3 ud = unit(r.d);
            const V3 refl = reflect(ud, n);
            const V3 fz = scale(rand_unit_on_sphere(rng), m.fuzz);
            const V3 s = add(refl, fz);
            if (!(dot(s, n) > 0.0f)) return acc;                    // absorbed: Emit() = 0
            thr = mul(thr, v3(m.albedo[0], m.albedo[1], m.albedo[2]));
            r = Ray{pt, s};
        } else if (m.type == RTX_MAT_DIELECTRIC) {                  // materials.go:91-113
            const float eta = front ? 1.0f / m.ior : m.ior;
            const V3 ud = unit(r.d);
            const float d = dot(scale(ud, -1.0f), n);
            const float cos_t = d < 1.0f ? d : (d != d ? d : 1.0f); // float32(math.Min(float64(d), 1))
            const float sin_t = (float)__builtin_sqrt(1.0 - (double)(cos_t * cos_t));
            bool refl = sin_t * eta > 1.0f;
            if (!refl) {                                            // short-circuit: draw only here
                float r0 = (1.0f - eta) / (1.0f + eta);             // materials.go:116-118
                r0 *= r0;
                const float rf = r0 + (1.0f - r0) * (float)go_pow5(1.0 - (double)cos_t);
                refl = rf > rng.next();
            }
            const V3 dir = refl ? reflect(ud, n) : refract(ud, n, eta);
            r = Ray{pt, dir};                                       // attenuation (1,1,1)
        } else {                                                    // DiffuseLight: emit, no scatter
            const V3 em = texture_value<COUNT>(p, m.texture, u, v, pt, cnt);
            return add(acc, mul(thr, em));
        }
    }
    return acc;  // depth exhausted: ray.go:33-35
}

}  // namespace rtxd
