// rtx_device.h — device-side building blocks of the megakernel (gfx950).
//
// Float semantics.  Every decision on a path (hit/miss, dot > 0, reflectance > u,
// rejection-sampling acceptance) is chaotic, so the kernel performs exactly the IEEE
// float32 operations of the Go source, in the same association order, with no
// contraction (built with -ffp-contract=off) and with the correctly rounded division
// and square root hipcc emits by default for gfx950.  Where Go widens to float64
// (Dielectric, materials.go:100, 118; sphere UV, hittables.go:122-123) the kernel does
// too.  The cited lines are the reference's; the structure (iterative, stackless,
// lockstep RNG) is the GPU's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtx.h"
#include "rtx_layout.h"

namespace rtxd {

// Wave vote on a bool (HIP's __ballot takes an int).
__device__ __forceinline__ uint64_t ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }

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
__device__ __forceinline__ V3 cross(V3 l, V3 r) {                                                 // vec3.go:129-135
    return v3(l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x);
}
// 1 / x, correctly rounded.  When every active lane's |x| lies in [2^-125, 2^125] (exponent
// field 2..252): one Newton step with fma on v_rcp_f32 (3 VALU), which equals the IEEE quotient
// on all 4.2e9 such inputs (scripts/micro/fastrcp_check.hip, exhaustive on the GPU); else the
// compiler's division (~10 VALU).  The vote is wave-uniform, so the branch does not diverge.
__device__ __forceinline__ bool rcp_fast_ok(float x) { return ((__float_as_uint(x) >> 23) & 0xFFu) - 2u <= 250u; }
__device__ __forceinline__ float rcp_newton(float x) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float rcp_ieee(float x) {
    if (__builtin_amdgcn_ballot_w64(!rcp_fast_ok(x)) == 0) return rcp_newton(x);
    return 1.0f / x;
}
// sqrt(x) correctly rounded, as the compiler expands an f32 sqrt: v_sqrt, then the neighbour
// whose fma residual changes sign.  The expansion's 2^32 pre-scaling is needed only below 2^-96,
// so it runs (the builtin) only when a lane of the wave has 0 <= x < 2^-96; its +-0 / +inf
// pass-through is left out: v_sqrt returns those exactly and both residuals then keep them.
__device__ __forceinline__ float sqrt_rn(float x) {
    if (__builtin_amdgcn_ballot_w64(x < 0x1p-96f && x >= 0.0f) != 0) return __builtin_sqrtf(x);
    float s = __builtin_amdgcn_sqrtf(x);
    const float sp = __uint_as_float(__float_as_uint(s) - 1u), sn = __uint_as_float(__float_as_uint(s) + 1u);
    const float rp = __builtin_fmaf(-sp, s, x), rn = __builtin_fmaf(-sn, s, x);
    if (rp <= 0.0f) s = sp;
    if (rn > 0.0f) s = sn;
    return s;
}
__device__ __forceinline__ V3 unit(V3 v) {                                                         // vec3.go:103-113
    float l = sqrt_rn(lensq(v));
    return scale(v, rcp_ieee(l));
}
__device__ __forceinline__ bool near_zero(V3 v) {                                                  // vec3.go:170-172
    return __builtin_fabsf(v.x) < 1e-8f && __builtin_fabsf(v.y) < 1e-8f && __builtin_fabsf(v.z) < 1e-8f;
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }   // vec3.go:212-214
__device__ __forceinline__ V3 refract(V3 uv, V3 n, float eta) {                                    // vec3.go:216-221
    float cos_t = dot(scale(uv, -1.0f), n);
    V3 perp = scale(add(uv, scale(n, cos_t)), eta);
    float s = sqrt_rn(__builtin_fabsf(1.0f - lensq(perp)));  // f64 sqrt of an f32, rounded back
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
// Go's math.Atan2 / math.Acos (Go 1.21 src/math/atan.go, asin.go, atan2.go — pure Go
// on amd64, Cephes rational approximations).  Restated op for op in float64, so the
// UV of hittables.go:122-123 is the same bits on the GPU, in the oracle and in Go.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ double go_xatan(double x) {  // atan.go xatan: [0, 0.66]
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
__device__ __forceinline__ double go_satan(double x) {  // atan.go satan: x >= 0
    const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
    const double PiO2 = 1.57079632679489661923, PiO4 = 0.785398163397448309616;
    if (x <= 0.66) return go_xatan(x);
    if (x > Tan3pio8) return PiO2 - go_xatan(1.0 / x) + Morebits;
    return PiO4 + go_xatan((x - 1.0) / (x + 1.0)) + 0.5 * Morebits;
}
__device__ __forceinline__ double go_atan(double x) {
    if (x == 0.0) return x;
    return x > 0.0 ? go_satan(x) : -go_satan(-x);
}
__device__ __forceinline__ double go_atan2(double y, double x) {  // atan2.go
    const double Pi = 3.14159265358979323846;
    if (y != y || x != x) return __builtin_nan("");
    if (y == 0.0) {
        if (x >= 0.0 && !__builtin_signbit(x)) return __builtin_copysign(0.0, y);
        return __builtin_copysign(Pi, y);
    }
    if (x == 0.0) return __builtin_copysign(Pi / 2.0, y);
    if (__builtin_isinf(x)) {
        if (x > 0.0) return __builtin_isinf(y) ? __builtin_copysign(Pi / 4.0, y) : __builtin_copysign(0.0, y);
        return __builtin_isinf(y) ? __builtin_copysign(3.0 * Pi / 4.0, y) : __builtin_copysign(Pi, y);
    }
    if (__builtin_isinf(y)) return __builtin_copysign(Pi / 2.0, y);
    const double q = go_atan(y / x);
    if (x < 0.0) return q <= 0.0 ? q + Pi : q - Pi;
    return q;
}
__device__ __forceinline__ double go_asin(double x) {  // asin.go
    const double PiO2 = 1.57079632679489661923;
    if (x == 0.0) return x;
    bool sign = false;
    if (x < 0.0) {
        x = -x;
        sign = true;
    }
    if (x > 1.0) return __builtin_nan("");
    double temp = __builtin_sqrt(1.0 - x * x);
    if (x > 0.7) temp = PiO2 - go_satan(temp / x);
    else temp = go_satan(x / temp);
    return sign ? -temp : temp;
}
__device__ __forceinline__ double go_acos(double x) { return 1.57079632679489661923 - go_asin(x); }

// Spherical UV, hittables.go:122-126 (float64 Acos / Atan2; typed float32 constants).
struct UV {
    float u, v;
};
__device__ __noinline__ UV sphere_uv(float nx, float ny, float nz) {
    const float pi32 = 3.14159274101257324f;
    const float theta = (float)go_acos(-(double)ny);
    const float phi = (float)(go_atan2(-(double)nz, (double)nx) + 3.14159265358979323846);
    return UV{(phi + 5.0f * pi32 / 12.0f) / (2.0f * pi32), theta / pi32};
}

// ---------------------------------------------------------------------------------
// Go's math.Sin (Go 1.21 sin.go + trig_reduce.go, pure Go on amd64) op for op, for
// NoiseTexture.GetTexture (materials.go:285-287); oracle/oracle.c has the same.
// ---------------------------------------------------------------------------------
__constant__ uint64_t kGoMPi4[20] = {
    0x0000000000000001ull, 0x45f306dc9c882a53ull, 0xf84eafa3ea69bb81ull, 0xb6c52b3278872083ull,
    0xfca2c757bd778ac3ull, 0x6e48dc74849ba5c0ull, 0x0c925dd413a32439ull, 0xfc3bd63962534e7dull,
    0xd1046bea5d768909ull, 0xd338e04d68befc82ull, 0x7323ac7306a673e9ull, 0x3908bf177bf25076ull,
    0x3ff12fffbc0b301full, 0xde5e2316b414da3eull, 0xda6cfd9e4f96136eull, 0x9e8c7ecd3cbfd45aull,
    0xea4f758fd7cbe2f6ull, 0x7a0e73ef14a525d4ull, 0xd7f6bf623f1aba10ull, 0xac06608df8f6d757ull};

__device__ __noinline__ double go_sin(double x) {
    const double S0 = 1.58962301576546568060e-10, S1 = -2.50507477628578072866e-8, S2 = 2.75573136213857245213e-6,
                 S3 = -1.98412698295895385996e-4, S4 = 8.33333333332211858878e-3, S5 = -1.66666666666666307295e-1;
    const double C0 = -1.13585365213876817300e-11, C1 = 2.08757008419747316778e-9, C2 = -2.75573141792967388112e-7,
                 C3 = 2.48015872888517045348e-5, C4 = -1.38888888888730564116e-3, C5 = 4.16666666666665929218e-2;
    const double PI4A = 7.85398125648498535156e-1, PI4B = 3.77489470793079817668e-8,
                 PI4C = 2.69515142907905952645e-15;
    if (x == 0 || x != x) return x;
    if (__builtin_isinf(x)) return __builtin_nan("");
    bool sign = false;
    if (x < 0) {
        x = -x;
        sign = true;
    }
    uint64_t j;
    double y, z;
    if (x >= (double)(1 << 29)) {  // trigReduce (Payne-Hanek)
        const double PI4 = 3.14159265358979323846 / 4;
        uint64_t ix = (uint64_t)__double_as_longlong(x);
        const int exp = (int)((ix >> 52) & 0x7FF) - 1023 - 52;
        ix &= ~(0x7FFull << 52);
        ix |= 1ull << 52;
        const unsigned digit = (unsigned)(exp + 61) / 64, bs = (unsigned)(exp + 61) % 64;
        auto shr = [](uint64_t v, unsigned s) { return s >= 64 ? 0ull : v >> s; };
        const uint64_t z0 = (kGoMPi4[digit] << bs) | shr(kGoMPi4[digit + 1], 64 - bs);
        const uint64_t z1 = (kGoMPi4[digit + 1] << bs) | shr(kGoMPi4[digit + 2], 64 - bs);
        const uint64_t z2 = (kGoMPi4[digit + 2] << bs) | shr(kGoMPi4[digit + 3], 64 - bs);
        const uint64_t z2hi = __umul64hi(z2, ix), z1hi = __umul64hi(z1, ix), z1lo = z1 * ix;
        const uint64_t z0lo = z0 * ix;
        const uint64_t lo = z1lo + z2hi;
        uint64_t hi = z0lo + z1hi + (lo < z1lo ? 1ull : 0ull);
        j = hi >> 61;
        hi = hi << 3 | lo >> 61;
        const unsigned lz = (unsigned)__builtin_clzll(hi);
        const uint64_t e = (uint64_t)(1023 - (int)(lz + 1));
        hi = (hi << (lz + 1)) | shr(lo, 64 - (lz + 1));
        hi >>= 64 - 52;
        hi |= e << 52;
        z = __longlong_as_double((long long)hi);
        if (j & 1) {
            j++;
            j &= 7;
            z--;
        }
        z = z * PI4;
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
        y = 1.0 - 0.5 * zz + zz * zz * ((((((C0 * zz) + C1) * zz + C2) * zz + C3) * zz + C4) * zz + C5);
    else
        y = z + z * zz * ((((((S0 * zz) + S1) * zz + S2) * zz + S3) * zz + S4) * zz + S5);
    return sign ? -y : y;
}

// Perlin noise and turbulence (materials.go:218-249, math.go:58-92) over the
// RTX_NOISE_TEXELS table of a NoiseTexture; NoiseTexture.GetTexture (:280-288).
__device__ __forceinline__ float go_lerp(float t, float x, float y) { return x * (1 - t) + y * t; }
__device__ __forceinline__ float go_smoothstep(float t) { return t * t * (3 - 2 * t); }
__device__ __forceinline__ int go_cell(float v) {  // int(float32) & 255; out of range -> MinInt64 & 255 = 0
    if (!(v >= -9.2233720368547758e18f && v < 9.2233720368547758e18f)) return 0;
    return (int)((long long)v & 255);
}
__device__ __forceinline__ float perlin_corner(const uint32_t* __restrict__ tab, int ix, int iy, int iz, float x,
                                               float y, float z) {
    const uint32_t h = tab[768 + ix] ^ tab[1024 + iy] ^ tab[1280 + iz];
    return __uint_as_float(tab[3 * h]) * x + __uint_as_float(tab[3 * h + 1]) * y + __uint_as_float(tab[3 * h + 2]) * z;
}
__device__ __noinline__ float noise_texture(const uint32_t* __restrict__ tab, float scale, float px, float py,
                                             float pz) {
    px = px * scale;
    py = py * scale;
    pz = pz * scale;
    const float z0 = pz;
    float sum = 0, weight = 1.0f;
    for (int o = 0; o < 7; ++o) {  // Turb(point, 7)
        const float xi = (float)__builtin_floor((double)px), yi = (float)__builtin_floor((double)py),
                    zi = (float)__builtin_floor((double)pz);
        const float tx = px - xi, ty = py - yi, tz = pz - zi;
        const int rx0 = go_cell(xi), rx1 = (rx0 + 1) & 255;
        const int ry0 = go_cell(yi), ry1 = (ry0 + 1) & 255;
        const int rz0 = go_cell(zi), rz1 = (rz0 + 1) & 255;
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
        sum += weight * go_lerp(sz, e, f);
        weight *= 0.5f;
        px = px * 2;
        py = py * 2;
        pz = pz * 2;
    }
    const float turb = __builtin_fabsf(sum);
    return 0.5f * (1 + (float)go_sin((double)(z0 + 10 * turb)));
}

// ---------------------------------------------------------------------------------
// RNG contract (GPU-first): Philox4x32-10 keyed by the seed, one block
// of four 32-bit words per (global pixel, sample, event, attempt); u = float32(w >> 8)
// * 2^-24 in [0, 1) (the range of rand.Float32).  The reference's draw ORDER is kept:
//   event 0 = GetRay (camera.go:265-299): block (0,0) = dx, dy, disk x, disk y of the
//             first unit-disk attempt; disk attempt a >= 1 uses words 0,1 of block (0,a);
//   event s+1 = the scatter after segment s (ray.go:42):
//             Lambertian / Metal unit-sphere attempt a (vec3.go:182-190) = words 0,1,2
//             of block (s+1, a); Dielectric's uniform (materials.go:103) = word 0 of
//             block (s+1, 0), drawn only when refraction is possible.
// Every lane of a wave evaluates its block at the same program point, so Philox runs
// in lockstep instead of at a per-lane word boundary inside divergent loops.
// ---------------------------------------------------------------------------------
struct U4 {
    uint32_t x, y, z, w;
};
// The round keys are bumped per call on SALU (the asm barrier keeps the compiler from hoisting the
// 20 round keys of the seed into SGPRs for the whole kernel): SGPR spills 43 -> 22, Cornell box
// -2.3 %, headline neutral (RTX_PHILOX_OPAQUE=0 for A/B).
#ifndef RTX_PHILOX_OPAQUE
#define RTX_PHILOX_OPAQUE 1
#endif
__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                            uint32_t k1) {
    if (RTX_PHILOX_OPAQUE) asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // One 32x32->64 product per word pair: a single v_mad_u64_u32 (near full rate on
        // gfx950, scripts/micro/pk_rate.hip) instead of v_mul_lo_u32 + v_mul_hi_u32, and
        // each three-way xor one v_bitop3_b32 (truth table 0x96) instead of two v_xor.
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    return U4{c0, c1, c2, c3};
}
__device__ __forceinline__ float unit_f32(uint32_t w) { return (float)(w >> 8) * 0x1.0p-24f; }
// RandF32N(-1, 1), math.go:30-32: -1 + u * (1 - (-1)).
__device__ __forceinline__ float signed_unit(uint32_t w) { return -1.0f + unit_f32(w) * 2.0f; }

struct PathRng {
    uint32_t k0, k1, pixel, sample;
    __device__ __forceinline__ U4 block(uint32_t event, uint32_t attempt) const {
        return philox4x32_10(pixel, sample, event, attempt, k0, k1);
    }
};

// NewVec3UnitRandOnUnitSphere32 (vec3.go:182-190) for event e, given its block 0.
__device__ __forceinline__ V3 rand_unit_on_sphere(const PathRng& rng, uint32_t e, U4 b, uint32_t& draws) {
    for (uint32_t a = 1;; ++a) {
        const float x = signed_unit(b.x), y = signed_unit(b.y), z = signed_unit(b.z);
        draws += 3;
        const V3 v = v3(x, y, z);
        if (lensq(v) < 1.0f) return unit(v);
        b = rng.block(e, a);
    }
}

// The scatter sample of one shading phase, drawn by the whole wave (coop_scatter).
struct Scatter {
    V3 s;            // unit vector on the sphere (Lambertian / Metal lanes)
    uint32_t u0;     // word 0 of block (e, 0): Dielectric's uniform
    uint32_t draws;  // rand draws NewVec3UnitRandOnUnitSphere32 made (3 per attempt)
};

__device__ __forceinline__ uint32_t lane_pull(uint32_t src_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane * 4u), (int)v);
}

// The scene's entries (rtx_layout.h) as two arrays of half-entries: a[i] and b[i].  An
// entry split this way spreads a wave's random reads over all 16 four-bank slots of
// the LDS (a 32-B-strided array of whole entries reaches only 8 with each 16-B read).
struct SceneRef {
    const float4* __restrict__ a;
    const float4* __restrict__ b;
    const float4* __restrict__ q;          // quad table, 4 float4 per quad (rtx_layout.h)
    const rtx_material* __restrict__ m;    // device materials (RTX_DEV_TEX_INLINE recoding)
    const rtx_texture* __restrict__ tx;    // device textures (only those materials reference; after m in LDS)
    // v3 on a scene too big for LDS: its first `hot` bytes of positions (the top levels,
    // stored first) are also in LDS, halves at la / lb (load_entry<HYB>)
    const float4* la;
    const float4* lb;
    uint32_t hot;
    uint32_t prim_end;  // the fixed layout: primitives stored below this position (Params::prim_end)
};
__device__ __forceinline__ SceneRef scene_ref(const float4* base, uint32_t n_entries, const rtx_material* mats) {
    const uint32_t m = n_entries + 1;  // + the sentinel
    return SceneRef{base, base + m, base + 2 * m, mats, nullptr, nullptr, nullptr, 0u, 0u};
}
// v3's LDS layout: the 'a' halves from LDS byte 0, the 'b' halves from byte LDS_B, the
// quad table after them.  A walk position is then the LDS address of its 'a' half and
// both halves load from one register (ds_read_b128 offset:0 / offset:LDS_B): no address
// arithmetic per step.  The material table, then the texture table (48 B per texture that a
// material reads: checkered, image, noise), go into the gap after the 'a' halves when they fit
// there (randSpheres: 15.5 KB of halves + 15.6 KB of materials + one checkered texture < 32 KB),
// else after the quad table.  (The texture record in LDS: a texture lookup used to be a chain of
// global loads, each waiting for the wave's outstanding sample-scratch stores.)
constexpr uint32_t LDS_B = 32768;
__host__ __device__ __forceinline__ uint32_t lds_mat_offset(uint32_t n_entries, uint32_t n_quads, uint32_t n_mats,
                                                            uint32_t n_tex) {
    const uint32_t halves = (n_entries + 1) * 16;
    return halves + n_mats * 32 + n_tex * 48 <= LDS_B ? halves : LDS_B + halves + n_quads * 64;
}
__host__ __device__ __forceinline__ uint32_t lds_fixed_bytes(uint32_t n_entries, uint32_t n_quads, uint32_t n_mats,
                                                             uint32_t n_tex) {
    const uint32_t end = LDS_B + (n_entries + 1) * 16 + n_quads * 64,
                   mo = lds_mat_offset(n_entries, n_quads, n_mats, n_tex);
    return mo < LDS_B ? end : mo + n_mats * 32 + n_tex * 48;
}
__device__ __forceinline__ SceneRef scene_ref_fixed(const float4* lds, uint32_t n_entries, uint32_t n_quads,
                                                    uint32_t n_mats, uint32_t n_tex) {
    const uint32_t mo = lds_mat_offset(n_entries, n_quads, n_mats, n_tex) / 16;
    return SceneRef{lds, lds + LDS_B / 16, lds + LDS_B / 16 + n_entries + 1,
                    reinterpret_cast<const rtx_material*>(lds + mo),
                    reinterpret_cast<const rtx_texture*>(lds + mo + 2 * n_mats), nullptr, nullptr, 0u, 0u};
}
// The LDS cache of a scene too big for the fixed layout: its first entries (the ones the walk
// reads most, rtx_capi.hip ensure_device), 'a' halves from LDS byte 0 and 'b' halves from
// HOT_B (reached by the ds_read offset field, as in the fixed layout).  Up to HOT_ENTRIES_8W
// three 8-wave workgroups share a CU; up to HOT_ENTRIES_MAX (80 KB: half of the CU's 160 KB)
// two 12-wave ones do — 6 waves per SIMD either way.  (2560 entries against 2048)
#ifndef RTX_HOT_B
#define RTX_HOT_B 40960
#endif
#ifndef RTX_HOT_MAX
#define RTX_HOT_MAX 2560
#endif
constexpr uint32_t HOT_B = RTX_HOT_B;
constexpr uint32_t HOT_ENTRIES_MAX = RTX_HOT_MAX;
constexpr uint32_t HOT_ENTRIES_8W = (160u * 1024u / 3u - HOT_B) / 16u / 64u * 64u;
static_assert(HOT_ENTRIES_MAX * 16 <= HOT_B && 2 * (HOT_B + HOT_ENTRIES_MAX * 16) <= 160u * 1024u,
              "two 12-wave workgroups' caches per CU");
__host__ __device__ __forceinline__ uint32_t lds_hot_bytes(uint32_t n_hot) { return HOT_B + n_hot * 16; }
// float4s of a scene's device table: both halves with their sentinels, then the quads.
__host__ __device__ __forceinline__ uint32_t scene_float4s(uint32_t n_entries, uint32_t n_quads) {
    return 2 * (n_entries + 1) + 4 * n_quads;
}
// Device material recoding (rtx_capi.hip ensure_device): a Lambertian / DiffuseLight
// whose texture is a SolidColor holds the colour in `albedo` and this texture index.
constexpr uint32_t RTX_DEV_TEX_INLINE = 0xFFFFFFFFu;

// ---------------------------------------------------------------------------------
// Kernel parameters
// ---------------------------------------------------------------------------------
constexpr uint32_t COUNTER_SLOTS = 26;  // device stats slots (rtx_capi.hip collect_on)

struct Params {
    const float4* entries;   // n_entries + 1 'a' halves, as many 'b', 4 * n_quads (SceneRef)
    uint32_t n_entries;
    uint32_t n_quads;
    uint32_t n_materials;
    const rtx_material* materials;
    const rtx_texture* textures;   // only the textures materials reference (ensure_device compacts them)
    uint32_t n_textures;
    const uint32_t* texels;
    rtx_camera cam;
    uint64_t seed;
    uint32_t x0, y0, width, rows, rank, world;
    uint32_t tile_w_log2;  // a tile of 64 pixels is (1 << tile_w_log2) wide (8 or 16) and 64 >> tile_w_log2 rows tall
    float* out;
    unsigned long long* counters;  // rtx_stats order when counting (COUNTER_SLOTS x u64)
    uint32_t shade_thresh;         // shade once this many lanes of a wave wait (1..64)
    uint32_t* tile_counter;        // global unit queue head (zeroed before each chunk's launch)
    uint32_t* error_flag;          // the device's sticky error word: KERR_* counters, never zeroed by a render
    uint64_t watchdog_ticks;       // per-wave limit in s_memrealtime ticks (100 MHz)
    uint32_t has_uv;               // scene has an image texture (UV needed at hits)
    uint32_t has_noise;            // scene has a Perlin NoiseTexture (v3 NOISE kernels)
    // v3 (render_items): samples [k0, k0 + kn) of every pixel, one colour per sample
    // into scratch[(k - k0) * width * rows + pixel] (3 floats), `sub` samples per unit.
    float* scratch;
    uint32_t k0, kn, sub;
    uint32_t item_waves;  // v3 waves per workgroup: 8 (one LDS scene copy each), or 4 for A/B
    uint32_t n_hot;       // entries stored first and cached in LDS by v3 when the scene does not fit
    uint32_t debug_launch;  // RTX_DEBUG_LAUNCH=1: v3 prints its launch shape to stderr
    uint32_t grid_pct;    // v3: percent of the resident grid launched (A/B knob; 100 = all resident waves)
    uint32_t prim_batch;  // v3: primitive tests wait for this many lanes (trav_step_batched); 0 = off
    uint32_t start;       // walk position of the walk's first entry (the root)
    uint32_t prim_end;    // scene in the LDS copy: its primitives are stored below this position
    // The tiered walk: the near pass walks the near tree and hands every path whose
    // next segment starts outside the near region [near_min, near_max] to the far pass, which walks
    // the guarded tree.  A path is handed over once, as a 64-B record at its segment start.
    uint32_t tier;          // 0: one walk; 1: the near pass; 2: the far pass (resumes the records)
    float near_min[3], near_max[3];
    float4* defer;          // the records: 4 float4 each (origin | pixel, dir | sample, thr | seg, acc | slot)
    uint32_t defer_cap;     // records the queue holds
    uint32_t* defer_count;  // records written (the far pass reads min(count, cap))
    // The samples whose records did not fit, by id = (k - k0) * n_tiles * 64 + pixel slot: rendered again
    // from their camera rays by the redo pass.  The near pass lists up to redo_cap ids in redo_ids (the
    // count, all of them, in *redo_count) and sets the bits of the others in redo_bits, one per scratch
    // slot of the chunk (zeroed per chunk); past redo_cap the list joins the bits (spill_redo_list) and
    // the redo pass scans them.
    uint32_t* redo_ids;
    uint32_t redo_cap;
    uint32_t* redo_count;
    uint32_t* redo_bits;
    // Tests of the wave-level claim guard (rtx_kernel.hip partial_wave): in the debug library
    // (librtx_dbgclaim.so, -DRTX_DEBUG_PARTIAL=1) claim site 1 (defer queue), 2 (redo list) or 3 (unit
    // queue) is entered by the even lanes only (RTX_DEBUG_PARTIAL_SITE); ignored by every other build.
    uint32_t debug_partial;
    uint32_t cam_pool;  // 1: the near pass takes camera rays from the wave's LDS pool when it fits (RTX_CAM_POOL=0: off)
    uint32_t refill_hits;  // POOL: a miss phase when fewer waiting lanes than this hit (RTX_REFILL_HITS; 0: never)
    // (last: the fields before it keep their kernel-argument offsets) a striped shard (rtx_region.stripe = 2^s > 1):
    // shard row lr is image row y0 + (((lr >> s) * world + rank) << s) + (lr & (2^s - 1)); render_items<ST>
    uint32_t stripe_log2;
    // The near pass's drain (render_drain): each workgroup of the near pass writes its records to a
    // region of its own, drain_region slots from blockIdx.x * drain_region, counted in drain_count[blockIdx.x], and
    // once its waves have no near work left it resumes them itself (its far phase), claiming units of 64 records
    // from drain_count[gridDim.x + blockIdx.x].  The far pass's launch is gone: a workgroup whose near work ends
    // early walks its far records while the others still render, and the long paths of the far tree start then.
    uint32_t* drain_count;   // 2 x the near grid, zeroed per chunk
    uint32_t drain_region;   // records per workgroup (the queue's capacity over the near grid)
    // render_drain (RTX_DRAIN_LDS): the workgroup's record count and far unit cursor are two LDS words at this float4
    // index of the dynamic LDS, past both phases' layouts, instead of drain_count's (a global atomic with return,
    // which the wave waits on, in every phase that defers)
    uint32_t drain_lds;
    uint32_t drain;          // 1: the timed tiered render drains (RTX_DRAIN=0: the far pass's own launch, A/B)
    // The layout is the paired walk's records (rtx_capi.hip build_w2): a layout in HBM with an LDS
    // cache, walked by trav_step_w2 (only the cache kernels, HYB, ever get one; never a drain launch).
    uint32_t w2;
};
constexpr uint32_t DRAIN_WORDS = 16384;  // Params::drain_count's words: near grids up to 8192 workgroups

// The camera-ray pool of render_items<POOL>: after the fixed layout's scene copy (16-B aligned), 64 rays
// of 2 float4 per wave (2 KB).
constexpr uint32_t POOL_BYTES_PER_WAVE = 64 * 32;
#ifndef RTX_POOL_WAVES  // waves per workgroup of the pooled kernels (two workgroups per CU) and their waves per SIMD
#define RTX_POOL_WAVES 12
#define RTX_POOL_MINW 6
#endif
__host__ __device__ __forceinline__ uint32_t pool_f4_offset(const Params& p) {
    return (lds_fixed_bytes(p.n_entries, p.n_quads, p.n_materials, p.n_textures) + 15u) / 16u;
}
// Whether a render of a scene in the LDS copy takes the camera-ray pool: wanted (Params::cam_pool) and two
// 12-wave workgroups' scene copies and pools fit a CU's 160 KB.
__host__ __device__ __forceinline__ bool pool_fits(const Params& p) {
    return p.cam_pool && (size_t)pool_f4_offset(p) * 16 + RTX_POOL_WAVES * POOL_BYTES_PER_WAVE <= 80u * 1024u;
}

// The words of Params::error_flag, the device's sticky error word (rtx_capi.hip KernErr): counters
// the kernel only adds to and no render zeroes, so a failed render stays visible behind any renders enqueued after
// it, until collect_on or rtx_device_check reads them (and turns a change into RTX_ERR_HIP).
constexpr uint32_t KERR_WATCHDOG = 0u;      // waves that outlived RTX_WATCHDOG_S
constexpr uint32_t KERR_PARTIAL_WAVE = 1u;  // lanes of waves that reached a wave-level claim without the whole wave
constexpr uint32_t KERR_WORDS = 2u;

struct Ray {
    V3 o, d;
};

// The tiles of a region's rows (64 pixels each, tile_w_log2 wide): the work units' pixels and the
// sample scratch's blocks.  Square 8 x 8 tiles for one or two shards; a shard of N row-interleaved
// ones has its consecutive rows N image rows apart, so wider tiles keep a tile's rays coherent:
// 16 x 4 for N = 4 (16 x 16 image pixels instead of 8 x 32), 32 x 2 from N = 8 on (32 x 16 instead of
// 8 x 64).  Rank 0's rows alone (profiles/r04_tile_ab.jsonl): N = 4 25.66 / 25.66 ms (16 / 32 wide)
// against 25.94 (8); N = 8 13.45 / 13.39 against 13.74.
__host__ __device__ __forceinline__ uint32_t tile_w_log2_for(uint32_t world, uint32_t stripe = 1) {
    if (stripe >= 8) return 3u;  // 8-row stripes: an 8 x 8 tile is 8 x 8 image pixels again
    if (stripe > 1) return stripe == 4 ? 4u : 5u;  // a tile's rows within one stripe (render_items' u_y)
    return world >= 8 ? 5u : (world >= 4 ? 4u : 3u);
}
// The narrowest tile (log2 of its width) whose rows lie within one stripe of 2^s rows (s = 0: single rows, any).
__host__ __device__ __forceinline__ uint32_t tile_w_log2_min(uint32_t s) { return s == 0 ? 3u : (s >= 3 ? 3u : 6u - s); }
// The image row (relative to y0) of shard row lr (rtx.h rtx_region_row, stripes of 2^s rows).
__host__ __device__ __forceinline__ uint32_t region_row(uint32_t lr, uint32_t rank, uint32_t world, uint32_t s) {
    return (((lr >> s) * world + rank) << s) + (lr & ((1u << s) - 1u));
}
__host__ __device__ __forceinline__ uint32_t tiles_x_of(uint32_t width, uint32_t twl) { return (width + (1u << twl) - 1u) >> twl; }
__host__ __device__ __forceinline__ uint32_t tiles_y_of(uint32_t rows, uint32_t twl) {
    const uint32_t th = 64u >> twl;
    return (rows + th - 1u) / th;
}

struct Counters {
    uint32_t segments, node_visits, prim_tests, hits, texel_fetches, draws;
    uint32_t cache_hits;  // entries read from the LDS cache of a big scene (load_entry<HYB>)
};

// GetRay + sampleUnitSquare, camera.go:265-299, event 0.  base = (pixel00 + du*i) + dv*j.
// SKIP_DISK: without defocus the unit-disk sample is drawn but never used (camera.go:279-281)
// and no later draw depends on it (every event has its own Philox blocks), so a kernel that
// does not count draws may leave its rejection loop out (Cornell box -1.7 %).
// b = block (0, 0) of the sample, drawn by the caller (the shading phase draws it together with
// the other lanes' scatter blocks: one Philox evaluation for both).
template <bool SKIP_DISK = false>
__device__ __forceinline__ Ray camera_ray(const rtx_camera& c, V3 base, const PathRng& rng, U4 b, uint32_t& draws) {
    const V3 du = v3(c.pixel_du[0], c.pixel_du[1], c.pixel_du[2]);
    const V3 dv = v3(c.pixel_dv[0], c.pixel_dv[1], c.pixel_dv[2]);
    const float dx = -0.5f + unit_f32(b.x);                       // :290
    const float dy = -0.5f + unit_f32(b.y);                       // :291
    const V3 pc = add(base, add(scale(du, dx), scale(dv, dy)));   // :275
    float x = signed_unit(b.z), y = signed_unit(b.w);             // :277 disk, always drawn
    draws += 4;
    for (uint32_t a = 1; !(SKIP_DISK && !(c.defocus_angle > 0.0f)) && !(x * x + y * y < 1.0f); ++a) {  // vec3.go:203-210
        b = rng.block(0, a);
        x = signed_unit(b.x);
        y = signed_unit(b.y);
        draws += 2;
    }
    const V3 center = v3(c.center[0], c.center[1], c.center[2]);
    V3 origin = center;
    if (c.defocus_angle > 0.0f) {                                 // :279-281
        const V3 ddu = v3(c.defocus_disk_u[0], c.defocus_disk_u[1], c.defocus_disk_u[2]);
        const V3 ddv = v3(c.defocus_disk_v[0], c.defocus_disk_v[1], c.defocus_disk_v[2]);
        origin = add(center, add(scale(ddu, x), scale(ddv, y)));
    }
    return Ray{origin, sub(pc, origin)};                          // :283-286
}

__device__ __forceinline__ V3 pixel_base(const rtx_camera& c, uint32_t x, uint32_t y) {  // camera.go:266-274
    return add(add(v3(c.pixel00[0], c.pixel00[1], c.pixel00[2]),
                   scale(v3(c.pixel_du[0], c.pixel_du[1], c.pixel_du[2]), (float)x)),
               scale(v3(c.pixel_dv[0], c.pixel_dv[1], c.pixel_dv[2]), (float)y));
}

// Texture.GetTexture, materials.go:127-193, 267-288.  NOISE: the scene has a Perlin
// texture (its evaluation is an out-of-line call that costs the caller registers, so
// only kernels built for such scenes contain it).
template <bool COUNT, bool NOISE = false>
__device__ __forceinline__ V3 texture_value(const Params& p, const SceneRef E, uint32_t ti, float u, float v, V3 pt,
                                            Counters& cnt) {
    const rtx_texture& t = E.tx[ti];
    if (t.type == RTX_TEX_SOLID) return v3(t.even[0], t.even[1], t.even[2]);
    if (t.type == RTX_TEX_CHECKERED) {
        const float inv = t.pad;  // float32(1 / scale), materials.go:128 (computed on the host, upload_copy)
        const float fx = __builtin_floorf(inv * pt.x), fy = __builtin_floorf(inv * pt.y), fz = __builtin_floorf(inv * pt.z);
        bool odd;
        // int(math.Floor(...)) is an int64; only the parity of x + y + z matters, so when every lane's
        // floors are below 2^31 in magnitude 32-bit conversions (wrapping sums keep the parity) do it
        if (__builtin_amdgcn_ballot_w64(!(__builtin_fabsf(fx) < 0x1p31f && __builtin_fabsf(fy) < 0x1p31f &&
                                          __builtin_fabsf(fz) < 0x1p31f)) == 0) {
            odd = (((uint32_t)(int32_t)fx + (uint32_t)(int32_t)fy + (uint32_t)(int32_t)fz) & 1u) != 0;
        } else {
            odd = (((int64_t)fx + (int64_t)fy + (int64_t)fz) & 1) != 0;
        }
        return !odd ? v3(t.even[0], t.even[1], t.even[2]) : v3(t.odd[0], t.odd[1], t.odd[2]);
    }
    if (NOISE && t.type == RTX_TEX_NOISE) {
        const float g = noise_texture(p.texels + t.texel_offset, t.scale, pt.x, pt.y, pt.z);
        return v3(g, g, g);
    }
    // RTX_TEX_IMAGE: Dy() <= 0 -> the debug colour; else At(int(u*Dx), int(v*Dy)).RGBA()
    if ((int32_t)t.height <= 0) return v3(0.0f, 1.0f, 1.0f);
    const float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);  // Clamp passes NaN through
    const float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    const float vv = 1.0f - vc;
    const float fi = uu * (float)t.width;
    const float fj = vv * (float)t.height;
    if (COUNT) ++cnt.texel_fetches;
    // int(i), int(j) truncate; i == Dx (u == 1), j == Dy (v == 0) and NaN (int(NaN) =
    // MinInt64) lie outside the bounds: the border texel after the raster (rtx.h)
    uint64_t idx = (uint64_t)t.width * t.height;
    if (fi >= 0.0f && fj >= 0.0f) {
        const uint64_t i = (uint64_t)fi, j = (uint64_t)fj;
        if (i < t.width && j < t.height) idx = j * t.width + i;
    }
    const uint2 px = *reinterpret_cast<const uint2*>(p.texels + t.texel_offset + 2 * idx);  // RGBA16
    const float cs = 1.0f / 65535.0f;  // colScale = float32(1.0 / 65535.0)
    return v3((float)(px.x & 0xFFFFu) * cs, (float)(px.x >> 16) * cs, (float)(px.y & 0xFFFFu) * cs);
}

// Material index of the primitive at entry `hit`.
template <bool QUADS>
__device__ __forceinline__ uint32_t hit_material(const SceneRef E, uint32_t hit) {
    const float4 b = E.b[hit];
    if (QUADS && __float_as_int(b.w) == RTX_E_QUAD) return (uint32_t)__float_as_int(E.q[4u * __float_as_int(b.x)].w);
    return RTX_DEV_SPHERE_MATERIAL(__float_as_int(b.w));
}

// Wave-cooperative rejection sampling for NewVec3UnitRandOnUnitSphere32 (vec3.go:182-190).
// Must be called by the whole wave (converged).  A lane with hit >= 0 draws block (e, 0);
// its words 0-2 are attempt 0 of the unit-sphere loop.  The loop's result is the FIRST
// accepted attempt a, attempt a being words 0-2 of block (e, a) — a pure function of the
// counter, so any lane can evaluate any lane's attempt.  Instead of every lane looping
// until the unluckiest one accepts (acceptance pi/6 per attempt: ~6-7 rounds for 40
// lanes), the n lanes still rejecting get 64/n consecutive lanes each, which evaluate
// attempts base .. base+64/n-1 of that owner in one round; the owner takes the first
// accepted one.  Same attempt, same bits, about 3 Philox rounds per phase.
// b0 = block (e, 0) of a lane with hit >= 0, drawn by the caller.
template <bool QUADS>
__device__ __forceinline__ Scatter coop_scatter(const Params& p, const SceneRef E, const PathRng& rng,
                                                uint32_t e, int32_t hit, const U4 b0) {
    Scatter out{v3(0.0f, 0.0f, 0.0f), 0u, 0u};
    bool need = false;
    float x = 0.0f, y = 0.0f, z = 0.0f;
    uint32_t ty = 0xFFFFFFFFu;  // (no hit: no material)
    if (hit >= 0) {
        const uint32_t mi = hit_material<QUADS>(E, (uint32_t)hit);
        ty = E.m[mi].type;
        out.u0 = b0.x;
        x = signed_unit(b0.x);
        y = signed_unit(b0.y);
        z = signed_unit(b0.z);
    }
    static_assert(RTX_MAT_LAMBERTIAN == 0 && RTX_MAT_METAL == 1, "need: one unsigned compare");
    need = ty < 2u;  // Lambertian or Metal (a single compare: its ballot needs no lane-mask materialisation)
    uint32_t att = 0;
    uint64_t pend = ballot(need) & ~ballot(x * x + y * y + z * z < 1.0f);  // lensq(v) < 1
    const uint32_t lane = __lane_id();
    const uint64_t below_mask = (1ull << lane) - 1ull;
    for (uint32_t base = 1; pend != 0;) {
        const uint32_t np = (uint32_t)__popcll(pend);
        // K = 64 / np attempts per owner this round, and q = lane / K below, by float reciprocals:
        // 64.5 / np and (lane + 0.5) / K lie at least 1/128 from the next integer, far beyond
        // v_rcp_f32's 1-ulp error, so truncation gives the integer quotients (the compiler's
        // integer divisions took ~25 VALU per round).
        const uint32_t K = __builtin_amdgcn_readfirstlane((uint32_t)(64.5f * __builtin_amdgcn_rcpf((float)np)));
        const bool mine = (pend >> lane) & 1ull;
        const uint32_t below = (uint32_t)__popcll(pend & below_mask);
        // Lane q (< np) learns the lane id of the q-th pending lane (a permutation push).
        const uint32_t dst = mine ? below : np + (lane - below);
        const uint32_t owner_of = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4u), (int)lane);
        const uint32_t q = (uint32_t)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)K)), k = lane - q * K;
        const bool slot = q < np;
        const uint32_t owner = lane_pull(slot ? q : 0u, owner_of);
        const uint32_t opix = lane_pull(owner, rng.pixel), osmp = lane_pull(owner, rng.sample);
        const uint32_t oe = lane_pull(owner, e);
        const U4 b = philox4x32_10(opix, osmp, oe, base + k, rng.k0, rng.k1);
        const float bx = signed_unit(b.x), by = signed_unit(b.y), bz = signed_unit(b.z);
        const uint64_t good = ballot(slot) & ballot(bx * bx + by * by + bz * bz < 1.0f);
        const uint64_t kmask = K >= 64u ? ~0ull : ((1ull << K) - 1ull);
        const uint64_t mine_good = mine ? ((good >> (below * K)) & kmask) : 0ull;
        const uint32_t kk = mine_good ? (uint32_t)__builtin_ctzll(mine_good) : 0u;
        const uint32_t src = mine_good ? below * K + kk : lane;
        const float fx = __int_as_float((int)lane_pull(src, __float_as_uint(bx)));
        const float fy = __int_as_float((int)lane_pull(src, __float_as_uint(by)));
        const float fz = __int_as_float((int)lane_pull(src, __float_as_uint(bz)));
        if (mine_good) {
            x = fx;
            y = fy;
            z = fz;
            att = base + kk;
        }
        pend &= ~ballot(mine_good != 0ull);  // (ballot(mine) is pend)
        base += K;
    }
    if (need) {
        out.s = unit(v3(x, y, z));
        out.draws = 3u * (att + 1u);
    }
    return out;
}

// One step of the closest-hit walk over the threaded pre-order layout (rtx_layout.h):
// entry i is a node (Aabb.Hit, bvh.go:52-61, 84-102) or a sphere (Sphere.Hit,
// hittables.go:96-116).  The sequence of steps is the reference recursion's, with
// running bound `closest` = the closest hit so far (bvh.go:227-232).
struct Trav {
    uint32_t i;  // walk position: the byte offset of the current entry's half, 16 * index
    int32_t hit;
    float closest, ix, iy, iz, a;
    float ra;   // RN(1 / a): the sphere test's divisions as div_by (SAFE rays)
    bool nx, ny, nz;
    bool safe;  // 1/dir and the origin finite, a in [2^-60, 2^60]: the SAFE step forms are exact
};

// The near walk's FMA slab form (box_step FMA) needs products that cannot overflow:
// |1/d| <= 2^64 per axis and an origin within 2^32 (the near tree's boxes lie within 2^32, topology).
// Rays outside these bounds take the reference's form, ray by ray (oracle.c restates the rule).
__device__ __forceinline__ bool near_fma_ok(const Ray& r, const Trav& t) {
    return __builtin_fabsf(t.ix) <= 0x1p64f && __builtin_fabsf(t.iy) <= 0x1p64f && __builtin_fabsf(t.iz) <= 0x1p64f &&
           __builtin_fabsf(r.o.x) <= 0x1p32f && __builtin_fabsf(r.o.y) <= 0x1p32f && __builtin_fabsf(r.o.z) <= 0x1p32f;
}

// FMA (the near pass): a ray is `safe` for the walk's fast forms only when the FMA form applies too.
template <bool FMA = false>
__device__ __forceinline__ void trav_begin(Trav& t, const Ray& r, uint32_t start) {
    // InBoundary computes 1/dir per node; hoisting it is bit-identical.
    if (__builtin_amdgcn_ballot_w64(!(rcp_fast_ok(r.d.x) && rcp_fast_ok(r.d.y) && rcp_fast_ok(r.d.z))) == 0) {
        t.ix = rcp_newton(r.d.x);
        t.iy = rcp_newton(r.d.y);
        t.iz = rcp_newton(r.d.z);
    } else {
        t.ix = 1.0f / r.d.x;
        t.iy = 1.0f / r.d.y;
        t.iz = 1.0f / r.d.z;
    }
    t.nx = t.ix < 0.0f;
    t.ny = t.iy < 0.0f;
    t.nz = t.iz < 0.0f;
    t.a = lensq(r.d);  // hittables.go:98, loop-invariant
    t.ra = rcp_ieee(t.a);
    t.safe = __builtin_isfinite(t.ix) && __builtin_isfinite(t.iy) && __builtin_isfinite(t.iz) &&
             __builtin_isfinite(r.o.x) && __builtin_isfinite(r.o.y) && __builtin_isfinite(r.o.z) &&
             t.a >= 0x1p-60f && t.a <= 0x1p60f;
    if (FMA) t.safe = t.safe && near_fma_ok(r, t);
    t.closest = __builtin_inff();
    t.hit = -1;
    t.i = start;
}

// Entry index of a walk position (a byte offset, 16 per entry: Trav::i).
__device__ __forceinline__ int32_t entry_of(uint32_t pos) { return (int32_t)(pos >> 4); }

// The entry at walk position `pos`: its two halves in one LDS / memory round trip.
template <bool FIXED, bool HYB = false>
__device__ __forceinline__ void load_entry(const SceneRef E, uint32_t pos, float4& ea, float4& eb) {
    if constexpr (HYB) {
        // The top levels from the LDS cache (v3's fixed layout at LDS address 0), the rest from
        // HBM: the global reads of the lanes past the cache and the LDS reads of the others are
        // both issued, under their exec masks, before one wait, so a wave with lanes on both sides
        // waits for the slower read only (two branches, each with its own wait, paid both in
        // turn).  The global reads take the table bases in SGPRs and the position as the offset.
        // (A flat load for both cost +4.6 % over a global one, config 4.)
        uint64_t sv, m;
        asm volatile("s_mov_b64 %[sv], exec\n\t"
                     "v_cmp_gt_u32_e64 %[m], %[hot], %[pos]\n\t" /* the LDS cache's lanes */
                     "s_andn2_b64 exec, %[sv], %[m]\n\t"
                     "s_cbranch_execz LG%=\n\t"
                     "global_load_dwordx4 %[ea], %[pos], %[ba]\n\t"
                     "global_load_dwordx4 %[eb], %[pos], %[bb]\n"
                     "LG%=:\n\t"
                     "s_and_b64 exec, %[sv], %[m]\n\t"
                     "s_cbranch_execz LL%=\n\t"
                     "ds_read_b128 %[ea], %[pos]\n\t"
                     "ds_read_b128 %[eb], %[pos] offset:%[lb]\n"
                     "LL%=:\n\t"
                     "s_mov_b64 exec, %[sv]\n\t"
                     "s_waitcnt vmcnt(0) lgkmcnt(0)"
                     : [ea] "=&v"(ea), [eb] "=&v"(eb), [sv] "=&s"(sv), [m] "=&s"(m)
                     : [pos] "v"(pos), [hot] "s"(E.hot), [ba] "s"(E.a), [bb] "s"(E.b), [lb] "i"(HOT_B)
                     : "scc");
    } else if constexpr (FIXED) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:%3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(ea), "=&v"(eb)
                     : "v"(pos), "i"(LDS_B));
    } else {
        ea = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(E.a) + pos);
        eb = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(E.b) + pos);
        // Both halves are consumed here, so the whole entry arrives in one round trip (two
        // 128-bit loads); otherwise the compiler sinks the node-only dwords into the box
        // branch behind a second, dependent read.
        asm volatile("" ::"v"(ea.x), "v"(ea.y), "v"(ea.z), "v"(ea.w), "v"(eb.x), "v"(eb.y), "v"(eb.z), "v"(eb.w));
    }
}

// (Quad).Hit, hittables.go:167-194, of the quad entry (ea, eb) at `pos` against (tmin, closest).
template <bool COUNT>
__device__ __forceinline__ void quad_test(Trav& t, const Ray& r, const SceneRef E, const float4 ea, const float4 eb,
                                          uint32_t pos, Counters& cnt) {
    const float tmin = 0.001f;  // ray.go:37
    if (COUNT) ++cnt.prim_tests;
    const float denom = r.d.x * ea.x + r.d.y * ea.y + r.d.z * ea.z;                 // :168
    if (!(__builtin_fabs((double)denom) < 1e-8)) {                                   // :170
        const float tt = (ea.w - (ea.x * r.o.x + ea.y * r.o.y + ea.z * r.o.z)) / denom;  // :174
        if (tmin < tt && tt < t.closest) {                                           // :176
            const uint32_t qi = 4u * (uint32_t)__float_as_int(eb.x);
            const float4 q0 = E.q[qi], q1 = E.q[qi + 1], q2 = E.q[qi + 2], q3 = E.q[qi + 3];
            const V3 php = sub(add(scale(r.d, tt), r.o), v3(q0.x, q0.y, q0.z));     // :180-181
            const V3 w = v3(q3.x, q3.y, q3.z);
            const float alpha = dot(w, cross(php, v3(q2.x, q2.y, q2.z)));           // :182
            const float beta = dot(w, cross(v3(q1.x, q1.y, q1.z), php));            // :183
            if (!(alpha < 0.0f || 1.0f < alpha || beta < 0.0f || 1.0f < beta)) {   // :185, :193
                t.closest = tt;
                t.hit = entry_of(pos);
            }
        }
    }
}

// n / a correctly rounded, given y = RN(1 / a) (Markstein: q0 = RN(n y) is within 1 ulp of n / a,
// the residual e = n - a q0 is exact by fma, and RN(q0 + e y) = RN(n / a) when y is the
// correctly rounded reciprocal), for a in [2^-60, 2^60] (Trav::safe): every quotient that can
// pass `tmin < t < closest` is then a normal number and so exactly the division's.  Quotients
// that overflow may come out NaN instead of inf, which fails the same tests.  3 VALU instead
// of the 11 of a division (scripts/micro/fastdiv_check.hip checks it against v_div_* on the GPU).
__device__ __forceinline__ float div_by(float n, float a, float y) {
    const float q0 = n * y;
    const float e = __builtin_fmaf(-a, q0, n);
    return __builtin_fmaf(e, y, q0);
}

// (*Sphere).Hit, hittables.go:96-116, of the sphere entry (ea, eb) at `pos` against (tmin, closest).
// SAFE: the two divisions by a as div_by.
// RANKED (the LDS layout, whose primitives are stored in the reference walk's order): a root equal
// to `closest` also wins when the sphere comes before the current hit in the reference's order —
// the tie bvh.go:220-249 resolves for the sphere it meets first (the right subtree is clipped to the
// left's hit, strictly).  A walk over another tree (rtx_topology.h) meets equal roots in another
// order; this rule gives every order the reference's answer.  (A no-op on the reference's own order.)
// RANK_WORD (a layout in HBM, whose storage order is the hot set's): the same rule on the rank word
// every sphere entry carries in b.y (ensure_layout: its place in the reference walk), the current
// hit's read from bt = the 'b' halves — only on an exact tie.
template <bool COUNT, bool SAFE = false, bool RANKED = false, bool RANK_WORD = false>
__device__ __forceinline__ void sphere_test(Trav& t, const Ray& r, const float4 ea, const float4 eb, uint32_t pos,
                                            Counters& cnt, const float4* __restrict__ bt = nullptr) {
    const float tmin = 0.001f;  // ray.go:37
    if (COUNT) ++cnt.prim_tests;
    const float ox = r.o.x - ea.x, oy = r.o.y - ea.y, oz = r.o.z - ea.z;  // :97
    const float hb = r.d.x * ox + r.d.y * oy + r.d.z * oz;                 // :99
    const float c = (ox * ox + oy * oy + oz * oz) - eb.x;                  // :100
    const float disc = hb * hb - t.a * c;                                  // :102
    if (disc >= 0.0f) {                                                    // :104 (NaN: miss either way)
        const float sq = __builtin_sqrtf(disc);                            // :108
        float tt = SAFE ? div_by(-hb - sq, t.a, t.ra) : (-hb - sq) / t.a;  // :110
        bool ok = tmin < tt && tt < t.closest;
        // The second root (:112) only when the first is not beyond tmin (or NaN): a
        // first root at or past closest makes the second, (-hb + sq) / a >= it, fail too.
        if (!(tmin < tt)) {
            tt = SAFE ? div_by(-hb + sq, t.a, t.ra) : (-hb + sq) / t.a;    // :112
            ok = tmin < tt && tt < t.closest;
        }
        if (RANKED && tt == t.closest && entry_of(pos) < t.hit) ok = true;  // (t.hit = -1: no hit yet)
        if (RANK_WORD && tt == t.closest && t.hit >= 0 && __float_as_uint(eb.y) < __float_as_uint(bt[t.hit].y))
            ok = true;
        if (ok) {
            t.closest = tt;
            t.hit = entry_of(pos);
        }
    }
}

// v_med3_f32 (no canonicalisation of the operands: they are products, tmin or the running bound).
__device__ __forceinline__ float med3(float a, float b, float c) {
    float d;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Aabb.Hit (bvh.go:52-61, 84-102) of the node entry (ea, eb) with next position `tag`:
// the walk moves to the next entry on a hit, else to the escape.
//
// MED3 (rays with t.safe): per axis ta = (min - o) * invD and tb = (max - o) * invD
// without the sign selects, and both bounds clamped into [min(ta, tb), max(ta, tb)] by one
// v_med3_f32 each: lo = clamp(lo, n, f), hi = clamp(hi, n, f).  While [lo, hi] and the axis
// slab overlap, the clamps leave lo = max(lo, n) and hi = min(hi, f) — the reference's swap and
// bound updates; once they are disjoint, lo and hi collapse onto the same slab end and stay
// ordered lo >= hi (clamping is monotone), so `lo < hi` after three axes is exactly the
// reference's per-axis early-exit result.  It needs NaN-free slab distances: finite 1/dir and
// origin (a zero direction component gives 1/dir = inf and 0 * inf = NaN when the origin lies
// on a slab plane, which the reference ignores (`t0 > min` is false for NaN) — those rays take
// the select path).  20 VALU per box instead of 24.
// The tiered walk's hit check: whether the sphere (centre, radius) = sa's own box,
// NewAabb(c - r, c + r) as NewSphere makes it (hittables.go:85-94), passes Aabb.Hit (bvh.go:52-61,
// 84-102) for the ray with interval [0.001, the float after t.closest] — the bound at which the
// guarded walk's test of the sphere's leaf box (a superset) would still accept this hit.
__device__ __forceinline__ void own_box_interval(const Trav& t, const Ray& r, const float4 sa, float& lo, float& hi) {
    const float rr = sa.w * -1.0f;
    const float ax = sa.x + rr, bx = sa.x + sa.w, ay = sa.y + rr, by = sa.y + sa.w, az = sa.z + rr, bz = sa.z + sa.w;
    const float mnx = __builtin_fminf(ax, bx), mxx = __builtin_fmaxf(ax, bx);
    const float mny = __builtin_fminf(ay, by), mxy = __builtin_fmaxf(ay, by);
    const float mnz = __builtin_fminf(az, bz), mxz = __builtin_fmaxf(az, bz);
    const float t0x = ((t.nx ? mxx : mnx) - r.o.x) * t.ix, t1x = ((t.nx ? mnx : mxx) - r.o.x) * t.ix;
    const float t0y = ((t.ny ? mxy : mny) - r.o.y) * t.iy, t1y = ((t.ny ? mny : mxy) - r.o.y) * t.iy;
    const float t0z = ((t.nz ? mxz : mnz) - r.o.z) * t.iz, t1z = ((t.nz ? mnz : mxz) - r.o.z) * t.iz;
    const float bound = __int_as_float(__float_as_int(t.closest) + 1);  // t.closest > 0, finite
    lo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(0.001f, t0x), t0y), t0z);
    hi = __builtin_fminf(__builtin_fminf(__builtin_fminf(bound, t1x), t1y), t1z);
}
__device__ __forceinline__ bool own_box_pass(const Trav& t, const Ray& r, const float4 sa) {
    float lo, hi;
    own_box_interval(t, r, sa, lo, hi);
    return lo < hi;
}

// Go's math.Min / math.Max on float32 operands (math.go:38-44, bvh.go:28-34): NaN wins, -0 below +0.
__device__ __forceinline__ float go_minf(float a, float b) {
    if (a != a || b != b) return __builtin_nanf("");
    if (a == 0.0f && b == 0.0f) return __builtin_signbit(a) ? a : b;
    return a < b ? a : b;
}
__device__ __forceinline__ float go_maxf(float a, float b) {
    if (a != a || b != b) return __builtin_nanf("");
    if (a == 0.0f && b == 0.0f) return __builtin_signbit(a) ? b : a;
    return a > b ? a : b;
}

// The tiered walk's hit check for a quad: whether NewQuad's own box — NewAabb(Q, Q + u + v)
// .GetPaddedAabb(), hittables.go:162, bvh.go:28-34, 63-84, formed in float32 as Go does from the quad record's
// (Q, material), (u, 0), (v, 0) — passes Aabb.Hit (bvh.go:52-61, 84-102) with [0.001, the float after t.closest].
// Every box the guarded walk tests above the quad contains it (NewAabbFromBoxes unions), so it reaches the quad with
// a bound past the hit, as for a sphere (own_box_pass).
__device__ __forceinline__ bool quad_own_box_pass(const Trav& t, const Ray& r, const float4 q0, const float4 q1,
                                                  const float4 q2) {
    const float eps = 0.0001f;
    auto axis = [&](float qk, float uk, float vk, float& lo, float& hi) {
        const float c = (qk + uk) + vk;
        lo = go_minf(qk, c);
        hi = go_maxf(qk, c);
        if (hi - lo < eps) {
            lo = lo - eps;
            hi = hi + eps;
        }
    };
    float mnx, mxx, mny, mxy, mnz, mxz;
    axis(q0.x, q1.x, q2.x, mnx, mxx);
    axis(q0.y, q1.y, q2.y, mny, mxy);
    axis(q0.z, q1.z, q2.z, mnz, mxz);
    // InBoundary per axis as the reference writes it: the NaN rules of `t0 > min` / `t1 < max` keep the bound
    float lo = 0.001f, hi = __int_as_float(__float_as_int(t.closest) + 1);  // t.closest > 0, finite
    auto slab = [&](float mn, float mx, float o, float inv, bool neg) {
        float t0 = (mn - o) * inv, t1 = (mx - o) * inv;
        if (neg) {
            const float x = t0;
            t0 = t1;
            t1 = x;
        }
        if (t0 > lo) lo = t0;
        if (t1 < hi) hi = t1;
    };
    slab(mnx, mxx, r.o.x, t.ix, t.nx);
    if (!(lo < hi)) return false;
    slab(mny, mxy, r.o.y, t.iy, t.ny);
    if (!(lo < hi)) return false;
    slab(mnz, mxz, r.o.z, t.iz, t.nz);
    return lo < hi;
}

// FMA (the near walk): the slab distances as fma(b, 1/d, no) with no = -(o * (1/d))
// per axis (the caller's, once per phase) — one rounding of b/d - o/d instead of two of (b - o) * (1/d).
// The near tree's boxes carry the slack for either form (sphere_margin), and its walk is exact by the hit
// check whatever boxes pass (§14-15), so only the work counts change — as the oracle's near walk restates.
// Rays outside near_fma_ok take the reference's form (per lane in the select form; the MED3 form runs
// only when every walking lane's ray is safe, which for the near pass includes near_fma_ok).
template <bool MED3 = false, bool FMA = false>
__device__ __forceinline__ bool box_hit(const Trav& t, const Ray& r, const float4 ea, const float4 eb,
                                        const V3 no = V3{0.0f, 0.0f, 0.0f}) {
    const float tmin = 0.001f;  // ray.go:37
    if constexpr (MED3) {
        float tax, tbx, tay, tby, taz, tbz;
        if constexpr (FMA) {
            tax = __builtin_fmaf(ea.x, t.ix, no.x), tbx = __builtin_fmaf(eb.x, t.ix, no.x);
            tay = __builtin_fmaf(ea.y, t.iy, no.y), tby = __builtin_fmaf(eb.y, t.iy, no.y);
            taz = __builtin_fmaf(ea.z, t.iz, no.z), tbz = __builtin_fmaf(eb.z, t.iz, no.z);
        } else {
            tax = (ea.x - r.o.x) * t.ix, tbx = (eb.x - r.o.x) * t.ix;
            tay = (ea.y - r.o.y) * t.iy, tby = (eb.y - r.o.y) * t.iy;
            taz = (ea.z - r.o.z) * t.iz, tbz = (eb.z - r.o.z) * t.iz;
        }
        const float lo = med3(med3(med3(tmin, tax, tbx), tay, tby), taz, tbz);
        const float hi = med3(med3(med3(t.closest, tax, tbx), tay, tby), taz, tbz);
        return lo < hi;
    }
    // Per axis: t0 = (min - o) * invD, t1 = (max - o) * invD, swapped if invD < 0.
    // (Scalar FP32 throughout: a v_pk_mul_f32 / v_pk_add_f32 issues at a quarter of
    // v_mul_f32's rate on gfx950, scripts/micro/pk_rate.hip, so packing loses 2x.)
    float t0x = ((t.nx ? eb.x : ea.x) - r.o.x) * t.ix;
    float t1x = ((t.nx ? ea.x : eb.x) - r.o.x) * t.ix;
    float t0y = ((t.ny ? eb.y : ea.y) - r.o.y) * t.iy;
    float t1y = ((t.ny ? ea.y : eb.y) - r.o.y) * t.iy;
    float t0z = ((t.nz ? eb.z : ea.z) - r.o.z) * t.iz;
    float t1z = ((t.nz ? ea.z : eb.z) - r.o.z) * t.iz;
    if (FMA && near_fma_ok(r, t)) {
        t0x = __builtin_fmaf(t.nx ? eb.x : ea.x, t.ix, no.x);
        t1x = __builtin_fmaf(t.nx ? ea.x : eb.x, t.ix, no.x);
        t0y = __builtin_fmaf(t.ny ? eb.y : ea.y, t.iy, no.y);
        t1y = __builtin_fmaf(t.ny ? ea.y : eb.y, t.iy, no.y);
        t0z = __builtin_fmaf(t.nz ? eb.z : ea.z, t.iz, no.z);
        t1z = __builtin_fmaf(t.nz ? ea.z : eb.z, t.iz, no.z);
    }
    // `if t0 > min { min = t0 }` keeps min on NaN (0 * inf): fmaxf's NaN rule.  The
    // bound only shrinks, so one min < max test after all three axes equals the
    // reference's per-axis early exit.
    const float lo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tmin, t0x), t0y), t0z);
    // hi = fminf(fminf(fminf(closest, t1x), t1y), t1z) as v_min3 + v_min: the builtin
    // would first canonicalize `closest` (one more VALU per box).  Same IEEE-mode
    // result: the operands are arithmetic results or +inf, never signalling NaNs.
    float hi;
    asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4" : "=&v"(hi) : "v"(t.closest), "v"(t1x), "v"(t1y), "v"(t1z));
    return lo < hi;
}

template <bool COUNT, bool MED3 = false, bool FMA = false>
__device__ __forceinline__ void box_step(Trav& t, const Ray& r, const float4 ea, const float4 eb, int32_t tag,
                                         Counters& cnt, const V3 no = V3{0.0f, 0.0f, 0.0f}) {
    if (COUNT && __float_as_int(ea.w) != tag) ++cnt.node_visits;  // (not the sentinel: escape == next)
    // the next entry on a box hit, else the escape (both stored as walk positions): a
    // mask select (a ?: here became a branch).
    const uint32_t take = 0u - (uint32_t)box_hit<MED3, FMA>(t, r, ea, eb, no);
    t.i = ((uint32_t)tag & take) | ((uint32_t)__float_as_int(ea.w) & ~take);
}

// One step of the closest-hit walk over the threaded pre-order layout (rtx_layout.h):
// entry i is a node (Aabb.Hit, bvh.go:52-61, 84-102) or a sphere (Sphere.Hit,
// hittables.go:96-116).  The sequence of steps is the reference recursion's, with
// running bound `closest` = the closest hit so far (bvh.go:227-232).
// QUADS: the scene holds quads (a third entry kind); false compiles the sphere-only step.
// FIXED: E is v3's LDS layout at LDS address 0 (scene_ref_fixed).
template <bool COUNT, bool QUADS = false, bool FIXED = false, bool HYB = false, bool MED3 = false, bool FMA = false>
__device__ __forceinline__ void trav_step(Trav& t, const Ray& r, const SceneRef E, Counters& cnt,
                                          const V3 no = V3{0.0f, 0.0f, 0.0f}) {
    float4 ea, eb;
    load_entry<FIXED, HYB>(E, t.i, ea, eb);
    if (COUNT && HYB && t.i < E.hot) ++cnt.cache_hits;
    const int32_t tag = __float_as_int(eb.w);  // device recoding, rtx_layout.h
    // (tag > -2, not tag >= 0: a sign test became a 64-bit compare of eb.z:eb.w)
    if (tag > -2) {  // a node (or the sentinel)
        box_step<COUNT, MED3, FMA>(t, r, ea, eb, tag, cnt, no);
    } else {
        if (QUADS && tag == RTX_E_QUAD) quad_test<COUNT>(t, r, E, ea, eb, t.i, cnt);
        else sphere_test<COUNT, MED3, FIXED, !FIXED>(t, r, ea, eb, t.i, cnt, E.b);
        t.i = (uint32_t)__float_as_int(eb.z);  // the primitive's successor
    }
}

// The record at walk position `pos` of the paired walk (build_w2): entries pos and pos + 16, both halves, in one
// round trip — from the LDS cache (its 'a' halves at 0, 'b' halves at HOT_B) below E.hot, else from HBM, both kinds
// issued under their exec masks before one wait (load_entry<HYB>).
__device__ __forceinline__ void load_record(const SceneRef E, uint32_t pos, float4& a0, float4& b0, float4& a1, float4& b1) {
    uint64_t sv, m;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "v_cmp_gt_u32_e64 %[m], %[hot], %[pos]\n\t" /* the LDS cache's lanes */
                 "s_andn2_b64 exec, %[sv], %[m]\n\t"
                 "s_cbranch_execz LG%=\n\t"
                 "global_load_dwordx4 %[a0], %[pos], %[ba]\n\t"
                 "global_load_dwordx4 %[a1], %[pos], %[ba] offset:16\n\t"
                 "global_load_dwordx4 %[b0], %[pos], %[bb]\n\t"
                 "global_load_dwordx4 %[b1], %[pos], %[bb] offset:16\n"
                 "LG%=:\n\t"
                 "s_and_b64 exec, %[sv], %[m]\n\t"
                 "s_cbranch_execz LL%=\n\t"
                 "ds_read_b128 %[a0], %[pos]\n\t"
                 "ds_read_b128 %[a1], %[pos] offset:16\n\t"
                 "ds_read_b128 %[b0], %[pos] offset:%[lb]\n\t"
                 "ds_read_b128 %[b1], %[pos] offset:%[lb16]\n"
                 "LL%=:\n\t"
                 "s_mov_b64 exec, %[sv]\n\t"
                 "s_waitcnt vmcnt(0) lgkmcnt(0)"
                 : [a0] "=&v"(a0), [b0] "=&v"(b0), [a1] "=&v"(a1), [b1] "=&v"(b1), [sv] "=&s"(sv), [m] "=&s"(m)
                 : [pos] "v"(pos), [hot] "s"(E.hot), [ba] "s"(E.a), [bb] "s"(E.b), [lb] "i"(HOT_B), [lb16] "i"(HOT_B + 16)
                 : "scc");
}

// One step of the paired walk (rtx_capi.hip build_w2) for a layout in HBM with its LDS cache: the
// record at t.i holds the threaded walk's entry p and its fail successor q(p).  Slot 0: a node whose box passes
// descends (the record of its first child, b.w); otherwise (a failed box, a primitive tested) the lane goes on to
// slot 1 in the same step: a node to its first child's record (b.w) or its escape's (a.w), a primitive tested and to
// its successor's record (b.z).  The same tests in the same order with the same bounds as trav_step on the threaded
// layout — so the same hits, draws and work counters — in fewer dependent reads.  Lanes at the walk's end (the
// sentinel position) read nothing.
template <bool COUNT, bool QUADS = false, bool MED3 = false, bool FMA = false>
__device__ __forceinline__ void trav_step_w2(Trav& t, const Ray& r, const SceneRef E, Counters& cnt, uint32_t end,
                                             const V3 no = V3{0.0f, 0.0f, 0.0f}) {
    if (t.i >= end) return;
    const uint32_t pos = t.i;
    float4 a0, b0, a1, b1;
    load_record(E, pos, a0, b0, a1, b1);
    if (COUNT && pos < E.hot) ++cnt.cache_hits;
    const int32_t tag0 = __float_as_int(b0.w);
    bool down = false;
    if (tag0 > -2) {  // a node (slot 0 is never the sentinel)
        if (COUNT) ++cnt.node_visits;
        down = box_hit<MED3, FMA>(t, r, a0, b0, no);
    } else if (QUADS && tag0 == RTX_E_QUAD) {
        quad_test<COUNT>(t, r, E, a0, b0, pos, cnt);
    } else {
        sphere_test<COUNT, MED3, false, true>(t, r, a0, b0, pos, cnt, E.b);
    }
    if (down) {
        t.i = (uint32_t)tag0;
        return;
    }
    const int32_t tag1 = __float_as_int(b1.w);
    if (tag1 > -2) {  // a node, or the sentinel (escape == next: not a test)
        if (COUNT && __float_as_int(a1.w) != tag1) ++cnt.node_visits;
        t.i = box_hit<MED3, FMA>(t, r, a1, b1, no) ? (uint32_t)tag1 : (uint32_t)__float_as_int(a1.w);
    } else {
        if (QUADS && tag1 == RTX_E_QUAD) quad_test<COUNT>(t, r, E, a1, b1, pos + 16, cnt);
        else sphere_test<COUNT, MED3, false, true>(t, r, a1, b1, pos + 16, cnt, E.b);
        t.i = (uint32_t)__float_as_int(b1.z);
    }
}

// The walk step with primitive batching (v3, RTX_PRIM_BATCH = kmin > 0): every lane reads its
// entry, then the wave runs EITHER the box tests of its lanes on nodes OR the primitive tests of
// its lanes on primitives — the primitive tests once at least `kmin` lanes wait on one (or no
// lane has a node to test).  Lanes of the other kind keep their position and read the entry
// again next step.  Each lane still takes the reference's steps in the reference's order with
// the current bound, so every result is unchanged; the wave no longer pays both paths in the
// ~75 % of steps where a few lanes sit on primitives.
// Returns (COUNT only) the lanes whose entry the step processed, wave-uniform; `idle` gets the
// lanes parked on the sentinel (low 16 bits) and the lanes whose entry kind the step did not
// run (high 16 bits).
template <bool COUNT, bool QUADS, bool FIXED, bool HYB, bool MED3, bool FMA = false>
__device__ __forceinline__ uint32_t trav_step_batched(Trav& t, const Ray& r, const SceneRef E, Counters& cnt,
                                                      uint32_t end, uint32_t kmin, uint32_t& idle,
                                                      const V3 no = V3{0.0f, 0.0f, 0.0f}) {
    float4 ea, eb;
    load_entry<FIXED, HYB>(E, t.i, ea, eb);
    const int32_t tag = __float_as_int(eb.w);
    const bool prim = tag < -1;
    const uint64_t pm = ballot(prim);
    // lanes on a node: SALU on two compare masks (a vote on `!prim && t.i < end` itself was
    // materialised as v_cndmask + v_cmp, two VALU per step)
    const uint64_t bm = ballot(t.i < end) & ~pm;
    const bool prims = (uint32_t)__popcll(pm) >= kmin || bm == 0;
    if (prims) {
        if (__builtin_amdgcn_inverse_ballot_w64(pm)) {  // = prim, as the vote's mask (no second compare)
            if (COUNT && HYB && t.i < E.hot) ++cnt.cache_hits;
            if (QUADS && tag == RTX_E_QUAD) quad_test<COUNT>(t, r, E, ea, eb, t.i, cnt);
            else sphere_test<COUNT, MED3, FIXED, !FIXED>(t, r, ea, eb, t.i, cnt, E.b);
            t.i = (uint32_t)__float_as_int(eb.z);
        }
    } else if (__builtin_amdgcn_inverse_ballot_w64(bm)) {  // lanes on a node (the sentinel's step is a no-op)
        if (COUNT && HYB && t.i < E.hot) ++cnt.cache_hits;
        box_step<COUNT, MED3, FMA>(t, r, ea, eb, tag, cnt, no);
    }
    if (COUNT) {
        const uint32_t walking = (uint32_t)__popcll(pm | bm);
        idle += (64u - walking) | ((uint32_t)__popcll(prims ? bm : pm) << 16);
    }
    return COUNT ? (uint32_t)__popcll(prims ? pm : bm) : 0u;
}

// trav_step_batched<false, false, true, false, true> x 6 — the timed kernel's walk between two
// wave votes, for a sphere scene in LDS whose walking lanes all have t.safe rays — written out in
// GCN assembly.  Same decisions, same IEEE operations in the same order, same results
// (tests/test_gpu_parity.py compares it with the counting kernel, which keeps the C++ step, and
// with the oracle).  What the compiler could not be talked out of: the uniform choice box /
// primitive went through s_cselect + s_and vcc, exec + vccz branches, the box test through
// saveexec + execz + exec restore + phi copies of the position, and the sphere test through
// three nested divergent ifs: 45 issued instructions per box step, 31 here; the sphere test runs
// branch-free on the primitive lanes (both roots, then one select).  One asm statement for all
// six steps: the compiler puts an s_nop at every asm boundary, and a read into a register tuple
// cannot hand its components to another asm statement without copies, so the entry lives in the
// clobbered v0-v7 (halves a, b) with v8-v9 as scratch.
//   - kind: primitive = tag < -1; node lanes = walking & ~primitive, walking = the lanes with
//     pos < end at the last vote (an SGPR mask: no compare per step; a lane that reaches the
//     sentinel between two votes stays a node lane there, and a box step on the sentinel
//     changes nothing; -1.7 % at 100 spp)
//   - the primitive tests run when >= kmin lanes wait on one or no node lane is left; after a box
//     step the count test is skipped and box steps follow while a node lane is left (box runs:
//     the primitive tests gather more lanes; -1.8 % at 100 spp, Cornell box -7.4 %)
//   - box (MED3, box_step): per axis (min - o) * inv, (max - o) * inv; lo/hi clamped by v_med3
//   - sphere (sphere_test<false, true>): hb, c, disc as hittables.go:97-102; sqrt correctly
//     rounded as the compiler expands an f32 sqrt — v_sqrt, then the neighbour whose fma
//     residual changes sign; inputs below 2^-96 scaled by 2^32 first and the root by 2^-16
//     after, a path taken only when some lane has 0 <= disc < 2^-96.  (The expansion's last
//     step, passing +-0 and +inf through, is left out: v_sqrt returns them exactly and both
//     neighbour residuals are then NaN or a zero, which keeps them.)  Both roots by div_by;
//     the first root when tmin < t1, else the second (hittables.go:110-114).  disc < 0 needs no
//     test of its own (:104): v_sqrt returns NaN there, and NaN roots fail tmin < t.
// gfx950 hazards: a VALU-written SGPR/VCC read as a v_cndmask mask by the next VALU needs
// s_nop 1; a v_sqrt result read by the next VALU needs s_nop 0 (as the compiler emits them).
// Entry read of the prefetching walk, under the current exec: both halves from the fixed layout.
#define RTX_LOAD_LDS                                                         \
        "ds_read_b128 v[0:3], %[pos]\n\t"                                    \
        "ds_read_b128 v[4:7], %[pos] offset:32768\n\t" /* LDS_B */
#define RTX_WAIT_LDS "s_waitcnt lgkmcnt(0)\n\t"
// End of a box step: back to the full wave, then the next step's header (RTX_BOX_NEXT), or a box run
// (RTX_BOX_FAST): the lanes of this step still on a node test their next box at once, under the
// same exec minus the lanes now on a primitive (only these lanes moved), without the next step's
// primitive-count test; back to the full wave and the header when no node lane is left.
#define RTX_BOX_NEXT(K) "s_mov_b64 exec, %[save]\n\t" "s_branch LE%=_" #K "\n"
#define RTX_BOX_FAST(K, KN)                                                  \
        "v_cmp_gt_u32_e64 %[pm], %[pe], %[pos]\n\t" /* (exec: node lanes) now on a primitive */\
        "s_andn2_b64 exec, exec, %[pm]\n\t" /* the node lanes left (scc) */  \
        "s_cbranch_scc1 LB%=_" #KN "\n\t"                                    \
        "s_mov_b64 exec, %[save]\n\t"                                        \
        "s_branch LE%=_" #K "\n"
// Primitive runs (sphere scenes): the lanes of a primitive step whose successor is a primitive
// again (a reference leaf's second sphere, or a World's next item) test it at once, in the same step,
// under the step's exec narrowed to them — as box runs do for nodes (no header, no count test, no
// exec restore between the two sphere tests).  Each lane still tests its entries in its own order with
// its own bound.  Measured +0.5 % at C2 (128.75 / 129.04 vs 128.17 / 128.22 ms, images identical):
// off; RTX_PRIM_RUN=1 for A/B.
#ifndef RTX_PRIM_RUN
#define RTX_PRIM_RUN 0
#endif
#if RTX_PRIM_RUN
#define RTX_PRIM_RUN_TAIL(K, WAIT)                                           \
        "v_cmp_gt_u32_e64 %[pm], %[pe], %[pos]\n\t" /* (exec: this step's lanes) on a primitive again */\
        "s_and_b64 exec, exec, %[pm]\n\t"                                    \
        "s_cbranch_scc0 LR%=_" #K "\n\t"                                     \
        WAIT /* its read, issued in the test */                              \
        "s_branch LU%=_" #K "\n"
#else
#define RTX_PRIM_RUN_TAIL(K, WAIT) ""
#endif
// A box step's slab distances, lo / hi clamped by v_med3 (box_step MED3): the reference's
// (b - o) * (1/d), or the near walk's fma(b, 1/d, -(o/d)) (box_step FMA: 12 VALU instead of 18).
#define RTX_SLABS_SUBMUL \
        "v_sub_f32 v0, v0, %[ox]\n\t"                                        \
        "v_sub_f32 v4, v4, %[ox]\n\t"                                        \
        "v_sub_f32 v1, v1, %[oy]\n\t"                                        \
        "v_sub_f32 v5, v5, %[oy]\n\t"                                        \
        "v_mul_f32 v0, v0, %[ix]\n\t"                                        \
        "v_mul_f32 v4, v4, %[ix]\n\t"                                        \
        "v_sub_f32 v2, v2, %[oz]\n\t"                                        \
        "v_sub_f32 v6, v6, %[oz]\n\t"                                        \
        "v_mul_f32 v1, v1, %[iy]\n\t"                                        \
        "v_mul_f32 v5, v5, %[iy]\n\t"                                        \
        "v_med3_f32 v8, %[tmin], v0, v4\n\t"                                 \
        "v_med3_f32 v9, %[cl], v0, v4\n\t"                                   \
        "v_mul_f32 v2, v2, %[iz]\n\t"                                        \
        "v_mul_f32 v6, v6, %[iz]\n\t"                                        \
        "v_med3_f32 v8, v8, v1, v5\n\t"                                      \
        "v_med3_f32 v9, v9, v1, v5\n\t"                                      \
        "v_med3_f32 v8, v8, v2, v6\n\t"                                      \
        "v_med3_f32 v9, v9, v2, v6\n\t"
#define RTX_SLABS_FMA                                                        \
        "v_fma_f32 v0, v0, %[ix], %[nox]\n\t"                                \
        "v_fma_f32 v4, v4, %[ix], %[nox]\n\t"                                \
        "v_fma_f32 v1, v1, %[iy], %[noy]\n\t"                                \
        "v_fma_f32 v5, v5, %[iy], %[noy]\n\t"                                \
        "v_med3_f32 v8, %[tmin], v0, v4\n\t"                                 \
        "v_med3_f32 v9, %[cl], v0, v4\n\t"                                   \
        "v_fma_f32 v2, v2, %[iz], %[noz]\n\t"                                \
        "v_fma_f32 v6, v6, %[iz], %[noz]\n\t"                                \
        "v_med3_f32 v8, v8, v1, v5\n\t"                                      \
        "v_med3_f32 v9, v9, v1, v5\n\t"                                      \
        "v_med3_f32 v8, v8, v2, v6\n\t"                                      \
        "v_med3_f32 v9, v9, v2, v6\n\t"
#define RTX_WALK_STEP_PF(K, LOAD, WAIT, BEND, SLABS)                               \
        "v_cmp_gt_u32_e64 %[pm], %[pe], %[pos]\n\t" /* primitive: pos < prim_end */\
        "s_bcnt1_i32_b64 %[cnt], %[pm]\n\t"                                  \
        "s_cmp_ge_u32 %[cnt], %[kmin]\n\t"                                   \
        "s_cbranch_scc1 LP%=_" #K "\n\t"                                     \
        "s_andn2_b64 %[wm], %[wk], %[pm]\n\t" /* scc: a node lane */         \
        "s_cbranch_scc0 LP%=_" #K "\n\t"                                     \
        /* ---- box tests on the node lanes, then their next entries */      \
        "s_and_saveexec_b64 %[save], %[wm]\n\t"                              \
        "LB%=_" #K ":\n\t" /* a box run continues here, exec = its node lanes */\
        WAIT                                                                 \
        SLABS                                                                \
        "v_cmp_lt_f32_e32 vcc, v8, v9\n\t"                                   \
        "s_nop 1\n\t"                                                        \
        "v_cndmask_b32_e32 %[pos], v3, v7, vcc\n\t"                          \
        LOAD                                                                 \
        BEND                                                                 \
        /* ---- sphere tests on the primitive lanes, successor read first */ \
        "LP%=_" #K ":\n\t"                                                   \
        WAIT                                                                 \
        "s_and_saveexec_b64 %[save], %[pm]\n\t"                              \
        "s_cbranch_execz LR%=_" #K "\n"                                       \
        "LU%=_" #K ":\n\t" /* a primitive run continues here, exec = its lanes */\
        "v_sub_f32 v10, %[ox], v0\n\t" /* oc = o - center */                 \
        "v_sub_f32 v11, %[oy], v1\n\t"                                       \
        "v_sub_f32 v12, %[oz], v2\n\t"                                       \
        "v_mul_f32 v13, v10, v10\n\t" /* c = |oc|^2 - r^2 */                 \
        "v_mul_f32 v9, v11, v11\n\t"                                         \
        "v_add_f32 v13, v13, v9\n\t"                                         \
        "v_mul_f32 v9, v12, v12\n\t"                                         \
        "v_add_f32 v13, v13, v9\n\t"                                         \
        "v_sub_f32 v13, v13, v4\n\t"                                         \
        "v_lshrrev_b32_e32 v14, 4, %[pos]\n\t" /* this entry's index */      \
        "v_mov_b32 %[pos], v6\n\t"     /* successor */                       \
        LOAD                                                                 \
        "v_mul_f32 v8, %[dx], v10\n\t" /* hb = d.oc */                       \
        "v_mul_f32 v9, %[dy], v11\n\t"                                       \
        "v_add_f32 v8, v8, v9\n\t"                                           \
        "v_mul_f32 v9, %[dz], v12\n\t"                                       \
        "v_add_f32 v8, v8, v9\n\t"                                           \
        "v_mul_f32 v10, %[a], v13\n\t" /* disc = hb*hb - a*c */              \
        "v_mul_f32 v9, v8, v8\n\t"                                           \
        "v_sub_f32 v10, v9, v10\n\t"                                         \
        "v_sqrt_f32_e32 v12, v10\n\t"                                        \
        "v_cmp_gt_u32_e32 vcc, 0xf800000, v10\n\t" /* 0 <= x < 2^-96 (by its bits; in the v_sqrt hazard slot) */\
        "s_cbranch_vccnz LS%=_" #K "\n\t" /* here: x >= 2^-96, -0 or x < 0 (NaN root: no hit) */\
        "v_add_u32_e32 v9, -1, v12\n\t"                                      \
        "v_add_u32_e32 v11, 1, v12\n\t"                                      \
        "v_fma_f32 v13, -v9, v12, v10\n\t"                                   \
        "v_fma_f32 v15, -v11, v12, v10\n\t"                                  \
        "v_cmp_ge_f32_e64 %[g1], 0, v13\n\t"                                 \
        "v_cmp_lt_f32_e64 %[l1], 0, v15\n\t"                                 \
        "s_nop 0\n\t"                                                        \
        "v_cndmask_b32_e64 v12, v12, v9, %[g1]\n\t"                          \
        "v_cndmask_b32_e64 v12, v12, v11, %[l1]\n\t"                         \
        "LQ%=_" #K ":\n\t" /* v12 = sqrt(disc) */                            \
        "v_sub_f32_e64 v11, -v8, v12\n\t" /* -hb - sq */                     \
        "v_add_f32_e64 v13, -v8, v12\n\t" /* -hb + sq */                     \
        "v_mul_f32 v15, v11, %[ra]\n\t"   /* div_by: q0 = n y */             \
        "v_mul_f32 v16, v13, %[ra]\n\t"                                      \
        "v_fma_f32 v11, -%[a], v15, v11\n\t" /* e = n - a q0 */              \
        "v_fmac_f32 v15, v11, %[ra]\n\t" /* t1 = q0 + e y */                 \
        "v_cmp_lt_f32_e64 %[g1], %[tmin], v15\n\t" /* tmin < t1 */           \
        "v_fma_f32 v13, -%[a], v16, v13\n\t" /* (2 wait states for g1) */    \
        "v_fmac_f32 v16, v13, %[ra]\n\t" /* t2 */                            \
        "v_cndmask_b32_e64 v16, v16, v15, %[g1]\n\t" /* t: t1 if tmin < t1, else t2 */\
        "v_cmp_lt_f32_e64 %[l1], %[tmin], v16\n\t" /* tmin < t < closest */  \
        "v_cmp_lt_f32_e64 %[l2], v16, %[cl]\n\t"                             \
        "s_and_b64 %[l1], %[l1], %[l2]\n\t" /* (disc < 0: NaN roots fail) */ \
        "v_cmp_eq_f32_e64 %[l2], v16, %[cl]\n\t" /* or a tie won by the     */ \
        "v_cmp_lt_i32_e64 %[g1], v14, %[hit]\n\t" /* reference's earlier sphere */\
        "s_and_b64 %[l2], %[l2], %[g1]\n\t" /* (sphere_test RANKED) */       \
        "s_or_b64 %[l1], %[l1], %[l2]\n\t"                                  \
        "v_cndmask_b32_e64 %[cl], %[cl], v16, %[l1]\n\t"                     \
        "v_cndmask_b32_e64 %[hit], %[hit], v14, %[l1]\n\t"                   \
        RTX_PRIM_RUN_TAIL(K, WAIT)                                           \
        "LR%=_" #K ":\n\t"                                                   \
        "s_mov_b64 exec, %[save]\n"                                          \
        "LE%=_" #K ":\n\t"
#define RTX_WALK_STEP_PFQ(K, LOAD, WAIT, BEND, SLABS)                               \
        "v_cmp_gt_u32_e64 %[pm], %[pe], %[pos]\n\t" /* primitive: pos < prim_end */\
        "s_bcnt1_i32_b64 %[cnt], %[pm]\n\t"                                  \
        "s_cmp_ge_u32 %[cnt], %[kmin]\n\t"                                   \
        "s_cbranch_scc1 LP%=_" #K "\n\t"                                     \
        "s_andn2_b64 %[wm], %[wk], %[pm]\n\t" /* scc: a node lane */         \
        "s_cbranch_scc0 LP%=_" #K "\n\t"                                     \
        /* ---- box tests on the node lanes, then their next entries */      \
        "s_and_saveexec_b64 %[save], %[wm]\n\t"                              \
        "LB%=_" #K ":\n\t" /* a box run continues here, exec = its node lanes */\
        WAIT                                                                 \
        SLABS                                                                \
        "v_cmp_lt_f32_e32 vcc, v8, v9\n\t"                                   \
        "s_nop 1\n\t"                                                        \
        "v_cndmask_b32_e32 %[pos], v3, v7, vcc\n\t"                          \
        LOAD                                                                 \
        BEND                                                                 \
        /* ---- sphere tests on the primitive lanes, successor read first */ \
        "LP%=_" #K ":\n\t"                                                   \
        WAIT                                                                 \
        "s_and_saveexec_b64 %[save], %[pm]\n\t"                              \
        "s_cbranch_execz LR%=_" #K "\n\t"                                    \
        "v_mov_b32 v10, v0\n\t" /* centre / normal */                        \
        "v_mov_b32 v11, v1\n\t"                                              \
        "v_mov_b32 v12, v2\n\t"                                              \
        "v_mov_b32 v19, v3\n\t" /* quad: D */                                \
        "v_mov_b32 v13, v4\n\t" /* r^2 / quad index */                       \
        "v_mov_b32 v18, v7\n\t" /* tag */                                    \
        "v_lshrrev_b32_e32 v14, 4, %[pos]\n\t" /* this entry's index */      \
        "v_mov_b32 %[pos], v6\n\t" /* successor */                           \
        LOAD                                                                 \
        "v_cmp_gt_i32_e64 %[qs], -2, v18\n\t" /* sphere: tag < -2 */         \
        "s_and_saveexec_b64 %[qm], %[qs]\n\t"                                \
        "s_cbranch_execz LT%=_" #K "\n\t"                                    \
        "v_sub_f32 v10, %[ox], v10\n\t" /* oc = o - center */                \
        "v_sub_f32 v11, %[oy], v11\n\t"                                      \
        "v_sub_f32 v12, %[oz], v12\n\t"                                      \
        "v_mul_f32 v8, %[dx], v10\n\t" /* hb = d.oc */                       \
        "v_mul_f32 v9, %[dy], v11\n\t"                                       \
        "v_add_f32 v8, v8, v9\n\t"                                           \
        "v_mul_f32 v9, %[dz], v12\n\t"                                       \
        "v_add_f32 v8, v8, v9\n\t"                                           \
        "v_mul_f32 v10, v10, v10\n\t" /* c = |oc|^2 - r^2 */                 \
        "v_mul_f32 v11, v11, v11\n\t"                                        \
        "v_add_f32 v10, v10, v11\n\t"                                        \
        "v_mul_f32 v12, v12, v12\n\t"                                        \
        "v_add_f32 v10, v10, v12\n\t"                                        \
        "v_sub_f32 v10, v10, v13\n\t"                                        \
        "v_mul_f32 v10, %[a], v10\n\t" /* disc = hb*hb - a*c */              \
        "v_mul_f32 v9, v8, v8\n\t"                                           \
        "v_sub_f32 v10, v9, v10\n\t"                                         \
        "v_sqrt_f32_e32 v12, v10\n\t"                                        \
        "v_cmp_gt_u32_e32 vcc, 0xf800000, v10\n\t" /* 0 <= x < 2^-96 (by its bits; in the v_sqrt hazard slot) */\
        "s_cbranch_vccnz LS%=_" #K "\n\t" /* here: x >= 2^-96, -0 or x < 0 (NaN root: no hit) */\
        "v_add_u32_e32 v9, -1, v12\n\t"                                      \
        "v_add_u32_e32 v11, 1, v12\n\t"                                      \
        "v_fma_f32 v13, -v9, v12, v10\n\t"                                   \
        "v_fma_f32 v15, -v11, v12, v10\n\t"                                  \
        "v_cmp_ge_f32_e64 %[g1], 0, v13\n\t"                                 \
        "v_cmp_lt_f32_e64 %[l1], 0, v15\n\t"                                 \
        "s_nop 0\n\t"                                                        \
        "v_cndmask_b32_e64 v12, v12, v9, %[g1]\n\t"                          \
        "v_cndmask_b32_e64 v12, v12, v11, %[l1]\n\t"                         \
        "LQ%=_" #K ":\n\t" /* v12 = sqrt(disc) */                            \
        "v_sub_f32_e64 v11, -v8, v12\n\t" /* -hb - sq */                     \
        "v_add_f32_e64 v13, -v8, v12\n\t" /* -hb + sq */                     \
        "v_mul_f32 v15, v11, %[ra]\n\t"   /* div_by: q0 = n y */             \
        "v_mul_f32 v16, v13, %[ra]\n\t"                                      \
        "v_fma_f32 v11, -%[a], v15, v11\n\t" /* e = n - a q0 */              \
        "v_fmac_f32 v15, v11, %[ra]\n\t" /* t1 = q0 + e y */                 \
        "v_cmp_lt_f32_e64 %[g1], %[tmin], v15\n\t" /* tmin < t1 */           \
        "v_fma_f32 v13, -%[a], v16, v13\n\t" /* (2 wait states for g1) */    \
        "v_fmac_f32 v16, v13, %[ra]\n\t" /* t2 */                            \
        "v_cndmask_b32_e64 v16, v16, v15, %[g1]\n\t" /* t: t1 if tmin < t1, else t2 */\
        "v_cmp_lt_f32_e64 %[l1], %[tmin], v16\n\t" /* tmin < t < closest */  \
        "v_cmp_lt_f32_e64 %[l2], v16, %[cl]\n\t"                             \
        "s_and_b64 %[l1], %[l1], %[l2]\n\t" /* (disc < 0: NaN roots fail) */ \
        "v_cmp_eq_f32_e64 %[l2], v16, %[cl]\n\t" /* or a tie won by the     */ \
        "v_cmp_lt_i32_e64 %[g1], v14, %[hit]\n\t" /* reference's earlier sphere */\
        "s_and_b64 %[l2], %[l2], %[g1]\n\t" /* (sphere_test RANKED) */       \
        "s_or_b64 %[l1], %[l1], %[l2]\n\t"                                  \
        "v_cndmask_b32_e64 %[cl], %[cl], v16, %[l1]\n\t"                     \
        "v_cndmask_b32_e64 %[hit], %[hit], v14, %[l1]\n"                     \
        "LT%=_" #K ":\n\t"                                                   \
        "s_andn2_b64 exec, %[qm], %[qs]\n\t" /* quad lanes */                \
        "s_cbranch_execz LR%=_" #K "\n\t"                                    \
        "v_mul_f32 v8, %[dx], v10\n\t" /* denom = d . n (hittables.go:168) */\
        "v_mul_f32 v9, %[dy], v11\n\t"                                       \
        "v_add_f32 v8, v8, v9\n\t"                                           \
        "v_mul_f32 v9, %[dz], v12\n\t"                                       \
        "v_add_f32 v8, v8, v9\n\t"                                           \
        "v_mul_f32 v15, v10, %[ox]\n\t" /* n . o */                          \
        "v_mul_f32 v16, v11, %[oy]\n\t"                                      \
        "v_add_f32 v15, v15, v16\n\t"                                        \
        "v_mul_f32 v16, v12, %[oz]\n\t"                                      \
        "v_add_f32 v15, v15, v16\n\t"                                        \
        "v_sub_f32 v15, v19, v15\n\t" /* D - n . o  (:174) */                \
        "v_rcp_f32_e32 v16, v8\n\t" /* y = RN(1 / denom): fma Newton step */ \
        "v_and_b32_e32 v9, 0x7fffffff, v8\n\t"                               \
        "v_cmp_gt_f32_e32 vcc, 0x322bcc78, v9\n\t" /* |denom| < 1e-8 (:170): parallel */\
        "v_fma_f32 v17, -v8, v16, 1.0\n\t"                                   \
        "v_fma_f32 v16, v17, v16, v16\n\t"                                   \
        "v_mul_f32 v17, v15, v16\n\t" /* div_by: t = (D - n.o) / denom */    \
        "v_fma_f32 v15, -v8, v17, v15\n\t"                                   \
        "v_fmac_f32 v17, v15, v16\n\t" /* t */                               \
        "v_cmp_lt_f32_e64 %[l1], %[tmin], v17\n\t" /* tmin < t < closest (:176) */\
        "v_cmp_lt_f32_e64 %[l2], v17, %[cl]\n\t"                             \
        "s_and_b64 %[l1], %[l1], %[l2]\n\t"                                  \
        "s_andn2_b64 %[l1], %[l1], vcc\n\t"                                  \
        "s_and_saveexec_b64 %[g1], %[l1]\n\t" /* lanes on the plane inside the bound */\
        "s_cbranch_execz LR%=_" #K "\n\t"                                    \
        "v_lshlrev_b32_e32 v9, 6, v13\n\t" /* the quad record: Q, u, v, w (rtx_layout.h) */\
        "v_add_u32_e32 v9, %[qbase], v9\n\t"                                 \
        "ds_read_b96 v[20:22], v9\n\t"                                       \
        "ds_read_b96 v[24:26], v9 offset:16\n\t"                             \
        "ds_read_b96 v[28:30], v9 offset:32\n\t"                             \
        "ds_read_b96 v[32:34], v9 offset:48\n\t"                             \
        "v_mul_f32 v10, %[dx], v17\n\t" /* r.At(t) = d t + o (:180) */       \
        "v_mul_f32 v11, %[dy], v17\n\t"                                      \
        "v_mul_f32 v12, %[dz], v17\n\t"                                      \
        "v_add_f32 v10, v10, %[ox]\n\t"                                      \
        "v_add_f32 v11, v11, %[oy]\n\t"                                      \
        "v_add_f32 v12, v12, %[oz]\n\t"                                      \
        "s_waitcnt lgkmcnt(0)\n\t" /* (the successor read returns first) */  \
        "v_sub_f32 v10, v10, v20\n\t" /* php = p - Q (:181) */               \
        "v_sub_f32 v11, v11, v21\n\t"                                        \
        "v_sub_f32 v12, v12, v22\n\t"                                        \
        "v_mul_f32 v15, v11, v30\n\t" /* cross(php, v) (:182) */             \
        "v_mul_f32 v16, v12, v29\n\t"                                        \
        "v_sub_f32 v15, v15, v16\n\t"                                        \
        "v_mul_f32 v16, v12, v28\n\t"                                        \
        "v_mul_f32 v19, v10, v30\n\t"                                        \
        "v_sub_f32 v16, v16, v19\n\t"                                        \
        "v_mul_f32 v19, v10, v29\n\t"                                        \
        "v_mul_f32 v20, v11, v28\n\t"                                        \
        "v_sub_f32 v19, v19, v20\n\t"                                        \
        "v_mul_f32 v15, v32, v15\n\t" /* alpha = w . c */                    \
        "v_mul_f32 v16, v33, v16\n\t"                                        \
        "v_add_f32 v15, v15, v16\n\t"                                        \
        "v_mul_f32 v16, v34, v19\n\t"                                        \
        "v_add_f32 v15, v15, v16\n\t"                                        \
        "v_mul_f32 v16, v25, v12\n\t" /* cross(u, php) (:183) */             \
        "v_mul_f32 v19, v26, v11\n\t"                                        \
        "v_sub_f32 v16, v16, v19\n\t"                                        \
        "v_mul_f32 v19, v26, v10\n\t"                                        \
        "v_mul_f32 v20, v24, v12\n\t"                                        \
        "v_sub_f32 v19, v19, v20\n\t"                                        \
        "v_mul_f32 v20, v24, v11\n\t"                                        \
        "v_mul_f32 v21, v25, v10\n\t"                                        \
        "v_sub_f32 v20, v20, v21\n\t"                                        \
        "v_mul_f32 v16, v32, v16\n\t" /* beta = w . c */                     \
        "v_mul_f32 v19, v33, v19\n\t"                                        \
        "v_add_f32 v16, v16, v19\n\t"                                        \
        "v_mul_f32 v19, v34, v20\n\t"                                        \
        "v_add_f32 v16, v16, v19\n\t"                                        \
        "v_cmp_gt_f32_e64 %[l1], 0, v15\n\t" /* outside: a < 0 || 1 < a || b < 0 || 1 < b (:185) */\
        "v_cmp_lt_f32_e64 %[l2], 1.0, v15\n\t"                               \
        "s_or_b64 %[l1], %[l1], %[l2]\n\t"                                   \
        "v_cmp_gt_f32_e64 %[l2], 0, v16\n\t"                                 \
        "s_or_b64 %[l1], %[l1], %[l2]\n\t"                                   \
        "v_cmp_lt_f32_e64 %[l2], 1.0, v16\n\t"                               \
        "s_or_b64 %[l1], %[l1], %[l2]\n\t"                                   \
        "s_andn2_b64 %[l1], exec, %[l1]\n\t" /* hit (NaN alpha or beta: inside, as in Go) */\
        "v_cndmask_b32_e64 %[cl], %[cl], v17, %[l1]\n\t"                     \
        "v_cndmask_b32_e64 %[hit], %[hit], v14, %[l1]\n\t"                   \
        "LR%=_" #K ":\n\t"                                                   \
        "s_mov_b64 exec, %[save]\n\t"                                        \
        "LE%=_" #K ":\n\t"
// The whole traversal phase (traverse_loop's !COUNT body for this case): RTX_ASM_BLOCK asm steps
// (RTX_ASM_BLOCK_Q with quads), then the
// vote — at_end = pos >= end, walking lanes W, waiting lanes P0 — until no lane walks or at
// least `thresh` wait; returns the final at_end mask.  Termination: storage positions do NOT
// increase along a walk (a scene in the LDS copy stores its primitives first), but every step
// moves a lane to a later entry of the threaded pre-order (a node's next is its first child, its
// escape the entry after its subtree; a primitive's next the entry after it), the upload emits
// that order from an acyclic tree (check_acyclic, rtx_capi.hip), and the sentinel ends it: every
// lane reaches the sentinel within n_entries steps.  The watchdog (RTX_WATCHDOG_S) is checked
// only between phases in render_items' loop and cannot interrupt this asm loop.
#define RTX_WALK_VOTE                                                        \
        "v_cmp_ge_u32_e64 %[pm], %[pos], %[end]\n\t"                         \
        "s_andn2_b64 %[wk], %[W], %[pm]\n\t" /* still walking (scc: any) */  \
        "s_cbranch_scc0 LX%=\n\t"                                            \
        "s_and_b64 %[l1], %[W], %[pm]\n\t"                                   \
        "s_or_b64 %[l1], %[l1], %[P0]\n\t" /* waiting to shade */            \
        "s_bcnt1_i32_b64 %[cnt], %[l1]\n\t"                                  \
        "s_cmp_lt_u32 %[cnt], %[thresh]\n\t"                                 \
        "s_cbranch_scc1 LW%=\n"                                               \
        "LX%=:"
#define RTX_WALK_OUTS                                                                                        \
    [pos] "+v"(t.i), [cl] "+v"(t.closest), [hit] "+v"(t.hit), [pm] "=&s"(pm), [wm] "=&s"(wm),              \
        [save] "=&s"(save), [g1] "=&s"(g1), [l1] "=&s"(l1), [l2] "=&s"(l2), [cnt] "=&s"(cnt), [wk] "=&s"(wk)
#define RTX_WALK_INS                                                                                         \
    [ox] "v"(r.o.x), [oy] "v"(r.o.y), [oz] "v"(r.o.z), [dx] "v"(r.d.x), [dy] "v"(r.d.y), [dz] "v"(r.d.z),  \
        [ix] "v"(t.ix), [iy] "v"(t.iy), [iz] "v"(t.iz), [a] "v"(t.a), [ra] "v"(t.ra), [end] "s"(end),      \
        [kmin] "s"(kmin), [tmin] "s"(tmin), [W] "s"(W), [P0] "s"(P0), [thresh] "s"(thresh), [pe] "s"(prim_end)
#define RTX_WALK_CLOBBERS                                                                                    \
    "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15",    \
        "v16", "vcc", "scc"
// Steps per vote (A/B with box runs, 100 spp / Cornell box 600x600x50: 4 steps -0.1 % / -2.4 %,
// 5 -0.4 % / +2.4 %, 8 +0.6 % / +2.5 %, 12 +6 % / +14 % against 6).  Every step but a block's last
// continues a box run into the next step (RTX_BOX_FAST).
#ifndef RTX_ASM_BLOCK  // sphere scenes
#define RTX_ASM_BLOCK 6
#endif
#ifndef RTX_ASM_BLOCK_Q  // scenes with quads
#define RTX_ASM_BLOCK_Q 4
#endif
#define RTX_WALK_4 S(0, RTX_BOX_FAST(0, 1)) S(1, RTX_BOX_FAST(1, 2)) S(2, RTX_BOX_FAST(2, 3)) S(3, RTX_BOX_NEXT(3))
#define RTX_WALK_5 \
    S(0, RTX_BOX_FAST(0, 1)) S(1, RTX_BOX_FAST(1, 2)) S(2, RTX_BOX_FAST(2, 3)) S(3, RTX_BOX_FAST(3, 4)) S(4, RTX_BOX_NEXT(4))
#define RTX_WALK_6                                                                                          \
    S(0, RTX_BOX_FAST(0, 1)) S(1, RTX_BOX_FAST(1, 2)) S(2, RTX_BOX_FAST(2, 3)) S(3, RTX_BOX_FAST(3, 4)) S(4, RTX_BOX_FAST(4, 5)) \
        S(5, RTX_BOX_NEXT(5))
#define RTX_WALK_8                                                                                          \
    S(0, RTX_BOX_FAST(0, 1)) S(1, RTX_BOX_FAST(1, 2)) S(2, RTX_BOX_FAST(2, 3)) S(3, RTX_BOX_FAST(3, 4)) S(4, RTX_BOX_FAST(4, 5)) \
        S(5, RTX_BOX_FAST(5, 6)) S(6, RTX_BOX_FAST(6, 7)) S(7, RTX_BOX_NEXT(7))
#define RTX_WALK_BLOCK_(n) RTX_WALK_##n
#define RTX_WALK_BLOCK(n) RTX_WALK_BLOCK_(n)
// The sqrt of a primitive step when some lane has 0 <= disc < 2^-96 (scaled by 2^32), out of the
// hot path: placed after the loop, it returns to the step (one taken branch fewer per step).
#define RTX_WALK_COLD(K)                                                     \
        "LS%=_" #K ":\n\t" /* some lane: 0 <= x < 2^-96, scaled by 2^32 */   \
        "v_mul_f32 v13, 0x4f800000, v10\n\t"                                 \
        "v_cndmask_b32_e32 v13, v10, v13, vcc\n\t"                           \
        "v_sqrt_f32_e32 v12, v13\n\t"                                        \
        "s_nop 0\n\t"                                                        \
        "v_add_u32_e32 v9, -1, v12\n\t"                                      \
        "v_add_u32_e32 v11, 1, v12\n\t"                                      \
        "v_fma_f32 v10, -v9, v12, v13\n\t"                                   \
        "v_fma_f32 v15, -v11, v12, v13\n\t"                                  \
        "v_cmp_ge_f32_e64 %[g1], 0, v10\n\t"                                 \
        "v_cmp_lt_f32_e64 %[l1], 0, v15\n\t"                                 \
        "s_nop 0\n\t"                                                        \
        "v_cndmask_b32_e64 v12, v12, v9, %[g1]\n\t"                          \
        "v_cndmask_b32_e64 v12, v12, v11, %[l1]\n\t"                         \
        "v_mul_f32 v9, 0x37800000, v12\n\t" /* x 2^-16 when scaled */        \
        "v_cndmask_b32_e32 v12, v12, v9, vcc\n"                              \
        "s_branch LQ%=_" #K "\n"
#define RTX_COLD_4 RTX_WALK_COLD(0) RTX_WALK_COLD(1) RTX_WALK_COLD(2) RTX_WALK_COLD(3)
#define RTX_COLD_5 RTX_COLD_4 RTX_WALK_COLD(4)
#define RTX_COLD_6 RTX_COLD_5 RTX_WALK_COLD(5)
#define RTX_COLD_8 RTX_COLD_6 RTX_WALK_COLD(6) RTX_WALK_COLD(7)
#define RTX_COLD_BLOCK_(n) RTX_COLD_##n
#define RTX_COLD_BLOCK(n) RTX_COLD_BLOCK_(n)
// QUADS: the scene holds quads (RTX_WALK_STEP_PFQ; the quad table at LDS byte qbase).
// FMA: the near walk's slab form (box_step FMA), no = -(o * (1/d)) per axis (sphere scenes).
template <bool QUADS = false, bool FMA = false>
__device__ __forceinline__ uint64_t walk_phase_asm(Trav& t, const Ray& r, uint32_t end, uint32_t kmin, float tmin,
                                                   uint64_t W, uint64_t P0, uint32_t thresh, uint32_t prim_end,
                                                   uint32_t qbase = 0, const V3 no = V3{0.0f, 0.0f, 0.0f}) {
    static_assert(LDS_B == 32768, "the asm reads the 'b' halves at offset:32768");
    static_assert(!(QUADS && FMA), "the FMA form is the near walk's: sphere scenes");
    uint64_t pm, wm, save, g1, l1, l2, wk;
    uint32_t cnt;
    if constexpr (QUADS) {
        uint64_t qm, qs;
#define S(K, BEND) RTX_WALK_STEP_PFQ(K, RTX_LOAD_LDS, RTX_WAIT_LDS, BEND, RTX_SLABS_SUBMUL)
        asm volatile(RTX_LOAD_LDS "v_cmp_lt_u32_e64 %[wk], %[pos], %[end]\nLW%=:\n\t" RTX_WALK_BLOCK(RTX_ASM_BLOCK_Q) RTX_WALK_VOTE
                     "\n\ts_branch LZ%=\n" RTX_COLD_BLOCK(RTX_ASM_BLOCK_Q) "LZ%=:\n\ts_waitcnt lgkmcnt(0)"
                     : RTX_WALK_OUTS, [qm] "=&s"(qm), [qs] "=&s"(qs)
                     : RTX_WALK_INS, [qbase] "s"(qbase)
                     : RTX_WALK_CLOBBERS, "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27",
                       "v28", "v29", "v30", "v31", "v32", "v33", "v34");
#undef S
    } else if constexpr (FMA) {
#define S(K, BEND) RTX_WALK_STEP_PF(K, RTX_LOAD_LDS, RTX_WAIT_LDS, BEND, RTX_SLABS_FMA)
        asm volatile(RTX_LOAD_LDS "v_cmp_lt_u32_e64 %[wk], %[pos], %[end]\nLW%=:\n\t" RTX_WALK_BLOCK(RTX_ASM_BLOCK) RTX_WALK_VOTE
                     "\n\ts_branch LZ%=\n" RTX_COLD_BLOCK(RTX_ASM_BLOCK) "LZ%=:\n\ts_waitcnt lgkmcnt(0)"
                     : RTX_WALK_OUTS
                     : RTX_WALK_INS, [nox] "v"(no.x), [noy] "v"(no.y), [noz] "v"(no.z)
                     : RTX_WALK_CLOBBERS);
#undef S
    } else {
#define S(K, BEND) RTX_WALK_STEP_PF(K, RTX_LOAD_LDS, RTX_WAIT_LDS, BEND, RTX_SLABS_SUBMUL)
        asm volatile(RTX_LOAD_LDS "v_cmp_lt_u32_e64 %[wk], %[pos], %[end]\nLW%=:\n\t" RTX_WALK_BLOCK(RTX_ASM_BLOCK) RTX_WALK_VOTE
                     "\n\ts_branch LZ%=\n" RTX_COLD_BLOCK(RTX_ASM_BLOCK) "LZ%=:\n\ts_waitcnt lgkmcnt(0)"
                     : RTX_WALK_OUTS
                     : RTX_WALK_INS
                     : RTX_WALK_CLOBBERS);
#undef S
    }
    return pm;  // at_end
}
#undef RTX_WALK_STEP_PF
#undef RTX_WALK_STEP_PFQ
#undef RTX_SLABS_SUBMUL
#undef RTX_SLABS_FMA
#undef RTX_PRIM_RUN_TAIL
#undef RTX_WALK_4
#undef RTX_WALK_5
#undef RTX_WALK_6
#undef RTX_WALK_8
#undef RTX_WALK_BLOCK_
#undef RTX_WALK_BLOCK
#undef RTX_WALK_COLD
#undef RTX_COLD_4
#undef RTX_COLD_5
#undef RTX_COLD_6
#undef RTX_COLD_8
#undef RTX_COLD_BLOCK_
#undef RTX_COLD_BLOCK
#undef RTX_BOX_NEXT
#undef RTX_BOX_FAST
#undef RTX_LOAD_LDS
#undef RTX_WAIT_LDS
#undef RTX_WALK_VOTE
#undef RTX_WALK_OUTS
#undef RTX_WALK_INS
#undef RTX_WALK_CLOBBERS

// Shade the result of segment `seg` (ray.go:36-53, materials.go:33-113).  Returns true
// when the path ends, with its colour in `color`; otherwise r / thr hold the next
// segment.  Lockstep RNG: every hitting lane evaluates block (seg+1, 0) first.
template <bool COUNT, bool QUADS = false, bool NOISE = false>
__device__ __forceinline__ bool shade(const Params& p, const SceneRef E, const Trav& t, uint32_t seg,
                                      Ray& r, V3& thr, V3& acc, const PathRng& rng, Counters& cnt, V3& color,
                                      const Scatter* pre = nullptr) {
    if (t.hit < 0) {  // miss: background (ray.go:52)
        color = add(acc, mul(thr, v3(p.cam.background[0], p.cam.background[1], p.cam.background[2])));
        return true;
    }
    if (COUNT) ++cnt.hits;
    const uint32_t e = seg + 1;
    U4 b0{0u, 0u, 0u, 0u};
    if (pre) b0.x = pre->u0;  // drawn by coop_scatter
    else b0 = rng.block(e, 0);
    const float4 sa = E.a[t.hit];
    const float4 sb = E.b[t.hit];
    const V3 pt = add(scale(r.d, t.closest), r.o);              // ray.go:25-30
    const bool quad = QUADS && __float_as_int(sb.w) == RTX_E_QUAD;
    uint32_t mi;
    V3 n;
    float4 q0, q1, q2, q3;
    if (quad) {                                                 // hittables.go:167-190
        const uint32_t qi = 4u * (uint32_t)__float_as_int(sb.x);
        q0 = E.q[qi];
        q1 = E.q[qi + 1];
        q2 = E.q[qi + 2];
        q3 = E.q[qi + 3];
        mi = (uint32_t)__float_as_int(q0.w);
        n = v3(sa.x, sa.y, sa.z);                               // q.normal
    } else {
        mi = RTX_DEV_SPHERE_MATERIAL(__float_as_int(sb.w));
        n = unit(scale(sub(pt, v3(sa.x, sa.y, sa.z)), sa.w));   // hittables.go:119-120
    }
    const bool front = dot(r.d, n) < 0.0f;                      // hittables.go:23
    const rtx_material m = E.m[mi];
    float u = 0.0f, v = 0.0f;
    const bool inl = m.texture == RTX_DEV_TEX_INLINE;  // SolidColor, colour in m.albedo
    if (p.has_uv && (m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_DIFFUSE_LIGHT) && !inl &&
        E.tx[m.texture].type == RTX_TEX_IMAGE) {           // only an image texture reads UV
        if (quad) {  // (alpha, beta) of the hit, recomputed as quad_test did (hittables.go:181-183)
            const V3 php = sub(pt, v3(q0.x, q0.y, q0.z));
            const V3 w = v3(q3.x, q3.y, q3.z);
            u = dot(w, cross(php, v3(q2.x, q2.y, q2.z)));
            v = dot(w, cross(v3(q1.x, q1.y, q1.z), php));
        } else {
            const UV uv = sphere_uv(n.x, n.y, n.z);
            u = uv.u;
            v = uv.v;
        }
    }
    if (!front) n = scale(n, -1.0f);                            // hittables.go:24-26
    // Metal and Dielectric both start from Unit(dir) and its mirror direction: computed once,
    // so a wave holding both materials runs the sqrt, divide and reflect once, not twice.
    V3 ud = v3(0.0f, 0.0f, 0.0f), mirror = ud;
    if (m.type == RTX_MAT_METAL || m.type == RTX_MAT_DIELECTRIC) {
        ud = unit(r.d);                                         // materials.go:61, 96
        mirror = reflect(ud, n);                                // materials.go:62, 108
    }

    if (m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_METAL) {
        uint32_t draws = 0;
        V3 s;                                                   // shared by both materials
        if (pre) {
            s = pre->s;
            draws = pre->draws;
        } else {
            s = rand_unit_on_sphere(rng, e, b0, draws);
        }
        if (COUNT) cnt.draws += draws;
        if (m.type == RTX_MAT_LAMBERTIAN) {                     // materials.go:33-42
            V3 dir = add(n, s);
            if (near_zero(dir)) dir = n;
            const V3 att = inl ? v3(m.albedo[0], m.albedo[1], m.albedo[2])
                               : texture_value<COUNT, NOISE>(p, E, m.texture, u, v, pt, cnt);
            thr = mul(thr, att);
            r = Ray{pt, dir};
            return false;
        }
        const V3 refl = mirror;                                 // materials.go:60-75
        const V3 sc = add(refl, scale(s, m.fuzz));
        if (!(dot(sc, n) > 0.0f)) {                             // absorbed: Emit() = 0
            color = acc;
            return true;
        }
        thr = mul(thr, v3(m.albedo[0], m.albedo[1], m.albedo[2]));
        r = Ray{pt, sc};
        return false;
    }
    if (m.type == RTX_MAT_DIELECTRIC) {                         // materials.go:91-113
        // 1/ior and both r0 values precomputed per material (ensure_device, rtx_capi.hip)
        const float eta = front ? m.albedo[0] : m.ior;
        const float d = dot(scale(ud, -1.0f), n);
        const float cos_t = d < 1.0f ? d : (d != d ? d : 1.0f); // float32(math.Min(float64(d), 1))
        const float sin_t = (float)__builtin_sqrt(1.0 - (double)(cos_t * cos_t));
        bool refl = sin_t * eta > 1.0f;
        if (!refl) {                                            // short-circuit: draw only here
            const float r0 = front ? m.albedo[1] : m.albedo[2];  // ((1-eta)/(1+eta))^2, materials.go:116-118
            const float rf = r0 + (1.0f - r0) * (float)go_pow5(1.0 - (double)cos_t);
            refl = rf > unit_f32(b0.x);
            if (COUNT) cnt.draws += 1;
        }
        r = Ray{pt, refl ? mirror : refract(ud, n, eta)};          // attenuation (1,1,1)
        return false;
    }
    // DiffuseLight: emit, never scatters (materials.go:303-313)
    const V3 em = inl ? v3(m.albedo[0], m.albedo[1], m.albedo[2]) : texture_value<COUNT, NOISE>(p, E, m.texture, u, v, pt, cnt);
    color = add(acc, mul(thr, em));
    return true;
}

}  // namespace rtxd
