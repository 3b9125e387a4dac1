// Check of the sphere test's fast division (rtx_device.h div_by) against the correctly
// rounded IEEE division hipcc emits (v_div_scale / v_div_fmas / v_div_fixup), on the GPU.
//
// div_by(n, a, y) = fma(fma(-a, n*y, n), y, n*y) with y = RN(1/a).  Claim: for a in
// [2^-60, 2^60], div_by(n, a, y) == n / a bit for bit whenever n / a is a normal finite
// number (Markstein's theorem); any other quotient either stays non-normal or becomes NaN
// for an overflowing one.  The sphere test only uses quotients that pass tmin < t < closest.
//
// Sweep: every one of the 2^23 significands of a, at 41 exponents spread over [-60, 60],
// times 64 numerators per (a) drawn from a hash over exponents [-40, 40] and both signs,
// plus numerators of n = a * t for t near the tmin 0.001 and near 1.  Prints the mismatch
// counts by class of the reference quotient; exit status 1 if any normal quotient differs.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o fastdiv_check fastdiv_check.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float div_by(float n, float a, float y) {
    const float q0 = n * y;
    const float e = __builtin_fmaf(-a, q0, n);
    return __builtin_fmaf(e, y, q0);
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {  // a 32-bit integer hash
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// counts[0]: normal reference quotients that differ; [1]: checked normal quotients;
// [2]: non-normal references (zero, subnormal, inf) where the fast one differs (allowed).
__global__ void check(unsigned long long* counts, int exp_a) {
    const uint32_t mant = blockIdx.x * blockDim.x + threadIdx.x;
    if (mant >= (1u << 23)) return;
    const float a = __uint_as_float(((uint32_t)(exp_a + 127) << 23) | mant);
    const float y = 1.0f / a;
    unsigned long long bad = 0, ok = 0, other = 0;
    for (uint32_t k = 0; k < 64 + 8; ++k) {
        float n;
        const uint32_t h = mix(mant * 977u + k * 0x9E3779B9u + (uint32_t)exp_a * 131u);
        if (k < 64) {
            const int e = (int)(h % 81u) - 40;
            n = __uint_as_float((h & 0x80000000u) | ((uint32_t)(e + 127) << 23) | (mix(h) & 0x7FFFFFu));
        } else {  // quotients near tmin = 0.001 and near 1: n = a * t (rounded)
            const float t = (k & 1) ? 0.001f * (1.0f + (float)(h & 0xFFFF) * 0x1p-20f)
                                    : 1.0f + (float)(h & 0xFFFF) * 0x1p-18f;
            n = a * t;
        }
        const float q = n / a;
        const float f = div_by(n, a, y);
        const uint32_t qb = __float_as_uint(q), fb = __float_as_uint(f);
        const uint32_t ex = (qb >> 23) & 0xFF;
        if (ex != 0 && ex != 0xFF) {
            ++ok;
            if (qb != fb) ++bad;
        } else if (qb != fb) {
            ++other;
        }
    }
    atomicAdd(&counts[0], bad);
    atomicAdd(&counts[1], ok);
    atomicAdd(&counts[2], other);
}

int main() {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 3 * sizeof(unsigned long long)) != hipSuccess) return 2;
    if (hipMemset(d, 0, 3 * sizeof(unsigned long long)) != hipSuccess) return 2;
    for (int e = -60; e <= 60; e += 3) {
        hipLaunchKernelGGL(check, dim3((1u << 23) / 256), dim3(256), 0, 0, d, e);
        if (hipGetLastError() != hipSuccess) return 2;
    }
    unsigned long long h[3] = {0, 0, 0};
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("fastdiv_check: %llu normal quotients checked, %llu differ; %llu non-normal differ (allowed)\n", h[1],
           h[0], h[2]);
    (void)hipFree(d);
    return h[0] == 0 ? 0 : 1;
}
