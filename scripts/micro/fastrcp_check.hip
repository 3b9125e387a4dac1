// Exhaustive check of a short correctly rounded float32 reciprocal against the IEEE division
// hipcc emits for 1.0f / x (v_div_scale / v_div_fmas / v_div_fixup), on the GPU.
//
// rcp_fast(x) = fma(fma(-x, y0, 1), y0, y0) with y0 = v_rcp_f32(x) (within 1 ulp): one
// Newton-Raphson step evaluated with fma.  Every one of the 2^32 bit patterns is tried; the
// mismatches are counted by class of x: |x| in [2^-125, 2^125] (both x and 1/x normal, away
// from the ends of the range), and the rest (zero, subnormal, huge, inf, NaN).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o fastrcp_check fastrcp_check.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float rcp_fast(float x) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}

// counts[0]: mid-range mismatches, [1]: mid-range checked, [2]: other mismatches, [3]: first
// mid-range mismatching bit pattern + 1 (0: none)
__global__ void check(unsigned long long* counts, uint32_t hi) {
    const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const float q = 1.0f / x;
    const float f = rcp_fast(x);
    const uint32_t ex = (bits >> 23) & 0xFF;
    const bool mid = ex >= 127 - 125 && ex <= 127 + 125;
    const bool same = __float_as_uint(q) == __float_as_uint(f) || (q != q && f != f);
    if (mid) {
        atomicAdd(&counts[1], 1ull);
        if (!same) {
            atomicAdd(&counts[0], 1ull);
            atomicCAS(&counts[3], 0ull, (unsigned long long)bits + 1ull);
        }
    } else if (!same) {
        atomicAdd(&counts[2], 1ull);
    }
}

int main() {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 4 * sizeof(unsigned long long)) != hipSuccess) return 2;
    if (hipMemset(d, 0, 4 * sizeof(unsigned long long)) != hipSuccess) return 2;
    for (uint32_t hi = 0; hi < 256; ++hi) {
        hipLaunchKernelGGL(check, dim3((1u << 24) / 256), dim3(256), 0, 0, d, hi);
        if (hipGetLastError() != hipSuccess) return 2;
    }
    unsigned long long h[4] = {0, 0, 0, 0};
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("fastrcp_check: %llu mid-range inputs, %llu differ (first 0x%08llx); %llu other inputs differ\n", h[1],
           h[0], h[3] ? h[3] - 1 : 0ull, h[2]);
    (void)hipFree(d);
    return h[0] == 0 ? 0 : 1;
}
