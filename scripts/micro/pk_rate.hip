// Microbenchmark: throughput of v_mul_f32 vs v_pk_mul_f32 / v_pk_add_f32 (and the
// quarter-rate v_mad_u64_u32) on gfx950, 8 independent chains per wave, full occupancy.
// Build: hipcc --offload-arch=gfx950 -O3 -o pk_rate pk_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// 8 independent scalar multiplies per iteration
__global__ void scalar_mul(float* out, int iters) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    const float m = 0.99999f;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_mul_f32 %0, %0, %8\n\tv_mul_f32 %1, %1, %8\n\tv_mul_f32 %2, %2, %8\n\tv_mul_f32 %3, %3, %8\n\t"
            "v_mul_f32 %4, %4, %8\n\tv_mul_f32 %5, %5, %8\n\tv_mul_f32 %6, %6, %8\n\tv_mul_f32 %7, %7, %8"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(m));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 8 independent packed multiplies per iteration (16 products)
__global__ void packed_mul(float* out, int iters) {
    float2 a0 = make_float2(threadIdx.x * 1e-3f, 1), a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;
    const float2 m = make_float2(0.99999f, 0.99998f);
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_pk_mul_f32 %0, %0, %8\n\tv_pk_mul_f32 %1, %1, %8\n\tv_pk_mul_f32 %2, %2, %8\n\tv_pk_mul_f32 %3, %3, %8\n\t"
            "v_pk_mul_f32 %4, %4, %8\n\tv_pk_mul_f32 %5, %5, %8\n\tv_pk_mul_f32 %6, %6, %8\n\tv_pk_mul_f32 %7, %7, %8"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(m));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0.x + a1.x + a2.x + a3.x + a4.y + a5.y + a6.y + a7.y;
}

// 8 independent packed adds with a negated, op_sel-broadcast operand
__global__ void packed_sub_bcast(float* out, int iters) {
    float2 a0 = make_float2(threadIdx.x * 1e-3f, 1), a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;
    const float2 m = make_float2(1e-6f, 2e-6f);
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_pk_add_f32 %0, %0, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %1, %1, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %2, %2, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %3, %3, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %4, %4, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %5, %5, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %6, %6, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %7, %7, %8 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(m));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0.x + a1.x + a2.x + a3.x + a4.y + a5.y + a6.y + a7.y;
}

// 8 independent 32x32->64 multiply-adds (Philox's product)
__global__ void mad_u64(float* out, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t m = 0xD2511F53u, x = threadIdx.x * 7u;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_mad_u64_u32 %0, s[0:1], %8, %9, %0\n\tv_mad_u64_u32 %1, s[0:1], %8, %9, %1\n\t"
            "v_mad_u64_u32 %2, s[0:1], %8, %9, %2\n\tv_mad_u64_u32 %3, s[0:1], %8, %9, %3\n\t"
            "v_mad_u64_u32 %4, s[0:1], %8, %9, %4\n\tv_mad_u64_u32 %5, s[0:1], %8, %9, %5\n\t"
            "v_mad_u64_u32 %6, s[0:1], %8, %9, %6\n\tv_mad_u64_u32 %7, s[0:1], %8, %9, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(m), "v"(x)
            : "s0", "s1");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

template <typename K>
float run(K kern, float* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters);  // warm
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    int dev = 0, cus = 0, clk_khz = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    const int blocks = cus * 8;  // 8 waves per SIMD (4 waves per block x 8 blocks per CU / 4 SIMDs)
    const int iters = 20000;
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
    const double waves_per_simd = (double)blocks * 4 / (cus * 4);
    const double instr = 8.0 * iters * waves_per_simd;  // per SIMD
    struct {
        const char* name;
        float ms;
    } r[] = {{"v_mul_f32", run(scalar_mul, out, blocks, iters)},
             {"v_pk_mul_f32", run(packed_mul, out, blocks, iters)},
             {"v_pk_add_f32 op_sel/neg", run(packed_sub_bcast, out, blocks, iters)},
             {"v_mad_u64_u32", run(mad_u64, out, blocks, iters)}};
    for (auto& x : r) {
        const double cycles = x.ms * 1e-3 * clk_khz * 1e3;
        printf("%-26s %8.3f ms  %6.2f cycles per wave64 instruction per SIMD (clock %d MHz)\n", x.name, x.ms,
               cycles / instr, clk_khz / 1000);
    }
    hipFree(out);
    return 0;
}
