// Microbenchmark: cost of a wave64 VALU chain as a function of the exec mask.
// Build: hipcc --offload-arch=gfx950 -O3 -o exec_mask exec_mask.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void chain(float* out, int iters) {
    const uint32_t lane = threadIdx.x & 63u;
    bool on;
    if (MODE == 0) on = true;                   // all 64 lanes
    else if (MODE == 1) on = lane < 32;         // low half only
    else if (MODE == 2) on = (lane & 1) == 0;   // every other lane (both halves)
    else if (MODE == 3) on = lane < 16;         // quarter, low half
    else on = lane == 0;                        // one lane
    float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.9999f, d = 0.5f;
    if (on) {
        for (int i = 0; i < iters; ++i) {
            a = a * b + c; b = b * c + d; c = c * d + a; d = d * a + b;
            a = a * b + c; b = b * c + d; c = c * d + a; d = d * a + b;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

template <int MODE>
float run(float* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    float* out;
    const int blocks = 256 * 16;  // 16 waves... 4 waves per block, 64 waves per CU
    hipMalloc(&out, sizeof(float) * blocks * 256);
    const int iters = 4096;
    const char* names[] = {"all 64", "low 32", "alternate 32", "low 16", "one lane"};
    float t[5] = {run<0>(out, blocks, iters), run<1>(out, blocks, iters), run<2>(out, blocks, iters),
                  run<3>(out, blocks, iters), run<4>(out, blocks, iters)};
    for (int m = 0; m < 5; ++m) printf("%-14s %8.3f ms  (%.2f x all-64)\n", names[m], t[m], t[m] / t[0]);
    return 0;
}
