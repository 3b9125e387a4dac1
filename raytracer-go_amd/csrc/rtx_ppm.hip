// rtx_ppm.hip — the output tail of Camera.Render on the GPU.
//
// Per pixel (camera.go:212-215, vec3.go:141-166): ToGamma2 = float32(math.Sqrt(float64(c))),
// ToRGB = Clamp(0, 1, .) * 255.999 (float32), String = fmt "%d %d %d" of int(.), then
// "\n".  Go's int(float32) truncates toward zero and gives MinInt64 for NaN on amd64;
// Clamp passes NaN through (math.go:20-28), so a NaN channel prints
// "-9223372036854775808".  The P3 header is "P3\n<W> <H>\n255\n" (camera.go:183-188).
//
// Three steps over the float32 RGB framebuffer already in HBM: quantise and measure each
// line (one thread per pixel), an exclusive scan of the line lengths (hipCUB), and
// write each line at its offset.  The text is then one contiguous buffer — the 2M-line
// fmt.Sprintf + channel pipeline of the reference becomes two memory-bound passes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

#include "rtx_ppm.h"

namespace rtxd {

namespace {

constexpr int32_t NAN_CODE = -1;  // stands for int(NaN) = MinInt64
__device__ const char kMinInt64[] = "-9223372036854775808";
constexpr uint32_t kMinInt64Len = 20;

__device__ __forceinline__ int32_t quantize(float x) {
    float g = (float)__builtin_sqrt((double)x);          // ToGamma2, vec3.go:162-166
    if (g < 0.0f) g = 0.0f;                               // Clamp(0, 1, g), math.go:20-28
    else if (g > 1.0f) g = 1.0f;                          //   (NaN compares false: passes)
    const float v = g * 255.999f;                         // ToRGB, vec3.go:145-152
    if (v != v) return NAN_CODE;                          // int(NaN) = MinInt64
    return (int32_t)v;                                    // truncation; v in [0, 255.999]
}

__device__ __forceinline__ uint32_t digits(int32_t q) {
    if (q == NAN_CODE) return kMinInt64Len;
    return q >= 100 ? 3u : (q >= 10 ? 2u : 1u);
}

__device__ __forceinline__ char* put(char* o, int32_t q) {
    if (q == NAN_CODE) {
        for (uint32_t i = 0; i < kMinInt64Len; ++i) o[i] = kMinInt64[i];
        return o + kMinInt64Len;
    }
    if (q >= 100) *o++ = (char)('0' + q / 100);
    if (q >= 10) *o++ = (char)('0' + (q / 10) % 10);
    *o++ = (char)('0' + q % 10);
    return o;
}

__global__ __launch_bounds__(256) void ppm_measure(const float* __restrict__ rgb, uint64_t n,
                                                   uint32_t* __restrict__ q, uint32_t* __restrict__ len) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int32_t r = quantize(rgb[3 * i]), g = quantize(rgb[3 * i + 1]), b = quantize(rgb[3 * i + 2]);
    // packed: 3 x 9 bits (0..255, 511 = NaN)
    q[i] = ((uint32_t)(r & 511)) | ((uint32_t)(g & 511) << 9) | ((uint32_t)(b & 511) << 18);
    len[i] = digits(r) + digits(g) + digits(b) + 3;  // two spaces and the newline
}

__device__ __forceinline__ int32_t unpack(uint32_t v) { return v == 511u ? NAN_CODE : (int32_t)v; }

__global__ __launch_bounds__(256) void ppm_write(const uint32_t* __restrict__ q, const uint64_t* __restrict__ off,
                                                 uint64_t n, char* __restrict__ text) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = q[i];
    char* o = text + off[i];
    o = put(o, unpack(v & 511u));
    *o++ = ' ';
    o = put(o, unpack((v >> 9) & 511u));
    *o++ = ' ';
    o = put(o, unpack((v >> 18) & 511u));
    *o = '\n';
}

// Lengths widened to 64-bit offsets by the scan's output type.
struct Widen {
    __device__ __forceinline__ uint64_t operator()(uint32_t x) const { return x; }
};

}  // namespace

uint64_t ppm_header(uint32_t width, uint32_t height, char* out) {
    char buf[64];
    int n = snprintf(buf, sizeof(buf), "P3\n%u %u\n255\n", width, height);
    if (out) for (int i = 0; i < n; ++i) out[i] = buf[i];
    return (uint64_t)n;
}

uint64_t ppm_max_bytes(uint32_t width, uint32_t height) {
    return ppm_header(width, height, nullptr) + (uint64_t)width * height * (3 * kMinInt64Len + 3);
}

hipError_t ppm_scratch_bytes(uint64_t n, size_t* bytes) {
    size_t scan = 0;
    hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t*> in(nullptr, Widen{});
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan, in, (uint64_t*)nullptr, (int)n);
    if (e != hipSuccess) return e;
    *bytes = n * (4 + 4 + 8) + scan + 256;
    return hipSuccess;
}

hipError_t ppm_encode(const float* d_rgb, uint32_t width, uint32_t height, char* d_text, void* d_scratch,
                      size_t scratch_bytes, uint64_t header_len, hipStream_t stream) {
    const uint64_t n = (uint64_t)width * height;
    if (n == 0) return hipSuccess;
    auto* base = (unsigned char*)d_scratch;
    auto* q = (uint32_t*)base;
    auto* len = (uint32_t*)(base + n * 4);
    auto* off = (uint64_t*)(base + ((n * 8 + 255) / 256) * 256);
    void* scan_tmp = (void*)(off + n);
    const size_t used = (size_t)((unsigned char*)scan_tmp - base);
    size_t scan_bytes = scratch_bytes > used ? scratch_bytes - used : 0;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(ppm_measure, dim3(blocks), dim3(256), 0, stream, d_rgb, n, q, len);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t*> in(len, Widen{});
    e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, in, off, (int)n, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ppm_write, dim3(blocks), dim3(256), 0, stream, q, off, n, d_text + header_len);
    return hipGetLastError();
}

}  // namespace rtxd
