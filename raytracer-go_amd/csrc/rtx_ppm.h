// rtx_ppm.h — device PPM encoder (rtx_ppm.hip), used by the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rtxd {
// "P3\n<W> <H>\n255\n" into out (if non-null); returns its length.
uint64_t ppm_header(uint32_t width, uint32_t height, char* out);
// Upper bound of the whole PPM text (header + 63 bytes per pixel).
uint64_t ppm_max_bytes(uint32_t width, uint32_t height);
// Device scratch ppm_encode needs for n pixels.
hipError_t ppm_scratch_bytes(uint64_t n, size_t* bytes);
// Enqueue the pixel lines of d_rgb (W*H*3 float32) at d_text + header_len.  The line
// offsets end up in the scratch: see ppm_text_end.
hipError_t ppm_encode(const float* d_rgb, uint32_t width, uint32_t height, char* d_text, void* d_scratch,
                      size_t scratch_bytes, uint64_t header_len, hipStream_t stream);
// Byte offsets (relative to the first pixel line) of the last line's start and its
// length live at these scratch locations after ppm_encode.
inline const uint64_t* ppm_last_offset(const void* scratch, uint64_t n) {
    return (const uint64_t*)((const unsigned char*)scratch + ((n * 8 + 255) / 256) * 256) + (n - 1);
}
inline const uint32_t* ppm_last_length(const void* scratch, uint64_t n) {
    return (const uint32_t*)((const unsigned char*)scratch + n * 4) + (n - 1);
}
}  // namespace rtxd
