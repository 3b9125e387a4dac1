// image.cpp — the parts of Go's image and image/color packages (Go 1.21) that
// ImageTexture.GetTexture reaches through image.Image (materials.go:175-193): Bounds(),
// At(x, y) and Color.RGBA() for *image.RGBA and *image.YCbCr (jpeg.Decode's type for
// colour JPEGs, file.go:20-28).  Restated from the published Go sources.
#include "internal.h"

namespace internal {

Rectangle Rect(int64_t x0, int64_t y0, int64_t x1, int64_t y1) {  // image/geom.go Rect
    if (x0 > x1) std::swap(x0, x1);
    if (y0 > y1) std::swap(y0, y1);
    return Rectangle{x0, y0, x1, y1};
}

// ---- *image.RGBA --------------------------------------------------------------------
std::shared_ptr<RGBAImage> NewRGBA(Rectangle r) {
    auto m = std::make_shared<RGBAImage>();
    m->Rect = r;
    m->Stride = 4 * r.Dx();
    m->Pix.assign((size_t)(4 * r.Dx() * r.Dy()), 0);
    return m;
}

RGBA64 RGBAImage::At(int64_t x, int64_t y) const {  // RGBAAt, then color.RGBA.RGBA()
    if (!Rect.In(x, y)) return RGBA64{};            // color.RGBA{}
    const size_t i = (size_t)((y - Rect.MinY) * Stride + (x - Rect.MinX) * 4);
    auto w = [](uint32_t c) { return c | c << 8; };
    return RGBA64{w(Pix[i]), w(Pix[i + 1]), w(Pix[i + 2]), w(Pix[i + 3])};
}

// ---- *image.YCbCr ---------------------------------------------------------------------
std::shared_ptr<YCbCrImage> NewYCbCr(Rectangle r, YCbCrSubsampleRatio ratio) {  // image/ycbcr.go
    const int64_t w = r.Dx(), h = r.Dy();
    int64_t cw = w, ch = h;  // yCbCrSize
    switch (ratio) {
    case YCbCrSubsampleRatio::R422: cw = (r.MaxX + 1) / 2 - r.MinX / 2; break;
    case YCbCrSubsampleRatio::R420:
        cw = (r.MaxX + 1) / 2 - r.MinX / 2;
        ch = (r.MaxY + 1) / 2 - r.MinY / 2;
        break;
    case YCbCrSubsampleRatio::R440: ch = (r.MaxY + 1) / 2 - r.MinY / 2; break;
    case YCbCrSubsampleRatio::R411: cw = (r.MaxX + 3) / 4 - r.MinX / 4; break;
    case YCbCrSubsampleRatio::R410:
        cw = (r.MaxX + 3) / 4 - r.MinX / 4;
        ch = (r.MaxY + 1) / 2 - r.MinY / 2;
        break;
    default: break;
    }
    auto m = std::make_shared<YCbCrImage>();
    m->Y.assign((size_t)(w * h), 0);
    m->Cb.assign((size_t)(cw * ch), 0);
    m->Cr.assign((size_t)(cw * ch), 0);
    m->YStride = w;
    m->CStride = cw;
    m->SubsampleRatio = ratio;
    m->Rect = r;
    return m;
}

int64_t YCbCrImage::YOffset(int64_t x, int64_t y) const { return (y - Rect.MinY) * YStride + (x - Rect.MinX); }

// Go's `/` truncates toward zero; the coordinates here are inside Rect.
int64_t YCbCrImage::COffset(int64_t x, int64_t y) const {
    switch (SubsampleRatio) {
    case YCbCrSubsampleRatio::R422: return (y - Rect.MinY) * CStride + (x / 2 - Rect.MinX / 2);
    case YCbCrSubsampleRatio::R420: return (y / 2 - Rect.MinY / 2) * CStride + (x / 2 - Rect.MinX / 2);
    case YCbCrSubsampleRatio::R440: return (y / 2 - Rect.MinY / 2) * CStride + (x - Rect.MinX);
    case YCbCrSubsampleRatio::R411: return (y - Rect.MinY) * CStride + (x / 4 - Rect.MinX / 4);
    case YCbCrSubsampleRatio::R410: return (y / 2 - Rect.MinY / 2) * CStride + (x / 4 - Rect.MinX / 4);
    default: return (y - Rect.MinY) * CStride + (x - Rect.MinX);  // 4:4:4
    }
}

RGBA64 YCbCrImage::At(int64_t x, int64_t y) const {  // YCbCrAt
    if (!Rect.In(x, y)) return YCbCrToRGBA(0, 0, 0);  // color.YCbCr{}
    const size_t yi = (size_t)YOffset(x, y), ci = (size_t)COffset(x, y);
    return YCbCrToRGBA(Y[yi], Cb[ci], Cr[ci]);
}

// color.YCbCr.RGBA(): yy1 = Y * 0x10101 (65536 Y + the rounding adjustment 257 Y), the
// 16.16 JFIF factors 91881, 22554, 46802, 116130, and a clamp of the 24-bit result
// (`uint32(r)&0xff000000 == 0 ? r >> 8 : ^(r >> 31) & 0xffff`).
RGBA64 YCbCrToRGBA(uint8_t y, uint8_t cb, uint8_t cr) {
    const int32_t yy1 = (int32_t)y * 0x10101;
    const int32_t cb1 = (int32_t)cb - 128, cr1 = (int32_t)cr - 128;
    auto clamp16 = [](int32_t v) -> uint32_t {
        if (((uint32_t)v & 0xff000000u) == 0) return (uint32_t)(v >> 8);
        return (uint32_t)(~(v >> 31)) & 0xffffu;
    };
    RGBA64 c;
    c.r = clamp16(yy1 + 91881 * cr1);
    c.g = clamp16(yy1 - 22554 * cb1 - 46802 * cr1);
    c.b = clamp16(yy1 + 116130 * cb1);
    c.a = 0xffff;
    return c;
}

}  // namespace internal
