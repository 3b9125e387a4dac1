// camera.cpp — internal/camera.go: options, init, and Render as the drop-in boundary.
//
// Render keeps the reference's contract (P3 header, one "r g b" line per pixel, rows
// top to bottom, `error` return) but replaces the goroutine-per-pixel fan-out and the
// TwFlem/pipe ordering stages (camera.go:198-230) with one call into librtx.so.
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

#include "internal.h"

namespace internal {

CameraOpt WithSamplesPerPixel(int samples) { return [=](Camera& c) { c.samplesPerPixel = samples; }; }  // :56
CameraOpt WithMaxRayDepth(int depth) { return [=](Camera& c) { c.bounceDepth = depth; }; }                // :62
CameraOpt WithFOVDegrees(float fov) { return [=](Camera& c) { c.fovRadians = ToRadians(fov); }; }       // :68
CameraOpt WithLookAt(Vec3 lookAt) { return [=](Camera& c) { c.lookAt = lookAt; }; }                     // :74
CameraOpt WithLookFrom(Vec3 lookFrom) { return [=](Camera& c) { c.lookFrom = lookFrom; }; }             // :80
CameraOpt WithDefocusAngleDegrees(float d) { return [=](Camera& c) { c.defocusAngleRadians = ToRadians(d); }; }  // :86
CameraOpt WithFocusDist(float dist) { return [=](Camera& c) { c.focusDistance = dist; }; }              // :92
CameraOpt WithBackgroundColor(Color color) { return [=](Camera& c) { c.background = color; }; }         // :98
CameraOpt WithSeed(uint64_t seed) { return [=](Camera& c) { c.seed = seed; }; }
CameraOpt WithGPUs(int n) { return [=](Camera& c) { c.gpus = n; }; }

CameraPtr NewCamera(float aspectRatio, int imageWidth, const std::vector<CameraOpt>& opts) {  // :104-126
    auto c = std::make_shared<Camera>();
    c->aspectRatio = aspectRatio;
    c->imageWidth = (float)imageWidth;
    c->fovRadians = (float)PiO2;
    c->samplesPerPixel = 100;
    c->bounceDepth = 50;
    c->focusDistance = 10;
    c->defocusAngleRadians = 0;
    c->lookAt = NewVec3(0, 0, 0);
    c->lookFrom = NewVec3(0, 0, -1);
    c->vup = NewVec3(0, 1, 0);
    c->background = NewVec3(0, 0, 0);
    for (const auto& fn : opts) fn(*c);
    c->init();
    return c;
}
CameraPtr NewCamera(float aspectRatio, int imageWidth, std::initializer_list<CameraOpt> opts) {
    return NewCamera(aspectRatio, imageWidth, std::vector<CameraOpt>(opts));
}

void Camera::init() {  // camera.go:128-165 (the worker pool of :167-175 has no equivalent)
    if (inited_) return;
    inited_ = true;
    center = lookFrom.Cpy();
    const Vec3 dist = Sub(lookFrom, lookAt);
    const float h = (float)std::tan((double)(fovRadians / 2.0f));
    viewportHeight = 2.0f * h * focusDistance;
    imageHeight = (float)(std::floor((double)imageWidth) / (double)aspectRatio);
    if (imageHeight < 1) imageHeight = 1;
    viewportWidth = viewportHeight * (imageWidth / imageHeight);
    w = Unit(dist);
    u = Unit(Cross(vup, w));
    v = Cross(w, u);
    viewportU = Scale(u, viewportWidth);
    viewportV = Scale(v, -viewportHeight);
    pixelDu = viewportU.Cpy();
    pixelDu.Scale(1 / imageWidth);
    pixelDv = viewportV.Cpy();
    pixelDv.Scale(1 / imageHeight);
    viewportUpperLeft = center.Cpy();
    viewportUpperLeft.Sub(Scale(w, focusDistance));
    viewportUpperLeft.Sub(Scale(viewportU, 0.5f));
    viewportUpperLeft.Sub(Scale(viewportV, 0.5f));
    pixel00 = viewportUpperLeft.Cpy();
    pixel00.Add(Scale(Add(pixelDu, pixelDv), 0.5f));
    const float defocusRadius = focusDistance * (float)std::tan((double)(defocusAngleRadians / 2.0f));
    defocusDiskU = Scale(u, defocusRadius);
    defocusDiskV = Scale(v, defocusRadius);

    std::memset(&derived_, 0, sizeof(derived_));
    derived_.image_width = (uint32_t)(int)imageWidth;
    derived_.image_height = (uint32_t)(int)imageHeight;
    derived_.samples_per_pixel = (uint32_t)samplesPerPixel;
    derived_.max_depth = bounceDepth > 0 ? (uint32_t)bounceDepth : 0u;
    derived_.defocus_angle = defocusAngleRadians;
    auto put = [](float* d, const Vec3& s) { d[0] = s.X; d[1] = s.Y; d[2] = s.Z; };
    put(derived_.center, center);
    put(derived_.pixel00, pixel00);
    put(derived_.pixel_du, pixelDu);
    put(derived_.pixel_dv, pixelDv);
    put(derived_.defocus_disk_u, defocusDiskU);
    put(derived_.defocus_disk_v, defocusDiskV);
    put(derived_.background, background);
}

static Error rtx_error(int code) {
    Error e;
    e.code = code;
    e.message = rtx_last_error();
    return e;
}

Error Camera::RenderLinear(const HittablePtr& world, std::vector<float>& rgb, rtx_stats* stats) {
    init();
    FlatScene fs;
    if (Error e = Flatten(world, fs)) return e;
    if (samplesPerPixel <= 0) return Error{RTX_ERR_INVALID_ARG, "samplesPerPixel must be > 0"};
    rtx_scene* scene = nullptr;
    if (int rc = rtx_scene_create(&fs.desc, &scene)) return rtx_error(rc);
    rgb.assign((size_t)derived_.image_width * derived_.image_height * 3, 0.0f);
    const int rc = rtx_render(scene, &derived_, seed, gpus, rgb.data(), stats);
    Error e;
    if (rc) e = rtx_error(rc);
    rtx_scene_destroy(scene);
    return e;
}

std::string EncodePPM(const float* rgb, int w, int h) {  // camera.go:212-215, 242
    std::string out;
    out.reserve((size_t)w * h * 12);
    for (size_t p = 0; p < (size_t)w * h; ++p) {
        Vec3 c = NewVec3(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2]);
        c.ToGamma2();
        c.ToRGB();
        out += c.String();
        out += '\n';
    }
    return out;
}

Error Camera::Render(const HittablePtr& world, std::ostream& writer) {  // camera.go:180-231
    init();
    const int W = (int)imageWidth, H = (int)imageHeight;
    std::ostringstream head;
    head << "P3\n" << W << " " << H << "\n255\n";  // :183-188, written before rendering
    writer << head.str();
    if (!writer) return Error{RTX_ERR_INVALID_ARG, "write failed"};
    if (gpus <= 1) {  // one device: render and encode on the GPU (rtx_render_ppm)
        FlatScene fs;
        if (Error e = Flatten(world, fs)) return e;
        if (samplesPerPixel <= 0) return Error{RTX_ERR_INVALID_ARG, "samplesPerPixel must be > 0"};
        rtx_scene* scene = nullptr;
        if (int rc = rtx_scene_create(&fs.desc, &scene)) return rtx_error(rc);
        std::string text(rtx_ppm_max_bytes((uint32_t)W, (uint32_t)H), '\0');
        uint64_t len = 0;
        const int rc = rtx_render_ppm(scene, &derived_, seed, text.data(), text.size(), &len, nullptr);
        rtx_scene_destroy(scene);
        if (rc) return rtx_error(rc);
        const size_t hl = head.str().size();  // the text repeats the header: skip it
        writer.write(text.data() + hl, (std::streamsize)(len - hl));  // :237-251
        if (!writer) return Error{RTX_ERR_INVALID_ARG, "write failed"};
        return Error{};
    }
    std::vector<float> rgb;
    if (Error e = RenderLinear(world, rgb)) return e;
    writer << EncodePPM(rgb.data(), W, H);  // :237-251 (multi-GPU: gathered on the host)
    if (!writer) return Error{RTX_ERR_INVALID_ARG, "write failed"};
    return Error{};
}

Error Overwrite(const std::string& fname, std::shared_ptr<std::ostream>& out) {  // file.go:9-18
    std::remove(fname.c_str());
    auto f = std::make_shared<std::ofstream>(fname, std::ios::binary | std::ios::trunc);
    if (!f->is_open()) return Error{RTX_ERR_INVALID_ARG, "open " + fname + ": cannot create"};
    out = f;
    return Error{};
}

}  // namespace internal
