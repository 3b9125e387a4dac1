// capi_host.cpp — C entry points of librtxhost.so (include/rtx_host.h).
#include <cstring>
#include <fstream>

#include "../../include/rtx_host.h"
#include "internal.h"
#include "scenes.h"

using namespace internal;

struct rtxhost_scene {
    SceneSpec spec;
    FlatScene flat;
};

namespace {
thread_local std::string g_err;
int set_err(const Error& e) {
    g_err = e.message;
    return e.code;
}
}  // namespace

extern "C" {

const char* rtxhost_last_error(void) { return g_err.c_str(); }

int rtxhost_build_scene(const char* name, uint64_t seed, rtxhost_scene** out) {
    g_err.clear();
    if (!name || !out) return set_err(Error{RTX_ERR_INVALID_ARG, "NULL argument"});
    auto* s = new rtxhost_scene();
    if (!BuildScene(name, seed, s->spec)) {
        delete s;
        return set_err(Error{RTX_ERR_INVALID_ARG, std::string("unknown scene ") + name});
    }
    if (Error e = Flatten(s->spec.world, s->flat)) {
        delete s;
        return set_err(e);
    }
    *out = s;
    return RTX_OK;
}

void rtxhost_scene_free(rtxhost_scene* s) { delete s; }

int64_t rtxhost_scene_world_spheres(const rtxhost_scene* s, rtx_sphere* out, uint64_t cap, uint64_t* bvh_draw0,
                                    uint64_t* seed) {
    g_err.clear();
    if (!s || !s->spec.list) return set_err(Error{RTX_ERR_INVALID_ARG, "scene has no World list"});
    const auto& hs = s->spec.list->hittables;
    for (size_t i = 0; i < hs.size(); ++i) {
        auto sp = dynamic_cast<const Sphere*>(hs[i].get());
        if (!sp) return set_err(Error{RTX_ERR_UNSUPPORTED, "the World holds a non-sphere"});
        auto it = s->flat.mat_index.find(sp->Mat.get());
        if (it == s->flat.mat_index.end()) return set_err(Error{RTX_ERR_INVALID_ARG, "material not flattened"});
        if (out && i < cap) {
            rtx_sphere r{};
            r.center[0] = sp->Center.X; r.center[1] = sp->Center.Y; r.center[2] = sp->Center.Z;
            r.radius = sp->Radius;
            r.material = it->second;
            out[i] = r;
        }
    }
    if (bvh_draw0) *bvh_draw0 = s->spec.bvh_draw0;
    if (seed) *seed = s->spec.seed;
    return (int64_t)hs.size();
}

const rtx_scene_desc* rtxhost_scene_desc(const rtxhost_scene* s) { return s ? &s->flat.desc : nullptr; }

int rtxhost_synthetic_earth_ycbcr(uint64_t seed, int32_t w, int32_t h, uint8_t* y, uint8_t* cb, uint8_t* cr) {
    g_err.clear();
    if (w <= 0 || h <= 0 || !y || !cb || !cr) return set_err(Error{RTX_ERR_INVALID_ARG, "bad arguments"});
    auto img = std::dynamic_pointer_cast<YCbCrImage>(SyntheticEarth(seed, w, h));
    std::memcpy(y, img->Y.data(), img->Y.size());
    std::memcpy(cb, img->Cb.data(), img->Cb.size());
    std::memcpy(cr, img->Cr.data(), img->Cr.size());
    return RTX_OK;
}

void rtxhost_ycbcr_rgba(uint8_t y, uint8_t cb, uint8_t cr, uint32_t out[4]) {
    const RGBA64 c = YCbCrToRGBA(y, cb, cr);
    out[0] = c.r;
    out[1] = c.g;
    out[2] = c.b;
    out[3] = c.a;
}

static CameraPtr make_camera(const SceneSpec& spec, int32_t w, int32_t spp, int32_t depth, uint64_t seed, int gpus) {
    std::vector<CameraOpt> opts = spec.opts;
    if (spp > 0) opts.push_back(WithSamplesPerPixel(spp));
    if (depth > 0) opts.push_back(WithMaxRayDepth(depth));
    opts.push_back(WithSeed(seed));
    opts.push_back(WithGPUs(gpus));
    return NewCamera(spec.aspect, w > 0 ? w : spec.width, opts);
}

int rtxhost_scene_camera(const rtxhost_scene* s, int32_t image_width, int32_t spp, int32_t depth, rtx_camera* out) {
    g_err.clear();
    if (!s || !out) return set_err(Error{RTX_ERR_INVALID_ARG, "NULL argument"});
    *out = make_camera(s->spec, image_width, spp, depth, 1, 1)->Derived();
    return RTX_OK;
}

int rtxhost_render_ppm(const char* scene_name, uint64_t scene_seed, int32_t image_width, int32_t spp, int32_t depth,
                       uint64_t render_seed, int32_t n_gpus, const char* path) {
    g_err.clear();
    if (!scene_name || !path) return set_err(Error{RTX_ERR_INVALID_ARG, "NULL argument"});
    SceneSpec spec;
    if (!BuildScene(scene_name, scene_seed, spec))
        return set_err(Error{RTX_ERR_INVALID_ARG, std::string("unknown scene ") + scene_name});
    std::shared_ptr<std::ostream> f;
    if (Error e = Overwrite(path, f)) return set_err(e);
    auto cam = make_camera(spec, image_width, spp, depth, render_seed, n_gpus);
    if (Error e = cam->Render(spec.world, *f)) return set_err(e);
    f->flush();
    return RTX_OK;
}

uint64_t rtxhost_ppm_encode(const float* rgb, uint32_t w, uint32_t h, char* out, uint64_t cap) {
    if (!rgb) return 0;
    const std::string s = EncodePPM(rgb, (int)w, (int)h);
    if (out && cap) std::memcpy(out, s.data(), std::min<uint64_t>(cap, s.size()));
    return s.size();
}

}  // extern "C"
