// scenes.cpp — main.go scene builders restated over the seeded streams.
#include "scenes.h"

#include <algorithm>
#include <cmath>

namespace internal {

namespace {

std::vector<CameraOpt> rand_spheres_camera() {  // main.go:228-239
    return {WithSamplesPerPixel(500),
            WithMaxRayDepth(50),
            WithLookFrom(NewVec3(13, 2, 3)),
            WithLookAt(NewVec3(0, 0, 0)),
            WithFOVDegrees(20),
            WithDefocusAngleDegrees(0.6f),
            WithFocusDist(10),
            WithBackgroundColor(NewVec3(0.7f, 0.8f, 1))};
}

MaterialPtr checkered_ground() {  // main.go:242-243
    auto checkered = NewCheckered(0.32f, NewVec3(0.2f, 0.3f, 0.1f), NewVec3(0.9f, 0.9f, 0.9f));
    return NewLambertian(checkered);
}

// The material draw of main.go:258-270 with configurable thresholds.
MaterialPtr random_material(Rand& randCtx, float matPer, float lamb, float metal) {
    if (matPer < lamb) {
        const Vec3 a = NewVec3Rand32(randCtx);
        const Vec3 b = NewVec3Rand32(randCtx);
        const Vec3 randCol = Mul(a, b);
        return NewLambertian(NewSolidColor(randCol.X, randCol.Y, randCol.Z));
    }
    if (matPer < metal) {
        const Vec3 albedo = NewVec3RandRange32(randCtx, 0.5f, 1);
        const float fuzz = RandF32N(randCtx, 0, 0.5f);
        return NewMetal(albedo, fuzz);
    }
    return NewDielectric(1.5f);
}

void grid_spheres(World& world, Rand& randCtx, float lamb, float metal) {  // main.go:248-276
    Rand& g = GlobalRand();
    const Vec3 p = NewVec3(4, 0.2f, 0);
    for (int i = -11; i < 11; ++i) {
        for (int j = -11; j < 11; ++j) {
            const float matPer = g.Float32();
            const float cx = (float)i + 0.9f * g.Float32();
            const float cz = (float)j + 0.9f * g.Float32();
            const Vec3 center = NewVec3(cx, 0.2f, cz);
            const Vec3 dist = Sub(center, p);
            const float ln = dist.Len();
            if (ln > 0.9f) world.Add(NewSphere(center, 0.2f, random_material(randCtx, matPer, lamb, metal)));
        }
    }
}

}  // namespace

SceneSpec RandSpheres(uint64_t seed) {
    SceneSpec s;
    s.name = "random_spheres";
    s.opts = rand_spheres_camera();
    Seed(seed);                       // rand.Float32() / rand.Intn global source
    auto randCtx = NewRand(seed);     // main.go:246-247
    auto world = NewWorld();
    world->Add(NewSphere(NewVec3(0, -1000, 0), 1000, checkered_ground()));  // :244
    grid_spheres(*world, *randCtx, 0.8f, 0.95f);
    world->Add(NewSphere(NewVec3(0, 1, 0), 1, NewDielectric(1.5f)));                         // :278-279
    world->Add(NewSphere(NewVec3(-4, 1, 0), 1, NewLambertian(NewSolidColor(0.4f, 0.2f, 0.1f))));  // :281-282
    world->Add(NewSphere(NewVec3(4, 1, 0), 1, NewMetal(NewVec3(0.7f, 0.6f, 0.5f), 0)));      // :284-285
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);                                                        // :287
    return s;
}

SceneSpec NestedWorlds(uint64_t seed) {
    SceneSpec s;
    s.name = "nested_worlds";
    s.opts = rand_spheres_camera();
    Seed(seed);
    auto randCtx = NewRand(seed);
    auto flat = NewWorld();
    grid_spheres(*flat, *randCtx, 0.8f, 0.95f);
    // The grid in Worlds of up to 22 spheres (one per grid row, in Add order), handed to
    // NewBVHFromWorld as children; row 3 holds a BVH of its first half and a World of the
    // rest, itself holding a World of two big spheres (hittables.go:55-72 nested 3 deep).
    auto top = NewWorld();
    top->Add(NewSphere(NewVec3(0, -1000, 0), 1000, checkered_ground()));
    const auto& hs = flat->hittables;
    for (size_t r = 0; r * 22 < hs.size(); ++r) {
        auto row = NewWorld();
        const size_t a = r * 22, b = std::min(hs.size(), a + 22);
        if (r == 3 && b - a > 4) {
            auto half = NewWorld();
            for (size_t k = a; k < (a + b) / 2; ++k) half->Add(hs[k]);
            auto rest = NewWorld();
            for (size_t k = (a + b) / 2; k < b; ++k) rest->Add(hs[k]);
            auto big = NewWorld();
            big->Add(NewSphere(NewVec3(0, 1, 0), 1, NewDielectric(1.5f)));
            big->Add(NewSphere(NewVec3(-4, 1, 0), 1, NewLambertian(NewSolidColor(0.4f, 0.2f, 0.1f))));
            rest->Add(big);
            row->Add(NewBVHFromWorld(*half));
            row->Add(rest);
        } else {
            for (size_t k = a; k < b; ++k) row->Add(hs[k]);
        }
        top->Add(row);
    }
    top->Add(NewSphere(NewVec3(4, 1, 0), 1, NewMetal(NewVec3(0.7f, 0.6f, 0.5f), 0)));
    s.world = NewBVHFromWorld(*top);
    return s;
}

SceneSpec StressSpheres(uint64_t seed, int n) {
    SceneSpec s;
    s.name = "stress_100k";
    s.opts = rand_spheres_camera();
    s.opts[0] = WithSamplesPerPixel(100);
    Seed(seed);
    auto randCtx = NewRand(seed);
    auto world = NewWorld();
    world->Add(NewSphere(NewVec3(0, -1000, 0), 1000, checkered_ground()));
    Rand& g = GlobalRand();
    for (int k = 0; k < n; ++k) {
        const float matPer = g.Float32();
        const float cx = -158.0f + 316.0f * g.Float32();
        const float cz = -158.0f + 316.0f * g.Float32();
        world->Add(NewSphere(NewVec3(cx, 0.2f, cz), 0.2f, random_material(*randCtx, matPer, 0.8f, 0.95f)));
    }
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

// The seeded earth-like colour of texel (x, y) of a w x h map, 8-bit RGB.
static void earth_rgb(const float ph[6], uint32_t grain, int x, int y, int w, int h, uint32_t rgb[3]) {
    const float lat = ((float)y + 0.5f) / (float)h;  // 0 top .. 1 bottom
    const float lon = ((float)x + 0.5f) / (float)w;
    const float a = std::sin(6.2831853f * 2.0f * lon + ph[0]) * std::sin(3.1415927f * 3.0f * lat + ph[1]);
    const float b = 0.5f * std::sin(6.2831853f * 5.0f * lon + ph[2]) * std::cos(3.1415927f * 4.0f * lat + ph[3]);
    const float c = 0.25f * std::sin(6.2831853f * 11.0f * lon + ph[4] + 3.0f * lat + ph[5]);
    const float land = a + b + c;
    if (lat < 0.07f || lat > 0.93f) {  // ice caps
        rgb[0] = 225 + (grain & 15); rgb[1] = 230 + (grain & 15); rgb[2] = 240 + (grain & 15);
    } else if (land > 0.35f) {         // land
        rgb[0] = 70 + grain * 2; rgb[1] = 110 + grain; rgb[2] = 40 + grain;
    } else {                           // ocean
        rgb[0] = 10 + grain / 2; rgb[1] = 40 + grain; rgb[2] = 120 + grain * 2;
    }
}

ImagePtr SyntheticEarthRGBA(uint64_t seed, int w, int h) {
    auto img = NewRGBA(Rect(0, 0, w, h));
    Rand r(seed, kStreamTexture);
    // A few seeded low-frequency waves decide land vs ocean; a per-texel draw adds grain.
    float ph[6];
    for (float& v : ph) v = 6.2831853f * r.Float32();
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            uint32_t rgb[3];
            earth_rgb(ph, r.Uint32() & 31u, x, y, w, h, rgb);
            uint8_t* p = &img->Pix[(size_t)(y * img->Stride + 4 * x)];
            p[0] = (uint8_t)rgb[0]; p[1] = (uint8_t)rgb[1]; p[2] = (uint8_t)rgb[2]; p[3] = 255;
        }
    return img;
}

// The planes a baseline JFIF encoder + jpeg.Decode would give for the same map: 4:2:0,
// Y per texel and Cb/Cr per 2x2 block (from the block's top-left texel), with
// integer JFIF forward transforms and a seeded +-1 grain on Y.  Only the decoder side
// (YCbCr.At / RGBA) has to match Go; this is just a deterministic source of planes.
ImagePtr SyntheticEarth(uint64_t seed, int w, int h) {
    auto img = NewYCbCr(Rect(0, 0, w, h), YCbCrSubsampleRatio::R420);
    Rand r(seed, kStreamTexture);
    float ph[6];
    for (float& v : ph) v = 6.2831853f * r.Float32();
    auto clamp8 = [](int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const uint32_t word = r.Uint32();
            uint32_t c[3];
            earth_rgb(ph, word & 31u, x, y, w, h, c);
            const int R = (int)c[0], G = (int)c[1], B = (int)c[2];
            const int yy = (19595 * R + 38470 * G + 7471 * B + (1 << 15)) >> 16;
            img->Y[(size_t)img->YOffset(x, y)] = clamp8(yy + (int)((word >> 5) % 3u) - 1);
            if ((x & 1) == 0 && (y & 1) == 0) {
                const int cb = ((-11056 * R - 21712 * G + 32768 * B + (1 << 15)) >> 16) + 128;
                const int cr = ((32768 * R - 27440 * G - 5328 * B + (1 << 15)) >> 16) + 128;
                const size_t ci = (size_t)img->COffset(x, y);
                img->Cb[ci] = clamp8(cb);
                img->Cr[ci] = clamp8(cr);
            }
        }
    return img;
}

SceneSpec EarthDielectric(uint64_t seed, int tex_w, int tex_h) {
    SceneSpec s;
    s.name = "earth_dielectric";
    s.opts = rand_spheres_camera();
    s.opts[0] = WithSamplesPerPixel(1000);
    s.width = 3840;
    Seed(seed);
    auto randCtx = NewRand(seed);
    auto world = NewWorld();
    world->Add(NewSphere(NewVec3(0, -1000, 0), 1000, checkered_ground()));
    grid_spheres(*world, *randCtx, 0.45f, 0.65f);
    auto earth = NewLambertian(NewImageTexture(SyntheticEarth(seed, tex_w, tex_h)));
    world->Add(NewSphere(NewVec3(0, 1, 0), 1, earth));
    world->Add(NewSphere(NewVec3(-4, 1, 0), 1, NewDielectric(1.5f)));
    world->Add(NewSphere(NewVec3(4, 1, 0), 1, NewMetal(NewVec3(0.7f, 0.6f, 0.5f), 0)));
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

SceneSpec Earth(uint64_t seed, int tex_w, int tex_h, ImagePtr img, float look_z) {  // main.go:80-104
    SceneSpec s;
    s.name = "earth";
    s.opts = {WithSamplesPerPixel(100),
              WithMaxRayDepth(50),
              WithLookFrom(NewVec3(0, 0, look_z)),
              WithLookAt(NewVec3(0, 0, 0)),
              WithFOVDegrees(20),
              WithDefocusAngleDegrees(0),
              WithBackgroundColor(NewVec3(0.7f, 0.8f, 1))};
    Seed(seed);
    auto world = NewWorld();
    auto mat = NewLambertian(NewImageTexture(img ? img : SyntheticEarth(seed, tex_w, tex_h)));
    world->Add(NewSphere(NewVec3(0, 0, 0), 2, mat));
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

SceneSpec QuadDemo(uint64_t seed) {  // main.go:132-160
    SceneSpec s;
    s.name = "quad_demo";
    s.aspect = 16.0f / 9.0f;
    s.width = 400;
    s.opts = {WithSamplesPerPixel(100),
              WithMaxRayDepth(50),
              WithLookFrom(NewVec3(0, 0, 9)),
              WithLookAt(NewVec3(0, 0, 0)),
              WithFOVDegrees(80),
              WithDefocusAngleDegrees(0),
              WithBackgroundColor(NewVec3(0.7f, 0.8f, 1))};
    Seed(seed);  // BVH axis choice (bvh.go:147)
    auto world = NewWorld();
    auto leftRed = NewLambertian(NewSolidColor(1, 0.2f, 0.2f));
    auto backGreen = NewLambertian(NewSolidColor(0.2f, 1, 0.2f));
    auto rightBlue = NewLambertian(NewSolidColor(0.2f, 0.2f, 1));
    auto upperOrange = NewLambertian(NewSolidColor(1, 0.5f, 0));
    auto lowerTeal = NewLambertian(NewSolidColor(0.2f, 0.8f, 0.8f));
    world->Add(NewQuad(NewVec3(-3, -2, 5), NewVec3(0, 0, -4), NewVec3(0, 4, 0), leftRed));
    world->Add(NewQuad(NewVec3(-2, -2, 0), NewVec3(4, 0, 0), NewVec3(0, 4, 0), backGreen));
    world->Add(NewQuad(NewVec3(3, -2, 1), NewVec3(0, 0, 4), NewVec3(0, 4, 0), rightBlue));
    world->Add(NewQuad(NewVec3(-2, 3, 1), NewVec3(4, 0, 0), NewVec3(0, 0, 4), upperOrange));
    world->Add(NewQuad(NewVec3(-2, -3, 5), NewVec3(4, 0, 0), NewVec3(0, 0, -4), lowerTeal));
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

SceneSpec CornellBox(uint64_t seed) {  // main.go:194-225 (main.go:55: the selected scene)
    SceneSpec s;
    s.name = "cornell_box";
    s.aspect = 1.0f;
    s.width = 600;
    s.opts = {WithSamplesPerPixel(200),
              WithMaxRayDepth(50),
              WithLookFrom(NewVec3(278, 278, -800)),
              WithLookAt(NewVec3(278, 278, 0)),
              WithFOVDegrees(40),
              WithDefocusAngleDegrees(0),
              WithBackgroundColor(NewVec3(0, 0, 0))};
    Seed(seed);
    auto world = NewWorld();
    auto red = NewLambertian(NewSolidColor(0.65f, 0.05f, 0.05f));
    auto white = NewLambertian(NewSolidColor(0.73f, 0.73f, 0.73f));
    auto green = NewLambertian(NewSolidColor(0.12f, 0.45f, 0.15f));
    auto light = NewDiffuseLight(NewSolidColor(15, 15, 15));
    world->Add(NewQuad(NewVec3(555, 0, 0), NewVec3(0, 555, 0), NewVec3(0, 0, 555), green));
    world->Add(NewQuad(NewVec3(0, 0, 0), NewVec3(0, 555, 0), NewVec3(0, 0, 555), red));
    world->Add(NewQuad(NewVec3(343, 554, 332), NewVec3(-130, 0, 0), NewVec3(0, 0, -105), light));
    world->Add(NewQuad(NewVec3(0, 0, 0), NewVec3(555, 0, 0), NewVec3(0, 0, 555), white));
    world->Add(NewQuad(NewVec3(555, 555, 555), NewVec3(-555, 0, 0), NewVec3(0, 0, -555), white));
    world->Add(NewQuad(NewVec3(0, 0, 555), NewVec3(555, 0, 0), NewVec3(0, 555, 0), white));
    world->Add(Box(NewVec3(130, 0, 65), NewVec3(295, 165, 230), white));
    world->Add(Box(NewVec3(265, 0, 295), NewVec3(430, 330, 460), white));
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

SceneSpec PerlinDemo(uint64_t seed) {  // main.go:106-130
    SceneSpec s;
    s.name = "perlin_demo";
    s.aspect = 16.0f / 9.0f;
    s.width = 400;
    s.opts = {WithSamplesPerPixel(100),
              WithMaxRayDepth(50),
              WithLookFrom(NewVec3(13, 2, 3)),
              WithLookAt(NewVec3(0, 0, 0)),
              WithFOVDegrees(20),
              WithDefocusAngleDegrees(0),
              WithBackgroundColor(NewVec3(0.7f, 0.8f, 1))};
    Seed(seed);                       // global rand: Permute (materials.go:259-265), BVH axis
    auto randCtx = NewRand(seed);     // main.go:122-123, time-seeded in the reference
    auto world = NewWorld();
    auto perlinTex = NewNoiseTexture(randCtx, 4);
    auto mat = NewLambertian(perlinTex);
    world->Add(NewSphere(NewVec3(0, -1000, 0), 1000, mat));
    world->Add(NewSphere(NewVec3(0, 2, 0), 2, mat));
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

SceneSpec SimpleLightDemo(uint64_t seed) {  // main.go:162-192
    SceneSpec s;
    s.name = "simple_light_demo";
    s.aspect = 16.0f / 9.0f;
    s.width = 400;
    s.opts = {WithSamplesPerPixel(500),
              WithMaxRayDepth(50),
              WithLookFrom(NewVec3(26, 3, 6)),
              WithLookAt(NewVec3(0, 2, 0)),
              WithFOVDegrees(20),
              WithDefocusAngleDegrees(0),
              WithBackgroundColor(NewVec3(0, 0, 0))};
    Seed(seed);
    auto randCtx = NewRand(seed);
    auto world = NewWorld();
    auto perlinTex = NewNoiseTexture(randCtx, 4);
    auto mat = NewLambertian(perlinTex);
    world->Add(NewSphere(NewVec3(0, -1000, 0), 1000, mat));
    world->Add(NewSphere(NewVec3(0, 2, 0), 2, mat));
    auto red = NewLambertian(NewSolidColor(1, 0, 0));
    world->Add(NewSphere(NewVec3(-4, 2, 4), 2, red));
    auto diffLight = NewDiffuseLight(NewSolidColor(4, 4, 4));
    world->Add(NewSphere(NewVec3(0, 7, 0), 2, diffLight));
    s.list = world;
    s.bvh_draw0 = GlobalRand().Drawn();
    s.world = NewBVHFromWorld(*world);
    return s;
}

bool BuildScene(const std::string& name, uint64_t seed, SceneSpec& out) {
    if (name == "random_spheres") out = RandSpheres(seed);
    else if (name == "stress_100k") out = StressSpheres(seed, 100000);
    else if (name == "earth_dielectric") out = EarthDielectric(seed, 2048, 1024);
    else if (name == "earth") out = Earth(seed, 2048, 1024);
    // main.go's earth with the map as an *image.RGBA instead of jpeg.Decode's *image.YCbCr
    else if (name == "earth_rgba") out = Earth(seed, 2048, 1024, SyntheticEarthRGBA(seed, 2048, 1024));
    // main.go's earth seen from -z: the far side, where u = (phi + 5 pi/12) / 2 pi reaches 1
    // (hittables.go:125) and GetTexture reads At(Dx, j), outside the image
    else if (name == "earth_far_side") out = Earth(seed, 2048, 1024, nullptr, -12.0f);
    else if (name == "quad_demo") out = QuadDemo(seed);
    else if (name == "cornell_box") out = CornellBox(seed);
    else if (name == "nested_worlds") out = NestedWorlds(seed);
    else if (name == "perlin_demo") out = PerlinDemo(seed);
    else if (name == "simple_light_demo") out = SimpleLightDemo(seed);
    else return false;
    out.seed = seed;
    return true;
}

}  // namespace internal
