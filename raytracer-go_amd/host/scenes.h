// scenes.h — the scene builders of main.go (and the BASELINE configs built from them),
// restated with seeded streams instead of time-seeded math/rand.
#pragma once
#include <string>
#include <vector>

#include "internal.h"

namespace internal {

struct SceneSpec {
    std::string name;
    HittablePtr world;  // what main.go passes to camera.Render (a *BVH)
    float aspect = 16.0f / 9.0f;
    int width = 400;
    std::vector<CameraOpt> opts;  // NewCamera options as main.go sets them
    // The World passed to NewBVHFromWorld and the global-rand position at that call
    // (the inputs of the GPU BVH build, rtx_scene_create_spheres), and the seed.
    std::shared_ptr<World> list;
    uint64_t bvh_draw0 = 0;
    uint64_t seed = 0;
};

// randSpheres, main.go:227-289 — the north-star scene (configs 1-3).
SceneSpec RandSpheres(uint64_t seed);
// randSpheres' grid in Worlds nested inside the BVH (a World as a BVH child, hittables.go:55-72;
// main.go never builds one, the API allows it): the ABI 5 list refs.
SceneSpec NestedWorlds(uint64_t seed);
// Config 4: 100 000 r=0.2 spheres, centres uniform on the y=0.2 plane over
// [-158,158)^2 (the randSpheres grid density), materials 80/15/5 as main.go:258-270,
// plus the checkered ground sphere; randSpheres camera.
SceneSpec StressSpheres(uint64_t seed, int n);
// Config 5: randSpheres layout with a Dielectric-heavy mix (45/20/35), the centre
// sphere Lambertian(ImageTexture(synthetic 2048x1024 earth)), defocus 0.6 / focus 10.
SceneSpec EarthDielectric(uint64_t seed, int tex_w, int tex_h);
// earth, main.go:80-104, with a synthetic texture standing in for the missing
// textures/earthmap.jpg (.MISSING_LARGE_BLOBS:2).
// img: the texture (default SyntheticEarth); look_z: the camera's z (main.go: 12).
SceneSpec Earth(uint64_t seed, int tex_w, int tex_h, ImagePtr img = nullptr, float look_z = 12.0f);
// A seeded "earth-like" map (oceans, continents, ice caps) as the *image.YCbCr 4:2:0 a
// colour JPEG decodes to (jpeg.Decode, file.go:20-28): what main.go's earth scene and
// config 5 texture with, standing in for the missing textures/earthmap.jpg.
ImagePtr SyntheticEarth(uint64_t seed, int w, int h);
// The same map as an *image.RGBA (8-bit channels, black outside the bounds).
ImagePtr SyntheticEarthRGBA(uint64_t seed, int w, int h);

// quadDemo, main.go:132-160: five Lambertian quads.
SceneSpec QuadDemo(uint64_t seed);
// cornellBox, main.go:194-225 (the scene main.go:55 selects): 6 walls/light + 2 Boxes
// = 18 quads, DiffuseLight(15) ceiling lamp, black background, 600x600 at 200 spp.
SceneSpec CornellBox(uint64_t seed);

// perlinDemo, main.go:106-130, and simpleLightDemo, main.go:162-192: Perlin
// NoiseTexture(scale 4) spheres (+ a red sphere and a DiffuseLight(4) sphere).
SceneSpec PerlinDemo(uint64_t seed);
SceneSpec SimpleLightDemo(uint64_t seed);

// By name: "random_spheres", "stress_100k", "earth_dielectric", "earth", "earth_rgba",
// "earth_far_side", "quad_demo", "cornell_box", "perlin_demo", "simple_light_demo".
bool BuildScene(const std::string& name, uint64_t seed, SceneSpec& out);

}  // namespace internal
