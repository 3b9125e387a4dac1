// main.cpp — the reference's main.go (main.go:22-78) on the GPU path.
//
//   rtx_main [scene] [width] [spp] [gpus]      scene: cornell_box (default, as main.go:55
//                                              selects), random_spheres, quad_demo, earth,
//                                              perlin_demo, simple_light_demo,
//                                              earth_dielectric, stress_100k
// Writes out/img.ppm (file.go Overwrite) and prints the wall time like main.go:77.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "internal.h"
#include "scenes.h"

using namespace internal;

int main(int argc, char** argv) {
    const auto now = std::chrono::steady_clock::now();
    const std::string name = argc > 1 ? argv[1] : "cornell_box";  // main.go:55
    const int width = argc > 2 ? std::atoi(argv[2]) : 0;
    const int spp = argc > 3 ? std::atoi(argv[3]) : 0;
    const int gpus = argc > 4 ? std::atoi(argv[4]) : 1;

    std::shared_ptr<std::ostream> f;
    if (Error e = Overwrite("out/img.ppm", f)) {  // main.go:43-46 panics here
        std::fprintf(stderr, "panic: %s\n", e.message.c_str());
        return 2;
    }
    SceneSpec spec;
    if (!BuildScene(name, 1, spec)) {
        std::fprintf(stderr, "panic: unknown scene %s\n", name.c_str());
        return 2;
    }
    std::vector<CameraOpt> opts = spec.opts;
    if (spp > 0) opts.push_back(WithSamplesPerPixel(spp));
    opts.push_back(WithGPUs(gpus));
    auto camera = NewCamera(spec.aspect, width > 0 ? width : spec.width, opts);
    if (Error e = camera->Render(spec.world, *f)) {  // main.go:74-76
        std::fprintf(stderr, "panic: %s\n", e.message.c_str());
        return 2;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - now).count();
    std::printf("Finished in: %.3fs\n", s);  // main.go:77
    return 0;
}
