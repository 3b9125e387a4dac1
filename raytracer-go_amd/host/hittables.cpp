// hittables.cpp — constructors of internal/hittables.go.  The intersection code
// (Sphere.Hit :96-132, World.Hit :55-72) runs on the device.
#include <algorithm>
#include "internal.h"

namespace internal {

void World::Add(HittablePtr h) {  // hittables.go:48-53
    hittables.push_back(h);
    bBox = NewAabbFromBoxes(bBox, h->GetBounds());
}
void World::Add(const std::vector<HittablePtr>& hs) {
    for (const auto& h : hs) Add(h);
}
std::shared_ptr<World> NewWorld() { return std::make_shared<World>(); }  // hittables.go:44-46

std::shared_ptr<Sphere> NewSphere(Vec3 center, float radius, MaterialPtr mat) {  // hittables.go:85-94
    auto s = std::make_shared<Sphere>();
    const Vec3 rvec = NewVec3(radius, radius, radius);
    s->Center = center;
    s->Radius = radius;
    s->Mat = std::move(mat);
    s->bBox = NewAabb(Add(center, Scale(rvec, -1)), Add(center, rvec));
    return s;
}

std::shared_ptr<Quad> NewQuad(Vec3 Q, Vec3 u, Vec3 v, MaterialPtr mat) {  // hittables.go:149-165
    auto q = std::make_shared<Quad>();
    const Vec3 n = Cross(u, v);
    const Vec3 norm = Unit(n);
    q->Q = Q;
    q->u = u;
    q->v = v;
    q->w = Scale(n, 1 / Dot(n, n));
    q->material = std::move(mat);
    q->bBox = NewAabb(Q, Add(Add(Q, u), v)).GetPaddedAabb();
    q->D = Dot(norm, Q);
    q->normal = norm;
    return q;
}

std::vector<HittablePtr> Box(Vec3 a, Vec3 b, MaterialPtr mat) {  // hittables.go:200-216
    const Vec3 mn = NewVec3(MinF32(a.X, b.X), MinF32(a.Y, b.Y), MinF32(a.Z, b.Z));
    const Vec3 mx = NewVec3(MaxF32(a.X, b.X), MaxF32(a.Y, b.Y), MaxF32(a.Z, b.Z));
    const Vec3 dx = NewVec3(mx.X - mn.X, 0, 0);
    const Vec3 dy = NewVec3(0, mx.Y - mn.Y, 0);
    const Vec3 dz = NewVec3(0, 0, mx.Z - mn.Z);
    return {
        NewQuad(NewVec3(mn.X, mn.Y, mx.Z), dx, dy, mat),
        NewQuad(NewVec3(mx.X, mn.Y, mx.Z), Scale(dz, -1), dy, mat),
        NewQuad(NewVec3(mx.X, mn.Y, mn.Z), Scale(dx, -1), dy, mat),
        NewQuad(NewVec3(mn.X, mn.Y, mn.Z), dz, dy, mat),
        NewQuad(NewVec3(mn.X, mx.Y, mx.Z), dx, Scale(dz, -1), mat),
        NewQuad(NewVec3(mn.X, mn.Y, mn.Z), dx, dz, mat),
    };
}

// ---- materials.go constructors ---------------------------------------------------------
std::shared_ptr<SolidColor> NewSolidColor(float x, float y, float z) { return std::make_shared<SolidColor>(NewVec3(x, y, z)); }
std::shared_ptr<Checkered> NewCheckered(float scale, Vec3 even, Vec3 odd) { return std::make_shared<Checkered>(scale, even, odd); }
std::shared_ptr<ImageTexture> NewImageTexture(ImagePtr img) { return std::make_shared<ImageTexture>(std::move(img)); }
static std::vector<int> Permute(std::vector<int> p) {  // materials.go:259-265, global rand
    for (int i = (int)p.size() - 1; i > 0; --i) {
        const int target = GlobalRand().Intn(i);
        std::swap(p[i], p[target]);
    }
    return p;
}

Perlin NewPerlin(Rand& randCtx) {  // materials.go:202-216
    const int pointCount = 256;
    Perlin per;
    per.randVec3.resize(pointCount);
    for (int i = 0; i < pointCount; ++i) per.randVec3[i] = NewVec3RandRange32(randCtx, -1, 1);
    std::vector<int> nums(pointCount);  // GetNums, :251-257
    for (int i = 0; i < pointCount; ++i) nums[i] = i;
    per.permX = Permute(nums);
    per.permY = Permute(nums);
    per.permZ = Permute(nums);
    return per;
}

std::shared_ptr<NoiseTexture> NewNoiseTexture(std::shared_ptr<Rand> randCtx, float scale) {  // :290-295
    return std::make_shared<NoiseTexture>(NewPerlin(*randCtx), scale);
}
std::shared_ptr<Lambertian> NewLambertian(TexturePtr albedo) { return std::make_shared<Lambertian>(std::move(albedo)); }
std::shared_ptr<Metal> NewMetal(Vec3 albedo, float fuzz) { return std::make_shared<Metal>(albedo, fuzz); }
std::shared_ptr<Dielectric> NewDielectric(float ior) { return std::make_shared<Dielectric>(ior); }
std::shared_ptr<DiffuseLight> NewDiffuseLight(TexturePtr emit) { return std::make_shared<DiffuseLight>(std::move(emit)); }

}  // namespace internal
