// internal.h — C++ mirror of the reference's Go package `internal`
// (TwFlem/raytracer-go internal/*.go), the host side above the C-ABI.
//
// Go is not available in this image, so the drop-in host is written in C++ with the
// same names, argument meanings and error behaviour as the Go API main.go uses
// (SURVEY.md §8b): NewCamera + functional options, NewWorld/Add, NewBVHFromWorld,
// NewSphere, NewQuad, Box, NewLambertian/Metal/Dielectric/DiffuseLight,
// NewSolidColor/Checkered/ImageTexture/NoiseTexture, Vec3 helpers, RandF32N, and
// (*Camera).Render(world, writer) error.  Render no longer spawns a goroutine per
// pixel: it flattens the Hittable tree into the rtx.h tables and calls librtx.so.
// Go's garbage-collected pointers become std::shared_ptr.
#pragma once
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <memory>
#include <ostream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rtx.h"

namespace internal {

// ---- vec3.go ------------------------------------------------------------------
struct Vec3 {
    float X = 0, Y = 0, Z = 0;
    Vec3 Cpy() const { return *this; }
    void Add(const Vec3& in);
    void Mul(const Vec3& in);
    void Sub(const Vec3& in);
    void Div(const Vec3& in);
    void Scale(float in);
    void Unit();
    float LenSq() const;
    float Len() const;
    std::string String() const;  // "%d %d %d" of int(X), int(Y), int(Z)
    void ToRGB();
    void ToGamma2();
    bool NearZero() const;
    Vec3 GetColor() const { return *this; }
};
using Color = Vec3;

Vec3 NewVec3(float x, float y, float z);
Vec3 NewVec3Zero();
Vec3 NewVec3Unit();
Vec3 Add(Vec3 a, const Vec3& b);
Vec3 Mul(Vec3 a, const Vec3& b);
Vec3 Sub(Vec3 a, const Vec3& b);
Vec3 Div(Vec3 a, const Vec3& b);
Vec3 Scale(Vec3 a, float s);
Vec3 Unit(Vec3 a);
Vec3 Cross(const Vec3& l, const Vec3& r);
float Dot(const Vec3& l, const Vec3& r);

// ---- math/rand, restated as the seeded counter streams of SURVEY.md §8c ----------
// Go seeds these from the clock (main.go:246, camera.go:170); here every stream is
// Philox4x32-10 keyed by a seed, so a render is reproducible and device-exact.
class Rand {
public:
    Rand(uint64_t seed, uint32_t stream) : seed_(seed), stream_(stream) {}
    uint32_t Uint32();
    float Float32();   // [0, 1), 24-bit
    int Intn(int n);   // multiply-shift of one word
    uint64_t Drawn() const { return n_; }

private:
    uint64_t seed_;
    uint32_t stream_;
    uint64_t n_ = 0;
};
constexpr uint32_t kStreamGlobal = 1;  // package-level math/rand (main.go:251-252, bvh.go:147)
constexpr uint32_t kStreamCtx = 2;     // rand.New(rand.NewSource(...)) (main.go:246-247)
constexpr uint32_t kStreamTexture = 3; // synthetic image textures (stand-in for earthmap.jpg)
Rand& GlobalRand();            // the global source
void Seed(uint64_t seed);      // rand.Seed: resets the global source
std::shared_ptr<Rand> NewRand(uint64_t seed);  // a randCtx

float RandF32N(Rand& r, float min, float max);      // math.go:30-32
Vec3 NewVec3Rand32(Rand& r);                        // vec3.go:174-176
Vec3 NewVec3RandRange32(Rand& r, float min, float max);  // vec3.go:178-180

// ---- math.go --------------------------------------------------------------------
template <typename T>
T Clamp(T min, T max, T val) {
    if (val < min) return min;
    if (val > max) return max;
    return val;
}
float MinF32(float a, float b);  // float32(math.Min(float64(a), float64(b)))
float MaxF32(float a, float b);
float ToRadians(float degrees);
constexpr float PiF32 = 3.14159274101257324f;
constexpr double PiO2 = 1.57079632679489661923;

// ---- bvh.go: Interval / Aabb -------------------------------------------------------
struct Interval {
    float min = 0, max = 0;
    bool In(float v, float padding) const { return min - padding < v && v < max + padding; }
};
Interval NewInterval(float min, float max);
struct Aabb {
    Interval x, y, z;
    Aabb GetPaddedAabb() const;
    Aabb GetBounds() const { return *this; }
};
Aabb NewAabb(const Vec3& p1, const Vec3& p2);
Aabb NewAabbFromIntervals(Interval x, Interval y, Interval z);
Aabb NewAabbFromBoxes(const Aabb& b1, const Aabb& b2);

// ---- materials.go: textures ---------------------------------------------------------
class Texture {
public:
    virtual ~Texture() = default;
};
using TexturePtr = std::shared_ptr<Texture>;

class SolidColor : public Texture {
public:
    explicit SolidColor(Color c) : albedo(c) {}
    Color albedo;
};
class Checkered : public Texture {
public:
    Checkered(float s, Vec3 e, Vec3 o) : scale(s), even(e), odd(o) {}
    float scale;
    Color even, odd;
};
// ---- Go's image package: what ImageTexture.GetTexture uses of an image.Image --------
// (Bounds() and At(x, y).RGBA(); materials.go:175-193).  Go's `int` is 64-bit.
struct Rectangle {  // image.Rectangle (image/geom.go)
    int64_t MinX = 0, MinY = 0, MaxX = 0, MaxY = 0;
    int64_t Dx() const { return MaxX - MinX; }
    int64_t Dy() const { return MaxY - MinY; }
    bool In(int64_t x, int64_t y) const { return MinX <= x && x < MaxX && MinY <= y && y < MaxY; }  // Point.In
};
Rectangle Rect(int64_t x0, int64_t y0, int64_t x1, int64_t y1);  // image.Rect (canonicalised)
struct RGBA64 {  // color.Color.RGBA(): alpha-premultiplied 16-bit channels in uint32
    uint32_t r = 0, g = 0, b = 0, a = 0;
};
class Image {  // image.Image
public:
    virtual ~Image() = default;
    virtual Rectangle Bounds() const = 0;
    virtual RGBA64 At(int64_t x, int64_t y) const = 0;  // At(x, y).RGBA()
};
using ImagePtr = std::shared_ptr<Image>;
// *image.RGBA (image/image.go): 4 bytes per pixel, Pix[(y-Min.Y)*Stride + (x-Min.X)*4].
// At outside Bounds is color.RGBA{} (0, 0, 0, 0); color.RGBA.RGBA() widens r to r | r<<8.
class RGBAImage : public Image {
public:
    Rectangle Rect;
    int64_t Stride = 0;
    std::vector<uint8_t> Pix;
    Rectangle Bounds() const override { return Rect; }
    RGBA64 At(int64_t x, int64_t y) const override;
};
std::shared_ptr<RGBAImage> NewRGBA(Rectangle r);  // image.NewRGBA
// *image.YCbCr (image/ycbcr.go), what jpeg.Decode returns for a colour JPEG: a Y plane and
// Cb/Cr planes subsampled by SubsampleRatio.  At outside Bounds is color.YCbCr{} (Y = Cb =
// Cr = 0), whose RGBA() is (0, 34678, 0, 65535) — a green, not black.
enum class YCbCrSubsampleRatio { R444 = 0, R422, R420, R440, R411, R410 };
class YCbCrImage : public Image {
public:
    std::vector<uint8_t> Y, Cb, Cr;
    int64_t YStride = 0, CStride = 0;
    YCbCrSubsampleRatio SubsampleRatio = YCbCrSubsampleRatio::R444;
    Rectangle Rect;
    Rectangle Bounds() const override { return Rect; }
    RGBA64 At(int64_t x, int64_t y) const override;  // YCbCrAt(x, y).RGBA()
    int64_t YOffset(int64_t x, int64_t y) const;
    int64_t COffset(int64_t x, int64_t y) const;
};
std::shared_ptr<YCbCrImage> NewYCbCr(Rectangle r, YCbCrSubsampleRatio ratio);  // image.NewYCbCr
// color.YCbCr{y, cb, cr}.RGBA() (image/color/ycbcr.go): 16-bit JFIF conversion.
RGBA64 YCbCrToRGBA(uint8_t y, uint8_t cb, uint8_t cr);
class ImageTexture : public Texture {
public:
    explicit ImageTexture(ImagePtr im) : img(std::move(im)) {}
    ImagePtr img;
};
// Perlin, materials.go:195-295.  NewPerlin draws the 256 gradient vectors from randCtx
// and the three permutations from the global rand (Permute, :259-265).
struct Perlin {
    std::vector<Vec3> randVec3;
    std::vector<int> permX, permY, permZ;
};
Perlin NewPerlin(Rand& randCtx);
class NoiseTexture : public Texture {  // materials.go:267-295
public:
    NoiseTexture(Perlin p, float s) : perlin(std::move(p)), scale(s) {}
    Perlin perlin;
    float scale;
};
std::shared_ptr<SolidColor> NewSolidColor(float x, float y, float z);
std::shared_ptr<Checkered> NewCheckered(float scale, Vec3 even, Vec3 odd);
std::shared_ptr<ImageTexture> NewImageTexture(ImagePtr img);
std::shared_ptr<NoiseTexture> NewNoiseTexture(std::shared_ptr<Rand> randCtx, float scale);

// ---- materials.go: materials ---------------------------------------------------------
class Material {
public:
    virtual ~Material() = default;
};
using MaterialPtr = std::shared_ptr<Material>;
class Lambertian : public Material {
public:
    explicit Lambertian(TexturePtr t) : albedo(std::move(t)) {}
    TexturePtr albedo;
};
class Metal : public Material {
public:
    Metal(Vec3 a, float f) : albedo(a), fuzz(f) {}
    Color albedo;
    float fuzz;
};
class Dielectric : public Material {
public:
    explicit Dielectric(float ior) : refractiveIndex(ior) {}
    float refractiveIndex;
};
class DiffuseLight : public Material {
public:
    explicit DiffuseLight(TexturePtr t) : emit(std::move(t)) {}
    TexturePtr emit;
};
std::shared_ptr<Lambertian> NewLambertian(TexturePtr albedo);
std::shared_ptr<Metal> NewMetal(Vec3 albedo, float fuzz);
std::shared_ptr<Dielectric> NewDielectric(float refractiveIndex);
std::shared_ptr<DiffuseLight> NewDiffuseLight(TexturePtr emit);

// ---- hittables.go / bvh.go: geometry --------------------------------------------------
class Hittable {
public:
    virtual ~Hittable() = default;
    virtual Aabb GetBounds() const = 0;
};
using HittablePtr = std::shared_ptr<Hittable>;

class Sphere : public Hittable {
public:
    Vec3 Center;
    float Radius = 0;
    MaterialPtr Mat;
    Aabb bBox;
    Aabb GetBounds() const override { return bBox; }
};
class Quad : public Hittable {
public:
    Vec3 Q, u, v, w, normal;
    float D = 0;
    MaterialPtr material;
    Aabb bBox;
    Aabb GetBounds() const override { return bBox; }
};
class World : public Hittable {
public:
    void Add(HittablePtr h);
    void Add(const std::vector<HittablePtr>& hs);
    Aabb GetBounds() const override { return bBox; }
    std::vector<HittablePtr> hittables;
    Aabb bBox;
};
class BVH : public Hittable {
public:
    HittablePtr left, right;
    Aabb bBox;
    Aabb GetBounds() const override { return bBox; }
};
std::shared_ptr<Sphere> NewSphere(Vec3 center, float radius, MaterialPtr mat);
std::shared_ptr<Quad> NewQuad(Vec3 Q, Vec3 u, Vec3 v, MaterialPtr mat);
std::vector<HittablePtr> Box(Vec3 a, Vec3 b, MaterialPtr mat);
std::shared_ptr<World> NewWorld();
std::shared_ptr<BVH> NewBVHFromWorld(const World& w);
std::shared_ptr<BVH> NewBVH(const std::vector<HittablePtr>& hittables);

// ---- camera.go -----------------------------------------------------------------------
// Go's `error`: empty message = nil.
struct Error {
    int code = RTX_OK;
    std::string message;
    explicit operator bool() const { return code != RTX_OK; }
};

class Camera;
using CameraOpt = std::function<void(Camera&)>;

class Camera {
public:
    // (*Camera).Render, camera.go:180-231: writes "P3\nW H\n255\n" and one
    // "r g b\n" line per pixel, rows top to bottom.
    Error Render(const HittablePtr& world, std::ostream& writer);
    // The linear float32 image (pre-gamma), W*H*3 — what Render quantises.
    Error RenderLinear(const HittablePtr& world, std::vector<float>& rgb, rtx_stats* stats = nullptr);
    // Derived state uploaded to the device (camera.go:128-165).
    const rtx_camera& Derived() const { return derived_; }
    int ImageWidth() const { return (int)imageWidth; }
    int ImageHeight() const { return (int)imageHeight; }

    // fields of camera.go:23-52
    float aspectRatio = 0, imageWidth = 0, imageHeight = 0, viewportHeight = 0, viewportWidth = 0;
    int samplesPerPixel = 100, bounceDepth = 50;
    float defocusAngleRadians = 0, focusDistance = 10, fovRadians = (float)PiO2;
    Vec3 viewportU, viewportV, pixelDu, pixelDv, viewportUpperLeft, pixel00, center, lookAt, lookFrom, vup, u, v, w,
        defocusDiskU, defocusDiskV;
    Color background;
    // options that the GPU framework adds
    uint64_t seed = 1;
    int gpus = 1;

    void init();  // camera.go:128-178

private:
    rtx_camera derived_{};
    bool inited_ = false;
};
using CameraPtr = std::shared_ptr<Camera>;

CameraPtr NewCamera(float aspectRatio, int imageWidth, std::initializer_list<CameraOpt> opts = {});
CameraPtr NewCamera(float aspectRatio, int imageWidth, const std::vector<CameraOpt>& opts);
CameraOpt WithSamplesPerPixel(int samples);
CameraOpt WithMaxRayDepth(int depth);
CameraOpt WithFOVDegrees(float fov);
CameraOpt WithLookAt(Vec3 lookAt);
CameraOpt WithLookFrom(Vec3 lookFrom);
CameraOpt WithDefocusAngleDegrees(float degrees);
CameraOpt WithFocusDist(float dist);
CameraOpt WithBackgroundColor(Color color);
CameraOpt WithSeed(uint64_t seed);  // RNG contract key (replaces time.Now seeding)
CameraOpt WithGPUs(int n);          // row-interleave the image over n devices

// ---- flattening (what a cgo Render does before crossing the boundary) -----------------
struct FlatScene {
    std::vector<rtx_bvh_node> nodes;
    std::vector<int32_t> roots;
    std::vector<rtx_sphere> spheres;
    std::vector<rtx_quad> quads;
    std::vector<rtx_material> materials;
    std::vector<rtx_texture> textures;
    std::vector<uint32_t> texels;
    std::vector<rtx_list> lists;       // Worlds nested in the tree (RTX_PRIM_LIST refs)
    std::vector<int32_t> list_refs;
    rtx_scene_desc desc{};  // views into the vectors above (valid while FlatScene lives)
    std::unordered_map<const Material*, uint32_t> mat_index;  // Material -> materials[]
};
Error Flatten(const HittablePtr& world, FlatScene& out);

// PPM body of camera.go:212-215 + 237-251 (ToGamma2, ToRGB, String per pixel).
std::string EncodePPM(const float* rgb, int w, int h);

// file.go
Error Overwrite(const std::string& fname, std::shared_ptr<std::ostream>& out);

}  // namespace internal
