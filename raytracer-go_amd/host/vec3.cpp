// vec3.cpp — internal/vec3.go, internal/math.go and the seeded math/rand streams.
#include <cmath>
#include <cstdio>

#include "internal.h"

namespace internal {

void Vec3::Add(const Vec3& in) { X += in.X; Y += in.Y; Z += in.Z; }  // vec3.go:43-47
void Vec3::Mul(const Vec3& in) { X *= in.X; Y *= in.Y; Z *= in.Z; }  // vec3.go:55-59
void Vec3::Sub(const Vec3& in) { X -= in.X; Y -= in.Y; Z -= in.Z; }  // vec3.go:67-71
void Vec3::Div(const Vec3& in) { X /= in.X; Y /= in.Y; Z /= in.Z; }  // vec3.go:79-83
void Vec3::Scale(float in) { X *= in; Y *= in; Z *= in; }            // vec3.go:91-95
void Vec3::Unit() {                                                  // vec3.go:103-107
    float lensq = LenSq();
    float l = (float)std::sqrt((double)lensq);
    Scale(1.0f / l);
}
float Vec3::LenSq() const { return X * X + Y * Y + Z * Z; }           // vec3.go:115-117
float Vec3::Len() const { return (float)std::sqrt((double)LenSq()); } // vec3.go:119-121

// int(float32) on amd64 (CVTTSS2SQ): truncation; NaN / out of range -> MinInt64.
static long long go_int(float f) {
    if (std::isnan(f) || f >= 9223372036854775808.0f || f < -9223372036854775808.0f) return INT64_MIN;
    return (long long)f;
}
std::string Vec3::String() const {  // vec3.go:141-143
    char buf[80];
    std::snprintf(buf, sizeof(buf), "%lld %lld %lld", go_int(X), go_int(Y), go_int(Z));
    return buf;
}
void Vec3::ToRGB() {  // vec3.go:145-152
    X = Clamp(0.0f, 1.0f, X);
    Y = Clamp(0.0f, 1.0f, Y);
    Z = Clamp(0.0f, 1.0f, Z);
    X *= 255.999f;
    Y *= 255.999f;
    Z *= 255.999f;
}
void Vec3::ToGamma2() {  // vec3.go:162-166
    X = (float)std::sqrt((double)X);
    Y = (float)std::sqrt((double)Y);
    Z = (float)std::sqrt((double)Z);
}
bool Vec3::NearZero() const {  // vec3.go:170-172
    const float eps = 1e-8f;
    return (float)std::fabs((double)X) < eps && (float)std::fabs((double)Y) < eps && (float)std::fabs((double)Z) < eps;
}

Vec3 NewVec3(float x, float y, float z) { return Vec3{x, y, z}; }
Vec3 NewVec3Zero() { return Vec3{0, 0, 0}; }
Vec3 NewVec3Unit() { return Vec3{1, 1, 1}; }
Vec3 Add(Vec3 a, const Vec3& b) { a.Add(b); return a; }
Vec3 Mul(Vec3 a, const Vec3& b) { a.Mul(b); return a; }
Vec3 Sub(Vec3 a, const Vec3& b) { a.Sub(b); return a; }
Vec3 Div(Vec3 a, const Vec3& b) { a.Div(b); return a; }
Vec3 Scale(Vec3 a, float s) { a.Scale(s); return a; }
Vec3 Unit(Vec3 a) { a.Unit(); return a; }
Vec3 Cross(const Vec3& l, const Vec3& r) {  // vec3.go:129-135
    return Vec3{l.Y * r.Z - l.Z * r.Y, l.Z * r.X - l.X * r.Z, l.X * r.Y - l.Y * r.X};
}
float Dot(const Vec3& l, const Vec3& r) { return l.X * r.X + l.Y * r.Y + l.Z * r.Z; }  // vec3.go:137-139

// ---- math.go --------------------------------------------------------------------
static double go_min(double a, double b) {
    if (std::isnan(a) || std::isnan(b)) return NAN;
    if (a == 0 && b == 0) return std::signbit(a) ? a : b;
    return a < b ? a : b;
}
static double go_max(double a, double b) {
    if (std::isnan(a) || std::isnan(b)) return NAN;
    if (a == 0 && b == 0) return std::signbit(a) ? b : a;
    return a > b ? a : b;
}
float MinF32(float a, float b) { return (float)go_min(a, b); }  // math.go:38-40
float MaxF32(float a, float b) { return (float)go_max(a, b); }  // math.go:42-44
// radRatio = float32(math.Pi / 180.0), math.go:46 (single and double rounding agree).
float ToRadians(float degrees) { return degrees * (float)(3.14159265358979323846 / 180.0); }

// ---- seeded streams ------------------------------------------------------------------
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
    }
}

uint32_t Rand::Uint32() {
    const uint64_t blk = n_ >> 2;
    uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0x80000000u | stream_};  // disjoint from pixel counters
    philox4x32_10(c, (uint32_t)seed_, (uint32_t)(seed_ >> 32));
    return c[n_++ & 3u];
}
float Rand::Float32() { return (float)(Uint32() >> 8) * 0x1.0p-24f; }
int Rand::Intn(int n) { return (int)(((uint64_t)Uint32() * (uint64_t)n) >> 32); }

static Rand g_global(1, kStreamGlobal);
Rand& GlobalRand() { return g_global; }
void Seed(uint64_t seed) { g_global = Rand(seed, kStreamGlobal); }
std::shared_ptr<Rand> NewRand(uint64_t seed) { return std::make_shared<Rand>(seed, kStreamCtx); }

float RandF32N(Rand& r, float min, float max) { return min + r.Float32() * (max - min); }  // math.go:30-32
Vec3 NewVec3Rand32(Rand& r) {  // vec3.go:174-176, arguments evaluated left to right
    const float x = r.Float32(), y = r.Float32(), z = r.Float32();
    return NewVec3(x, y, z);
}
Vec3 NewVec3RandRange32(Rand& r, float min, float max) {  // vec3.go:178-180
    const float x = RandF32N(r, min, max), y = RandF32N(r, min, max), z = RandF32N(r, min, max);
    return NewVec3(x, y, z);
}

}  // namespace internal
