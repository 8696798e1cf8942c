// rt_math.h -- float3 / mat4 arithmetic with the reference's exact evaluation order.
//
// Shared by the host scene code and the gfx950 kernels.  Every routine mirrors the
// template's definition (template/precomp.h) operation for operation, so that a
// kernel compiled with -ffp-contract=off and IEEE div/sqrt produces the same bits
// as the reference's x86-64 SSE build:
//   * dot = (x*x' + y*y') + z*z'                          precomp.h:805
//   * normalize = v * (1.0f / sqrtf(dot(v, v)))            precomp.h:827, 473
//   * std::min / std::max  = (b<a)?b:a / (a<b)?b:a        (slab tests, scene.h:417-446)
//   * template fminf/fmaxf = a<b?a:b / a>b?a:b             precomp.h:471-472
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_HD __host__ __device__ __forceinline__

namespace rt {

// template/common.h:7-12, template/precomp.h:1656-1657
constexpr float kPI = 3.14159265358979323846264f;
constexpr float kINVPI = 0.31830988618379067153777f;
constexpr float kINV2PI = 0.15915494309189533576888f;
constexpr float kTWOPI = 6.28318530717958647692528f;
constexpr float kEPS = 0.0001f;
constexpr float kSKY = 0.00392156862745f;
constexpr float kFLT_EPSILON = 1.192092896e-07f;
// CL_DBL_EPSILON (Primitive.h:128,258) = 2^-52, exactly representable: the
// float-vs-double comparison reduces to a float comparison against it.
constexpr float kDENOM_EPS = 2.220446049250313080847e-16f;

struct f3 { float x, y, z; };

RT_HD f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
RT_HD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RT_HD f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
RT_HD f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
RT_HD f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
RT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_HD f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
RT_HD float length(f3 v) { return sqrtf(dot(v, v)); }
RT_HD f3 normalize(f3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return v * inv; }
RT_HD f3 reflect(f3 i, f3 n) { return i - 2.0f * n * dot(n, i); }
RT_HD float smin(float a, float b) { return (b < a) ? b : a; }
RT_HD float smax(float a, float b) { return (a < b) ? b : a; }
RT_HD float tmin(float a, float b) { return a < b ? a : b; }
RT_HD float tmax(float a, float b) { return a > b ? a : b; }
RT_HD f3 fmin3(f3 a, f3 b) { return mk(tmin(a.x, b.x), tmin(a.y, b.y), tmin(a.z, b.z)); }
RT_HD f3 fmax3(f3 a, f3 b) { return mk(tmax(a.x, b.x), tmax(a.y, b.y), tmax(a.z, b.z)); }
RT_HD float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// TransformPosition / TransformVector: make_float3(float4(a, w) * M), template.cpp:825-839
RT_HD f3 tpos(const float *M, f3 a) {
    return mk(M[0] * a.x + M[1] * a.y + M[2] * a.z + M[3] * 1.0f,
              M[4] * a.x + M[5] * a.y + M[6] * a.z + M[7] * 1.0f,
              M[8] * a.x + M[9] * a.y + M[10] * a.z + M[11] * 1.0f);
}
RT_HD f3 tvec(const float *M, f3 a) {
    return mk(M[0] * a.x + M[1] * a.y + M[2] * a.z + M[3] * 0.0f,
              M[4] * a.x + M[5] * a.y + M[6] * a.z + M[7] * 0.0f,
              M[8] * a.x + M[9] * a.y + M[10] * a.z + M[11] * 0.0f);
}

// RNG: Marsaglia xorshift32 + WangHash seeding, template/template.cpp:673-704
RT_HD uint32_t wang_hash(uint32_t s) {
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u; s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
// InitSeed(base) = WangHash((base + 1) * 17) is a bijection, so exactly one base (1768515948)
// maps to 0, a fixed point of xorshift32: every draw would be 0 and the rejection loops of
// randomInUnitDisk / GetRandomPoint would never end.  With per-pixel seeds that base is
// reached (1080p spp 1: frame 852, pixel (108, 942)), so a zero seed is replaced by the
// reference's global start seed 0x12345678 (template/template.cpp:673); the oracle does the same.
RT_HD uint32_t init_seed(uint32_t base) {
    const uint32_t h = wang_hash((base + 1u) * 17u);
    return h ? h : 0x12345678u;
}
RT_HD uint32_t rnd_u(uint32_t &s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
RT_HD float rnd_f(uint32_t &s) { return (float)rnd_u(s) * 2.3283064365387e-10f; }
// rnd_f(s) * 2.0f - 1.0f with one rounding fewer to issue: the literal above is exactly 2^-32, so
// both products are exact power-of-two scalings and the fma's single rounding is the subtraction's
static_assert(2.3283064365387e-10f == 0x1p-32f, "rnd_f scales by exactly 2^-32");
RT_HD float rnd_sym(uint32_t &s) { return __builtin_fmaf((float)rnd_u(s), 0x1p-31f, -1.0f); }

}  // namespace rt
