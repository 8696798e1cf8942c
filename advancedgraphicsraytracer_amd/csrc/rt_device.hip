// rt_device.hip -- gfx950 kernels and the device half of the C-ABI.
//
// Hot path: Renderer::Tick -> Camera::GetPrimaryRay -> Renderer::Trace
// -> Scene::IntersectBVH / IsOccluded -> Primitive::Intersect / Hit, plus
// NextEventDirectIllumination, the Diffuse / Mirror / Dielectric / Checkerboard / Light
// materials, the sky lookup, the running-average accumulator and the RGB8 pack -- all in
// ONE kernel launch per frame (k_render).  Launch shape: 256-thread workgroups of four
// wave64s, one wave per 8x8 screen tile (the reference's PACKET_SIZE 64 / SQRT_PACKET_SIZE 8,
// Ray.h:3-5), one lane per pixel.  No MFMA: this is branchy scalar fp32.
//
// Device scene layout in HBM (built once by rt_scene_create):
//   nodes  : the reference's 32-byte BVHNode array (root 0, node 1 unused, sibling pairs
//            64-byte aligned) with (leftFirst, count) replaced by one packed word
//            (leftFirst << 8 | count) so a 64-byte sibling-pair load carries everything
//            the traversal needs;
//   prims  : leaf order (primitiveIndices applied), 48 B per slot: triangle A, B-A, C-A
//            (host-computed, bit-identical to the reference's per-test subtraction) and
//            the original primitive id -- no index indirection in the leaf loop;
//   shade  : per primitive id, 32 B: geometric normal (triangles, host-computed with the
//            reference's normalize(cross(..))), sphere centre / 1/r, material id;
//   per-lane traversal stack: LDS, [depth][256 lanes] u32, conflict-free.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rt_internal.h"
#include "rt_libm.h"

namespace rt {

enum : uint32_t { T_TRI = 4, T_SPH = 0, T_PLANE = 1, T_CUBE = 2, T_QUAD = 3 };
enum : int { F_DIFFUSE = 0, F_SPECULAR = 1, F_MIX = 2, F_DIELECTRIC = 3, F_LIGHT = 4 };

struct DevMaterial {
    int kind, flag;
    float c0[3], c1[3];
    float ior, diffuse, specular;
    uint32_t tex_off, tex_w, tex_h;   // TextureMaterial: texels at SceneView::tex + tex_off
};

struct SceneView {
    const float4 *__restrict__ nodes;   // 2 float4 per node
    const float4 *__restrict__ prims;   // 3 float4 per leaf slot
    const float4 *__restrict__ shade;   // 2 float4 per primitive id
    const DevMaterial *__restrict__ mats;
    const uint32_t *__restrict__ sky;
    const float4 *__restrict__ xprims;  // cubes / quads: 8 float4 each (Minv rows, M rows, data)
    const uint32_t *__restrict__ tex;   // all TextureMaterial texels
    uint32_t sky_w, sky_h;
    int sky_const;
    float sky_rgb[3];
    float light_M[12];                  // prim 0 Transform rows 0..2
    float light_c[3];
    float light_r, light_r2, light_invr;
    int light_mat;
    int light_quad;                     // prim 0 is a quad (else a sphere)
    float light_qsize, light_area;      // quad data[0].x; Primitive::GetArea
    float light_N[3];                   // quad normal TransformVector((0,-1,0), M)
    uint32_t root_word;
    int bounds_finite;                  // every node bound is a finite float
    uint32_t stack_entries;             // LDS stack entries per lane
    uint32_t node_f4;                   // node array size in float4s
    int wave_primary;                   // camera rays take the wave-coherent walk
};

struct FrameArgs {
    float cam_pos[3], cam_tl[3], cam_tr[3], cam_bl[3];
    float lens, rw, rh;
    uint32_t W, H, spp, depth, frame, reset;
    uint32_t shard, nshards, tiles_x, ntiles_local;
    int packed_out;
    float4 *acc;
    uint32_t *out;
    unsigned long long *counters;       // [0] shadow rays, [1] bounce rays
};

struct DRay {
    f3 O, D, rD;
    float t;
    int obj;
    int inside;
    float u, v;
};

__device__ __forceinline__ DRay make_ray(f3 O, f3 D, float t) {   // Ray.h:9-16
    DRay r;
    r.O = O; r.D = D; r.t = t; r.obj = -1; r.inside = 0; r.u = 0.0f; r.v = 0.0f;
    r.rD = mk(1 / D.x, 1 / D.y, 1 / D.z);
    return r;
}

// cold-path transcendentals (textured sky, sphere u/v): correctly rounded float via the
// double functions, as the oracle does; the hot cos/sin/exp come from rt_libm.h
__device__ __forceinline__ float cr_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
__device__ __forceinline__ float cr_acos(float x) { return (float)acos((double)x); }
__device__ __forceinline__ float cr_asin(float x) { return (float)asin((double)x); }

// float -> uint the way the reference's x86-64 build converts: (uint32)(int64)trunc(f)
__device__ __forceinline__ uint32_t f2u_wrap(float f) {
    if (!(f == f) || f >= 9.2e18f || f <= -9.2e18f) return 0u;
    return (uint32_t)(long long)f;
}

// ------------------------------------------------------------------ slab tests (scene.h:414-450)
// EXACT: the reference's std::min/std::max selects, NaN behaviour included.
// FAST (chosen per wave when every active ray has a finite origin and finite 1/D and the
// scene's node bounds are NaN-free): no slab product can then be NaN, and on non-NaN
// inputs the selects equal IEEE minNum/maxNum up to the sign of a zero result, which no
// consumer can observe (the values are only compared) -- so v_min3/v_max3 give the
// identical decisions with a third of the instructions.
template <bool FAST>
__device__ __forceinline__ void slab(const DRay &r, float4 a, float4 b, float &tmn, float &tmx) {
    float tx1 = (a.x - r.O.x) * r.rD.x, tx2 = (a.w - r.O.x) * r.rD.x;
    float ty1 = (a.y - r.O.y) * r.rD.y, ty2 = (b.x - r.O.y) * r.rD.y;
    float tz1 = (a.z - r.O.z) * r.rD.z, tz2 = (b.y - r.O.z) * r.rD.z;
    if (FAST) {
        tmn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
        tmx = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    } else {
        tmn = smin(tx1, tx2); tmx = smax(tx1, tx2);
        tmn = smax(tmn, smin(ty1, ty2)); tmx = smin(tmx, smax(ty1, ty2));
        tmn = smax(tmn, smin(tz1, tz2)); tmx = smin(tmx, smax(tz1, tz2));
    }
}
template <bool FAST>
__device__ __forceinline__ float slab_dist(const DRay &r, float4 a, float4 b) {
    float tmn, tmx;
    slab<FAST>(r, a, b, tmn, tmx);
    return (tmx >= tmn && tmn < r.t && tmx > 0) ? tmn : 1e30f;
}
template <bool FAST>
__device__ __forceinline__ bool slab_hit(const DRay &r, float4 a, float4 b) {
    float tmn, tmx;
    slab<FAST>(r, a, b, tmn, tmx);
    return tmx >= tmn && tmn < r.t && tmx > 0;
}
__device__ __forceinline__ bool ray_finite(const DRay &r) {
    return isfinite(r.O.x) && isfinite(r.O.y) && isfinite(r.O.z) && isfinite(r.rD.x) && isfinite(r.rD.y) &&
           isfinite(r.rD.z);
}

// ------------------------------------------------------------------ primitive tests (Primitive.h:64-279)
// TransformPosition / TransformVector with the matrix as three float4 rows (same order of
// operations as rt_math.h tpos / tvec)
__device__ __forceinline__ f3 tpos_rows(float4 r0, float4 r1, float4 r2, f3 a) {
    return mk(r0.x * a.x + r0.y * a.y + r0.z * a.z + r0.w * 1.0f, r1.x * a.x + r1.y * a.y + r1.z * a.z + r1.w * 1.0f,
              r2.x * a.x + r2.y * a.y + r2.z * a.z + r2.w * 1.0f);
}
__device__ __forceinline__ f3 tvec_rows(float4 r0, float4 r1, float4 r2, f3 a) {
    return mk(r0.x * a.x + r0.y * a.y + r0.z * a.z + r0.w * 0.0f, r1.x * a.x + r1.y * a.y + r1.z * a.z + r1.w * 0.0f,
              r2.x * a.x + r2.y * a.y + r2.z * a.z + r2.w * 0.0f);
}
// CUBE slab test in object space (Primitive.h:87-110 / 196-235); false on a miss
__device__ __forceinline__ bool cube_slab(const float4 *x, const DRay &r, float &tmin_o, float &tmax_o) {
    const f3 O = tpos_rows(x[0], x[1], x[2], r.O), D = tvec_rows(x[0], x[1], x[2], r.D);
    const float4 d0 = x[6], d1 = x[7];
    const float rDx = 1 / D.x, rDy = 1 / D.y, rDz = 1 / D.z;
    const bool sx = D.x < 0, sy = D.y < 0, sz = D.z < 0;
    float tmin = ((sx ? d1.x : d0.x) - O.x) * rDx;
    float tmax = ((sx ? d0.x : d1.x) - O.x) * rDx;
    const float tymin = ((sy ? d1.y : d0.y) - O.y) * rDy;
    const float tymax = ((sy ? d0.y : d1.y) - O.y) * rDy;
    if (tmin > tymax || tymin > tmax) return false;
    tmin = smax(tmin, tymin);
    tmax = smin(tmax, tymax);
    const float tzmin = ((sz ? d1.z : d0.z) - O.z) * rDz;
    const float tzmax = ((sz ? d0.z : d1.z) - O.z) * rDz;
    if (tmin > tzmax || tzmin > tmax) return false;
    tmin_o = smax(tmin, tzmin);
    tmax_o = smin(tmax, tzmax);
    return true;
}
// QUAD plane distance in object space (Primitive.h:111-117 / 236-247)
__device__ __forceinline__ float quad_t(const float4 *x, const DRay &r, f3 &O, f3 &D) {
    O = tpos_rows(x[0], x[1], x[2], r.O);
    D = tvec_rows(x[0], x[1], x[2], r.D);
    return O.y / -D.y;
}
// cubes and quads (off the hot path): Intersect; `tie` as in prim_intersect_t
__device__ __noinline__ void xprim_intersect(const SceneView &S, uint32_t type, uint32_t xi, int id, DRay &r,
                                             bool &tie) {
    const float4 *x = S.xprims + 8 * xi;
    if (type == T_CUBE) {   // the acceptance test is on tmax (Primitive.h:221-233)
        float tmin, tmax;
        if (!cube_slab(x, r, tmin, tmax)) return;
        float t;
        if (tmin > kEPS) t = tmin;
        else if (tmax > kEPS) t = tmax;
        else return;
        if (tmax < r.t) { r.t = t; r.obj = id; }
        else if (tmax == r.t) tie = true;
    } else {
        f3 O, D;
        const float t = quad_t(x, r, O, D);
        const float size = x[6].x;
        if (t <= r.t && t > kEPS) {
            const f3 I = O + t * D;
            if (I.x > -size && I.x < size && I.z > -size && I.z < size) {
                if (t == r.t) tie = true;
                else { r.t = t; r.obj = id; r.u = 0.0f; r.v = 0.0f; }   // u, v unset there: 0
            }
        }
    }
}
__device__ __noinline__ bool xprim_hit(const SceneView &S, uint32_t type, uint32_t xi, const DRay &r) {
    const float4 *x = S.xprims + 8 * xi;
    if (type == T_CUBE) {
        float tmin, tmax;
        if (!cube_slab(x, r, tmin, tmax)) return false;
        return (tmin > kEPS || tmax > kEPS) && tmax < r.t;
    }
    f3 O, D;
    const float t = quad_t(x, r, O, D);   // the quad's extent is not tested (reference quirk)
    return t < r.t && t > kEPS;
}
__device__ __forceinline__ void prim_intersect(const SceneView &S, uint32_t k, DRay &r) {
    float4 p0 = S.prims[3 * k], p1 = S.prims[3 * k + 1];
    uint32_t type = __float_as_uint(p1.w);
    int id = __float_as_int(p0.w);
    if (type == T_TRI) {
        float4 p2 = S.prims[3 * k + 2];
        f3 A = mk(p0.x, p0.y, p0.z), AB = mk(p1.x, p1.y, p1.z), AC = mk(p2.x, p2.y, p2.z);
        float denom = dot(cross(r.D, AC), AB);
        if (fabsf(denom) < kDENOM_EPS) return;
        f3 AO = r.O - A;
        float u = dot(cross(-r.D, AO), AC) / denom;
        if (u < 0 || u > 1) return;
        float v = dot(cross(-r.D, AB), AO) / denom;
        if (v < 0 || u + v > 1) return;
        float t = dot(cross(AO, AB), AC) / denom;
        if (t < r.t && t > kEPS) { r.t = t; r.obj = id; r.u = u; r.v = v; }
    } else if (type == T_SPH) {
        f3 oc = r.O - mk(p0.x, p0.y, p0.z);
        float b = dot(oc, r.D);
        float c = dot(oc, oc) - p1.x;
        float d = b * b - c;
        if (d <= 0) return;
        d = sqrtf(d);
        float t = -b - d;
        if (!(t < r.t && t > kEPS)) {
            t = d - b;
            if (!(t < r.t && t > kEPS)) return;
        }
        r.t = t; r.obj = id;            // u, v filled in after traversal (finish_uv)
    } else if (type == T_PLANE) {
        f3 N = mk(p0.x, p0.y, p0.z);
        float t = -(dot(r.O, N) + p1.x) / (dot(r.D, N));
        if (t < r.t && t > kEPS) { r.t = t; r.obj = id; }
    } else {
        bool tie = false;
        xprim_intersect(S, type, __float_as_uint(p1.x), id, r, tie);
    }
}

// prim_intersect plus `tie`: set when the candidate distance equals the current r.t
// exactly (a second primitive at the same distance: the visiting order would decide).
__device__ __forceinline__ void prim_intersect_t(const SceneView &S, uint32_t k, DRay &r, bool &tie) {
    float4 p0 = S.prims[3 * k], p1 = S.prims[3 * k + 1];
    uint32_t type = __float_as_uint(p1.w);
    int id = __float_as_int(p0.w);
    if (type == T_TRI) {
        float4 p2 = S.prims[3 * k + 2];
        f3 A = mk(p0.x, p0.y, p0.z), AB = mk(p1.x, p1.y, p1.z), AC = mk(p2.x, p2.y, p2.z);
        float denom = dot(cross(r.D, AC), AB);
        if (fabsf(denom) < kDENOM_EPS) return;
        f3 AO = r.O - A;
        float u = dot(cross(-r.D, AO), AC) / denom;
        if (u < 0 || u > 1) return;
        float v = dot(cross(-r.D, AB), AO) / denom;
        if (v < 0 || u + v > 1) return;
        float t = dot(cross(AO, AB), AC) / denom;
        if (t <= r.t && t > kEPS) {
            if (t == r.t) tie = true;
            else { r.t = t; r.obj = id; r.u = u; r.v = v; }
        }
    } else if (type == T_SPH) {
        f3 oc = r.O - mk(p0.x, p0.y, p0.z);
        float b = dot(oc, r.D);
        float c = dot(oc, oc) - p1.x;
        float d = b * b - c;
        if (d <= 0) return;
        d = sqrtf(d);
        float t = -b - d;
        if (t == r.t && t > kEPS) tie = true;
        if (!(t < r.t && t > kEPS)) {
            t = d - b;
            if (t == r.t && t > kEPS) tie = true;
            if (!(t < r.t && t > kEPS)) return;
        }
        r.t = t; r.obj = id;
    } else if (type == T_PLANE) {
        f3 N = mk(p0.x, p0.y, p0.z);
        float t = -(dot(r.O, N) + p1.x) / (dot(r.D, N));
        if (t == r.t && t > kEPS) tie = true;
        if (t < r.t && t > kEPS) { r.t = t; r.obj = id; }
    } else {
        xprim_intersect(S, type, __float_as_uint(p1.x), id, r, tie);
    }
}

__device__ __forceinline__ bool prim_hit(const SceneView &S, uint32_t k, const DRay &r) {
    float4 p0 = S.prims[3 * k], p1 = S.prims[3 * k + 1];
    uint32_t type = __float_as_uint(p1.w);
    if (type == T_TRI) {
        float4 p2 = S.prims[3 * k + 2];
        f3 A = mk(p0.x, p0.y, p0.z), AB = mk(p1.x, p1.y, p1.z), AC = mk(p2.x, p2.y, p2.z);
        float denom = dot(cross(r.D, AC), AB);
        if (fabsf(denom) < kDENOM_EPS) return false;
        f3 AO = r.O - A;
        float u = dot(cross(-r.D, AO), AC) / denom;
        if (u < 0 || u > 1) return false;
        float v = dot(cross(-r.D, AB), AO) / denom;
        if (v < 0 || u + v > 1) return false;
        float t = dot(cross(AO, AB), AC) / denom;
        return t < r.t && t > kEPS;
    } else if (type == T_SPH) {
        f3 oc = r.O - mk(p0.x, p0.y, p0.z);
        float b = dot(oc, r.D);
        float c = dot(oc, oc) - p1.x;
        float d = b * b - c;
        if (d <= 0) return false;
        d = sqrtf(d);
        float t = -b - d;
        if (t < r.t && t > kEPS) return true;
        t = d - b;
        return t < r.t && t > kEPS;
    } else if (type == T_PLANE) {
        f3 N = mk(p0.x, p0.y, p0.z);
        float t = -(dot(r.O, N) + p1.x) / (dot(r.D, N));
        return t < r.t && t > kEPS;
    } else {
        return xprim_hit(S, type, __float_as_uint(p1.x), r);
    }
}

// u, v of a sphere / plane hit, evaluated once for the final hit: identical to the
// reference's evaluation at acceptance time (same t, same centre).
__device__ __forceinline__ void finish_uv(const SceneView &S, DRay &r) {
    if (r.obj < 0) return;
    float4 s0 = S.shade[2 * r.obj], s1 = S.shade[2 * r.obj + 1];
    uint32_t type = __float_as_uint(s1.x);
    f3 I = r.O + r.t * r.D;
    if (type == T_SPH) {
        f3 cToI = normalize(I - mk(s0.x, s0.y, s0.z));
        r.u = 0.5f - cr_atan2(cToI.z, cToI.x) * kINV2PI;
        r.v = 0.5f - cr_asin(cToI.y) * kINVPI;
    } else if (type == T_PLANE) {
        if (s0.x < kFLT_EPSILON && s0.y < kFLT_EPSILON) { r.u = I.x; r.v = -I.y; }
        else if (s0.x < kFLT_EPSILON && s0.z < kFLT_EPSILON) { r.u = I.x; r.v = -I.z; }
        else if (s0.y < kFLT_EPSILON && s0.z < kFLT_EPSILON) { r.u = I.y; r.v = -I.z; }
        else { r.u = 0.0f; r.v = 0.0f; }   // left unset by the reference: defined as 0
    } else if (type == T_QUAD) {
        r.u = 0.0f; r.v = 0.0f;
    } else if (type == T_CUBE) {           // Primitive::setTextureCoordsCube, Primitive.h:752-797
        const float4 *x = S.xprims + 8 * __float_as_uint(s1.z);
        const f3 o = tpos_rows(x[0], x[1], x[2], I);
        const float4 d0 = x[6], d1 = x[7];
        float uc = o.z, vc = o.y;
        const float e0 = fabsf(o.x - d0.x), e1 = fabsf(o.x - d1.x), e2 = fabsf(o.y - d0.y), e3 = fabsf(o.y - d1.y);
        const float e4 = fabsf(o.z - d0.z), e5 = fabsf(o.z - d1.z);
        float minDist = e0;
        int face = 1;
        if (e1 < minDist) uc = -o.z, vc = o.y, face = 0, minDist = e1;
        if (e2 < minDist) uc = o.x, vc = o.z, face = 3, minDist = e2;
        if (e3 < minDist) uc = o.x, vc = -o.z, face = 2, minDist = e3;
        if (e4 < minDist) uc = -o.x, vc = o.y, face = 5, minDist = e4;
        if (e5 < minDist) uc = o.x, vc = o.y, face = 4;
        uc = -uc, vc = -vc;
        uc = 0.5f * (uc / d1.x + 1.0f);
        vc = 0.5f * (vc / d1.x + 1.0f);
        const float third = 1.0f / 3.0f;
        const float fu = face == 0 ? 2.0f : face == 1 ? 0.0f : face == 5 ? 3.0f : 1.0f;
        const float fv = face == 2 ? 0.0f : face == 3 ? 2.0f : 1.0f;
        r.u = 0.25f * (fu + uc);
        r.v = third * (fv + vc);
    }
}

// Scene::GetNormal (template/scene.h:489-497) of the hit primitive at I, not yet flipped:
// Primitive::GetNormal (Primitive.h:284-314)
__device__ __forceinline__ f3 prim_normal(const SceneView &S, int obj, f3 I) {
    const float4 s0 = S.shade[2 * obj], s1 = S.shade[2 * obj + 1];
    const uint32_t type = __float_as_uint(s1.x);
    if (type == T_SPH) return (I - mk(s0.x, s0.y, s0.z)) * s1.y;
    if (type != T_CUBE) return mk(s0.x, s0.y, s0.z);
    const float4 *x = S.xprims + 8 * __float_as_uint(s1.z);
    const f3 o = tpos_rows(x[0], x[1], x[2], I);
    const float4 d0 = x[6], d1 = x[7];
    f3 N = mk(-1, 0, 0);
    const float e0 = fabsf(o.x - d0.x), e1 = fabsf(o.x - d1.x), e2 = fabsf(o.y - d0.y), e3 = fabsf(o.y - d1.y);
    const float e4 = fabsf(o.z - d0.z), e5 = fabsf(o.z - d1.z);
    float minDist = e0;
    if (e1 < minDist) minDist = e1, N.x = 1;
    if (e2 < minDist) minDist = e2, N = mk(0, -1, 0);
    if (e3 < minDist) minDist = e3, N = mk(0, 1, 0);
    if (e4 < minDist) minDist = e4, N = mk(0, 0, -1);
    if (e5 < minDist) minDist = e5, N = mk(0, 0, 1);
    return tvec_rows(x[3], x[4], x[5], N);
}

// Scene::GetNormal (flipped against the ray) and Scene::GetMaterial of a hit; a
// TextureMaterial also needs the hit's u, v (deferred by the traversal, finish_uv)
__device__ __forceinline__ const DevMaterial &hit_surface(const SceneView &S, DRay &ray, f3 I, f3 &N) {
    N = prim_normal(S, ray.obj, I);
    if (dot(N, ray.D) > 0) N = -N;
    const DevMaterial &m = S.mats[__float_as_int(S.shade[2 * ray.obj].w)];
    if (m.kind == RT_TEXTURE) finish_uv(S, ray);
    return m;
}

// ------------------------------------------------------------------ traversal (scene.h:285-320, 452-487)
// Where a traversal reads its nodes and keeps its stack: `nodes` is the global node array
// or the workgroup's LDS copy of it; `stk` is this lane's column of the LDS stack, entry i
// at stk[i * STRIDE] (STRIDE = workgroup size: consecutive lanes, consecutive banks).
template <int STRIDE>
struct Trav {
    const float4 *nodes;
    uint32_t *stk;
};

template <bool FAST, int STRIDE>
__device__ __forceinline__ void closest_hit_t(const SceneView &S, const Trav<STRIDE> &T, DRay &r) {
    uint32_t *stk = T.stk;
    uint32_t word = S.root_word;
    int sp = 0;
    for (;;) {
        uint32_t cnt = word & 0xffu, lf = word >> 8;
        if (cnt) {
            for (uint32_t k = lf; k < lf + cnt; ++k) prim_intersect(S, k, r);
            if (sp == 0) break;
            word = stk[--sp * STRIDE];
            continue;
        }
        const float4 *q = T.nodes + 2 * lf;
        float4 a0 = q[0], b0 = q[1], a1 = q[2], b1 = q[3];
        float d1 = slab_dist<FAST>(r, a0, b0), d2 = slab_dist<FAST>(r, a1, b1);
        uint32_t w1 = __float_as_uint(b0.z), w2 = __float_as_uint(b1.z);
        if (d1 > d2) { float td = d1; d1 = d2; d2 = td; uint32_t tw = w1; w1 = w2; w2 = tw; }
        if (d1 == 1e30f) {
            if (sp == 0) break;
            word = stk[--sp * STRIDE];
        } else {
            word = w1;
            if (d2 != 1e30f) stk[sp++ * STRIDE] = w2;
        }
    }
}

template <bool FAST, int STRIDE>
__device__ __forceinline__ bool occluded_t(const SceneView &S, const Trav<STRIDE> &T, const DRay &r) {
    uint32_t *stk = T.stk;
    uint32_t word = S.root_word;
    int sp = 0;
    for (;;) {
        uint32_t cnt = word & 0xffu, lf = word >> 8;
        if (cnt) {
            for (uint32_t k = lf; k < lf + cnt; ++k)
                if (prim_hit(S, k, r)) return true;
            if (sp == 0) return false;
            word = stk[--sp * STRIDE];
            continue;
        }
        const float4 *q = T.nodes + 2 * lf;
        float4 a0 = q[0], b0 = q[1], a1 = q[2], b1 = q[3];
        bool h1 = slab_hit<FAST>(r, a0, b0), h2 = slab_hit<FAST>(r, a1, b1);
        uint32_t w1 = __float_as_uint(b0.z), w2 = __float_as_uint(b1.z);
        if (h1 && h2) { word = w1; stk[sp++ * STRIDE] = w2; }
        else if (!(h1 || h2)) { if (sp == 0) return false; word = stk[--sp * STRIDE]; }
        else word = h1 ? w1 : w2;
    }
}

// ---- wave-coherent closest hit: the calling lanes walk the union of their subtrees with
// a wave-uniform node and stack (the stack lives in the LDS column of the wave's lane 0 --
// a VGPR lane-stack cannot be used because the caller may have lanes switched off).
// Closest hit along the union of the lanes' subtrees; children are visited in the order
// most calling lanes prefer.  A lane tests a leaf only if its slab test passed with its t
// at that moment.  Results equal IntersectBVH's whenever the closest hit is unique: `tie`
// reports a lane that met a second primitive at exactly its current t, and `odd` a hit
// nearer than its leaf box's entry distance (float rounding at a box face) -- the two
// ways the visiting order could matter; such lanes are re-traced in the reference order.
template <int STRIDE>
__device__ __forceinline__ void wave_closest_hit_fast(const SceneView &S, const Trav<STRIDE> &T, DRay &r, bool &flag) {
    const float4 *nodes = T.nodes;
    uint32_t *ws = T.stk - __lane_id();               // the wave's uniform stack (node indices)
    uint32_t word = __builtin_amdgcn_readfirstlane(S.root_word);
    bool in = true;
    float tb = -1e30f;                                // my slab entry distance of the current node
    uint32_t sp = 0;
    for (;;) {
        const uint32_t cnt = word & 0xffu, lf = word >> 8;
        if (cnt) {
            if (in)
                for (uint32_t k = lf; k < lf + cnt; ++k) {
                    const float t0 = r.t;
                    prim_intersect_t(S, k, r, flag);
                    if (r.t != t0 && r.t < tb) flag = true;   // hit nearer than its box's entry
                }
        } else {
            const float4 *q = nodes + 2 * lf;
            const float4 a0 = q[0], b0 = q[1], a1 = q[2], b1 = q[3];
            const float d1 = in ? slab_dist<true>(r, a0, b0) : 1e30f, d2 = in ? slab_dist<true>(r, a1, b1) : 1e30f;
            const bool h1 = d1 != 1e30f, h2 = d2 != 1e30f;
            const uint64_t m1 = __ballot(h1), m2 = __ballot(h2);
            if (m1 | m2) {
                const uint32_t v1 = __popcll(__ballot(h1 && !(h2 && d2 < d1)));
                const uint32_t v2 = __popcll(__ballot(h2 && !(h1 && d1 <= d2)));
                const bool first1 = m1 && (!m2 || v1 >= v2);
                if (m1 && m2) {
                    ws[sp * STRIDE] = first1 ? lf + 1 : lf;
                    ++sp;
                }
                word = __builtin_amdgcn_readfirstlane(__float_as_uint(first1 ? b0.z : b1.z));
                in = first1 ? h1 : h2;
                tb = first1 ? d1 : d2;
                continue;
            }
        }
        // pop, re-testing each entry with the lanes' current t
        for (;;) {
            if (sp == 0) return;
            --sp;
            const uint32_t ni = __builtin_amdgcn_readfirstlane(ws[sp * STRIDE]);
            const float4 a = nodes[2 * ni], b = nodes[2 * ni + 1];
            tb = slab_dist<true>(r, a, b);
            in = tb != 1e30f;
            if (__ballot(in)) {
                word = __builtin_amdgcn_readfirstlane(__float_as_uint(b.z));
                break;
            }
        }
    }
}

template <int STRIDE>
__device__ __forceinline__ void closest_hit(const SceneView &S, const Trav<STRIDE> &T, DRay &r) {
    if (__all(S.bounds_finite && ray_finite(r))) closest_hit_t<true>(S, T, r);
    else closest_hit_t<false>(S, T, r);
}
// camera rays: the wave-coherent walk where the scene asks for it (SceneView::wave_primary)
template <int STRIDE>
__device__ __forceinline__ void closest_hit_primary(const SceneView &S, const Trav<STRIDE> &T, DRay &r) {
    if (S.wave_primary && __all(S.bounds_finite && ray_finite(r))) {
        const DRay r0 = r;
        bool flag = false;
        wave_closest_hit_fast(S, T, r, flag);
        if (flag) { r = r0; closest_hit_t<true>(S, T, r); }
        return;
    }
    closest_hit(S, T, r);
}
template <int STRIDE>
__device__ __forceinline__ bool occluded(const SceneView &S, const Trav<STRIDE> &T, const DRay &r) {
    if (__all(S.bounds_finite && ray_finite(r))) return occluded_t<true>(S, T, r);
    return occluded_t<false>(S, T, r);
}

// ------------------------------------------------------------------ packet traversal (scene.h:322-412)
// Scene::IntersectBVHPacket with the packet = the wave: lane l holds ray l of the 64-ray
// packet.  The node, the stack and the "first active" ray are wave-uniform (node and
// primitive loads are scalar, the stack lives in one VGPR: entry i in lane i); each lane
// tests its own ray and a ballot finds the lowest hitting lane.  Inactive lanes (past the
// end of the batch / off screen) never test and never lead.  The VGPR lane-stack needs all
// 64 lanes switched on: callers invoke it from wave-uniform control flow only.
__device__ __forceinline__ float readlane_f(float v, uint32_t l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l));
}

template <bool FAST>
__device__ __forceinline__ void packet_closest_hit_t(const SceneView &S, DRay &r, bool active) {
    const uint32_t lane = __lane_id();
    uint32_t fa = 0, ni = 0, sp = 0;
    int stackv = 0;                                   // lane i: stack entry i (node index, depth < 64)
    for (;;) {
        ni = __builtin_amdgcn_readfirstlane(ni);
        const float4 a = S.nodes[2 * ni], b = S.nodes[2 * ni + 1];
        const uint32_t word = __float_as_uint(b.z), cnt = word & 0xffu, lf = word >> 8;
        const uint64_t m = __ballot(active && slab_hit<FAST>(r, a, b));
        uint32_t first = 0;                           // lanes >= first test a leaf
        bool visit = true;
        if (!((m >> fa) & 1u)) {
            if (m == 0) visit = false;
            else first = fa = (uint32_t)__ffsll((long long)m) - 1u;
        }
        if (visit && cnt == 0) {                      // interior: order by the leader's distances
            const float4 *q = S.nodes + 2 * lf;
            float d1 = readlane_f(slab_dist<FAST>(r, q[0], q[1]), fa);
            float d2 = readlane_f(slab_dist<FAST>(r, q[2], q[3]), fa);
            uint32_t c1 = lf, c2 = lf + 1;
            if (d1 > d2) { c1 = lf + 1; c2 = lf; }
            stackv = lane == sp ? (int)c2 : stackv;   // writelane
            ++sp;
            ni = c1;
            continue;
        }
        if (visit && active && lane >= first)
            for (uint32_t k = lf; k < lf + cnt; ++k) prim_intersect(S, k, r);
        if (sp == 0) break;
        --sp;
        ni = (uint32_t)__builtin_amdgcn_readlane(stackv, (int)sp);
    }
}
__device__ __forceinline__ void packet_closest_hit(const SceneView &S, DRay &r, bool active) {
    if (__all(S.bounds_finite && (!active || ray_finite(r)))) packet_closest_hit_t<true>(S, r, active);
    else packet_closest_hit_t<false>(S, r, active);
}

// ------------------------------------------------------------------ shading
// TEX_SKY = false: every texel is equal (the synthetic sky), so the lookup's index is
// irrelevant and the colour is the precomputed texel -- bit-identical, no atan2/acos.
template <bool TEX_SKY>
__device__ __forceinline__ f3 sky_color(const SceneView &S, f3 D) {   // renderer.h:15-22
    if (!TEX_SKY) return mk(S.sky_rgb[0], S.sky_rgb[1], S.sky_rgb[2]);
    uint32_t u = f2u_wrap((float)S.sky_w * cr_atan2(D.z, D.x) * kINV2PI - 0.5f);
    uint32_t v = f2u_wrap((float)S.sky_h * cr_acos(D.y) * kINVPI - 0.5f);
    uint32_t p = S.sky[(u & (S.sky_w - 1)) + (v & (S.sky_h - 1)) * S.sky_w];
    return mk((float)((p >> 16) & 255), (float)((p >> 8) & 255), (float)(p & 255)) * kSKY;
}

// ObjectMaterial::DiffuseReflection + mapToNormalAxis (ObjectMaterial.h:18-53)
__device__ __forceinline__ f3 diffuse_dir(f3 N, uint32_t &seed) {
    float r0 = rnd_f(seed), r1 = rnd_f(seed);
    float r = sqrtf(r0), theta = kTWOPI * r1;
    float st, ct;
    sincos_f(theta, st, ct);
    float x = r * ct, y = r * st, z = sqrtf(1 - r0);
    f3 a0 = mk(0.0f, -1.0f, 0.0f), a1 = mk(-1.0f, 0.0f, 0.0f);
    if (N.z + 1.0f > kFLT_EPSILON) {
        float a = 1.0f / (1.0f + N.z);
        float b = -N.x * N.y * a;
        a0 = mk(1.0f - N.x * N.x * a, b, -N.x);
        a1 = mk(b, 1.0f - N.y * N.y * a, -N.y);
    }
    return normalize(x * a0 + y * a1 + z * N);
}

__device__ __forceinline__ float fresnel(float n1, float n2, float cost, float cosi) {   // ObjectMaterial.h:55-60
    float s = (n1 * cosi - n2 * cost) / (n1 * cosi + n2 * cost);
    float p = (n1 * cost - n2 * cosi) / (n1 * cost + n2 * cosi);
    return 0.5f * ((s * s) + (p * p));
}

// ObjectMaterial::scatter overrides.  With last = true the bounce ray is never traced
// (Trace(.., depth 0) returns 0), so only the RNG draws and the specular flag are kept.
__device__ __forceinline__ bool scatter(const DevMaterial &m, const DRay &in, f3 I, f3 N, DRay &out, uint32_t &seed,
                                        bool last) {
    switch (m.kind) {
    case RT_DIFFUSE:                                                   // Diffuse.h:16-19
        if (last) { rnd_u(seed); rnd_u(seed); }
        else out = make_ray(I, diffuse_dir(N, seed), 1e34f);
        return false;
    case RT_MIRROR:                                                    // Mirror.h:16-19
        if (!last) out = make_ray(I, normalize(reflect(in.D, N)), 1e34f);
        return true;
    case RT_DIELECTRIC: {                                              // Dielectric.h:23-54
        float n1 = 1, n2 = m.ior;
        float n12 = n1 / n2;
        float cosi = dot(N, in.D);
        if (in.inside) n12 = 1 / n12;
        float k = 1 - (n12 * n12) * (1 - (cosi * cosi));
        if (k < 0) {
            if (!last) { out = make_ray(I, normalize(reflect(in.D, N)), 1e34f); out.inside = 1; }
        } else {
            float Fr = 0;
            if (!in.inside) {
                float sini = length(cross(N, in.D));
                float sq = n12 * sini;
                float cost = sqrtf(1 - sq * sq);
                Fr = fresnel(n1, n2, cost, -cosi);
            }
            if (Fr > kFLT_EPSILON && rnd_f(seed) < Fr) {
                if (!last) out = make_ray(I, normalize(reflect(in.D, N)), 1e34f);
            } else if (!last) {
                f3 T = normalize(n12 * in.D - (n12 * cosi + sqrtf(k)) * N);
                out = make_ray(I, T, 1e34f);
                out.inside = !in.inside;
            }
        }
        return true;
    }
    case RT_LIGHT:
        return false;
    default:                                                           // Checkerboard.h:39-58
        if (m.diffuse < kFLT_EPSILON) {
            if (!last) out = make_ray(I, normalize(reflect(in.D, N)), 1e34f);
            return true;
        }
        if (m.specular < kFLT_EPSILON) {
            if (last) { rnd_u(seed); rnd_u(seed); }
            else out = make_ray(I, diffuse_dir(N, seed), 1e34f);
            return false;
        }
        if (rnd_f(seed) < m.specular) {
            if (!last) out = make_ray(I, normalize(reflect(in.D, N)), 1e34f);
            return true;
        }
        if (last) { rnd_u(seed); rnd_u(seed); }
        else out = make_ray(I, diffuse_dir(N, seed), 1e34f);
        return false;
    }
}

// TextureMaterial::GetColor (TextureMaterial.h:30-37); scale = 1/255 (correction) or
// SKYDOME_CORRECTION (getColorModifier) -- the same float
__device__ __forceinline__ f3 texture_color(const SceneView &S, const DevMaterial &m, const DRay &in) {
    const uint32_t u = f2u_wrap((float)m.tex_w * in.u), v = f2u_wrap((float)m.tex_h * in.v);
    const uint32_t p = S.tex[m.tex_off + (u & (m.tex_w - 1)) + (v & (m.tex_h - 1)) * m.tex_w];
    return mk((float)((p >> 16) & 255), (float)((p >> 8) & 255), (float)(p & 255)) * (1.0f / 255.0f);
}

__device__ __forceinline__ f3 mat_color(const SceneView &S, const DevMaterial &m, const DRay &in, f3 I) {
    if (m.kind == RT_TEXTURE) return texture_color(S, m, in);
    if (m.kind == RT_DIELECTRIC) {                                     // Dielectric.h:12-21
        f3 c = mk(1, 1, 1);
        if (in.inside) { c.x = exp_f(-m.c0[0] * in.t); c.y = exp_f(-m.c0[1] * in.t); c.z = exp_f(-m.c0[2] * in.t); }
        return c;
    }
    if (m.kind == RT_CHECKERBOARD) {                                   // Checkerboard.h:28-37
        bool ex = abs(((int)floorf(I.x)) % 2) == 0;
        bool ez = abs(((int)floorf(I.z)) % 2) == 0;
        return ex == ez ? mk(m.c0[0], m.c0[1], m.c0[2]) : mk(m.c1[0], m.c1[1], m.c1[2]);
    }
    return mk(m.c0[0], m.c0[1], m.c0[2]);
}

// Scene::GetLightPos = Primitive::GetRandomPoint of the light (Primitive.h:394-402, 423-427)
__device__ __forceinline__ f3 light_point(const SceneView &S, uint32_t &seed) {
    if (S.light_quad) {   // Primitive.h:423-427: the point lies in object z = 0 (reference quirk)
        const float a = S.light_qsize * (rnd_f(seed) - 1.0f);
        const float b = S.light_qsize * (rnd_f(seed) - 1.0f);
        return tpos(S.light_M, mk(a, b, 0.0f));
    }
    f3 pt = mk(1, 1, 1);
    while (dot(pt, pt) > 1) {
        float x = rnd_f(seed) * 2.0f - 1.0f;
        float y = rnd_f(seed) * 2.0f - 1.0f;
        float z = rnd_f(seed) * 2.0f - 1.0f;
        pt = mk(x, y, z);
    }
    return tpos(S.light_M, normalize(pt) * S.light_r);
}

// Renderer::NextEventDirectIllumination, renderer.h:44-75 (light = prim 0, a sphere)
template <int STRIDE>
__device__ __forceinline__ f3 nee(const SceneView &S, const Trav<STRIDE> &T, f3 I, f3 N, f3 BRDF, uint32_t &seed,
                                  uint32_t &nshadow) {
    f3 Il = light_point(S, seed);
    const float area = S.light_area;                                   // GetArea, Primitive.h:450-468
    f3 L = Il - I;
    float dist = length(L);
    L = L / dist;
    f3 Nl = S.light_quad ? mk(S.light_N[0], S.light_N[1], S.light_N[2])
                         : (Il - mk(S.light_c[0], S.light_c[1], S.light_c[2])) * S.light_invr;
    if (dot(Nl, L) > 0) Nl = -Nl;                                      // Scene::GetNormal flip
    float dotNL = dot(N, L), dotNlL = dot(Nl, -L);
    f3 Ld = mk(0, 0, 0);
    if (dotNL > 0 && dotNlL > 0) {
        DRay sh = make_ray(I, L, dist - 2.0f * kEPS);
        ++nshadow;
        if (!occluded(S, T, sh)) {
            float solid = (dotNlL * area) / (dist * dist);
            float lightPDF = 1.0f / solid;
            const DevMaterial &lm = S.mats[S.light_mat];                // GetLightColor(0, toLight)
            const f3 lc = lm.kind == RT_LIGHT ? mk(lm.c0[0], lm.c0[1], lm.c0[2]) : mat_color(S, lm, sh, sh.O + sh.t * sh.D);
            Ld = (lc * BRDF) * (dotNL / lightPDF);
        }
    }
    return Ld;
}

// Renderer::Trace (renderer.cpp:17-72) as a loop.  The recursion's result
// BRDF * ((Trace * dot) / PDF) + Ld is folded innermost-first from per-level records,
// so the float evaluation order is the reference's.
template <int MAXD, bool TEX_SKY, int STRIDE, bool CAMWAVE = false>
__device__ f3 trace_path(const SceneView &S, const Trav<STRIDE> &T, DRay ray, int depth, uint32_t &seed,
                         uint32_t &nshadow, uint32_t &nbounce, bool lastSpec = true) {
    f3 lv_mul[MAXD], lv_add[MAXD];
    float lv_c[MAXD];
    bool lv_diff[MAXD];
    int levels = 0;
    f3 term = mk(0, 0, 0);
    for (int d = depth; d > 0 && levels < MAXD; --d) {
        if (d != depth) ++nbounce;
        if (CAMWAVE && d == depth) closest_hit_primary(S, T, ray);
        else closest_hit(S, T, ray);
        if (ray.obj == -1) { term = sky_color<TEX_SKY>(S, ray.D); break; }
        f3 I = ray.O + ray.t * ray.D;
        f3 N;
        const DevMaterial &m = hit_surface(S, ray, I, N);
        if (m.flag == F_LIGHT) { term = lastSpec ? mk(m.c0[0], m.c0[1], m.c0[2]) : mk(0, 0, 0); break; }
        const bool last = MAXD == 1 || d == 1;   // MAXD 1: the bounce ray is never traced
        DRay out;
        bool spec = scatter(m, ray, I, N, out, seed, last);
        f3 albedo = mat_color(S, m, ray, I);
        if (m.flag == F_DIFFUSE || (m.flag == F_MIX && !spec)) {
            f3 BRDF = albedo * kINVPI;
            lv_add[levels] = nee(S, T, I, N, BRDF, seed, nshadow);
            lv_mul[levels] = BRDF;
            lv_c[levels] = last ? 0.0f : dot(N, out.D);
            lv_diff[levels] = true;
        } else {
            lv_mul[levels] = albedo;
            lv_add[levels] = mk(0, 0, 0);
            lv_c[levels] = 0.0f;
            lv_diff[levels] = false;
        }
        ++levels;
        if (last) break;
        ray = out;
        lastSpec = spec;
    }
    f3 r = term;
    for (int k = levels - 1; k >= 0; --k)
        r = lv_diff[k] ? lv_mul[k] * ((r * lv_c[k]) / kINV2PI) + lv_add[k] : lv_mul[k] * r;
    return r;
}

// Renderer::TracePacket's per-ray shading (renderer.cpp:78-133): the primary hit comes
// from the packet traversal, every bounce is a Trace(ray_out, specularBounce, depth).
template <int MAXD, bool TEX_SKY, int STRIDE>
__device__ f3 shade_packet(const SceneView &S, const Trav<STRIDE> &T, DRay ray, int depth, uint32_t &seed,
                           uint32_t &nshadow, uint32_t &nbounce) {
    if (ray.obj == -1) return sky_color<TEX_SKY>(S, ray.D);
    f3 I = ray.O + ray.t * ray.D;
    f3 N;
    const DevMaterial &m = hit_surface(S, ray, I, N);
    const bool last = depth == 0;                  // Trace(.., 0) returns 0: the bounce is never traced
    DRay out;
    bool spec = scatter(m, ray, I, N, out, seed, last);
    f3 albedo = mat_color(S, m, ray, I);
    if (m.flag == F_LIGHT) return albedo;
    const bool diffuse = m.flag == F_DIFFUSE || m.flag == F_MIX;
    // MIX + specular bounce: the ray is traced for a result that is then overwritten
    // (renderer.cpp:111-114) and traced again after NEE (116-120).  One call site.
    const int passes = (m.flag == F_MIX && spec) ? 2 : 1;
    const f3 BRDF = albedo * kINVPI;
    f3 Ld = mk(0, 0, 0), Li = mk(0, 0, 0);
    for (int p = 0; p < passes; ++p) {
        if (diffuse && p == passes - 1) Ld = nee(S, T, I, N, BRDF, seed, nshadow);
        nbounce += last ? 0u : 1u;
        Li = trace_path<MAXD, TEX_SKY>(S, T, out, depth, seed, nshadow, nbounce, spec);
    }
    if (!diffuse) return albedo * Li;
    f3 Ei = (Li * (last ? 0.0f : dot(N, out.D))) / kINV2PI;
    return BRDF * Ei + Ld;
}

// ------------------------------------------------------------------ Whitted (the K key)
// ObjectMaterial::getColorModifier overrides: colour in c, colorVars[3] in c3 and the
// refraction direction colorVars[4..6] in T (Diffuse.h:21-23, Mirror.h:21-23,
// Light.h:20-22, Checkerboard.h:60-71, Dielectric.h:56-85).
__device__ __forceinline__ void color_modifier(const SceneView &S, const DevMaterial &m, const DRay &in, f3 I, f3 N, f3 &c, float &c3,
                                               f3 &T) {
    c3 = 0.0f;
    T = mk(0, 0, 0);
    switch (m.kind) {
    case RT_LIGHT:   // clamp = fmaxf(a, fminf(f, b)), template/precomp.h:782
        c = mk(fmaxf(0.0f, fminf(m.c0[0], 1.0f)), fmaxf(0.0f, fminf(m.c0[1], 1.0f)), fmaxf(0.0f, fminf(m.c0[2], 1.0f)));
        return;
    case RT_CHECKERBOARD:
    case RT_TEXTURE:                 // TextureMaterial.h:62-71
        c = mat_color(S, m, in, I);
        c3 = m.diffuse;
        return;
    case RT_DSMIX:                   // DSMix.h:48-50
        c = mk(m.c0[0], m.c0[1], m.c0[2]);
        c3 = m.diffuse;
        return;
    case RT_DIELECTRIC: {
        float n1 = 1, n2 = m.ior, n12 = n1 / n2;
        float cosi = dot(N, in.D);
        c = mk(1, 1, 1);
        if (in.inside) {
            c = mk(exp_f(-m.c0[0] * in.t), exp_f(-m.c0[1] * in.t), exp_f(-m.c0[2] * in.t));
            n12 = 1 / n12;
        }
        float k = 1 - (n12 * n12) * (1 - (cosi * cosi));
        if (k < 0) { c3 = -1.0f; return; }   // TIR
        if (!in.inside) {
            float sini = length(cross(N, in.D));
            float sq = n12 * sini;
            float cost = sqrtf(1 - sq * sq);
            c3 = fresnel(n1, n2, cost, -cosi);
        }
        T = normalize(n12 * in.D - (n12 * cosi + sqrtf(k)) * N);
        return;
    }
    default:
        c = mk(m.c0[0], m.c0[1], m.c0[2]);
        return;
    }
}

// Renderer::DirectIllumination, renderer.h:24-42: 4 light-sphere samples, spotlight test
// against GetLightDir (0,-1,0), GetLightColor (24,24,22) (template/scene.h:234-242).
template <int STRIDE>
__device__ __forceinline__ f3 direct_illumination(const SceneView &S, const Trav<STRIDE> &T, f3 I, f3 N,
                                                  uint32_t &seed, uint32_t &nshadow) {
    f3 result = mk(0, 0, 0);
    const f3 ldir = mk(0.0f, -1.0f, 0.0f), lcol = mk(24.0f, 24.0f, 22.0f);
    for (int i = 0; i < 4; ++i) {
        f3 L = light_point(S, seed) - I;
        float dist = length(L);
        L = L / dist;
        float dotDN = dot(L, N);
        if (dotDN < 0 || dot(ldir, L) > 0) continue;
        DRay sh = make_ray(I, L, dist - (2 * kEPS));
        ++nshadow;
        if (occluded(S, T, sh)) continue;
        result = result + (dotDN / (dist * dist)) * lcol;
    }
    return result / 4.0f;
}

// Renderer::WhittedTrace (renderer.cpp:138-195) as a depth-first walk with an explicit
// frame stack.  A frame holds the parent's colour modifier and its partial sum; a child's
// value is added (scaled by Fr, Ft or 1 - diffuse) when it returns, and the dielectric's
// refraction child starts only after the reflection child is finished -- the reference's
// evaluation and RNG order, so results are bit-identical to the recursion.
constexpr int kWHITTED_MAX = 32;
struct WFrame {
    f3 col, res, I, T;
    float w, ft;
    int flags;   // 1: scale the child by w, 2: refraction child pending, 4: its inside flag
};

template <bool TEX_SKY, int STRIDE>
__device__ f3 trace_whitted(const SceneView &S, const Trav<STRIDE> &T, DRay ray, int depth, uint32_t &seed,
                            uint32_t &nshadow, uint32_t &nbounce) {
    WFrame st[kWHITTED_MAX];
    int sp = 0;
    bool primary = true;
    for (;;) {
        // ---- evaluate WhittedTrace(ray, depth - sp) up to its first child
        f3 ret = mk(0, 0, 0);
        if (depth - sp > 0) {
            if (!primary) ++nbounce;
            primary = false;
            closest_hit(S, T, ray);
            if (ray.obj == -1) {
                ret = sky_color<TEX_SKY>(S, ray.D);
            } else {
                f3 I = ray.O + ray.t * ray.D;
                f3 N;
                const DevMaterial &m = hit_surface(S, ray, I, N);
                f3 col, Tdir;
                float c3;
                color_modifier(S, m, ray, I, N, col, c3, Tdir);
                f3 res = mk(0, 0, 0);
                WFrame f;
                f.col = col; f.w = 1.0f; f.ft = 0.0f; f.flags = 0;
                bool push = false, child_inside = false;
                f3 childD = mk(0, 0, 0);
                if (m.flag == F_LIGHT) {
                    res = res + mk(24.0f, 24.0f, 22.0f);
                } else if (m.flag == F_DIFFUSE) {
                    res = res + direct_illumination(S, T, I, N, seed, nshadow);
                } else if (m.flag == F_SPECULAR) {
                    push = true; childD = normalize(reflect(ray.D, N));
                } else if (m.flag == F_MIX) {
                    res = res + c3 * direct_illumination(S, T, I, N, seed, nshadow);
                    push = true; childD = normalize(reflect(ray.D, N));
                    f.w = 1.0f - c3; f.flags = 1;
                } else if (m.flag == F_DIELECTRIC) {
                    if (c3 < 0) {
                        push = true; childD = normalize(reflect(ray.D, N)); child_inside = true;
                    } else {
                        float Fr = c3, Ft = 1 - Fr;
                        if (Fr > kFLT_EPSILON) {
                            push = true; childD = normalize(reflect(ray.D, N));
                            f.w = Fr; f.flags = 1;
                            if (Ft > kFLT_EPSILON) {
                                f.flags |= 2 | (ray.inside ? 0 : 4);
                                f.ft = Ft; f.I = I; f.T = Tdir;
                            }
                        } else if (Ft > kFLT_EPSILON) {
                            push = true; childD = Tdir; child_inside = !ray.inside;
                            f.w = Ft; f.flags = 1;
                        }
                    }
                }
                if (push) {
                    f.res = res;
                    st[sp++] = f;
                    ray = make_ray(I, childD, 1e34f);
                    ray.inside = child_inside ? 1 : 0;
                    continue;
                }
                ret = col * res;
            }
        }
        // ---- return ret to the parents until one has a child left to trace
        bool descend = false;
        while (sp > 0) {
            WFrame &f = st[sp - 1];
            f.res = f.res + ((f.flags & 1) ? f.w * ret : ret);
            if (f.flags & 2) {
                ray = make_ray(f.I, f.T, 1e34f);
                ray.inside = (f.flags & 4) ? 1 : 0;
                f.w = f.ft;
                f.flags &= ~2;
                descend = true;
                break;
            }
            ret = f.col * f.res;
            --sp;
        }
        if (!descend) return ret;
    }
}

// Camera::GetPrimaryRay (camera.h:43-52) + randomInUnitDisk (20-26)
__device__ __forceinline__ DRay primary_ray(const FrameArgs &F, uint32_t x, uint32_t y, uint32_t &seed) {
    float u = (float)x * F.rw + rnd_f(seed) * F.rw;
    float v = (float)y * F.rh + rnd_f(seed) * F.rh;
    f3 p;
    for (;;) {
        float px = rnd_f(seed) * 2.0f - 1.0f;
        float py = rnd_f(seed) * 2.0f - 1.0f;
        p = mk(px, py, 0);
        if (!(dot(p, p) >= 1)) break;
    }
    f3 rd = F.lens * p;
    f3 offset = mk(u * rd.x, v * rd.y, 0);
    f3 pos = mk(F.cam_pos[0], F.cam_pos[1], F.cam_pos[2]);
    f3 tl = mk(F.cam_tl[0], F.cam_tl[1], F.cam_tl[2]);
    f3 tr = mk(F.cam_tr[0], F.cam_tr[1], F.cam_tr[2]);
    f3 bl = mk(F.cam_bl[0], F.cam_bl[1], F.cam_bl[2]);
    f3 P = tl + u * (tr - tl) + v * (bl - tl);
    return make_ray(pos + offset, normalize(P - pos - offset), 1e34f);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// RGBF32_to_RGB8, template/precomp.h:441-444
__device__ __forceinline__ uint32_t pack_rgb8(float4 a) {
    uint32_t r = f2u_wrap(255.0f * smin(1.0f, a.x));
    uint32_t g = f2u_wrap(255.0f * smin(1.0f, a.y));
    uint32_t b = f2u_wrap(255.0f * smin(1.0f, a.z));
    return (r << 16) + (g << 8) + b;
}

// ------------------------------------------------------------------ kernels
// One screen tile (8x8, one wave) of one frame: per pixel spp x Trace / WhittedTrace /
// TracePacket (the tile is the packet, renderer.cpp:247-285), running average into the
// accumulator (renderer.cpp:235-241), RGB8 pack; per-wave ray counters.
enum : int { M_PATH = RT_MODE_PATH, M_WHITTED = RT_MODE_WHITTED, M_PACKET = RT_MODE_PACKET };

template <int MODE, int MAXD, bool TEX_SKY, int STRIDE>
__device__ __forceinline__ void render_tile(const SceneView &S, const FrameArgs &F, const Trav<STRIDE> &T,
                                            uint32_t local_tile, uint32_t lane) {
    const uint32_t tile = local_tile * F.nshards + F.shard;
    const uint32_t x = (tile % F.tiles_x) * 8u + (lane & 7u), y = (tile / F.tiles_x) * 8u + (lane >> 3);
    const bool on = x < F.W && y < F.H;
    const uint32_t px = x + y * F.W;
    // the wave-coherent camera-ray walk is compiled into the global-node primary+shadow
    // kernel only (SceneView::wave_primary picks it at run time)
    constexpr bool kCamWave = MODE == M_PATH && MAXD == 1 && STRIDE == 256;
    uint32_t nshadow = 0, nbounce = 0;
    f3 sum = mk(0, 0, 0);
    if (MODE == M_PACKET) {                           // the traversal is wave-wide: no early exit
        for (uint32_t s = 0; s < F.spp; ++s) {
            uint32_t seed = init_seed(px + F.W * F.H * (s + F.spp * F.frame));
            DRay ray = on ? primary_ray(F, x, y, seed) : make_ray(mk(0, 0, 0), mk(0, 0, 1), 1e34f);
            packet_closest_hit(S, ray, on);
            if (on) sum = sum + shade_packet<MAXD, TEX_SKY>(S, T, ray, (int)F.depth, seed, nshadow, nbounce);
        }
    } else if (on) {
        for (uint32_t s = 0; s < F.spp; ++s) {
            uint32_t seed = init_seed(px + F.W * F.H * (s + F.spp * F.frame));
            DRay ray = primary_ray(F, x, y, seed);
            if constexpr (MODE == M_WHITTED) sum = sum + trace_whitted<TEX_SKY>(S, T, ray, (int)F.depth, seed, nshadow, nbounce);
            else sum = sum + trace_path<MAXD, TEX_SKY, STRIDE, kCamWave>(S, T, ray, (int)F.depth, seed, nshadow, nbounce);
        }
    }
    if (on) {
        f3 res = (1.0f / (float)F.spp) * sum;
        float4 a = F.reset ? make_float4(0, 0, 0, 0) : F.acc[px];
        a.w += 1;                                                      // renderer.cpp:237-240
        const float w = a.w, inv = 1.0f / w;
        a = make_float4(a.x + inv * (res.x - a.x), a.y + inv * (res.y - a.y), a.z + inv * (res.z - a.z),
                        a.w + inv * (w - a.w));
        F.acc[px] = a;
        const uint32_t rgb = pack_rgb8(a);
        if (F.packed_out) F.out[local_tile * 64u + lane] = rgb;
        else F.out[px] = rgb;
    }
    nshadow = wave_sum(nshadow);
    nbounce = wave_sum(nbounce);
    if (lane == 0) {
        if (nshadow) atomicAdd(&F.counters[0], (unsigned long long)nshadow);
        if (nbounce) atomicAdd(&F.counters[1], (unsigned long long)nbounce);
    }
}

// Global-node variant: 256-thread workgroups, wave w of workgroup b owns local tile b*4+w.
#ifndef RT_RENDER_WAVES_PER_SIMD
#define RT_RENDER_WAVES_PER_SIMD 1
#endif
template <int MODE, int MAXD, bool TEX_SKY>
__global__ __launch_bounds__(256, RT_RENDER_WAVES_PER_SIMD) void k_render(SceneView S, FrameArgs F) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t tid = threadIdx.x;
    const uint32_t local_tile = blockIdx.x * 4u + (tid >> 6);
    if (local_tile >= F.ntiles_local) return;
    Trav<256> T{S.nodes, lds_stack + tid};
    render_tile<MODE, MAXD, TEX_SKY>(S, F, T, local_tile, tid & 63u);
}

// LDS-node variant for scenes whose node array fits beside the stacks (TEAPOT-F: 65 KB):
// a 1024-thread workgroup copies the node array into LDS, then its 16 waves render 16
// consecutive tiles (a 128x8 strip) reading every 64-byte sibling pair with ds_read_b128
// instead of a vector-memory load.  One strip per workgroup leaves the balancing across
// CUs to the hardware dispatcher: persistent grids with static or per-CU queues measured
// 5-13 % slower (profiles/r01/ab_lds_*.json).  LDS = [stack_entries][1024] u32 | nodes.
template <int MAXD, bool TEX_SKY>
__global__ __launch_bounds__(1024) void k_render_lds(SceneView S, FrameArgs F) {
    extern __shared__ uint32_t lds[];
    const uint32_t tid = threadIdx.x;
    float4 *lnodes = reinterpret_cast<float4 *>(lds + S.stack_entries * 1024u);
    for (uint32_t i = tid; i < S.node_f4; i += 1024u) lnodes[i] = S.nodes[i];
    __syncthreads();
    const uint32_t local_tile = blockIdx.x * 16u + (tid >> 6);
    if (local_tile >= F.ntiles_local) return;
    Trav<1024> T{lnodes, lds + tid};
    render_tile<M_PATH, MAXD, TEX_SKY>(S, F, T, local_tile, tid & 63u);
}

__global__ __launch_bounds__(256) void k_intersect(SceneView S, const rt_ray *__restrict__ rays, rt_hit *__restrict__ hits,
                                                   uint32_t n) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    rt_ray q = rays[i];
    DRay r = make_ray(mk(q.ox, q.oy, q.oz), mk(q.dx, q.dy, q.dz), q.tmax);
    Trav<256> T{S.nodes, lds_stack + threadIdx.x};
    closest_hit(S, T, r);
    finish_uv(S, r);
    rt_hit h;
    h.t = r.t; h.obj = r.obj; h.u = r.u; h.v = r.v;
    hits[i] = h;
}

// batched Scene::IntersectBVHPacket: wave w traces rays [64w, 64w + 64) as one packet
__global__ __launch_bounds__(256) void k_intersect_packet(SceneView S, const rt_ray *__restrict__ rays,
                                                          rt_hit *__restrict__ hits, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if ((i & ~63u) >= n) return;                      // whole waves only
    const bool active = i < n;
    DRay r = make_ray(mk(0, 0, 0), mk(0, 0, 1), 1e34f);
    if (active) {
        rt_ray q = rays[i];
        r = make_ray(mk(q.ox, q.oy, q.oz), mk(q.dx, q.dy, q.dz), q.tmax);
    }
    packet_closest_hit(S, r, active);
    if (!active) return;
    finish_uv(S, r);
    rt_hit h;
    h.t = r.t; h.obj = r.obj; h.u = r.u; h.v = r.v;
    hits[i] = h;
}

__global__ __launch_bounds__(256) void k_occluded(SceneView S, const rt_ray *__restrict__ rays, uint8_t *__restrict__ out,
                                                  uint32_t n) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    rt_ray q = rays[i];
    DRay r = make_ray(mk(q.ox, q.oy, q.oz), mk(q.dx, q.dy, q.dz), q.tmax);
    Trav<256> T{S.nodes, lds_stack + threadIdx.x};
    out[i] = occluded(S, T, r) ? 1 : 0;
}

// rank-0 side of the per-frame gather: packed shard tiles -> row-major frame
__global__ __launch_bounds__(256) void k_assemble(const uint32_t *__restrict__ gathered, uint32_t cap, uint32_t nshards,
                                                  uint32_t tiles_x, uint32_t ntiles, uint32_t W, uint32_t H,
                                                  uint32_t *__restrict__ out) {
    const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (tile >= ntiles) return;
    const uint32_t x = (tile % tiles_x) * 8u + (lane & 7u), y = (tile / tiles_x) * 8u + (lane >> 3);
    if (x >= W || y >= H) return;
    const uint32_t shard = tile % nshards, local = tile / nshards;
    out[x + y * W] = gathered[(size_t)shard * cap + local * 64u + lane];
}

}  // namespace rt

// ====================================================================== host side
using namespace rt;

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(e_ == hipErrorNoBinaryForGpu || e_ == hipErrorInvalidDeviceFunction    \
                            ? RT_ERR_NO_DEVICE : RT_ERR_HIP,                                   \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

struct rt_scene {
    int device = 0;
    SceneView view{};
    Bvh bvh;
    uint32_t num_prims = 0;
    uint32_t stack_depth = 0;   // LDS stack entries per lane
    bool lds_nodes = false;     // frame kernel keeps the node array in LDS (k_render_lds)
    uint32_t num_cus = 256;     // persistent grid size of k_render_lds
    bool has_cubes = false;     // cube acceptance depends on the visiting order: no wave walk
    void *d_nodes = nullptr, *d_prims = nullptr, *d_shade = nullptr, *d_mats = nullptr, *d_sky = nullptr;
    void *d_xprims = nullptr, *d_tex = nullptr;
    void *d_scratch = nullptr;  // staging for the host-pointer batched calls
    size_t scratch_bytes = 0;
    hipStream_t stream = nullptr;
};

struct rt_renderer {
    rt_scene *scene = nullptr;
    uint32_t W = 0, H = 0;
    float4 *d_acc = nullptr;
    unsigned long long *d_counters = nullptr;
    uint32_t *d_rgb = nullptr;   // staging frame for rt_render_frame_host
    uint64_t primary = 0, frames = 0;
    hipStream_t stream = nullptr;
};

namespace {

inline float ubits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline float ibits(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

uint32_t pick_stack(uint32_t depth) {   // entries needed <= tree depth; round up to 8
    uint32_t need = depth < 2 ? 2 : depth;
    return (need + 7u) & ~7u;
}

int material_flag(const rt_material &m, float diffuse, float specular) {   // getFlag overrides
    switch (m.kind) {
    case RT_DIFFUSE: return F_DIFFUSE;
    case RT_MIRROR: return F_SPECULAR;
    case RT_DIELECTRIC: return F_DIELECTRIC;
    case RT_LIGHT: return F_LIGHT;
    default:
        if (diffuse < kFLT_EPSILON) return F_SPECULAR;
        if (specular < kFLT_EPSILON) return F_DIFFUSE;
        return F_MIX;
    }
}

int validate_bvh(const Bvh &b, uint32_t n) {
    if (b.nodes_used < 2 || b.nodes_used > b.nodes.size()) return fail(RT_ERR_INVALID, "BVH node count out of range");
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (b.indices[i] >= n || seen[b.indices[i]]) return fail(RT_ERR_INVALID, "BVH indices are not a permutation");
        seen[b.indices[i]] = 1;
    }
    // walk from the root: children in range, leaves inside the index array
    std::vector<uint32_t> st{0};
    size_t visits = 0;
    while (!st.empty()) {
        uint32_t k = st.back();
        st.pop_back();
        if (++visits > 2 * (size_t)b.nodes_used) return fail(RT_ERR_INVALID, "BVH has a cycle");
        const Node &nd = b.nodes[k];
        if (nd.count > 0) {
            if ((uint64_t)nd.leftFirst + nd.count > n) return fail(RT_ERR_INVALID, "BVH leaf outside the index array");
            continue;
        }
        if (nd.leftFirst < 2 || nd.leftFirst + 1 >= b.nodes_used || (nd.leftFirst & 1u))
            return fail(RT_ERR_INVALID, "BVH child pair out of range / misaligned");
        st.push_back(nd.leftFirst);
        st.push_back(nd.leftFirst + 1);
    }
    return RT_OK;
}

void free_scene(rt_scene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipDeviceSynchronize();
    void *ptrs[] = {s->d_nodes, s->d_prims, s->d_shade, s->d_mats, s->d_sky, s->d_xprims, s->d_tex, s->d_scratch};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

template <typename T>
int upload(void **dst, const std::vector<T> &src) {
    HIP_TRY(hipMalloc(dst, std::max<size_t>(sizeof(T) * src.size(), 16)));
    if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice));
    return RT_OK;
}

int ensure_device(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(RT_ERR_NO_DEVICE, "no HIP device visible: the MI355X path has no CPU fallback");
    if (device < 0 || device >= count) return fail(RT_ERR_INVALID, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    return RT_OK;
}

inline f3 tvec_host(float4 r0, float4 r1, float4 r2, f3 a) {
    const float M[12] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w};
    return tvec(M, a);
}

int scene_create(const rt_scene_desc *d, rt_scene **out) {
    if (!d || !out || !d->prims || d->num_prims == 0 || !d->materials || d->num_materials == 0)
        return fail(RT_ERR_INVALID, "rt_scene_create: empty or null description");
    *out = nullptr;
    const uint32_t n = d->num_prims;
    if (n >= (1u << 24)) return fail(RT_ERR_UNSUPPORTED, "more than 2^24 primitives");
    for (uint32_t i = 0; i < n; ++i) {
        const rt_prim &p = d->prims[i];
        if (p.type < RT_SPHERE || p.type > RT_TRIANGLE)
            return fail(RT_ERR_INVALID, "primitive " + std::to_string(i) + ": unknown type");
        if (p.material < 0 || (uint32_t)p.material >= d->num_materials)
            return fail(RT_ERR_INVALID, "primitive " + std::to_string(i) + ": material out of range");
    }
    if (d->prims[0].type != RT_SPHERE && d->prims[0].type != RT_QUAD)
        return fail(RT_ERR_UNSUPPORTED, "primitive 0 must be the light, a sphere or a quad (Scene::GetRandomLight returns 0)");
    for (uint32_t i = 0; i < d->num_materials; ++i) {
        const rt_material &m = d->materials[i];
        if (m.kind < RT_DIFFUSE || m.kind > RT_TEXTURE) return fail(RT_ERR_INVALID, "unknown material kind");
        if (m.kind == RT_TEXTURE && (m.texture < 0 || (uint32_t)m.texture >= d->num_textures || !d->textures))
            return fail(RT_ERR_INVALID, "material " + std::to_string(i) + ": texture index out of range");
    }
    for (uint32_t i = 0; i < d->num_textures; ++i)
        if (!d->textures[i].pixels || !d->textures[i].width || !d->textures[i].height)
            return fail(RT_ERR_INVALID, "texture " + std::to_string(i) + " is empty");
    if (d->sky_pixels) {
        uint32_t w = d->sky_width, h = d->sky_height;
        if (!w || !h || (w & (w - 1)) || (h & (h - 1)))
            return fail(RT_ERR_INVALID, "sky texture must have power-of-two sides (renderer.h:18)");
    }
    int rc = ensure_device(d->device);
    if (rc != RT_OK) return rc;

    rt_scene *s = new rt_scene();
    s->device = d->device;
    s->num_prims = n;
    // ---- BVH: prebuilt (validated) or built here
    if (d->bvh_nodes) {
        if (!d->bvh_indices || d->bvh_num_nodes < 2) { delete s; return fail(RT_ERR_INVALID, "prebuilt BVH incomplete"); }
        s->bvh.nodes.resize(d->bvh_num_nodes);
        std::memcpy(s->bvh.nodes.data(), d->bvh_nodes, sizeof(Node) * d->bvh_num_nodes);
        s->bvh.indices.assign(d->bvh_indices, d->bvh_indices + n);
        s->bvh.nodes_used = d->bvh_num_nodes;
        if ((rc = validate_bvh(s->bvh, n)) != RT_OK) { delete s; return rc; }
        // depth + widest leaf
        // depth as Scene::maxDepthBVH (template/scene.h:144-154): interior levels, root leaf = 1
        std::vector<std::pair<uint32_t, uint32_t>> st{{0, 0}};
        while (!st.empty()) {
            auto [k, dd] = st.back();
            st.pop_back();
            const Node &nd = s->bvh.nodes[k];
            if (nd.count > 0) {
                s->bvh.max_leaf = std::max(s->bvh.max_leaf, nd.count);
                s->bvh.depth = std::max(s->bvh.depth, k == 0 ? 1u : dd);
                continue;
            }
            st.push_back({nd.leftFirst, dd + 1});
            st.push_back({nd.leftFirst + 1, dd + 1});
        }
    } else if ((rc = build_bvh(d->prims, d->transforms, n, s->bvh)) != RT_OK) {
        delete s;
        return rc;
    }
    if (s->bvh.max_leaf > 255) { delete s; return fail(RT_ERR_UNSUPPORTED, "BVH leaf with more than 255 primitives"); }
    if (s->bvh.depth > 64) { delete s; return fail(RT_ERR_UNSUPPORTED, "BVH deeper than 64 (the reference's stack[64])"); }
    s->stack_depth = pick_stack(s->bvh.depth);

    // ---- device node array: packed (leftFirst << 8 | count) word in b.z
    std::vector<float4> nodes(2 * (size_t)s->bvh.nodes_used);
    for (uint32_t i = 0; i < s->bvh.nodes_used; ++i) {
        const Node &nd = s->bvh.nodes[i];
        uint32_t word = (nd.leftFirst << 8) | nd.count;
        nodes[2 * i] = make_float4(nd.mn[0], nd.mn[1], nd.mn[2], nd.mx[0]);
        nodes[2 * i + 1] = make_float4(nd.mx[1], nd.mx[2], ubits(word), 0.0f);
    }
    // ---- leaf-order primitive records and per-id shading records; cubes and quads keep
    // their matrices and data in a side table (8 float4 each)
    static const float I16[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    std::vector<float4> prims(3 * (size_t)n), shade(2 * (size_t)n), xprims;
    std::vector<uint32_t> xindex(n, 0);
    for (uint32_t id = 0; id < n; ++id) {
        const rt_prim &p = d->prims[id];
        if (p.type != RT_CUBE && p.type != RT_QUAD) continue;
        if (p.type == RT_CUBE) s->has_cubes = true;
        PrimX x;
        prim_transform(p, d->transforms ? d->transforms + 16 * (size_t)id : nullptr, x);
        xindex[id] = (uint32_t)(xprims.size() / 8);
        for (int r = 0; r < 3; ++r) xprims.push_back(make_float4(x.Minv[4 * r], x.Minv[4 * r + 1], x.Minv[4 * r + 2], x.Minv[4 * r + 3]));
        for (int r = 0; r < 3; ++r) xprims.push_back(make_float4(x.M[4 * r], x.M[4 * r + 1], x.M[4 * r + 2], x.M[4 * r + 3]));
        if (p.type == RT_CUBE) {   // data[0] = -0.5 size, data[1] = 0.5 size (Primitive.h:724-725)
            const f3 sz = mk(p.v[3], p.v[4], p.v[5]), a = -0.5f * sz, b = 0.5f * sz;
            xprims.push_back(make_float4(a.x, a.y, a.z, 0.0f));
            xprims.push_back(make_float4(b.x, b.y, b.z, 0.0f));
        } else {                   // data[0].x = 0.5 size (Primitive.h:737)
            xprims.push_back(make_float4(0.5f * p.v[0], 0.0f, 0.0f, 0.0f));
            xprims.push_back(make_float4(0, 0, 0, 0));
        }
    }
    for (uint32_t id = 0; id < n; ++id) {
        const rt_prim &p = d->prims[id];
        float4 s0, s1 = make_float4(ubits((uint32_t)p.type), 0, 0, 0);
        if (p.type == RT_CUBE || p.type == RT_QUAD) {
            const float4 *x = &xprims[8 * (size_t)xindex[id]];
            // quad: constant normal TransformVector((0,-1,0), Transform) (Primitive.h:306-307)
            f3 N = p.type == RT_QUAD ? tvec_host(x[3], x[4], x[5], mk(0, -1, 0)) : mk(0, 0, 0);
            s0 = make_float4(N.x, N.y, N.z, ibits(p.material));
            s1.z = ubits(xindex[id]);
        } else if (p.type == RT_TRIANGLE) {
            f3 d0 = mk(p.v[0], p.v[1], p.v[2]), d1 = mk(p.v[3], p.v[4], p.v[5]), d2 = mk(p.v[6], p.v[7], p.v[8]);
            f3 N = tvec(I16, normalize(cross(d2 - d0, d1 - d0)));      // Primitive.h:308-310
            s0 = make_float4(N.x, N.y, N.z, ibits(p.material));
        } else if (p.type == RT_SPHERE) {
            float T[16];
            translate_matrix(p.v[0], p.v[1], p.v[2], T);
            f3 c = tpos(T, mk(0, 0, 0));
            s0 = make_float4(c.x, c.y, c.z, ibits(p.material));
            s1.y = 1.0f / p.v[3];                                      // data[0].z
        } else {
            s0 = make_float4(p.v[0], p.v[1], p.v[2], ibits(p.material));
        }
        shade[2 * id] = s0;
        shade[2 * id + 1] = s1;
    }
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t id = s->bvh.indices[k];
        const rt_prim &p = d->prims[id];
        float4 *q = &prims[3 * (size_t)k];
        if (p.type == RT_TRIANGLE) {
            f3 A = tpos(I16, mk(p.v[0], p.v[1], p.v[2]));                 // Intersect, Primitive.h:249-254
            f3 B = tpos(I16, mk(p.v[3], p.v[4], p.v[5]));
            f3 C = tpos(I16, mk(p.v[6], p.v[7], p.v[8]));
            f3 AB = B - A, AC = C - A;
            q[0] = make_float4(A.x, A.y, A.z, ibits((int)id));
            q[1] = make_float4(AB.x, AB.y, AB.z, ubits(T_TRI));
            q[2] = make_float4(AC.x, AC.y, AC.z, 0.0f);
        } else if (p.type == RT_SPHERE) {
            float T[16];
            translate_matrix(p.v[0], p.v[1], p.v[2], T);
            f3 c = tpos(T, mk(0, 0, 0));
            float r = p.v[3];
            q[0] = make_float4(c.x, c.y, c.z, ibits((int)id));
            q[1] = make_float4(r * r, 0.0f, 0.0f, ubits(T_SPH)); // data[0].y
            q[2] = make_float4(0, 0, 0, 0);
        } else if (p.type == RT_PLANE) {
            q[0] = make_float4(p.v[0], p.v[1], p.v[2], ibits((int)id));
            q[1] = make_float4(p.v[3], 0.0f, 0.0f, ubits(T_PLANE));
            q[2] = make_float4(0, 0, 0, 0);
        } else {
            q[0] = make_float4(0, 0, 0, ibits((int)id));
            q[1] = make_float4(ubits(xindex[id]), 0.0f, 0.0f, ubits(p.type == RT_CUBE ? T_CUBE : T_QUAD));
            q[2] = make_float4(0, 0, 0, 0);
        }
    }
    // ---- textures, concatenated
    std::vector<uint32_t> texels, tex_offsets;
    for (uint32_t i = 0; i < d->num_textures; ++i) {
        const rt_texture &t = d->textures[i];
        tex_offsets.push_back((uint32_t)texels.size());
        texels.insert(texels.end(), t.pixels, t.pixels + (size_t)t.width * t.height);
    }
    if (texels.empty()) texels.push_back(0);
    if (xprims.empty()) xprims.push_back(make_float4(0, 0, 0, 0));
    // ---- materials
    std::vector<DevMaterial> mats(d->num_materials);
    for (uint32_t i = 0; i < d->num_materials; ++i) {
        const rt_material &m = d->materials[i];
        DevMaterial &o = mats[i];
        std::memset(&o, 0, sizeof(o));
        o.kind = m.kind;
        for (int c = 0; c < 3; ++c) { o.c0[c] = m.color[c]; o.c1[c] = m.color2[c]; }
        o.ior = m.ior;
        // Checkerboard.h:6-14, TextureMaterial.h:6-17 (short ctor: diffuse 1, specular 0),
        // DSMix.h:6-9 (always clamped): clamp = fmaxf(a, fminf(f, b)), precomp.h:782
        if (m.kind == RT_CHECKERBOARD || m.kind == RT_TEXTURE || m.kind == RT_DSMIX) {
            if (m.diffuse < 0.0f && m.kind != RT_DSMIX) { o.diffuse = 1.0f; o.specular = 0.0f; }
            else { o.diffuse = tmax(0.0f, tmin(m.diffuse, 1.0f)); o.specular = 1.0f - o.diffuse; }
        }
        if (m.kind == RT_TEXTURE) {
            const rt_texture &t = d->textures[m.texture];
            o.tex_off = tex_offsets[m.texture];
            o.tex_w = t.width; o.tex_h = t.height;
        }
        o.flag = material_flag(m, o.diffuse, o.specular);
    }
    // ---- sky
    std::vector<uint32_t> sky;
    uint32_t sw = 1024, sh = 512;
    if (d->sky_pixels) {
        sw = d->sky_width; sh = d->sky_height;
        sky.assign(d->sky_pixels, d->sky_pixels + (size_t)sw * sh);
    } else {
        sky.assign((size_t)sw * sh, 0x406080u);
    }
    bool sky_const = std::all_of(sky.begin(), sky.end(), [&](uint32_t v) { return v == sky[0]; });

    rc = RT_OK;
    if (rc == RT_OK) rc = upload(&s->d_nodes, nodes);
    if (rc == RT_OK) rc = upload(&s->d_prims, prims);
    if (rc == RT_OK) rc = upload(&s->d_shade, shade);
    if (rc == RT_OK) rc = upload(&s->d_mats, mats);
    if (rc == RT_OK) rc = upload(&s->d_sky, sky);
    if (rc == RT_OK) rc = upload(&s->d_xprims, xprims);
    if (rc == RT_OK) rc = upload(&s->d_tex, texels);
    if (rc == RT_OK && hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        rc = fail(RT_ERR_HIP, "hipStreamCreate failed");
    if (rc != RT_OK) { free_scene(s); return rc; }

    SceneView &v = s->view;
    v.nodes = (const float4 *)s->d_nodes;
    v.prims = (const float4 *)s->d_prims;
    v.shade = (const float4 *)s->d_shade;
    v.mats = (const DevMaterial *)s->d_mats;
    v.sky = (const uint32_t *)s->d_sky;
    v.xprims = (const float4 *)s->d_xprims;
    v.tex = (const uint32_t *)s->d_tex;
    v.sky_w = sw; v.sky_h = sh;
    v.sky_const = sky_const ? 1 : 0;
    {
        uint32_t p = sky[0];
        f3 c = mk((float)((p >> 16) & 255), (float)((p >> 8) & 255), (float)(p & 255)) * kSKY;
        v.sky_rgb[0] = c.x; v.sky_rgb[1] = c.y; v.sky_rgb[2] = c.z;
    }
    const rt_prim &L = d->prims[0];
    PrimX LX;
    prim_transform(L, d->transforms ? d->transforms : nullptr, LX);
    std::memcpy(v.light_M, LX.M, sizeof(v.light_M));
    f3 lc = tpos(LX.M, mk(0, 0, 0));
    v.light_c[0] = lc.x; v.light_c[1] = lc.y; v.light_c[2] = lc.z;
    v.light_mat = L.material;
    v.light_quad = L.type == RT_QUAD;
    if (v.light_quad) {
        v.light_qsize = 0.5f * L.v[0];
        const float side = 2.0f * v.light_qsize;                      // GetArea, Primitive.h:461-463
        v.light_area = side * side;
        const f3 N = tvec(LX.M, mk(0, -1, 0));
        v.light_N[0] = N.x; v.light_N[1] = N.y; v.light_N[2] = N.z;
    } else {
        v.light_r = L.v[3];
        v.light_r2 = L.v[3] * L.v[3];
        v.light_invr = 1.0f / L.v[3];
        v.light_area = 4.0f * kPI * v.light_r2;                        // Primitive.h:452
    }
    const Node &root = s->bvh.nodes[0];
    v.root_word = (root.leftFirst << 8) | root.count;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, s->device) == hipSuccess && prop.multiProcessorCount > 0)
            s->num_cus = (uint32_t)prop.multiProcessorCount;
    }
    v.stack_entries = s->stack_depth;
    v.node_f4 = 2u * s->bvh.nodes_used;
#ifndef RT_DISABLE_LDS_SCENE
    s->lds_nodes = (size_t)s->stack_depth * 4096u + (size_t)s->bvh.nodes_used * 32u <= 160u * 1024u;
#endif
    // camera-ray walk: wave-coherent vs per-lane (RT_WAVE_PRIMARY=0/1 overrides the policy)
    v.wave_primary = 0;
    if (const char *e = std::getenv("RT_WAVE_PRIMARY")) v.wave_primary = std::atoi(e) != 0 && !s->has_cubes;
    v.bounds_finite = 1;
    for (uint32_t i = 0; i < s->bvh.nodes_used && v.bounds_finite; ++i) {
        if (i == 1) continue;
        const Node &nd = s->bvh.nodes[i];
        for (int c = 0; c < 3; ++c)
            if (!std::isfinite(nd.mn[c]) || !std::isfinite(nd.mx[c])) v.bounds_finite = 0;
    }
    *out = s;
    return RT_OK;
}

size_t stack_bytes(const rt_scene *s) { return (size_t)s->stack_depth * 256u * sizeof(uint32_t); }
// k_render_lds: [stack_entries][1024] u32 stacks, then the node array
size_t lds_scene_bytes(const rt_scene *s) {
    return (size_t)s->stack_depth * 1024u * sizeof(uint32_t) + (size_t)s->bvh.nodes_used * 32u;
}

int launch_render(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                  uint32_t *out, int packed, void *stream) {
    if (!r || !cam || !p || !out) return fail(RT_ERR_INVALID, "rt_render: null argument");
    if (p->width != r->W || p->height != r->H)
        return fail(RT_ERR_INVALID, "frame size differs from the renderer's accumulator");
    if (p->spp == 0) return fail(RT_ERR_INVALID, "spp must be >= 1");
    if (p->mode > RT_MODE_PACKET) return fail(RT_ERR_INVALID, "unknown integrator mode");
    if (nshards == 0 || shard >= nshards) return fail(RT_ERR_INVALID, "bad shard index");
    rt_scene *s = r->scene;
    HIP_TRY(hipSetDevice(s->device));
    FrameArgs F{};
    for (int i = 0; i < 3; ++i) {
        F.cam_pos[i] = cam->pos[i]; F.cam_tl[i] = cam->top_left[i];
        F.cam_tr[i] = cam->top_right[i]; F.cam_bl[i] = cam->bottom_left[i];
    }
    F.lens = cam->lens_radius;
    F.rw = 1.0f / (float)r->W;   // Camera::rWidth / rHeight (camera.h:98-99)
    F.rh = 1.0f / (float)r->H;
    F.W = r->W; F.H = r->H; F.spp = p->spp; F.depth = p->depth; F.frame = p->frame; F.reset = p->reset ? 1 : 0;
    const uint32_t tiles_x = (r->W + 7) / 8, tiles_y = (r->H + 7) / 8, ntiles = tiles_x * tiles_y;
    F.shard = shard; F.nshards = nshards; F.tiles_x = tiles_x;
    F.ntiles_local = shard < ntiles ? (ntiles - shard + nshards - 1) / nshards : 0;
    F.packed_out = packed;
    F.acc = r->d_acc;
    F.out = out;
    F.counters = r->d_counters;
    if (F.ntiles_local == 0) return RT_OK;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t depth = p->depth;
    if (depth > 32) return fail(RT_ERR_UNSUPPORTED, "Trace depth above 32");   // = kWHITTED_MAX
    const int md = depth <= 1 ? 1 : depth <= 4 ? 4 : depth <= 10 ? 10 : 32;
    const bool tex = !s->view.sky_const;
    const int mode = (int)p->mode;
    // LDS nodes pay off where registers allow 1024-thread workgroups without spilling:
    // the primary+shadow kernel with the constant sky (103 VGPRs); the path-tracing
    // variants keep the 256-thread global-node kernel (A/B in profiles/r01).
    const bool use_lds = s->lds_nodes && mode == RT_MODE_PATH && md == 1 && !tex;
    dim3 grid, block;
    size_t lds;
    if (use_lds) {
        grid = dim3((F.ntiles_local + 15) / 16);
        block = dim3(1024);
        lds = lds_scene_bytes(s);
    } else {
        grid = dim3((F.ntiles_local + 3) / 4);
        block = dim3(256);
        lds = stack_bytes(s);
    }
#define RT_LAUNCH(MO, MD, TX) hipLaunchKernelGGL((k_render<MO, MD, TX>), grid, block, lds, st, s->view, F)
    if (use_lds) hipLaunchKernelGGL((k_render_lds<1, false>), grid, block, lds, st, s->view, F);
    else if (mode == RT_MODE_WHITTED) {
        if (tex) RT_LAUNCH(M_WHITTED, 1, true); else RT_LAUNCH(M_WHITTED, 1, false);
    } else if (mode == RT_MODE_PACKET) {                // depth = the bounces' Trace depth (0 allowed)
        const int pd = depth <= 1 ? 1 : depth <= 10 ? 10 : 32;
        switch (pd * 2 + (tex ? 1 : 0)) {
        case 2: RT_LAUNCH(M_PACKET, 1, false); break;
        case 3: RT_LAUNCH(M_PACKET, 1, true); break;
        case 20: RT_LAUNCH(M_PACKET, 10, false); break;
        case 21: RT_LAUNCH(M_PACKET, 10, true); break;
        case 64: RT_LAUNCH(M_PACKET, 32, false); break;
        default: RT_LAUNCH(M_PACKET, 32, true); break;
        }
    } else switch (md * 2 + (tex ? 1 : 0)) {
    case 2: RT_LAUNCH(M_PATH, 1, false); break;
    case 3: RT_LAUNCH(M_PATH, 1, true); break;
    case 8: RT_LAUNCH(M_PATH, 4, false); break;
    case 9: RT_LAUNCH(M_PATH, 4, true); break;
    case 20: RT_LAUNCH(M_PATH, 10, false); break;
    case 21: RT_LAUNCH(M_PATH, 10, true); break;
    case 64: RT_LAUNCH(M_PATH, 32, false); break;
    default: RT_LAUNCH(M_PATH, 32, true); break;
    }
#undef RT_LAUNCH
    HIP_TRY(hipGetLastError());
    // pixels covered by this launch (primary rays per sample)
    uint64_t px = (uint64_t)F.ntiles_local * 64u;
    if ((r->W & 7u) || (r->H & 7u)) {
        px = 0;
        for (uint32_t t = shard; t < ntiles; t += nshards) {
            uint32_t tx = t % tiles_x, ty = t / tiles_x;
            px += (uint64_t)std::min(8u, r->W - tx * 8) * std::min(8u, r->H - ty * 8);
        }
    }
    (void)tiles_y;
    r->primary += px * p->spp;
    r->frames += 1;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_device_count(int *count) {
    if (!count) return fail(RT_ERR_INVALID, "null count");
    *count = 0;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) return fail(RT_ERR_NO_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    *count = c;
    return RT_OK;
}

int rt_scene_create(const rt_scene_desc *desc, rt_scene **out) {
    try {
        return scene_create(desc, out);
    } catch (const std::exception &e) {
        return fail(RT_ERR_INVALID, std::string("rt_scene_create: ") + e.what());
    }
}

int rt_scene_create_recipe(const char *name, const char *mesh_dir, int32_t device, rt_scene **out) {
    if (!name || !mesh_dir || !out) return fail(RT_ERR_INVALID, "rt_scene_create_recipe: null argument");
    try {
        SceneSource src;
        int rc = recipe_source(name, mesh_dir, src);
        if (rc != RT_OK) return rc;
        rt_scene_desc d{};
        d.prims = src.prims.data();
        d.num_prims = (uint32_t)src.prims.size();
        d.materials = src.materials.data();
        d.num_materials = (uint32_t)src.materials.size();
        d.device = device;
        return scene_create(&d, out);
    } catch (const std::exception &e) {
        return fail(RT_ERR_INVALID, std::string("rt_scene_create_recipe: ") + e.what());
    }
}

int rt_scene_destroy(rt_scene *s) {
    free_scene(s);
    return RT_OK;
}

int rt_scene_get_info(const rt_scene *s, rt_scene_info *info) {
    if (!s || !info) return fail(RT_ERR_INVALID, "null argument");
    info->num_prims = s->num_prims;
    info->nodes_used = s->bvh.nodes_used;
    info->depth = s->bvh.depth;
    info->max_leaf = s->bvh.max_leaf;
    return RT_OK;
}

int rt_scene_set_camera_walk(rt_scene *s, int walk) {
    if (!s) return fail(RT_ERR_INVALID, "null argument");
    if (walk != RT_WALK_LANE && walk != RT_WALK_WAVE) return fail(RT_ERR_INVALID, "unknown camera walk");
    if (walk == RT_WALK_WAVE && s->has_cubes)
        return fail(RT_ERR_UNSUPPORTED, "the wave walk needs order-independent hits; cubes accept on tmax (Primitive.h:221-233)");
    s->view.wave_primary = walk == RT_WALK_WAVE;
    return RT_OK;
}

int rt_scene_copy_bvh(const rt_scene *s, void *nodes, uint32_t *indices) {
    if (!s || !nodes || !indices) return fail(RT_ERR_INVALID, "null argument");
    std::memcpy(nodes, s->bvh.nodes.data(), sizeof(Node) * s->bvh.nodes_used);
    std::memcpy(indices, s->bvh.indices.data(), sizeof(uint32_t) * s->num_prims);
    return RT_OK;
}

int rt_intersect(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !hits))) return fail(RT_ERR_INVALID, "rt_intersect: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_intersect, dim3((n + 255) / 256), dim3(256), stack_bytes(s), st, s->view, rays, hits, n);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_occluded(rt_scene *s, const rt_ray *rays, uint8_t *out, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !out))) return fail(RT_ERR_INVALID, "rt_occluded: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_occluded, dim3((n + 255) / 256), dim3(256), stack_bytes(s), st, s->view, rays, out, n);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_intersect_packets(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !hits))) return fail(RT_ERR_INVALID, "rt_intersect_packets: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_intersect_packet, dim3((n + 255) / 256), dim3(256), 0, st, s->view, rays, hits, n);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}
enum { CALL_INTERSECT, CALL_OCCLUDED, CALL_PACKETS };
static int staged_call(rt_scene *s, const rt_ray *rays, void *out, size_t out_elem, uint32_t n, int kind) {
    if (!s || (n && (!rays || !out))) return fail(RT_ERR_INVALID, "null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    size_t need = (size_t)n * (sizeof(rt_ray) + out_elem) + 256;
    if (need > s->scratch_bytes) {
        if (s->d_scratch) HIP_TRY(hipFree(s->d_scratch));
        s->d_scratch = nullptr;
        s->scratch_bytes = 0;
        HIP_TRY(hipMalloc(&s->d_scratch, need));
        s->scratch_bytes = need;
    }
    rt_ray *d_rays = (rt_ray *)s->d_scratch;
    char *d_out = (char *)s->d_scratch + (((size_t)n * sizeof(rt_ray) + 255) & ~(size_t)255);
    HIP_TRY(hipMemcpyAsync(d_rays, rays, sizeof(rt_ray) * n, hipMemcpyHostToDevice, s->stream));
    int rc = kind == CALL_OCCLUDED ? rt_occluded(s, d_rays, (uint8_t *)d_out, n, s->stream)
             : kind == CALL_PACKETS ? rt_intersect_packets(s, d_rays, (rt_hit *)d_out, n, s->stream)
                                    : rt_intersect(s, d_rays, (rt_hit *)d_out, n, s->stream);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out, out_elem * n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return RT_OK;
}

int rt_intersect_host(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n) {
    return staged_call(s, rays, hits, sizeof(rt_hit), n, CALL_INTERSECT);
}
int rt_occluded_host(rt_scene *s, const rt_ray *rays, uint8_t *out, uint32_t n) {
    return staged_call(s, rays, out, 1, n, CALL_OCCLUDED);
}
int rt_intersect_packets_host(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n) {
    return staged_call(s, rays, hits, sizeof(rt_hit), n, CALL_PACKETS);
}

int rt_renderer_create(rt_scene *s, uint32_t W, uint32_t H, rt_renderer **out) {
    if (!s || !out || !W || !H) return fail(RT_ERR_INVALID, "rt_renderer_create: bad argument");
    if ((uint64_t)W * H >= (1ull << 31)) return fail(RT_ERR_UNSUPPORTED, "frame too large");
    HIP_TRY(hipSetDevice(s->device));
    rt_renderer *r = new rt_renderer();
    r->scene = s;
    r->W = W; r->H = H;
    hipError_t e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&r->d_acc, sizeof(float4) * (size_t)W * H);   // Renderer::Init, renderer.cpp:6-12
    if (e == hipSuccess) e = hipMemsetAsync(r->d_acc, 0, sizeof(float4) * (size_t)W * H, r->stream);
    if (e == hipSuccess) e = hipMalloc(&r->d_counters, 4 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemsetAsync(r->d_counters, 0, 4 * sizeof(unsigned long long), r->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(r->stream);   // ready before any caller stream uses it
    if (e != hipSuccess) {
        if (r->d_acc) (void)hipFree(r->d_acc);
        if (r->d_counters) (void)hipFree(r->d_counters);
        if (r->stream) (void)hipStreamDestroy(r->stream);
        delete r;
        return fail(RT_ERR_HIP, std::string("rt_renderer_create: ") + hipGetErrorString(e));
    }
    *out = r;
    return RT_OK;
}

int rt_renderer_destroy(rt_renderer *r) {
    if (!r) return RT_OK;
    (void)hipSetDevice(r->scene->device);
    (void)hipDeviceSynchronize();   // kernels on caller streams may still read the buffers
    (void)hipFree(r->d_acc);
    (void)hipFree(r->d_counters);
    if (r->d_rgb) (void)hipFree(r->d_rgb);
    (void)hipStreamDestroy(r->stream);
    delete r;
    return RT_OK;
}

int rt_render_frame(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t *rgb8, void *stream) {
    return launch_render(r, cam, p, 0, 1, rgb8, 0, stream);
}

int rt_render_frame_host(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t *rgb8) {
    if (!r || !rgb8) return fail(RT_ERR_INVALID, "rt_render_frame_host: null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    if (!r->d_rgb) HIP_TRY(hipMalloc(&r->d_rgb, sizeof(uint32_t) * (size_t)r->W * r->H));
    int rc = launch_render(r, cam, p, 0, 1, r->d_rgb, 0, r->stream);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(rgb8, r->d_rgb, sizeof(uint32_t) * (size_t)r->W * r->H, hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    return RT_OK;
}

int rt_shard_capacity(uint32_t W, uint32_t H, uint32_t nshards, uint32_t *pixels) {
    if (!pixels || !nshards || !W || !H) return fail(RT_ERR_INVALID, "rt_shard_capacity: bad argument");
    uint32_t ntiles = ((W + 7) / 8) * ((H + 7) / 8);
    *pixels = ((ntiles + nshards - 1) / nshards) * 64u;
    return RT_OK;
}

int rt_render_shard(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                    uint32_t *tiles, void *stream) {
    return launch_render(r, cam, p, shard, nshards, tiles, 1, stream);
}

int rt_assemble_shards(rt_renderer *r, const uint32_t *gathered, uint32_t nshards, uint32_t *rgb8, void *stream) {
    if (!r || !gathered || !rgb8 || !nshards) return fail(RT_ERR_INVALID, "rt_assemble_shards: bad argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    uint32_t cap = 0;
    rt_shard_capacity(r->W, r->H, nshards, &cap);
    uint32_t tiles_x = (r->W + 7) / 8, ntiles = tiles_x * ((r->H + 7) / 8);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_assemble, dim3((ntiles + 3) / 4), dim3(256), 0, st, gathered, cap, nshards, tiles_x, ntiles,
                       r->W, r->H, rgb8);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_renderer_counters(rt_renderer *r, rt_counters *out) {
    if (!r || !out) return fail(RT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long c[4];
    HIP_TRY(hipMemcpy(c, r->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    out->primary = r->primary;
    out->shadow = c[0];
    out->bounce = c[1];
    out->frames = r->frames;
    return RT_OK;
}

int rt_renderer_read_accumulator(rt_renderer *r, float *host) {
    if (!r || !host) return fail(RT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(host, r->d_acc, sizeof(float4) * (size_t)r->W * r->H, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_renderer_stream(rt_renderer *r, void **stream) {
    if (!r || !stream) return fail(RT_ERR_INVALID, "null argument");
    *stream = (void *)r->stream;
    return RT_OK;
}

int rt_synchronize(rt_renderer *r) {
    if (!r) return fail(RT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    HIP_TRY(hipDeviceSynchronize());
    return RT_OK;
}

}  // extern "C"
