/*
 * rt_oracle.c -- CPU restatement of the reference's hot path (TEST INFRASTRUCTURE).
 *
 * See rt_oracle.h for scope and the parity-pin statement ("partial": pinned by
 * the reference-run statistics of SURVEY.md, the reference itself being
 * unbuildable here without stand-in headers).
 *
 * Arithmetic rules: float32 throughout, no FMA
 * contraction (built with -ffp-contract=off), correctly rounded / and sqrtf,
 * std::min/max = (b<a)?b:a / (a<b)?b:a, the template's fminf/fmaxf = a<b?a:b,
 * left-to-right sums exactly as the reference writes them.
 * In-path transcendentals (cosf, sinf, expf, atan2f, acosf, asinf) are taken as
 * the correctly rounded float of the double-precision function; the device
 * kernels do the same so parity does not hinge on libm last-ulp choices (the
 * reference's MSVC CRT is unpinnable anyway).  mat4 construction uses libm
 * cosf/sinf, as the Linux build of template/precomp.h:1007-1009 does.
 */
#include "rt_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* template/common.h:7-12, template/precomp.h:1656-1657 */
#define PI_F 3.14159265358979323846264f
#define INVPI_F 0.31830988618379067153777f
#define INV2PI_F 0.15915494309189533576888f
#define TWOPI_F 6.28318530717958647692528f
#define EPS_F 0.0001f
#define SKYDOME_CORRECTION_F 0.00392156862745f
#define FLT_EPS_F 1.192092896e-07f
#define CL_DBL_EPS 2.220446049250313080847e-16 /* compared as double, Primitive.h:128,258 */
#define BIN_COUNT 32                           /* BVHNode.h:3 */

/* ------------------------------------------------------------------ math */
typedef struct { float x, y, z; } f3;

static inline f3 mk(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }     /* float3*float */
static inline f3 smul(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }     /* float*float3 */
static inline f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* precomp.h:805 */
static inline f3 cross(f3 a, f3 b) {                                               /* precomp.h:855 */
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float length3(f3 v) { return sqrtf(dot(v, v)); }                     /* precomp.h:816 */
static inline f3 normalize(f3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return muls(v, inv); } /* 827 */
static inline f3 reflect(f3 i, f3 n) { return sub(i, muls(smul(2.0f, n), dot(n, i))); }      /* 853 */
static inline float smin(float a, float b) { return (b < a) ? b : a; }  /* std::min */
static inline float smax(float a, float b) { return (a < b) ? b : a; }  /* std::max */
static inline float tmin_(float a, float b) { return a < b ? a : b; }   /* precomp.h:471 fminf */
static inline float tmax_(float a, float b) { return a > b ? a : b; }   /* precomp.h:472 fmaxf */
static inline f3 fmin3(f3 a, f3 b) { return mk(tmin_(a.x, b.x), tmin_(a.y, b.y), tmin_(a.z, b.z)); }
static inline f3 fmax3(f3 a, f3 b) { return mk(tmax_(a.x, b.x), tmax_(a.y, b.y), tmax_(a.z, b.z)); }
static inline float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* In-path cosf/sinf/expf (ObjectMaterial.h:32-33, Dielectric.h:15-17): double evaluation of
 * fdlibm's minimax kernels with basic operations only, rounded once to float -- the same
 * operation sequence as the kernels' csrc/rt_libm.h, so both sides agree bit for bit. */
static inline double rint_small(double v) { const double sh = 6755399441055744.0; return (v + sh) - sh; }
static inline double ksin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}
static inline double kcos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}
static inline void sincos_f(float a, float *s, float *c) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11;
    double x = (double)a;
    double k = rint_small(x * invpio2);
    double r = (x - k * pio2_1) - k * pio2_1t;
    double sr = ksin(r), cr = kcos(r);
    int q = (int)k & 3;
    *s = (float)(q == 0 ? sr : q == 1 ? cr : q == 2 ? -sr : -cr);
    *c = (float)(q == 0 ? cr : q == 1 ? -sr : q == 2 ? -cr : sr);
}
static inline float exp_f(float a) {
    if (!(a == a)) return a;
    if (a > 88.8f) return 1.0f / 0.0f;
    if (a < -104.0f) return 0.0f;
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10,
                 invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    double x = (double)a;
    double k = rint_small(x * invln2);
    double hi = x - k * ln2hi, lo = k * ln2lo;
    double r = hi - lo, t = r * r;
    double cc = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * cc) / (2.0 - cc)) - hi);
    uint64_t bits = (uint64_t)((int64_t)k + 1023) << 52;
    double p;
    memcpy(&p, &bits, 8);
    return (float)(y * p);
}
static inline float cr_cosf(float x) { float s, c; sincos_f(x, &s, &c); return c; }
static inline float cr_sinf(float x) { float s, c; sincos_f(x, &s, &c); return s; }
static inline float cr_expf(float x) { return exp_f(x); }
/* cold-path transcendentals (textured sky, sphere u/v): correctly rounded via libm double */
static inline float cr_atan2f(float y, float x) { return (float)atan2((double)y, (double)x); }
static inline float cr_acosf(float x) { return (float)acos((double)x); }
static inline float cr_asinf(float x) { return (float)asin((double)x); }

/* float -> uint as x86-64 does it: (uint32)(int64)trunc(f)  (renderer.h:16-17) */
static inline uint32_t f2u_wrap(float f) {
    if (!(f == f) || f >= 9.2e18f || f <= -9.2e18f) return 0u; /* cvttss2si indefinite -> low 32 bits 0 */
    return (uint32_t)(int64_t)f;
}

/* ------------------------------------------------------------------ mat4 */
void or_mat4_identity(float m[16]) { memset(m, 0, 64); m[0] = m[5] = m[10] = m[15] = 1.0f; }
void or_mat4_translate(float m[16], float x, float y, float z) { or_mat4_identity(m); m[3] = x; m[7] = y; m[11] = z; }
void or_mat4_scale(float m[16], float s) { or_mat4_identity(m); m[0] = m[5] = m[10] = s; }
void or_mat4_rotate_x(float m[16], float a) { or_mat4_identity(m); m[5] = cosf(a); m[6] = -sinf(a); m[9] = sinf(a); m[10] = cosf(a); }
void or_mat4_rotate_y(float m[16], float a) { or_mat4_identity(m); m[0] = cosf(a); m[2] = sinf(a); m[8] = -sinf(a); m[10] = cosf(a); }
void or_mat4_rotate_z(float m[16], float a) { or_mat4_identity(m); m[0] = cosf(a); m[1] = -sinf(a); m[4] = sinf(a); m[5] = cosf(a); }
/* template/template.cpp:779-792 */
void or_mat4_mul(float r[16], const float a[16], const float b[16]) {
    float t[16];
    for (int i = 0; i < 16; i += 4)
        for (int j = 0; j < 4; ++j)
            t[i + j] = (a[i + 0] * b[j + 0]) + (a[i + 1] * b[j + 4]) + (a[i + 2] * b[j + 8]) + (a[i + 3] * b[j + 12]);
    memcpy(r, t, 64);
}
/* TransformPosition / TransformVector: float4(a, w) * M (template/template.cpp:825-839) */
static inline f3 tpos(const float *M, f3 a) {
    return mk(M[0] * a.x + M[1] * a.y + M[2] * a.z + M[3] * 1.0f,
              M[4] * a.x + M[5] * a.y + M[6] * a.z + M[7] * 1.0f,
              M[8] * a.x + M[9] * a.y + M[10] * a.z + M[11] * 1.0f);
}
static inline f3 tvec(const float *M, f3 a) {
    return mk(M[0] * a.x + M[1] * a.y + M[2] * a.z + M[3] * 0.0f,
              M[4] * a.x + M[5] * a.y + M[6] * a.z + M[7] * 0.0f,
              M[8] * a.x + M[9] * a.y + M[10] * a.z + M[11] * 0.0f);
}
static const float IDENT[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};

/* ------------------------------------------------------------------ RNG (template/template.cpp:673-704) */
static uint32_t wang_hash(uint32_t s) {
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u, s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
/* per-pixel seeds: InitSeed (template/template.cpp:697-704); the single base whose WangHash is
 * 0 (a fixed point of xorshift32: the rejection loops would never end) gets the reference's
 * global start seed 0x12345678 (template/template.cpp:673) -- as rt_math.h init_seed */
uint32_t or_init_seed(uint32_t base) {
    const uint32_t h = wang_hash((base + 1u) * 17u);
    return h ? h : 0x12345678u;
}
static inline uint32_t rnd_u(uint32_t *s) { uint32_t x = *s; x ^= x << 13; x ^= x >> 17; x ^= x << 5; *s = x; return x; }
static inline float rnd_f(uint32_t *s) { return (float)rnd_u(s) * 2.3283064365387e-10f; }

/* ------------------------------------------------------------------ scene types */
typedef struct {
    int kind;         /* OR_* material kind */
    f3 c0, c1;        /* colour / absorption ; checkerboard colour2 */
    float ior, diffuse, specular;
    int tex;          /* TextureMaterial: texture index */
} material;

typedef struct {
    int type, mat;
    /* triangles: TransformPosition(data[i], Transform) and its edges, and the GetNormal base
     * normal, evaluated once when the triangle is added -- the same float values Intersect /
     * Hit / GetNormal recompute per call (Primitive.h:249-254, 308-310), since Transform is
     * fixed -- so the hot tests read 40 contiguous bytes instead of two matrices */
    f3 tA, tAB, tAC, tN;
    f3 d[3];          /* Primitive::data (Primitive.h:25) */
    float M[16];      /* Primitive::Transform */
    float Minv[16];   /* Primitive::InvertedTransform (FastInvertedTransformNoScale) */
} prim;

typedef struct { int w, h; uint32_t *px; } texture_t;

typedef struct {      /* BVHNode.h:5-14 -- 32 bytes */
    float mn[3], mx[3];
    uint32_t leftFirst, count;
} node;

struct or_scene {
    prim *p; int np, capp;
    material *m; int nm, capm;
    node *nodes; int nodesUsed, depth;
    uint32_t *idx;
    int skyW, skyH; uint32_t *sky;
    texture_t *tex; int ntex;
    int integrator;   /* 0 = Renderer::Trace, 1 = Renderer::WhittedTrace (the K key, renderer.h:136-139) */
};

typedef struct {      /* Ray.h:7-32 */
    f3 O, D, rD;
    float t; int obj; int inside; float u, v;
} ray_t;

static inline ray_t mkray(f3 O, f3 D, float t) {
    ray_t r; r.O = O; r.D = D; r.t = t; r.obj = -1; r.inside = 0; r.u = r.v = 0.0f;
    r.rD = mk(1 / D.x, 1 / D.y, 1 / D.z);
    return r;
}

typedef struct { int64_t aabb, prim, isect, occl, shadow, aabb_o, prim_o; } counters;

or_scene *or_scene_new(void) {
    or_scene *s = (or_scene *)calloc(1, sizeof(or_scene));
    s->skyW = 1024; s->skyH = 512;  /* synthetic power-of-two sky, SURVEY 8(d) */
    s->sky = (uint32_t *)malloc(sizeof(uint32_t) * 1024 * 512);
    for (int i = 0; i < 1024 * 512; i++) s->sky[i] = 0x406080u;
    return s;
}
void or_scene_free(or_scene *s) {
    if (!s) return;
    for (int i = 0; i < s->ntex; i++) free(s->tex[i].px);
    free(s->tex);
    free(s->p); free(s->m); free(s->nodes); free(s->idx); free(s->sky); free(s);
}
void or_scene_set_sky(or_scene *s, int w, int h, const uint32_t *px) {
    free(s->sky); s->skyW = w; s->skyH = h;
    s->sky = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)w * h);
    memcpy(s->sky, px, sizeof(uint32_t) * (size_t)w * h);
}
int or_scene_add_texture(or_scene *s, int w, int h, const uint32_t *px) {
    s->tex = (texture_t *)realloc(s->tex, sizeof(texture_t) * (s->ntex + 1));
    texture_t *t = &s->tex[s->ntex];
    t->w = w; t->h = h;
    t->px = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)w * h);
    memcpy(t->px, px, sizeof(uint32_t) * (size_t)w * h);
    return s->ntex++;
}
int or_scene_add_material(or_scene *s, int kind, const float c0[3], const float c1[3], float ior, float diffuse) {
    return or_scene_add_material_tex(s, kind, c0, c1, ior, diffuse, -1);
}
int or_scene_add_material_tex(or_scene *s, int kind, const float c0[3], const float c1[3], float ior, float diffuse,
                              int texture) {
    if (s->nm == s->capm) { s->capm = s->capm ? 2 * s->capm : 16; s->m = (material *)realloc(s->m, sizeof(material) * s->capm); }
    material *m = &s->m[s->nm];
    memset(m, 0, sizeof(*m));
    m->kind = kind;
    if (c0) m->c0 = mk(c0[0], c0[1], c0[2]);
    if (c1) m->c1 = mk(c1[0], c1[1], c1[2]);
    m->ior = ior;
    m->tex = texture;
    /* Checkerboard.h:6-14 / TextureMaterial.h:6-17: short ctor diffuse=1, specular=0;
     * with a diffuse argument clamp(diffuse, 0, 1) (precomp.h:782) and 1 - diffuse.
     * DSMix.h:6-9 always takes the diffuse argument. */
    if (kind == OR_CHECKER || kind == OR_TEXTURE || kind == OR_DSMIX) {
        if (diffuse < 0.0f && kind != OR_DSMIX) { m->diffuse = 1.0f; m->specular = 0.0f; }
        else { m->diffuse = tmax_(0.0f, tmin_(diffuse, 1.0f)); m->specular = 1.0f - m->diffuse; }
    }
    return s->nm++;
}
static prim *push_prim(or_scene *s) {
    if (s->np == s->capp) { s->capp = s->capp ? 2 * s->capp : 1024; s->p = (prim *)realloc(s->p, sizeof(prim) * s->capp); }
    prim *p = &s->p[s->np++];
    memset(p, 0, sizeof(*p));
    memcpy(p->M, IDENT, 64);
    memcpy(p->Minv, IDENT, 64);
    return p;
}
/* Primitive.h:690-698 */
int or_scene_add_sphere(or_scene *s, const float pos[3], float r, int mat) {
    prim *p = push_prim(s);
    p->type = OR_SPHERE; p->mat = mat;
    p->d[0] = mk(r, r * r, 1.0f / r);
    or_mat4_translate(p->M, pos[0], pos[1], pos[2]);
    return s->np - 1;
}
/* mat4::FastInvertedTransformNoScale, template/precomp.h:1061-1085 (the non-SSE branch,
 * same values): transpose of the 3x3 part, translation -(R^T t) */
static void fast_inv(const float *c, float *r) {
    memcpy(r, IDENT, 64);
    r[0] = c[0], r[1] = c[4], r[2] = c[8];
    r[4] = c[1], r[5] = c[5], r[6] = c[9];
    r[8] = c[2], r[9] = c[6], r[10] = c[10];
    r[3] = -(c[3] * r[0] + c[7] * r[1] + c[11] * r[2]);
    r[7] = -(c[3] * r[4] + c[7] * r[5] + c[11] * r[6]);
    r[11] = -(c[3] * r[8] + c[7] * r[9] + c[11] * r[10]);
}
/* Primitive.h:717-728 */
int or_scene_add_cube(or_scene *s, const float pos[3], const float size[3], const float T[16], int mat) {
    prim *p = push_prim(s);
    p->type = OR_CUBE; p->mat = mat;
    memcpy(p->M, T, 64);
    f3 ps = mk(pos[0], pos[1], pos[2]);
    if (length3(ps) > FLT_EPS_F) {
        float Tr[16];
        or_mat4_translate(Tr, pos[0], pos[1], pos[2]);
        or_mat4_mul(p->M, T, Tr);
    }
    f3 sz = mk(size[0], size[1], size[2]);
    p->d[0] = smul(-0.5f, sz); p->d[1] = smul(0.5f, sz);
    fast_inv(p->M, p->Minv);
    return s->np - 1;
}
/* Primitive.h:735-739 */
int or_scene_add_quad(or_scene *s, float size, const float T[16], int mat) {
    prim *p = push_prim(s);
    p->type = OR_QUAD; p->mat = mat;
    memcpy(p->M, T, 64);
    p->d[0] = mk(0.5f * size, 0.0f, 0.0f);
    fast_inv(p->M, p->Minv);
    return s->np - 1;
}
/* Primitive.h:705-710 */
int or_scene_add_plane(or_scene *s, const float n[3], float d, int mat) {
    prim *p = push_prim(s);
    p->type = OR_PLANE; p->mat = mat;
    p->d[0] = mk(n[0], n[1], n[2]); p->d[1] = mk(d, 0.0f, 0.0f);
    return s->np - 1;
}
/* Primitive.h:741-747 */
int or_scene_add_triangle(or_scene *s, const float v0[3], const float v1[3], const float v2[3], int mat) {
    prim *p = push_prim(s);
    p->type = OR_TRIANGLE; p->mat = mat;
    p->d[0] = mk(v0[0], v0[1], v0[2]); p->d[1] = mk(v1[0], v1[1], v1[2]); p->d[2] = mk(v2[0], v2[1], v2[2]);
    const f3 A = tpos(p->M, p->d[0]), B = tpos(p->M, p->d[1]), C = tpos(p->M, p->d[2]);
    p->tA = A; p->tAB = sub(B, A); p->tAC = sub(C, A);
    p->tN = tvec(p->M, normalize(cross(sub(p->d[2], p->d[0]), sub(p->d[1], p->d[0]))));
    return s->np - 1;
}
/* Scene::LoadModel face loop, template/scene.h:173-198 */
int or_scene_add_mesh(or_scene *s, const float *V, int nv, const int *T, int nt, const float M[16], int mat) {
    (void)nv;
    for (int f = 0; f < nt; f++) {
        f3 tv[3];
        for (int k = 0; k < 3; k++) {
            const float *q = V + 3 * (size_t)T[3 * f + k];
            tv[k] = tpos(M, mk(q[0], q[1], q[2]));
        }
        float a[3] = {tv[0].x, tv[0].y, tv[0].z}, b[3] = {tv[1].x, tv[1].y, tv[1].z}, c[3] = {tv[2].x, tv[2].y, tv[2].z};
        or_scene_add_triangle(s, a, b, c, mat);
    }
    return nt;
}

/* ------------------------------------------------------------------ primitive geometry (Primitive.h) */
static inline f3 prim_centroid(const prim *p) {   /* ctor 42-50, GetCentroid 443-445 */
    f3 c = mk(0, 0, 0);
    if (p->type == OR_PLANE) c = muls(neg(p->d[0]), p->d[1].x);
    else if (p->type == OR_TRIANGLE) c = divs(add(add(p->d[0], p->d[1]), p->d[2]), 3.0f);
    return tpos(p->M, c);
}
/* the 8 cube corners / 4 quad corners in GetAABBMin/Max's order (Primitive.h:325-341) */
static int box_corners(const prim *p, f3 *c) {
    if (p->type == OR_CUBE) {
        f3 a = p->d[0], b = p->d[1];
        c[0] = tpos(p->M, a);
        c[1] = tpos(p->M, mk(b.x, a.y, a.z));
        c[2] = tpos(p->M, mk(a.x, b.y, a.z));
        c[3] = tpos(p->M, mk(a.x, a.y, b.z));
        c[4] = tpos(p->M, b);
        c[5] = tpos(p->M, mk(a.x, b.y, b.z));
        c[6] = tpos(p->M, mk(b.x, a.y, b.z));
        c[7] = tpos(p->M, mk(b.x, b.y, a.z));
        return 8;
    }
    float sz = p->d[0].x;   /* QUAD, Primitive.h:336-341 */
    c[0] = tpos(p->M, mk(-sz, 0, -sz));
    c[1] = tpos(p->M, mk(-sz, 0, sz));
    c[2] = tpos(p->M, mk(sz, 0, -sz));
    c[3] = tpos(p->M, mk(sz, 0, sz));
    return 4;
}
static inline f3 prim_aabb_min(const prim *p) {   /* 319-351 */
    if (p->type == OR_SPHERE) return sub(tpos(p->M, mk(0, 0, 0)), mk(p->d[0].x, p->d[0].x, p->d[0].x));
    if (p->type == OR_PLANE) return mk(-1e30f, -1e30f, -1e30f);
    if (p->type == OR_CUBE || p->type == OR_QUAD) {
        f3 c[8];
        int n = box_corners(p, c);
        f3 m = c[0];
        for (int i = 1; i < n; i++) m = fmin3(m, c[i]);
        return m;
    }
    f3 A = tpos(p->M, p->d[0]), B = tpos(p->M, p->d[1]), C = tpos(p->M, p->d[2]);
    return fmin3(A, fmin3(B, C));
}
static inline f3 prim_aabb_max(const prim *p) {   /* 356-388 */
    if (p->type == OR_SPHERE) return add(tpos(p->M, mk(0, 0, 0)), mk(p->d[0].x, p->d[0].x, p->d[0].x));
    if (p->type == OR_PLANE) return mk(1e30f, 1e30f, 1e30f);
    if (p->type == OR_CUBE || p->type == OR_QUAD) {
        f3 c[8];
        int n = box_corners(p, c);
        f3 m = c[0];
        for (int i = 1; i < n; i++) m = fmax3(m, c[i]);
        return m;
    }
    f3 A = tpos(p->M, p->d[0]), B = tpos(p->M, p->d[1]), C = tpos(p->M, p->d[2]);
    return fmax3(A, fmax3(B, C));
}

/* CUBE slab test in object space (Primitive.h:87-110 / 196-235); returns 0 on a miss */
static int cube_slab(const prim *p, const ray_t *r, float *tmin_o, float *tmax_o) {
    f3 O = tpos(p->Minv, r->O), D = tvec(p->Minv, r->D);
    float rDx = 1 / D.x, rDy = 1 / D.y, rDz = 1 / D.z;
    int sx = D.x < 0, sy = D.y < 0, sz = D.z < 0;
    const f3 *d = p->d;
    float tmin = (d[sx].x - O.x) * rDx;
    float tmax = (d[1 - sx].x - O.x) * rDx;
    float tymin = (d[sy].y - O.y) * rDy;
    float tymax = (d[1 - sy].y - O.y) * rDy;
    if (tmin > tymax || tymin > tmax) return 0;
    tmin = smax(tmin, tymin);
    tmax = smin(tmax, tymax);
    float tzmin = (d[sz].z - O.z) * rDz;
    float tzmax = (d[1 - sz].z - O.z) * rDz;
    if (tmin > tzmax || tzmin > tmax) return 0;
    *tmin_o = smax(tmin, tzmin);
    *tmax_o = smin(tmax, tzmax);
    return 1;
}
/* Primitive::setTextureCoordsCube, Primitive.h:752-797 */
static void cube_uv(const prim *p, ray_t *r) {
    f3 objI = tpos(p->Minv, add(r->O, smul(r->t, r->D)));
    const f3 *d = p->d;
    float uc, vc;
    float d0 = fabsf(objI.x - d[0].x), d1 = fabsf(objI.x - d[1].x);
    float d2 = fabsf(objI.y - d[0].y), d3 = fabsf(objI.y - d[1].y);
    float d4 = fabsf(objI.z - d[0].z), d5 = fabsf(objI.z - d[1].z);
    float minDist = d0;
    int face = 1;
    uc = objI.z, vc = objI.y;
    if (d1 < minDist) uc = -objI.z, vc = objI.y, face = 0, minDist = d1;
    if (d2 < minDist) uc = objI.x, vc = objI.z, face = 3, minDist = d2;
    if (d3 < minDist) uc = objI.x, vc = -objI.z, face = 2, minDist = d3;
    if (d4 < minDist) uc = -objI.x, vc = objI.y, face = 5, minDist = d4;
    if (d5 < minDist) uc = objI.x, vc = objI.y, face = 4;
    uc = -uc, vc = -vc;
    uc = 0.5f * (uc / d[1].x + 1.0f);
    vc = 0.5f * (vc / d[1].x + 1.0f);
    const float third = 1.0f / 3.0f;
    switch (face) {
    case 0: r->u = 0.25f * (2 + uc); r->v = third * (1 + vc); break;
    case 1: r->u = 0.25f * (0 + uc); r->v = third * (1 + vc); break;
    case 2: r->u = 0.25f * (1 + uc); r->v = third * vc; break;
    case 3: r->u = 0.25f * (1 + uc); r->v = third * (2 + vc); break;
    case 4: r->u = 0.25f * (1 + uc); r->v = third * (1 + vc); break;
    default: r->u = 0.25f * (3 + uc); r->v = third * (1 + vc); break;
    }
}

/* Primitive::Intersect, 149-279 */
static void prim_intersect(const prim *p, ray_t *r, int idx) {
    if (p->type == OR_CUBE) {   /* 195-235: note the acceptance test is on tmax */
        float tmin, tmax;
        if (!cube_slab(p, r, &tmin, &tmax)) return;
        if (tmin > EPS_F) {
            if (tmax < r->t) { r->t = tmin; r->obj = idx; cube_uv(p, r); }
        } else if (tmax > EPS_F) {
            if (tmax < r->t) { r->t = tmax; r->obj = idx; cube_uv(p, r); }
        }
        return;
    }
    if (p->type == OR_QUAD) {   /* 236-247; u, v are left unset there: defined as 0 here */
        f3 O = tpos(p->Minv, r->O), D = tvec(p->Minv, r->D);
        float t = O.y / -D.y;
        float size = p->d[0].x;
        if (t < r->t && t > EPS_F) {
            f3 I = add(O, smul(t, D));
            if (I.x > -size && I.x < size && I.z > -size && I.z < size) { r->t = t; r->obj = idx; r->u = r->v = 0.0f; }
        }
        return;
    }
    if (p->type == OR_SPHERE) {
        f3 pos = tpos(p->M, mk(0, 0, 0));
        f3 oc = sub(r->O, pos);
        float b = dot(oc, r->D);
        float c = dot(oc, oc) - p->d[0].y;
        float t, d = b * b - c;
        if (d <= 0) return;
        d = sqrtf(d), t = -b - d;
        if (!(t < r->t && t > EPS_F)) {
            t = d - b;
            if (!(t < r->t && t > EPS_F)) return;
        }
        r->t = t; r->obj = idx;
        f3 cToI = normalize(sub(add(r->O, smul(r->t, r->D)), pos));
        r->u = 0.5f - cr_atan2f(cToI.z, cToI.x) * INV2PI_F;
        r->v = 0.5f - cr_asinf(cToI.y) * INVPI_F;
    } else if (p->type == OR_PLANE) {
        float t = -(dot(r->O, p->d[0]) + p->d[1].x) / (dot(r->D, p->d[0]));
        if (t < r->t && t > EPS_F) {
            r->t = t; r->obj = idx;
            f3 I = add(r->O, smul(r->t, r->D));
            f3 N = p->d[0];
            if (N.x < FLT_EPS_F && N.y < FLT_EPS_F) { r->u = I.x; r->v = -I.y; }
            else if (N.x < FLT_EPS_F && N.z < FLT_EPS_F) { r->u = I.x; r->v = -I.z; }
            else if (N.y < FLT_EPS_F && N.z < FLT_EPS_F) { r->u = I.y; r->v = -I.z; }
            else { r->u = r->v = 0.0f; }   /* left unset by the reference: defined as 0 */
        }
    } else {
        const f3 A = p->tA, AB = p->tAB, AC = p->tAC;
        float denom = dot(cross(r->D, AC), AB);
        if ((double)fabsf(denom) < CL_DBL_EPS) return;
        f3 AO = sub(r->O, A);
        float u = dot(cross(neg(r->D), AO), AC) / denom;
        if (u < 0 || u > 1) return;
        float v = dot(cross(neg(r->D), AB), AO) / denom;
        if (v < 0 || u + v > 1) return;
        float t = dot(cross(AO, AB), AC) / denom;
        if (t < r->t && t > EPS_F) { r->t = t; r->obj = idx; r->u = u; r->v = v; }
    }
}

/* Primitive::Hit, 64-144 */
static int prim_hit(const prim *p, const ray_t *r) {
    if (p->type == OR_CUBE) {   /* Primitive.h:83-110 */
        float tmin, tmax;
        if (!cube_slab(p, r, &tmin, &tmax)) return 0;
        return (tmin > EPS_F || tmax > EPS_F) && tmax < r->t;
    }
    if (p->type == OR_QUAD) {   /* 111-117: the quad's extent is not tested (reference quirk) */
        f3 O = tpos(p->Minv, r->O), D = tvec(p->Minv, r->D);
        float t = O.y / -D.y;
        return t < r->t && t > EPS_F;
    }
    if (p->type == OR_SPHERE) {
        f3 pos = tpos(p->M, mk(0, 0, 0));
        f3 oc = sub(r->O, pos);
        float b = dot(oc, r->D);
        float c = dot(oc, oc) - p->d[0].y;
        float d = b * b - c;
        if (d <= 0) return 0;
        d = sqrtf(d);
        float t = -b - d;
        if (t < r->t && t > EPS_F) return 1;
        t = d - b;
        return t < r->t && t > EPS_F;
    } else if (p->type == OR_PLANE) {
        float t = -(dot(r->O, p->d[0]) + p->d[1].x) / (dot(r->D, p->d[0]));
        return t < r->t && t > EPS_F;
    } else {
        const f3 A = p->tA, AB = p->tAB, AC = p->tAC;
        float denom = dot(cross(r->D, AC), AB);
        if ((double)fabsf(denom) < CL_DBL_EPS) return 0;
        f3 AO = sub(r->O, A);
        float u = dot(cross(neg(r->D), AO), AC) / denom;
        if (u < 0 || u > 1) return 0;
        float v = dot(cross(neg(r->D), AB), AO) / denom;
        if (v < 0 || u + v > 1) return 0;
        float t = dot(cross(AO, AB), AC) / denom;
        return t < r->t && t > EPS_F;
    }
}

/* Primitive::GetNormal 284-314 */
static inline f3 prim_normal(const prim *p, f3 I) {
    if (p->type == OR_SPHERE) return muls(sub(I, tpos(p->M, mk(0, 0, 0))), p->d[0].z);
    if (p->type == OR_PLANE) return p->d[0];
    if (p->type == OR_CUBE) {   /* Primitive.h:290-305 */
        f3 objI = tpos(p->Minv, I);
        const f3 *d = p->d;
        f3 N = mk(-1, 0, 0);
        float d0 = fabsf(objI.x - d[0].x), d1 = fabsf(objI.x - d[1].x);
        float d2 = fabsf(objI.y - d[0].y), d3 = fabsf(objI.y - d[1].y);
        float d4 = fabsf(objI.z - d[0].z), d5 = fabsf(objI.z - d[1].z);
        float minDist = d0;
        if (d1 < minDist) minDist = d1, N.x = 1;
        if (d2 < minDist) minDist = d2, N = mk(0, -1, 0);
        if (d3 < minDist) minDist = d3, N = mk(0, 1, 0);
        if (d4 < minDist) minDist = d4, N = mk(0, 0, -1);
        if (d5 < minDist) minDist = d5, N = mk(0, 0, 1);
        return tvec(p->M, N);
    }
    if (p->type == OR_QUAD) return tvec(p->M, mk(0, -1, 0));   /* 306-307 */
    return p->tN;   /* tvec(M, normalize(cross(C - A, B - A))), 308-310: cached at add time */
}

/* ------------------------------------------------------------------ plain BVH build (template/scene.h:845-976) */
typedef struct { f3 mn, mx; int count; } bin_t; /* BVHBin with aabb default +-1e34 (precomp.h:928) */

static inline float aabb_area(f3 mn, f3 mx) {     /* aabb::Area, precomp.h:912-917 */
    float e0 = mx.x - mn.x, e1 = mx.y - mn.y, e2 = mx.z - mn.z;
    return smax(0.0f, e0 * e1 + e0 * e2 + e1 * e2);
}
/* _mm_min_ps(a,b) = a<b?a:b ; _mm_max_ps(a,b) = a>b?a:b */
static inline f3 mmmin(f3 a, f3 b) { return fmin3(a, b); }
static inline f3 mmmax(f3 a, f3 b) { return fmax3(a, b); }

static void update_bounds(or_scene *s, uint32_t ni) {   /* 855-865 */
    node *n = &s->nodes[ni];
    f3 mn = mk(1e30f, 1e30f, 1e30f), mx = mk(-1e30f, -1e30f, -1e30f);
    for (uint32_t i = 0; i < n->count; i++) {
        const prim *p = &s->p[s->idx[n->leftFirst + i]];
        mn = fmin3(mn, prim_aabb_min(p));
        mx = fmax3(mx, prim_aabb_max(p));
    }
    n->mn[0] = mn.x; n->mn[1] = mn.y; n->mn[2] = mn.z;
    n->mx[0] = mx.x; n->mx[1] = mx.y; n->mx[2] = mx.z;
}

static float find_best_split(or_scene *s, const node *n, int *axis, float *splitPos) {  /* 914-976 */
    float bestCost = 1e30f;
    for (int a = 0; a < 3; a++) {
        float bmin = 1e30f, bmax = -1e30f;
        for (uint32_t i = 0; i < n->count; i++) {
            float c = comp(prim_centroid(&s->p[s->idx[n->leftFirst + i]]), a);
            bmin = smin(bmin, c);
            bmax = smax(bmax, c);
        }
        if (bmin == bmax) continue;
        bin_t bin[BIN_COUNT];
        for (int b = 0; b < BIN_COUNT; b++) { bin[b].mn = mk(1e34f, 1e34f, 1e34f); bin[b].mx = mk(-1e34f, -1e34f, -1e34f); bin[b].count = 0; }
        float scale = BIN_COUNT / (bmax - bmin);
        for (uint32_t i = 0; i < n->count; i++) {
            const prim *p = &s->p[s->idx[n->leftFirst + i]];
            int bi = (int)((comp(prim_centroid(p), a) - bmin) * scale);
            if (BIN_COUNT - 1 < bi) bi = BIN_COUNT - 1;   /* std::min(BIN_COUNT-1, bi) */
            bin[bi].count++;
            f3 pmn = prim_aabb_min(p), pmx = prim_aabb_max(p);
            bin[bi].mn = mmmin(bin[bi].mn, pmn); bin[bi].mx = mmmax(bin[bi].mx, pmn);
            bin[bi].mn = mmmin(bin[bi].mn, pmx); bin[bi].mx = mmmax(bin[bi].mx, pmx);
        }
        float leftArea[BIN_COUNT - 1], rightArea[BIN_COUNT - 1];
        int leftCount[BIN_COUNT - 1], rightCount[BIN_COUNT - 1];
        f3 lmn = mk(1e34f, 1e34f, 1e34f), lmx = mk(-1e34f, -1e34f, -1e34f);
        f3 rmn = lmn, rmx = lmx;
        int leftSum = 0, rightSum = 0;
        for (int i = 0; i < BIN_COUNT - 1; i++) {
            leftSum += bin[i].count;
            leftCount[i] = leftSum;
            lmn = mmmin(lmn, bin[i].mn); lmx = mmmax(lmx, bin[i].mx);
            leftArea[i] = aabb_area(lmn, lmx);
            rightSum += bin[BIN_COUNT - 1 - i].count;
            rightCount[BIN_COUNT - 2 - i] = rightSum;
            rmn = mmmin(rmn, bin[BIN_COUNT - 1 - i].mn); rmx = mmmax(rmx, bin[BIN_COUNT - 1 - i].mx);
            rightArea[BIN_COUNT - 2 - i] = aabb_area(rmn, rmx);
        }
        scale = (bmax - bmin) / BIN_COUNT;
        for (int i = 0; i < BIN_COUNT - 1; i++) {
            float planeCost = (float)leftCount[i] * leftArea[i] + (float)rightCount[i] * rightArea[i];
            if (planeCost < bestCost) { *axis = a; *splitPos = bmin + scale * (float)(i + 1); bestCost = planeCost; }
        }
    }
    return bestCost;
}

static void subdivide(or_scene *s, uint32_t ni) {   /* 867-912 */
    node *n = &s->nodes[ni];
    int axis = 0; float splitPos = 0.0f;
    float splitCost = find_best_split(s, n, &axis, &splitPos);
    float ex = n->mx[0] - n->mn[0], ey = n->mx[1] - n->mn[1], ez = n->mx[2] - n->mn[2];
    float nosplit = (float)n->count * (ex * ey + ey * ez + ez * ex);   /* calculateNodeCost 203-207 */
    if (splitCost >= nosplit) return;
    int i = (int)n->leftFirst, j = i + (int)n->count - 1;
    while (i <= j) {
        if (comp(prim_centroid(&s->p[s->idx[i]]), axis) < splitPos) i++;
        else { uint32_t tmp = s->idx[i]; s->idx[i] = s->idx[j]; s->idx[j--] = tmp; }
    }
    int leftCount = i - (int)n->leftFirst;
    if (leftCount == 0 || leftCount == (int)n->count) return;
    uint32_t L = (uint32_t)s->nodesUsed++, R = (uint32_t)s->nodesUsed++;
    s->nodes[L].leftFirst = n->leftFirst; s->nodes[L].count = (uint32_t)leftCount;
    s->nodes[R].leftFirst = (uint32_t)i; s->nodes[R].count = n->count - (uint32_t)leftCount;
    n->leftFirst = L; n->count = 0;
    update_bounds(s, L); update_bounds(s, R);
    subdivide(s, L); subdivide(s, R);
}

static int max_depth(const or_scene *s, uint32_t ni) {   /* 144-154 */
    const node *n = &s->nodes[ni];
    if (n->count > 0) return ni == 0 ? 1 : 0;
    int l = max_depth(s, n->leftFirst), r = max_depth(s, n->leftFirst + 1);
    return (l > r ? l : r) + 1;
}

int or_scene_build_bvh(or_scene *s) {   /* BuildBVH 845-853 with the 2N+1 pool of 112-116 */
    free(s->idx); free(s->nodes);
    s->idx = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(s->np > 0 ? s->np : 1));
    for (int i = 0; i < s->np; i++) s->idx[i] = (uint32_t)i;
    s->nodes = (node *)calloc((size_t)(2 * s->np + 2), sizeof(node));
    node *root = &s->nodes[0];
    root->leftFirst = 0; root->count = (uint32_t)s->np;
    s->nodesUsed = 2;
    update_bounds(s, 0);
    subdivide(s, 0);
    s->depth = max_depth(s, 0);
    return s->nodesUsed;
}
/* A prebuilt BVH (BVHNode.h:5-14 nodes + primitiveIndices) instead of BuildBVH: the analytic
 * known-answer tests fix the tree so that slab outcomes follow from the boxes alone, and the
 * SBVH test runs the library's spatial-split tree (nidx references) through this traversal. */
int or_scene_set_bvh(or_scene *s, const void *nodes, int nodes_used, const uint32_t *idx, int nidx) {
    if (nodes_used < 2 || nidx < 1) return -1;
    free(s->idx); free(s->nodes);
    s->idx = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)nidx);   /* nidx > np: an SBVH's references */
    memcpy(s->idx, idx, sizeof(uint32_t) * (size_t)nidx);
    s->nodes = (node *)calloc((size_t)nodes_used, sizeof(node));
    memcpy(s->nodes, nodes, sizeof(node) * (size_t)nodes_used);
    s->nodesUsed = nodes_used;
    s->depth = max_depth(s, 0);
    return nodes_used;
}
int or_scene_num_prims(const or_scene *s) { return s->np; }
int or_scene_nodes_used(const or_scene *s) { return s->nodesUsed; }
int or_scene_depth(const or_scene *s) { return s->depth; }
const void *or_scene_nodes(const or_scene *s) { return s->nodes; }
const uint32_t *or_scene_indices(const or_scene *s) { return s->idx; }

/* ------------------------------------------------------------------ traversal (template/scene.h) */
static inline float intersect_aabb(const ray_t *r, const node *n) {   /* 432-450 */
    float tx1 = (n->mn[0] - r->O.x) * r->rD.x, tx2 = (n->mx[0] - r->O.x) * r->rD.x;
    float tmin = smin(tx1, tx2), tmax = smax(tx1, tx2);
    float ty1 = (n->mn[1] - r->O.y) * r->rD.y, ty2 = (n->mx[1] - r->O.y) * r->rD.y;
    tmin = smax(tmin, smin(ty1, ty2)); tmax = smin(tmax, smax(ty1, ty2));
    float tz1 = (n->mn[2] - r->O.z) * r->rD.z, tz2 = (n->mx[2] - r->O.z) * r->rD.z;
    tmin = smax(tmin, smin(tz1, tz2)); tmax = smin(tmax, smax(tz1, tz2));
    if (tmax >= tmin && tmin < r->t && tmax > 0) return tmin;
    return 1e30f;
}
static inline int hits_aabb(const ray_t *r, const node *n) {          /* 414-430 */
    float tx1 = (n->mn[0] - r->O.x) * r->rD.x, tx2 = (n->mx[0] - r->O.x) * r->rD.x;
    float tmin = smin(tx1, tx2), tmax = smax(tx1, tx2);
    float ty1 = (n->mn[1] - r->O.y) * r->rD.y, ty2 = (n->mx[1] - r->O.y) * r->rD.y;
    tmin = smax(tmin, smin(ty1, ty2)); tmax = smin(tmax, smax(ty1, ty2));
    float tz1 = (n->mn[2] - r->O.z) * r->rD.z, tz2 = (n->mx[2] - r->O.z) * r->rD.z;
    tmin = smax(tmin, smin(tz1, tz2)); tmax = smin(tmax, smax(tz1, tz2));
    return tmax >= tmin && tmin < r->t && tmax > 0;
}

/* Traversal work counters of or_pixel_work (NULL otherwise): per pixel [0] closest-hit node
 * visits (interior + leaf), [1] closest-hit primitive tests, [2] any-hit node visits, [3] any-hit
 * primitive tests, [4] / [5] closest-hit pops of an interior / leaf entry whose entry distance
 * (at its push, IntersectAABB's tmin) is >= the ray's t at the pop -- the library's dry-run work
 * map (rt_renderer_tile_work) counts the same. */
static __thread uint32_t *tl_work;

/* slab entry distance with the reference's selects (intersect_aabb's tmin before the accept test) */
static inline float slab_entry(const ray_t *r, const node *n) {
    float tx1 = (n->mn[0] - r->O.x) * r->rD.x, tx2 = (n->mx[0] - r->O.x) * r->rD.x;
    float tmin = smin(tx1, tx2);
    float ty1 = (n->mn[1] - r->O.y) * r->rD.y, ty2 = (n->mx[1] - r->O.y) * r->rD.y;
    tmin = smax(tmin, smin(ty1, ty2));
    float tz1 = (n->mn[2] - r->O.z) * r->rD.z, tz2 = (n->mx[2] - r->O.z) * r->rD.z;
    return smax(tmin, smin(tz1, tz2));
}

static void intersect_bvh(const or_scene *s, ray_t *r, counters *k) {   /* 285-320 */
    const node *n = &s->nodes[0];
    const node *stack[64];
    float sdist[64];   /* counting only: each entry's IntersectAABB distance at its push */
    uint32_t sp = 0;
    if (k) k->isect++;
    for (;;) {
        if (tl_work) tl_work[0]++;
        if (n->count > 0) {
            if (tl_work) tl_work[1] += n->count;
            for (uint32_t i = 0; i < n->count; i++) {
                int oi = (int)s->idx[n->leftFirst + i];
                prim_intersect(&s->p[oi], r, oi);
            }
            if (k) k->prim += n->count;
            if (sp == 0) break;
            n = stack[--sp];
            if (tl_work && sdist[sp] >= r->t) tl_work[n->count > 0 ? 5 : 4]++;
            continue;
        }
        const node *c1 = &s->nodes[n->leftFirst], *c2 = &s->nodes[n->leftFirst + 1];
        float d1 = intersect_aabb(r, c1), d2 = intersect_aabb(r, c2);
        if (k) k->aabb += 2;
        if (d1 > d2) { float td = d1; d1 = d2; d2 = td; const node *tn = c1; c1 = c2; c2 = tn; }
        if (d1 == 1e30f) {
            if (sp == 0) break;
            n = stack[--sp];
            if (tl_work && sdist[sp] >= r->t) tl_work[n->count > 0 ? 5 : 4]++;
        } else {
            n = c1;
            if (d2 != 1e30f) { sdist[sp] = d2; stack[sp++] = c2; }
        }
    }
}

static int is_occluded(const or_scene *s, const ray_t *r, counters *k) {   /* 452-487 */
    const node *n = &s->nodes[0], *stack[64];
    uint32_t sp = 0;
    if (k) k->occl++;
    for (;;) {
        if (tl_work) tl_work[2]++;
        if (n->count > 0) {
            for (uint32_t i = 0; i < n->count; i++) {
                int oi = (int)s->idx[n->leftFirst + i];
                if (k) { k->prim++; k->prim_o++; }
                if (tl_work) tl_work[3]++;
                if (prim_hit(&s->p[oi], r)) return 1;
            }
            if (sp == 0) break;
            n = stack[--sp];
            continue;
        }
        const node *c1 = &s->nodes[n->leftFirst], *c2 = &s->nodes[n->leftFirst + 1];
        int h1 = hits_aabb(r, c1), h2 = hits_aabb(r, c2);
        if (k) { k->aabb += 2; k->aabb_o += 2; }
        if (h1 && h2) {
            /* counting (or_pixel_work): the library's child order for shadow rays, the box the ray
             * enters later first -- the answer is the same bool in any order, only the counts move */
            if (tl_work && slab_entry(r, c2) > slab_entry(r, c1)) { n = c2; stack[sp++] = c1; }
            else { n = c1; stack[sp++] = c2; }
        }
        else if (!(h1 || h2)) { if (sp == 0) break; n = stack[--sp]; }
        else if (h1) n = c1;
        else n = c2;
    }
    return 0;
}

static inline f3 scene_normal(const or_scene *s, int obj, f3 I, f3 wo) {   /* 489-497 */
    if (obj == -1) return mk(0, 0, 0);
    f3 N = prim_normal(&s->p[obj], I);
    if (dot(N, wo) > 0) N = neg(N);
    return N;
}

/* Primitive::GetRandomPoint SPHERE 394-402 (x drawn first: left-to-right argument order) */
static f3 sphere_random_point(const prim *p, uint32_t *seed) {
    f3 pt = mk(1, 1, 1);
    while (dot(pt, pt) > 1) {
        float x = rnd_f(seed) * 2.0f - 1.0f;
        float y = rnd_f(seed) * 2.0f - 1.0f;
        float z = rnd_f(seed) * 2.0f - 1.0f;
        pt = mk(x, y, z);
    }
    return tpos(p->M, muls(normalize(pt), p->d[0].x));
}
static inline float prim_area(const prim *p) {   /* 450-468 */
    if (p->type == OR_SPHERE) return 4.0f * PI_F * p->d[0].y;
    if (p->type == OR_PLANE) return 1e30f;
    if (p->type == OR_CUBE) {
        f3 sz = smul(2.0f, p->d[1]);
        return 2.0f * (sz.x * sz.y + sz.x * sz.z + sz.y * sz.z);
    }
    if (p->type == OR_QUAD) { float sz = 2.0f * p->d[0].x; return sz * sz; }
    f3 AB = sub(p->d[1], p->d[0]), AC = sub(p->d[2], p->d[0]);
    return 0.5f * length3(cross(AB, AC));
}
static f3 light_random_point(const prim *p, uint32_t *seed) {
    if (p->type == OR_SPHERE) return sphere_random_point(p, seed);
    if (p->type == OR_PLANE) return muls(neg(p->d[0]), p->d[1].x);
    if (p->type == OR_CUBE) {   /* Primitive.h:405-422 (Rand(6) = RandomFloat() * 6) */
        float u = rnd_f(seed) * 2.0f - 1.0f;
        float v = rnd_f(seed) * 2.0f - 1.0f;
        float face = rnd_f(seed) * 6.0f;
        f3 q;
        if (face < 1) q = mk(-1, u, v);
        else if (face < 2) q = mk(1, u, v);
        else if (face < 3) q = mk(u, -1, v);
        else if (face < 4) q = mk(u, 1, v);
        else if (face < 5) q = mk(u, v, -1);
        else q = mk(u, v, 1);
        return tpos(p->M, mul(q, p->d[1]));
    }
    if (p->type == OR_QUAD) {   /* 423-427: the point lies in object z = 0 (reference quirk) */
        float size = p->d[0].x;
        float a = size * (rnd_f(seed) - 1.0f);
        float b = size * (rnd_f(seed) - 1.0f);
        return tpos(p->M, mk(a, b, 0.0f));
    }
    float u = rnd_f(seed), v = rnd_f(seed);   /* Primitive.h:429-437 */
    while ((u + v) > 1) { u = rnd_f(seed); v = rnd_f(seed); }
    return tpos(p->M, add(add(p->d[0], smul(u, p->d[1])), smul(v, p->d[2])));
}

/* ------------------------------------------------------------------ camera (camera.h) */
void or_camera_default(or_camera *c, int W, int H) {   /* ctor 28-41 + members 93-100 */
    float aperture = (float)0.000005;
    float lensRadius = aperture / 2.0f, focus = 1.0f, FOV = 1.0f;
    float aspect = (float)W / (float)H;
    f3 pos = mk(0, 0, -FOV);
    f3 tl = add(pos, smul(focus, mk(-aspect, 1, FOV)));
    f3 tr = add(pos, smul(focus, mk(aspect, 1, FOV)));
    f3 bl = add(pos, smul(focus, mk(-aspect, -1, FOV)));
    c->pos[0] = pos.x; c->pos[1] = pos.y; c->pos[2] = pos.z;
    c->tl[0] = tl.x; c->tl[1] = tl.y; c->tl[2] = tl.z;
    c->tr[0] = tr.x; c->tr[1] = tr.y; c->tr[2] = tr.z;
    c->bl[0] = bl.x; c->bl[1] = bl.y; c->bl[2] = bl.z;
    c->lens_radius = lensRadius;
    c->rwidth = 1.0f / (float)W;
    c->rheight = 1.0f / (float)H;
}
static ray_t primary_ray(const or_camera *c, int x, int y, uint32_t *seed) {   /* 43-52, disk 20-26 */
    float u = (float)x * c->rwidth + rnd_f(seed) * c->rwidth;
    float v = (float)y * c->rheight + rnd_f(seed) * c->rheight;
    f3 p;
    for (;;) {
        float px = rnd_f(seed) * 2.0f - 1.0f;
        float py = rnd_f(seed) * 2.0f - 1.0f;
        p = mk(px, py, 0);
        if (dot(p, p) >= 1) continue;
        break;
    }
    f3 rd = smul(c->lens_radius, p);
    f3 offset = mk(u * rd.x, v * rd.y, 0);
    f3 pos = mk(c->pos[0], c->pos[1], c->pos[2]);
    f3 tl = mk(c->tl[0], c->tl[1], c->tl[2]), tr = mk(c->tr[0], c->tr[1], c->tr[2]), bl = mk(c->bl[0], c->bl[1], c->bl[2]);
    f3 P = add(add(tl, smul(u, sub(tr, tl))), smul(v, sub(bl, tl)));
    return mkray(add(pos, offset), normalize(sub(sub(P, pos), offset)), 1e34f);
}

/* ------------------------------------------------------------------ shading (renderer.h / renderer.cpp / materials) */
static inline f3 sky_color(const or_scene *s, f3 D) {   /* renderer.h:15-22 */
    uint32_t u = f2u_wrap((float)s->skyW * cr_atan2f(D.z, D.x) * INV2PI_F - 0.5f);
    uint32_t v = f2u_wrap((float)s->skyH * cr_acosf(D.y) * INVPI_F - 0.5f);
    uint32_t idx = (u & (uint32_t)(s->skyW - 1)) + (v & (uint32_t)(s->skyH - 1)) * (uint32_t)s->skyW;
    uint32_t p = s->sky[idx];
    return muls(mk((float)((p >> 16) & 255), (float)((p >> 8) & 255), (float)(p & 255)), SKYDOME_CORRECTION_F);
}

enum { FLAG_DIFFUSE = 0, FLAG_SPECULAR = 1, FLAG_MIX = 2, FLAG_DIELECTRIC = 3, FLAG_LIGHT = 4 };
static inline int mat_flag(const material *m) {
    switch (m->kind) {
    case OR_DIFFUSE: return FLAG_DIFFUSE;
    case OR_MIRROR: return FLAG_SPECULAR;
    case OR_DIELECTRIC: return FLAG_DIELECTRIC;
    case OR_LIGHT: return FLAG_LIGHT;
    default:  /* Checkerboard.h:16-26 */
        if (m->diffuse < FLT_EPS_F) return FLAG_SPECULAR;
        if (m->specular < FLT_EPS_F) return FLAG_DIFFUSE;
        return FLAG_MIX;
    }
}
/* ObjectMaterial.h:18-53 */
static f3 diffuse_reflection(f3 N, uint32_t *seed) {
    float r0 = rnd_f(seed), r1 = rnd_f(seed);
    float r = sqrtf(r0), theta = TWOPI_F * r1;
    float x = r * cr_cosf(theta), y = r * cr_sinf(theta), z = sqrtf(1 - r0);
    f3 a0 = mk(0.0f, -1.0f, 0.0f), a1 = mk(-1.0f, 0.0f, 0.0f), a2 = N;
    if (N.z + 1.0f > FLT_EPS_F) {
        float a = 1.0f / (1.0f + N.z);
        float b = -N.x * N.y * a;
        a0 = mk(1.0f - N.x * N.x * a, b, -N.x);
        a1 = mk(b, 1.0f - N.y * N.y * a, -N.y);
    }
    return normalize(add(add(smul(x, a0), smul(y, a1)), smul(z, a2)));
}
static inline float fresnel(float n1, float n2, float cost, float cosi) {   /* ObjectMaterial.h:55-60 */
    float s = (n1 * cosi - n2 * cost) / (n1 * cosi + n2 * cost);
    float p = (n1 * cost - n2 * cosi) / (n1 * cost + n2 * cosi);
    return 0.5f * ((s * s) + (p * p));
}
/* ObjectMaterial::scatter overrides; returns specularBounce */
static int mat_scatter(const material *m, const ray_t *in, f3 I, f3 N, ray_t *out, uint32_t *seed) {
    switch (m->kind) {
    case OR_DIFFUSE:   /* Diffuse.h:16-19 */
        *out = mkray(I, diffuse_reflection(N, seed), 1e34f);
        return 0;
    case OR_MIRROR:    /* Mirror.h:16-19 */
        *out = mkray(I, normalize(reflect(in->D, N)), 1e34f);
        return 1;
    case OR_DIELECTRIC: {   /* Dielectric.h:23-54 */
        float n1 = 1, n2 = m->ior;
        float n12 = n1 / n2;
        float cosi = dot(N, in->D);
        if (in->inside) n12 = 1 / n12;
        float k = 1 - (n12 * n12) * (1 - (cosi * cosi));
        if (k < 0) {
            *out = mkray(I, normalize(reflect(in->D, N)), 1e34f);
            out->inside = 1;
        } else {
            float Fr = 0;
            if (!in->inside) {
                float sini = length3(cross(N, in->D));
                float sq = n12 * sini;
                float cost = sqrtf(1 - sq * sq);
                Fr = fresnel(n1, n2, cost, -cosi);
            }
            if (Fr > FLT_EPS_F && rnd_f(seed) < Fr) {
                *out = mkray(I, normalize(reflect(in->D, N)), 1e34f);
            } else {
                f3 T = normalize(sub(smul(n12, in->D), smul(n12 * cosi + sqrtf(k), N)));
                *out = mkray(I, T, 1e34f);
                out->inside = !in->inside;
            }
        }
        return 1;
    }
    case OR_LIGHT:
        return 0;
    default:   /* Checkerboard.h:39-58 */
        if (m->diffuse < FLT_EPS_F) { *out = mkray(I, normalize(reflect(in->D, N)), 1e34f); return 1; }
        else if (m->specular < FLT_EPS_F) { *out = mkray(I, diffuse_reflection(N, seed), 1e34f); return 0; }
        if (rnd_f(seed) < m->specular) { *out = mkray(I, normalize(reflect(in->D, N)), 1e34f); return 1; }
        *out = mkray(I, diffuse_reflection(N, seed), 1e34f);
        return 0;
    }
}
/* TextureMaterial::GetColor, TextureMaterial.h:30-37 */
static f3 texture_color(const or_scene *s, const material *m, const ray_t *in, float scale) {
    const texture_t *t = &s->tex[m->tex];
    uint32_t u = f2u_wrap((float)t->w * in->u);
    uint32_t v = f2u_wrap((float)t->h * in->v);
    uint32_t idx = (u & (uint32_t)(t->w - 1)) + (v & (uint32_t)(t->h - 1)) * (uint32_t)t->w;
    uint32_t p = t->px[idx];
    return muls(mk((float)((p >> 16) & 255), (float)((p >> 8) & 255), (float)(p & 255)), scale);
}
static f3 mat_color(const or_scene *s, const material *m, const ray_t *in) {
    switch (m->kind) {
    case OR_TEXTURE:
        return texture_color(s, m, in, 1.0f / 255.0f);   /* TextureMaterial::correction */
    case OR_DIELECTRIC: {   /* Dielectric.h:12-21 */
        f3 c = mk(1, 1, 1);
        if (in->inside) {
            c.x = cr_expf(-m->c0.x * in->t);
            c.y = cr_expf(-m->c0.y * in->t);
            c.z = cr_expf(-m->c0.z * in->t);
        }
        return c;
    }
    case OR_CHECKER: {      /* Checkerboard.h:28-37 */
        f3 I = add(in->O, smul(in->t, in->D));
        int ex = abs(((int)floorf(I.x)) % 2) == 0;
        int ez = abs(((int)floorf(I.z)) % 2) == 0;
        return ex == ez ? m->c0 : m->c1;
    }
    default:
        return m->c0;
    }
}

/* Renderer::NextEventDirectIllumination, renderer.h:44-75 */
static f3 nee(const or_scene *s, f3 I, f3 N, f3 BRDF, uint32_t *seed, counters *k) {
    const int light = 0;   /* Scene::GetRandomLight, scene.h:225-227 */
    const prim *lp = &s->p[light];
    f3 Il = light_random_point(lp, seed);
    float area = prim_area(lp);
    f3 L = sub(Il, I);
    float dist = length3(L);
    L = divs(L, dist);
    f3 Nl = scene_normal(s, light, Il, L);
    float dotNL = dot(N, L), dotNlL = dot(Nl, neg(L));
    f3 Ld = mk(0, 0, 0);
    if (dotNL > 0 && dotNlL > 0) {
        ray_t sh = mkray(I, L, dist - 2.0f * EPS_F);
        if (k) k->shadow++;
        if (!is_occluded(s, &sh, k)) {
            float solid = (dotNlL * area) / (dist * dist);
            float lightPDF = 1.0f / solid;
            Ld = muls(mul(mat_color(s, &s->m[lp->mat], &sh), BRDF), (dotNL / lightPDF));
        }
    }
    return Ld;
}

/* Renderer::Trace, renderer.cpp:17-72 */
static f3 trace(const or_scene *s, ray_t *ray, int lastSpecular, int depth, uint32_t *seed, counters *k) {
    if (depth == 0) return mk(0, 0, 0);
    intersect_bvh(s, ray, k);
    if (ray->obj == -1) return sky_color(s, ray->D);
    f3 I = add(ray->O, smul(ray->t, ray->D));
    f3 N = scene_normal(s, ray->obj, I, ray->D);
    const material *m = &s->m[s->p[ray->obj].mat];
    ray_t out = mkray(mk(0, 0, 0), mk(1, 1, 1), 1e34f);
    int spec = mat_scatter(m, ray, I, N, &out, seed);
    f3 albedo = mat_color(s, m, ray);
    int flag = mat_flag(m);
    if (flag == FLAG_DIFFUSE || (flag == FLAG_MIX && !spec)) {
        f3 BRDF = muls(albedo, INVPI_F);
        float PDF = INV2PI_F;
        f3 Ld = nee(s, I, N, BRDF, seed, k);
        f3 Ei = divs(muls(trace(s, &out, spec, depth - 1, seed, k), dot(N, out.D)), PDF);
        return add(mul(BRDF, Ei), Ld);
    } else if (flag == FLAG_SPECULAR || flag == FLAG_MIX || flag == FLAG_DIELECTRIC) {
        return mul(albedo, trace(s, &out, spec, depth - 1, seed, k));
    } else {   /* LIGHT */
        if (lastSpecular) return albedo;
        return mk(0, 0, 0);
    }
}

/* ObjectMaterial::getColorModifier overrides (Whitted colour + parameters):
 * Diffuse.h:21-23, Mirror.h:21-23, Light.h:20-22, Checkerboard.h:60-71, Dielectric.h:56-85 */
static void color_modifier(const or_scene *s, const material *m, const ray_t *in, f3 N, float cv[7]) {
    memset(cv, 0, 7 * sizeof(float));
    switch (m->kind) {
    case OR_LIGHT:
        /* template/precomp.h:782 clamp = fmaxf(a, fminf(f, b)) */
        cv[0] = tmax_(0.0f, tmin_(m->c0.x, 1.0f)); cv[1] = tmax_(0.0f, tmin_(m->c0.y, 1.0f));
        cv[2] = tmax_(0.0f, tmin_(m->c0.z, 1.0f));
        return;
    case OR_CHECKER: {
        f3 c = mat_color(s, m, in);
        cv[0] = c.x; cv[1] = c.y; cv[2] = c.z; cv[3] = m->diffuse;
        return;
    }
    case OR_DSMIX:   /* DSMix.h:48-50 */
        cv[0] = m->c0.x; cv[1] = m->c0.y; cv[2] = m->c0.z; cv[3] = m->diffuse;
        return;
    case OR_TEXTURE: {   /* TextureMaterial.h:62-71 (SKYDOME_CORRECTION) */
        f3 c = texture_color(s, m, in, SKYDOME_CORRECTION_F);
        cv[0] = c.x; cv[1] = c.y; cv[2] = c.z; cv[3] = m->diffuse;
        return;
    }
    case OR_DIELECTRIC: {
        float n1 = 1, n2 = m->ior, n12 = n1 / n2;
        float cosi = dot(N, in->D);
        f3 beers = mk(1, 1, 1);
        if (in->inside) {
            beers.x = cr_expf(-m->c0.x * in->t); beers.y = cr_expf(-m->c0.y * in->t); beers.z = cr_expf(-m->c0.z * in->t);
            n12 = 1 / n12;
        }
        float k = 1 - (n12 * n12) * (1 - (cosi * cosi));
        cv[0] = beers.x; cv[1] = beers.y; cv[2] = beers.z;
        if (k < 0) { cv[3] = -1.0f; return; }
        float Fr = 0;
        if (!in->inside) {
            float sini = length3(cross(N, in->D));
            float sq = n12 * sini;
            float cost = sqrtf(1 - sq * sq);
            Fr = fresnel(n1, n2, cost, -cosi);
        }
        f3 T = normalize(sub(smul(n12, in->D), smul(n12 * cosi + sqrtf(k), N)));
        cv[3] = Fr; cv[4] = T.x; cv[5] = T.y; cv[6] = T.z;
        return;
    }
    default:
        cv[0] = m->c0.x; cv[1] = m->c0.y; cv[2] = m->c0.z;
        return;
    }
}

/* Renderer::DirectIllumination, renderer.h:24-42 (4 light samples, GetLightDir (0,-1,0)) */
static f3 direct_illumination(const or_scene *s, f3 I, f3 N, uint32_t *seed, counters *k) {
    f3 result = mk(0, 0, 0);
    int samples = 0;
    const f3 ldir = mk(0.0f, -1.0f, 0.0f), lcol = mk(24, 24, 22);   /* scene.h:237-242 */
    for (; samples < 4; samples++) {
        f3 L = sub(light_random_point(&s->p[0], seed), I);
        float dist = length3(L);
        L = divs(L, dist);
        float dotDN = dot(L, N);
        if (dotDN < 0 || dot(ldir, L) > 0) continue;
        ray_t toLight = mkray(I, L, dist - (2 * EPS_F));
        if (k) k->shadow++;
        if (is_occluded(s, &toLight, k)) continue;
        result = add(result, smul(dotDN / (dist * dist), lcol));
    }
    return divs(result, (float)samples);
}

/* Renderer::WhittedTrace, renderer.cpp:138-195 */
static f3 whitted(const or_scene *s, ray_t *ray, int depth, uint32_t *seed, counters *k) {
    f3 result = mk(0, 0, 0);
    if (depth == 0) return result;
    intersect_bvh(s, ray, k);
    if (ray->obj == -1) return sky_color(s, ray->D);
    f3 I = add(ray->O, smul(ray->t, ray->D));
    f3 N = scene_normal(s, ray->obj, I, ray->D);
    const material *m = &s->m[s->p[ray->obj].mat];
    int flag = mat_flag(m);
    float cv[7];
    color_modifier(s, m, ray, N, cv);
    if (flag == FLAG_LIGHT) {
        result = add(result, mk(24, 24, 22));
    } else if (flag == FLAG_DIFFUSE) {
        result = add(result, direct_illumination(s, I, N, seed, k));
    } else if (flag == FLAG_SPECULAR) {
        ray_t r = mkray(I, normalize(reflect(ray->D, N)), 1e34f);
        result = add(result, whitted(s, &r, depth - 1, seed, k));
    } else if (flag == FLAG_MIX) {
        result = add(result, smul(cv[3], direct_illumination(s, I, N, seed, k)));
        ray_t r = mkray(I, normalize(reflect(ray->D, N)), 1e34f);
        result = add(result, smul(1.0f - cv[3], whitted(s, &r, depth - 1, seed, k)));
    } else if (flag == FLAG_DIELECTRIC) {
        if (cv[3] < 0) {
            ray_t r = mkray(I, normalize(reflect(ray->D, N)), 1e34f);
            r.inside = 1;
            result = add(result, whitted(s, &r, depth - 1, seed, k));
        } else {
            float Fr = cv[3], Ft = 1 - Fr;
            if (Fr > FLT_EPS_F) {
                ray_t r = mkray(I, normalize(reflect(ray->D, N)), 1e34f);
                result = add(result, smul(Fr, whitted(s, &r, depth - 1, seed, k)));
            }
            if (Ft > FLT_EPS_F) {
                ray_t r = mkray(I, mk(cv[4], cv[5], cv[6]), 1e34f);
                r.inside = !ray->inside;
                result = add(result, smul(Ft, whitted(s, &r, depth - 1, seed, k)));
            }
        }
    }
    return mul(mk(cv[0], cv[1], cv[2]), result);
}

/* Scene::IntersectBVHPacket, template/scene.h:322-412: 64 rays share one traversal led by
 * the "first active" ray.  The reference fills off-screen slots of edge packets with
 * uninitialised rays; here they are inactive (never tested, never lead). */
static void intersect_packet(const or_scene *s, ray_t *R, const int *active, counters *k) {
    int fa = 0;                                  /* slot 0 is always on screen */
    const node *n = &s->nodes[0];
    const node *stack[64];
    uint32_t sp = 0;
    if (k) for (int i = 0; i < 64; i++) k->isect += active[i];
    for (;;) {
        if (hits_aabb(&R[fa], n)) {
            if (n->count > 0) {
                for (int i = 0; i < 64; i++) {
                    if (!active[i]) continue;
                    for (uint32_t j = 0; j < n->count; j++) {
                        int oi = (int)s->idx[n->leftFirst + j];
                        prim_intersect(&s->p[oi], &R[i], oi);
                    }
                }
                if (sp == 0) break;
                n = stack[--sp];
                continue;
            }
        } else {
            int found = -1;
            for (int i = 0; i < 64; i++)
                if (active[i] && hits_aabb(&R[i], n)) { found = i; break; }
            if (found < 0) {
                if (sp == 0) break;
                n = stack[--sp];
                continue;
            }
            fa = found;
            if (n->count > 0) {
                for (int i = fa; i < 64; i++) {
                    if (!active[i]) continue;
                    for (uint32_t j = 0; j < n->count; j++) {
                        int oi = (int)s->idx[n->leftFirst + j];
                        prim_intersect(&s->p[oi], &R[i], oi);
                    }
                }
                if (sp == 0) break;
                n = stack[--sp];
                continue;
            }
        }
        const node *c1 = &s->nodes[n->leftFirst], *c2 = &s->nodes[n->leftFirst + 1];
        float d1 = intersect_aabb(&R[fa], c1), d2 = intersect_aabb(&R[fa], c2);
        if (d1 > d2) { float td = d1; d1 = d2; d2 = td; const node *tn = c1; c1 = c2; c2 = tn; }
        n = c1;
        if (sp == 64) { fprintf(stderr, "oracle: packet stack overflow\n"); abort(); }
        stack[sp++] = c2;
    }
}

/* Renderer::TracePacket's per-ray shading, renderer.cpp:78-133 (bounces: Trace, depth given) */
static f3 shade_packet_ray(const or_scene *s, ray_t *ray, int depth, uint32_t *seed, counters *k) {
    if (ray->obj == -1) return sky_color(s, ray->D);
    f3 I = add(ray->O, smul(ray->t, ray->D));
    f3 N = scene_normal(s, ray->obj, I, ray->D);
    const material *m = &s->m[s->p[ray->obj].mat];
    ray_t out = mkray(mk(0, 0, 0), mk(1, 1, 1), 1e34f);
    int spec = mat_scatter(m, ray, I, N, &out, seed);
    f3 albedo = mat_color(s, m, ray);
    int flag = mat_flag(m);
    if (flag == FLAG_DIFFUSE || flag == FLAG_MIX) {
        /* MIX: a specular bounce is traced once for a result that is then overwritten
         * (renderer.cpp:111-114), and the same ray is traced again below (116-120) */
        if (flag == FLAG_MIX && spec) (void)trace(s, &out, spec, depth, seed, k);
        f3 BRDF = muls(albedo, INVPI_F);
        float PDF = INV2PI_F;
        f3 Ld = nee(s, I, N, BRDF, seed, k);
        f3 Ei = divs(muls(trace(s, &out, spec, depth, seed, k), dot(N, out.D)), PDF);
        return add(mul(BRDF, Ei), Ld);
    } else if (flag == FLAG_SPECULAR || flag == FLAG_DIELECTRIC) {
        return mul(albedo, trace(s, &out, spec, depth, seed, k));
    }
    return albedo;   /* LIGHT */
}

static uint32_t pixel_seed(int W, int H, int pixel, int sample, int spp, int frame);

/* One 8x8 packet tile (the PACKET_TRAVERSAL branch of Renderer::Tick, renderer.cpp:247-285),
 * averaged over spp packets; out[lane] for lane = xp + 8 * yp. */
static void packet_tile(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
                        int tx, int ty, f3 *out, counters *k) {
    ray_t R[64];
    uint32_t seed[64];
    int active[64];
    for (int l = 0; l < 64; l++) out[l] = mk(0, 0, 0);
    for (int smp = 0; smp < spp; smp++) {
        for (int l = 0; l < 64; l++) {
            int x = tx * 8 + (l & 7), y = ty * 8 + (l >> 3);
            active[l] = x < W && y < H;
            if (!active[l]) continue;
            seed[l] = pixel_seed(W, H, x + y * W, smp, spp, frame);
            R[l] = primary_ray(c, x, y, &seed[l]);
        }
        intersect_packet(s, R, active, k);
        for (int l = 0; l < 64; l++)
            if (active[l]) out[l] = add(out[l], shade_packet_ray(s, &R[l], depth, &seed[l], k));
    }
    for (int l = 0; l < 64; l++) out[l] = smul(1.0f / (float)spp, out[l]);
}

void or_scene_set_integrator(or_scene *s, int mode) { s->integrator = mode; }

/* ------------------------------------------------------------------ drivers */
static uint32_t pixel_seed(int W, int H, int pixel, int sample, int spp, int frame) {
    return or_init_seed((uint32_t)pixel + (uint32_t)W * (uint32_t)H * (uint32_t)(sample + spp * frame));
}

void or_camera_rays(const or_camera *c, int W, int H, int frame, const int32_t *pixels, int n, float *rays7) {
    for (int i = 0; i < n; i++) {
        int px = pixels[i];
        uint32_t seed = pixel_seed(W, H, px, 0, 1, frame);
        ray_t r = primary_ray(c, px % W, px / W, &seed);
        float *q = rays7 + 7 * (size_t)i;
        q[0] = r.O.x; q[1] = r.O.y; q[2] = r.O.z; q[3] = r.D.x; q[4] = r.D.y; q[5] = r.D.z; q[6] = r.t;
    }
}

void or_primary_hits(const or_scene *s, const or_camera *c, int W, int H, int frame,
                     const int32_t *pixels, int n, float *t, int32_t *obj, float *u, float *v) {
    #pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < n; i++) {
        int px = pixels[i];
        uint32_t seed = pixel_seed(W, H, px, 0, 1, frame);
        ray_t r = primary_ray(c, px % W, px / W, &seed);
        intersect_bvh(s, &r, NULL);
        t[i] = r.t; obj[i] = r.obj; u[i] = r.u; v[i] = r.v;
    }
}

static void add_counters(or_stats *st, const counters *k) {
    if (!st) return;
    #pragma omp atomic
    st->isect += k->isect;
    #pragma omp atomic
    st->occl += k->occl;
    #pragma omp atomic
    st->shadow += k->shadow;
    #pragma omp atomic
    st->aabb_tests += k->aabb;
    #pragma omp atomic
    st->prim_tests += k->prim;
    #pragma omp atomic
    st->aabb_occl += k->aabb_o;
    #pragma omp atomic
    st->prim_occl += k->prim_o;
}

static f3 trace_pixel(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
                      int px, counters *k) {
    f3 res = mk(0, 0, 0);
    int x = px % W, y = px / W;
    if (s->integrator == 2) {   /* the pixel's whole packet is traced; its counters are not kept */
        f3 tile[64];
        packet_tile(s, c, W, H, spp, depth, frame, x / 8, y / 8, tile, NULL);
        return tile[(x & 7) + 8 * (y & 7)];
    }
    for (int smp = 0; smp < spp; smp++) {
        uint32_t seed = pixel_seed(W, H, px, smp, spp, frame);
        ray_t r = primary_ray(c, x, y, &seed);
        res = add(res, s->integrator == 1 ? whitted(s, &r, depth, &seed, k) : trace(s, &r, 1, depth, &seed, k));
    }
    return smul(1.0f / (float)spp, res);
}

void or_pixel_work(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
                   const int32_t *pixels, int n, uint32_t *work) {
    #pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++) {
        uint32_t *w = work + 8 * (size_t)i;
        for (int q = 0; q < 8; q++) w[q] = 0;
        tl_work = w;
        (void)trace_pixel(s, c, W, H, spp, depth, frame, pixels[i], NULL);
        tl_work = NULL;
    }
}

/* The wave camera walk's exactness precondition (the library's wave_closest_hit_fast,
 * rt_kernels.inc).  The walk returns IntersectBVH's answer R for a camera ray, or flags the lane and
 * re-traces it in the reference order, unless R's computed t_R lies at least the walk's cull margin
 * before the computed slab entry of R's own leaf box L_R: e_L >= t_R * (1 + margin).  Per camera ray
 * (sample 0 of `frame`) this returns need = (e_L - t_R) / t_R for R = the reference's answer (0 for a
 * miss or a hit at or past its leaf's entry).  all != 0: the max of the same quantity over EVERY
 * primitive the ray hits (Primitive::Intersect accepting it from a fresh ray), found by a traversal
 * that culls boxes only on a slab miss -- a bound for any visiting order.  A frame whose rays all have
 * need < margin is rendered by the walk exactly as by the reference order.  obj (optional, all == 0):
 * R's primitive id per ray (-1 for a miss). */
void or_walk_need(const or_scene *s, const or_camera *c, int W, int H, int frame, const int32_t *pixels, int n,
                  int all, float *need, int32_t *obj) {
    #pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < n; i++) {
        uint32_t seed = pixel_seed(W, H, pixels[i], 0, 1, frame);
        const ray_t r = primary_ray(c, pixels[i] % W, pixels[i] / W, &seed);
        int target = -1;
        float t_target = 0.0f;
        if (!all) {
            ray_t q = r;
            intersect_bvh(s, &q, NULL);
            target = q.obj;
            t_target = q.t;
            if (obj) obj[i] = target;
            if (target < 0) { need[i] = 0.0f; continue; }
        }
        const node *stack[64];
        uint32_t sp = 0;
        const node *nd = &s->nodes[0];
        double worst = 0.0;
        for (;;) {
            if (nd->count > 0) {
                const float e = slab_entry(&r, nd);
                for (uint32_t k = 0; k < nd->count; k++) {
                    int oi = (int)s->idx[nd->leftFirst + k];
                    if (!all && oi != target) continue;
                    float tp = t_target;
                    if (all) {
                        ray_t q = r;
                        prim_intersect(&s->p[oi], &q, oi);
                        if (q.obj != oi) continue;
                        tp = q.t;
                    }
                    if (e > tp) {
                        double d = ((double)e - (double)tp) / (double)tp;
                        if (d > worst) worst = d;
                    }
                }
            } else {
                const node *c1 = &s->nodes[nd->leftFirst], *c2 = &s->nodes[nd->leftFirst + 1];
                int h1 = hits_aabb(&r, c1), h2 = hits_aabb(&r, c2);   /* r.t = 1e34: a miss only */
                if (h1 && h2) { nd = c1; stack[sp++] = c2; continue; }
                if (h1 || h2) { nd = h1 ? c1 : c2; continue; }
            }
            if (sp == 0) break;
            nd = stack[--sp];
        }
        need[i] = (float)worst;
    }
}

void or_trace_pixels(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
                     const int32_t *pixels, int n, float *rgb, or_stats *st) {
    #pragma omp parallel
    {
        counters k; memset(&k, 0, sizeof(k));
        #pragma omp for schedule(dynamic, 16)
        for (int i = 0; i < n; i++) {
            f3 r = trace_pixel(s, c, W, H, spp, depth, frame, pixels[i], &k);
            rgb[3 * i] = r.x; rgb[3 * i + 1] = r.y; rgb[3 * i + 2] = r.z;
        }
        add_counters(st, &k);
    }
}

/* Renderer::Trace(ray, lastSpecular, depth) (renderer.cpp:17-72) / WhittedTrace(ray, depth)
 * (renderer.cpp:138-195, integrator 1) on caller rays: ray i uses the RNG state seeds[i]
 * (RandomFloat's seed, template/template.cpp:673-704) and leaves the state after the call in
 * it; flags[i] bit 0 = lastSpecular, bit 1 = ray.inside (NULL: lastSpecular true, outside). */
void or_trace_rays(const or_scene *s, const float *rays7, int n, const uint8_t *flags, int depth, uint32_t *seeds,
                   float *rgb, or_stats *st) {
    #pragma omp parallel
    {
        counters k; memset(&k, 0, sizeof(k));
        #pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < n; i++) {
            const float *q = rays7 + 7 * (size_t)i;
            ray_t r = mkray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), q[6]);
            const int fl = flags ? flags[i] : 1;
            r.inside = (fl & 2) != 0;
            f3 v = s->integrator == 1 ? whitted(s, &r, depth, &seeds[i], &k) : trace(s, &r, fl & 1, depth, &seeds[i], &k);
            rgb[3 * i] = v.x; rgb[3 * i + 1] = v.y; rgb[3 * i + 2] = v.z;
        }
        add_counters(st, &k);
    }
}

/* RGBF32_to_RGB8, template/precomp.h:441-444 (the _MSC_VER_ typo keeps this path) */
static inline uint32_t rgb8(const float *a) {
    uint32_t r = f2u_wrap(255.0f * smin(1.0f, a[0]));
    uint32_t g = f2u_wrap(255.0f * smin(1.0f, a[1]));
    uint32_t b = f2u_wrap(255.0f * smin(1.0f, a[2]));
    return (r << 16) + (g << 8) + b;
}

/* running average + RGB8, renderer.cpp:235-241 */
static void accumulate(float *acc, uint32_t *out, int px, f3 r) {
    float *a = acc + 4 * (size_t)px;
    a[3] += 1;
    float w = a[3], inv = 1.0f / w;
    float nx = a[0] + inv * (r.x - a[0]);
    float ny = a[1] + inv * (r.y - a[1]);
    float nz = a[2] + inv * (r.z - a[2]);
    float nw = a[3] + inv * (w - a[3]);
    a[0] = nx; a[1] = ny; a[2] = nz; a[3] = nw;
    if (out) out[px] = rgb8(a);
}

void or_tick(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
             int y0, int y1, float *acc, uint32_t *out, or_stats *st, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    if (s->integrator == 2) {   /* packet mode: whole 8x8 tiles; rows [y0, y1) rounded out to tiles */
        int tx_n = (W + 7) / 8, ty0 = y0 / 8, ty1 = (y1 + 7) / 8;
        #pragma omp parallel
        {
            counters k; memset(&k, 0, sizeof(k));
            #pragma omp for schedule(dynamic)
            for (int t = ty0 * tx_n; t < ty1 * tx_n; t++) {
                f3 tile[64];
                int tx = t % tx_n, ty = t / tx_n;
                packet_tile(s, c, W, H, spp, depth, frame, tx, ty, tile, &k);
                for (int l = 0; l < 64; l++) {
                    int x = tx * 8 + (l & 7), y = ty * 8 + (l >> 3);
                    if (x < W && y < H) accumulate(acc, out, x + y * W, tile[l]);
                }
            }
            add_counters(st, &k);
        }
        return;
    }
    #pragma omp parallel
    {
        counters k; memset(&k, 0, sizeof(k));
        #pragma omp for schedule(dynamic)
        for (int y = y0; y < y1; y++) {
            for (int x = 0; x < W; x++) {
                int px = x + y * W;
                accumulate(acc, out, px, trace_pixel(s, c, W, H, spp, depth, frame, px, &k));
            }
        }
        add_counters(st, &k);
    }
}

void or_intersect(const or_scene *s, const float *R, int n, float *t, int32_t *obj, float *u, float *v, int brute) {
    #pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < n; i++) {
        const float *q = R + 7 * (size_t)i;
        ray_t r = mkray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), q[6]);
        if (brute) { for (int j = 0; j < s->np; j++) prim_intersect(&s->p[j], &r, j); }
        else intersect_bvh(s, &r, NULL);
        t[i] = r.t; obj[i] = r.obj; u[i] = r.u; v[i] = r.v;
    }
}
void or_intersect_packets(const or_scene *s, const float *R, int n, float *t, int32_t *obj, float *u, float *v) {
    int np = (n + 63) / 64;
    #pragma omp parallel for schedule(dynamic, 16)
    for (int pk = 0; pk < np; pk++) {
        ray_t P[64];
        int active[64];
        for (int l = 0; l < 64; l++) {
            int i = pk * 64 + l;
            active[l] = i < n;
            if (!active[l]) continue;
            const float *q = R + 7 * (size_t)i;
            P[l] = mkray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), q[6]);
        }
        intersect_packet(s, P, active, NULL);
        for (int l = 0; l < 64; l++) {
            int i = pk * 64 + l;
            if (i < n) { t[i] = P[l].t; obj[i] = P[l].obj; u[i] = P[l].u; v[i] = P[l].v; }
        }
    }
}

void or_occluded(const or_scene *s, const float *R, int n, uint8_t *out) {
    #pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < n; i++) {
        const float *q = R + 7 * (size_t)i;
        ray_t r = mkray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), q[6]);
        out[i] = (uint8_t)is_occluded(s, &r, NULL);
    }
}

/* Single-thread probe with the shipped global RNG (seed 0x12345678), replaying the
 * SURVEY.md Appendix A driver: a coverage pass (+ brute-force check on every 16th
 * pixel in x and y), then the mode pass; ps = primary + NEE-style shadow ray for
 * every non-light hit, Nl taken at I + d*L exactly as that driver did. */
void or_probe(const or_scene *s, int W, int H, int mode, int depth, int spp, int brute, or_stats *st) {
    uint32_t seed = 0x12345678u;
    or_camera cam; or_camera_default(&cam, W, H);
    counters k; memset(&k, 0, sizeof(k));
    memset(st, 0, sizeof(*st));
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            ray_t a = primary_ray(&cam, x, y, &seed), b = a;
            intersect_bvh(s, &a, NULL);
            st->coverage += a.obj >= 0;
            if (brute && (x % 16 == 0) && (y % 16 == 0)) {
                for (int j = 0; j < s->np; j++) prim_intersect(&s->p[j], &b, j);
                st->bf_tested++;
                st->bf_mismatch += a.obj != b.obj;
            }
        }
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            if (mode == OR_PROBE_PRIMARY) {
                ray_t r = primary_ray(&cam, x, y, &seed);
                intersect_bvh(s, &r, &k);
            } else if (mode == OR_PROBE_PS) {
                ray_t r = primary_ray(&cam, x, y, &seed);
                intersect_bvh(s, &r, &k);
                if (r.obj > 0) {
                    f3 I = add(r.O, smul(r.t, r.D));
                    f3 N = scene_normal(s, r.obj, I, r.D);
                    f3 L = sub(light_random_point(&s->p[0], &seed), I);
                    float d = length3(L);
                    L = divs(L, d);
                    f3 Nl = scene_normal(s, 0, add(I, smul(d, L)), L);
                    if (dot(N, L) > 0 && dot(Nl, neg(L)) > 0) {
                        ray_t sh = mkray(I, L, d - 2.0f * EPS_F);
                        is_occluded(s, &sh, &k);
                        k.shadow++;
                    }
                }
            } else {
                for (int smp = 0; smp < spp; smp++) {
                    ray_t r = primary_ray(&cam, x, y, &seed);
                    (void)trace(s, &r, 1, depth, &seed, &k);
                }
            }
        }
    st->shadow = k.shadow; st->isect = k.isect; st->occl = k.occl;
    st->aabb_tests = k.aabb; st->prim_tests = k.prim;
    st->aabb_occl = k.aabb_o; st->prim_occl = k.prim_o;
}

/* ------------------------------------------------------------------ OBJ parsing (tinyobj restatement) */
#define IS_DIGIT(x) ((unsigned)((x) - '0') < 10u)
/* tryParseDouble, template/tiny_obj_loader.h:887-1016 */
static int try_parse_double(const char *s, const char *s_end, double *result) {
    if (s >= s_end) return 0;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+', exp_sign = '+';
    const char *curr = s;
    int read = 0, end_not_reached = 0, leading_dot = 0;
    if (*curr == '+' || *curr == '-') {
        sign = *curr; curr++;
        if ((curr != s_end) && (*curr == '.')) leading_dot = 1;
    } else if (IS_DIGIT(*curr)) {
    } else if (*curr == '.') {
        leading_dot = 1;
    } else return 0;
    end_not_reached = (curr != s_end);
    if (!leading_dot) {
        while (end_not_reached && IS_DIGIT(*curr)) {
            mantissa *= 10;
            mantissa += (int)(*curr - 0x30);
            curr++; read++;
            end_not_reached = (curr != s_end);
        }
        if (read == 0) return 0;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++; read = 1;
        end_not_reached = (curr != s_end);
        while (end_not_reached && IS_DIGIT(*curr)) {
            static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            mantissa += (int)(*curr - 0x30) * (read < 8 ? pow_lut[read] : pow(10.0, -read));
            read++; curr++;
            end_not_reached = (curr != s_end);
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else goto assemble;
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = (curr != s_end);
        if (end_not_reached && (*curr == '+' || *curr == '-')) { exp_sign = *curr; curr++; }
        else if (IS_DIGIT(*curr)) {
        } else return 0;
        read = 0;
        end_not_reached = (curr != s_end);
        while (end_not_reached && IS_DIGIT(*curr)) {
            if (exponent > (2147483647 / 10)) return 0;
            exponent *= 10;
            exponent += (int)(*curr - 0x30);
            curr++; read++;
            end_not_reached = (curr != s_end);
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) return 0;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * (exponent ? ldexp(mantissa * pow(5.0, exponent), exponent) : mantissa);
    return 1;
}
/* parseReal, 1019-1027 */
static float parse_real(const char **tok, double def) {
    *tok += strspn(*tok, " \t");
    const char *end = *tok + strcspn(*tok, " \t\r");
    double val = def;
    try_parse_double(*tok, end, &val);
    *tok = end;
    return (float)val;
}
/* fixIndex: 1-based positive, negative relative */
static int fix_index(int idx, int n, int *ret) {
    if (idx > 0) { *ret = idx - 1; return 1; }
    if (idx == 0) return 0;
    *ret = n + idx;
    return *ret >= 0;
}

typedef struct { float *v; int nv, capv; int *t; int nt, capt; } meshbuf;
static void mb_vert(meshbuf *m, float x, float y, float z) {
    if (m->nv == m->capv) { m->capv = m->capv ? 2 * m->capv : 4096; m->v = (float *)realloc(m->v, sizeof(float) * 3 * m->capv); }
    m->v[3 * m->nv] = x; m->v[3 * m->nv + 1] = y; m->v[3 * m->nv + 2] = z; m->nv++;
}
static void mb_tri(meshbuf *m, int a, int b, int c) {
    if (m->nt == m->capt) { m->capt = m->capt ? 2 * m->capt : 4096; m->t = (int *)realloc(m->t, sizeof(int) * 3 * m->capt); }
    m->t[3 * m->nt] = a; m->t[3 * m->nt + 1] = b; m->t[3 * m->nt + 2] = c; m->nt++;
}

int or_obj_parse(const char *path, float **verts, int *nv, int **tris, int *nt) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    meshbuf m; memset(&m, 0, sizeof(m));
    char *line = NULL; size_t cap = 0; ssize_t len;
    int fi[256];
    while ((len = getline(&line, &cap, f)) != -1) {
        while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
        const char *tok = line + strspn(line, " \t");
        if (tok[0] == 0 || tok[0] == '#') continue;
        if (tok[0] == 'v' && (tok[1] == ' ' || tok[1] == '\t')) {   /* 2619-2640 */
            tok += 2;
            float x = parse_real(&tok, 0.0), y = parse_real(&tok, 0.0), z = parse_real(&tok, 0.0);
            mb_vert(&m, x, y, z);
        } else if (tok[0] == 'f' && (tok[1] == ' ' || tok[1] == '\t')) {   /* 2770-2800 */
            tok += 2; tok += strspn(tok, " \t");
            int n = 0, ok = 1;
            while (tok[0] != 0 && tok[0] != '\r' && tok[0] != '\n') {
                int vi;
                if (!fix_index(atoi(tok), m.nv, &vi)) { ok = 0; break; }
                if (n < 256) fi[n++] = vi;
                tok += strcspn(tok, " \t\r");
                tok += strspn(tok, " \t\r");
            }
            if (!ok) { fclose(f); free(line); free(m.v); free(m.t); return -2; }
            if (n < 3) continue;                          /* degenerate face, 1476-1482 */
            if (n == 3) { mb_tri(&m, fi[0], fi[1], fi[2]); continue; }
            if (n == 4) {                                 /* shortest-diagonal split, 1484-1580 */
                const float *v0 = m.v + 3 * fi[0], *v1 = m.v + 3 * fi[1], *v2 = m.v + 3 * fi[2], *v3 = m.v + 3 * fi[3];
                float e02x = v2[0] - v0[0], e02y = v2[1] - v0[1], e02z = v2[2] - v0[2];
                float e13x = v3[0] - v1[0], e13y = v3[1] - v1[1], e13z = v3[2] - v1[2];
                float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
                float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
                if (sqr02 < sqr13) { mb_tri(&m, fi[0], fi[1], fi[2]); mb_tri(&m, fi[0], fi[2], fi[3]); }
                else { mb_tri(&m, fi[0], fi[1], fi[3]); mb_tri(&m, fi[1], fi[2], fi[3]); }
                continue;
            }
            /* n > 4: none of the reference assets has such faces; fan as a fallback */
            for (int k = 1; k + 1 < n; k++) mb_tri(&m, fi[0], fi[k], fi[k + 1]);
        }
    }
    free(line); fclose(f);
    *verts = m.v; *nv = m.nv; *tris = m.t; *nt = m.nt;
    return 0;
}
void or_free(void *p) { free(p); }

/* RTMESH1 container: "RTMESH1\0", u32 nv, u32 nt, f32[3nv], i32[3nt] */
int or_mesh_write(const char *path, const float *V, int nv, const int *T, int nt) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    uint32_t h[2] = {(uint32_t)nv, (uint32_t)nt};
    fwrite("RTMESH1", 1, 8, f); fwrite(h, 4, 2, f);
    fwrite(V, 4, 3 * (size_t)nv, f); fwrite(T, 4, 3 * (size_t)nt, f);
    fclose(f);
    return 0;
}
int or_mesh_read(const char *path, float **V, int *nv, int **T, int *nt) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char mag[8]; uint32_t h[2];
    if (fread(mag, 1, 8, f) != 8 || memcmp(mag, "RTMESH1", 8) != 0 || fread(h, 4, 2, f) != 2) { fclose(f); return -2; }
    *V = (float *)malloc(4 * 3 * (size_t)h[0]); *T = (int *)malloc(4 * 3 * (size_t)h[1]);
    size_t a = fread(*V, 4, 3 * (size_t)h[0], f), b = fread(*T, 4, 3 * (size_t)h[1], f);
    fclose(f);
    if (a != 3 * (size_t)h[0] || b != 3 * (size_t)h[1]) { free(*V); free(*T); return -3; }
    *nv = (int)h[0]; *nt = (int)h[1];
    return 0;
}

/* ------------------------------------------------------------------ SURVEY 8(d) scene recipes */
static int add_mesh_file(or_scene *s, const char *dir, const char *name, const float M[16], int mat) {
    char path[1024];
    snprintf(path, sizeof(path), "%s/%s.rtmesh", dir, name);
    float *V; int *T; int nv, nt;
    if (or_mesh_read(path, &V, &nv, &T, &nt) != 0) return -1;
    or_scene_add_mesh(s, V, nv, T, nt, M, mat);
    free(V); free(T);
    return 0;
}
static void floor2(or_scene *s, int mat) {
    const float fy = -1.225f;
    float a[3] = {-20, fy, -1}, b[3] = {20, fy, -1}, c[3] = {20, fy, 40}, d[3] = {-20, fy, 40};
    or_scene_add_triangle(s, a, b, c, mat);
    or_scene_add_triangle(s, a, c, d, mat);
}
static void chain(float out[16], const float *const *ms, int n) {
    float acc[16]; memcpy(acc, ms[0], 64);
    for (int i = 1; i < n; i++) or_mat4_mul(acc, acc, ms[i]);
    memcpy(out, acc, 64);
}
or_scene *or_scene_recipe(const char *name, const char *dir) {
    or_scene *s = or_scene_new();
    const float lampc[3] = {24.0f, 24.0f, 22.0f};
    const float white[3] = {0.95f, 0.95f, 0.95f}, green[3] = {0.05f, 0.95f, 0.05f};
    const float ck1[3] = {0.1f, 0.1f, 0.1f}, ck2[3] = {0.9f, 0.9f, 0.9f};
    int lamp = or_scene_add_material(s, OR_LIGHT, lampc, NULL, 0, 0);          /* scene.h:55 */
    int mwhite = or_scene_add_material(s, OR_DIFFUSE, white, NULL, 0, 0);       /* scene.h:46 */
    int mgreen = or_scene_add_material(s, OR_DIFFUSE, green, NULL, 0, 0);       /* scene.h:44 */
    int mcheck = or_scene_add_material(s, OR_CHECKER, ck1, ck2, 0, -1.0f);      /* scene.h:50 */
    int teapot_like = !strcmp(name, "teapot") || !strcmp(name, "mig16") || !strcmp(name, "default");
    float lp[3] = {0.0f, teapot_like ? 6.0f : 4.0f, teapot_like ? 5.0f : -2.0f};
    or_scene_add_sphere(s, lp, 0.5f, lamp);
    float T[16], R[16], S[16], R2[16], R3[16], M[16];
    int rc = 0;
    if (!strcmp(name, "teapotF") || !strcmp(name, "teapot")) {
        int f = !strcmp(name, "teapotF");
        or_mat4_translate(T, 0, 0, f ? 2.0f : 1.5f);
        or_mat4_rotate_y(R, 0.5f * PI_F);
        or_mat4_scale(S, f ? 2.5f : 1.5f);
        const float *c[3] = {T, R, S}; chain(M, c, 3);
        rc |= add_mesh_file(s, dir, "teapot", M, mwhite);
        if (f) floor2(s, mcheck);
    } else if (!strcmp(name, "mig16")) {
        for (int i = 0; i < 16; i++) {
            float x = (float)(i % 4) - 1.5f, y = (float)(i / 4) - 1.5f;
            or_mat4_translate(T, x * 1.8f, y * 1.1f - 0.3f, 2.5f);
            or_mat4_rotate_x(R, 0.3f * PI_F);
            or_mat4_scale(S, 0.01f);
            const float *c[3] = {T, R, S}; chain(M, c, 3);
            rc |= add_mesh_file(s, dir, "mig29", M, mgreen);
        }
    } else if (!strcmp(name, "cfg3")) {
        const float ab[3] = {0.5f, 0.5f, 0.5f}, mc[3] = {0.9f, 0.75f, 0.0f};
        int glass = or_scene_add_material(s, OR_DIELECTRIC, ab, NULL, 1.52f, 0);
        int mirror = or_scene_add_material(s, OR_MIRROR, mc, NULL, 0, 0);
        or_mat4_translate(T, 0, -1, 2); or_mat4_scale(S, 8.0f);
        const float *c1[2] = {T, S}; chain(M, c1, 2);
        rc |= add_mesh_file(s, dir, "Shiba", M, glass);
        /* glider transform, template/scene.h:88 */
        or_mat4_translate(T, 1.0f, 0.0f, 0.0f);
        or_mat4_rotate_z(R, -0.15f * PI_F); or_mat4_rotate_y(R2, 0.05f * PI_F); or_mat4_rotate_x(R3, -0.55f * PI_F);
        or_mat4_scale(S, 0.025f);
        const float *c2[5] = {T, R, R2, R3, S}; chain(M, c2, 5);
        rc |= add_mesh_file(s, dir, "glider", M, mirror);
        floor2(s, mcheck);
    } else if (!strcmp(name, "default")) {
        /* the reference's as-shipped Scene() (template/scene.h:40-128): light (0,6,5), then
           cloud.obj, airways.obj, glider, piper_pa18.obj, mig29 -- cloud, airways and piper are
           not in assets/, and LoadModel returns without triangles for them (scene.h:164-168) */
        const float red[3] = {0.95f, 0.05f, 0.05f};
        int mred = or_scene_add_material(s, OR_DIFFUSE, red, NULL, 0, 0);       /* scene.h:43 */
        or_mat4_translate(T, 1.0f, 0.0f, 0.0f);                                   /* scene.h:88 */
        or_mat4_rotate_z(R, -0.15f * PI_F); or_mat4_rotate_y(R2, 0.05f * PI_F); or_mat4_rotate_x(R3, -0.55f * PI_F);
        or_mat4_scale(S, 0.025f);
        const float *c2[5] = {T, R, R2, R3, S}; chain(M, c2, 5);
        rc |= add_mesh_file(s, dir, "glider", M, mred);
        or_mat4_translate(T, 0.1f, 0.2f, -0.2f);                                  /* scene.h:94 */
        or_mat4_rotate_z(R, 1.1f * PI_F); or_mat4_rotate_y(R2, 0.05f * PI_F); or_mat4_rotate_x(R3, 0.2f * PI_F);
        or_mat4_scale(S, 0.001f);
        const float *c3[5] = {T, R, R2, R3, S}; chain(M, c3, 5);
        rc |= add_mesh_file(s, dir, "mig29", M, mgreen);
    } else if (!strcmp(name, "cfg5")) {
        or_mat4_translate(T, 0, -1.2f, 2.5f); or_mat4_scale(S, 12.0f);
        const float *c[2] = {T, S}; chain(M, c, 2);
        rc |= add_mesh_file(s, dir, "Shiba", M, mwhite);
        floor2(s, mcheck);
    } else {
        rc = -1;
    }
    if (rc != 0) { or_scene_free(s); return NULL; }
    or_scene_build_bvh(s);
    return s;
}
