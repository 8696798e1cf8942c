/*
 * rt_oracle.h -- CPU restatement of the reference ray tracer's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker, never the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so.  The shipped path is the HIP library under
 * advancedgraphicsraytracer_amd/csrc and fails loudly without it.
 *
 * PARITY PIN: partial.  The reference (pmichels19/AdvancedGraphicsRayTracer)
 * is unbuildable in this image without stand-ins (template/precomp.h:21,77
 * include <io.h> and "windows.h"; MSVC-only anonymous-union float3 and
 * rvalue->Ray& binding), so there is no oracle/_ref build.  The restatement is
 * pinned against the reference-run statistics recorded in SURVEY.md /
 * BASELINE.md (plain-BVH node counts and depths, coverage, exact shadow-ray
 * counts and rays/sample of the single-thread global-RNG runs), reproduced
 * by or_probe() below -- see tests/test_oracle_pins.py.
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* material kinds (MaterialType.h:3-9 + the concrete classes) */
enum { OR_DIFFUSE = 0, OR_MIRROR = 1, OR_DIELECTRIC = 2, OR_CHECKER = 3, OR_LIGHT = 4, OR_DSMIX = 5, OR_TEXTURE = 6 };
/* primitive kinds (Primitive.h:8-14) */
enum { OR_SPHERE = 0, OR_PLANE = 1, OR_CUBE = 2, OR_QUAD = 3, OR_TRIANGLE = 4 };
/* probe modes (SURVEY.md Appendix A / BASELINE.md section 2) */
enum { OR_PROBE_PRIMARY = 0, OR_PROBE_PS = 1, OR_PROBE_PT = 2 };

typedef struct or_scene or_scene;

typedef struct {
    float pos[3], tl[3], tr[3], bl[3];
    float lens_radius, rwidth, rheight;
} or_camera;

typedef struct {
    int64_t coverage;    /* primary rays that hit something */
    int64_t shadow;      /* shadow rays issued (ps mode) */
    int64_t isect;       /* Scene::IntersectBVH calls */
    int64_t occl;        /* Scene::IsOccluded calls */
    int64_t bf_tested;   /* brute-force cross-checked rays */
    int64_t bf_mismatch; /* of those, objIdx disagreements */
    int64_t aabb_tests;  /* child AABB tests, all traversals */
    int64_t prim_tests;  /* primitive tests, all traversals */
    int64_t aabb_occl;   /* of aabb_tests, those made by IsOccluded */
    int64_t prim_occl;   /* of prim_tests, those made by IsOccluded */
} or_stats;

/* OBJ parsing: restates tinyobj LoadObj (template/tiny_obj_loader.h:2554-2830,
 * tryParseDouble 887-1016, quad split 1484-1580) for v/f records. */
int or_obj_parse(const char *path, float **verts, int *nv, int **tris, int *nt);
void or_free(void *p);

/* mat4 (template/precomp.h:960-1199, template/template.cpp:779-792) */
void or_mat4_identity(float m[16]);
void or_mat4_translate(float m[16], float x, float y, float z);
void or_mat4_scale(float m[16], float s);
void or_mat4_rotate_x(float m[16], float a);
void or_mat4_rotate_y(float m[16], float a);
void or_mat4_rotate_z(float m[16], float a);
void or_mat4_mul(float r[16], const float a[16], const float b[16]);

/* scene assembly */
or_scene *or_scene_new(void);
void or_scene_free(or_scene *s);
int or_scene_add_material(or_scene *s, int kind, const float c0[3], const float c1[3], float ior, float diffuse);
/* TextureMaterial (TextureMaterial.h:6-17): texture = index from or_scene_add_texture */
int or_scene_add_material_tex(or_scene *s, int kind, const float c0[3], const float c1[3], float ior, float diffuse,
                              int texture);
/* Surface pixels 0x00RRGGBB (template/template.cpp:1579-1601), w x h */
int or_scene_add_texture(or_scene *s, int w, int h, const uint32_t *pixels);
/* Primitive::createCube (Primitive.h:717-728): T * Translate(pos) when |pos| > FLT_EPSILON */
int or_scene_add_cube(or_scene *s, const float pos[3], const float size[3], const float T[16], int mat);
/* Primitive::createQuad (Primitive.h:735-739) */
int or_scene_add_quad(or_scene *s, float size, const float T[16], int mat);
int or_scene_add_sphere(or_scene *s, const float pos[3], float r, int mat);
int or_scene_add_plane(or_scene *s, const float n[3], float d, int mat);
int or_scene_add_triangle(or_scene *s, const float v0[3], const float v1[3], const float v2[3], int mat);
int or_scene_add_mesh(or_scene *s, const float *verts, int nv, const int *tris, int nt, const float M[16], int mat);
int or_scene_build_bvh(or_scene *s);
int or_scene_set_bvh(or_scene *s, const void *nodes, int nodes_used, const uint32_t *idx, int nidx);
int or_scene_num_prims(const or_scene *s);
int or_scene_nodes_used(const or_scene *s);
int or_scene_depth(const or_scene *s);
const void *or_scene_nodes(const or_scene *s);    /* nodes_used x 32 B (BVHNode.h:5-14) */
const uint32_t *or_scene_indices(const or_scene *s);
void or_scene_set_sky(or_scene *s, int w, int h, const uint32_t *pixels);
/* build one of the SURVEY 8(d) scenes from RTMESH1 files in mesh_dir */
or_scene *or_scene_recipe(const char *name, const char *mesh_dir);
int or_mesh_read(const char *path, float **verts, int *nv, int **tris, int *nt);
int or_mesh_write(const char *path, const float *verts, int nv, const int *tris, int nt);

/* integrator used by or_trace_pixels / or_tick: 0 = Trace (default), 1 = WhittedTrace,
 * 2 = packet mode (IntersectBVHPacket + TracePacket; depth = the bounces' Trace depth) */
void or_scene_set_integrator(or_scene *s, int mode);

/* camera (camera.h:28-52) */
void or_camera_default(or_camera *c, int W, int H);

/* hot path, per-pixel seeded: seed = InitSeed(pixel + W*H*(sample + spp*frame)) */
uint32_t or_init_seed(uint32_t base);
/* Camera::GetPrimaryRay for sample 0 of a pixel list -> rays7 (O.xyz D.xyz t) */
void or_camera_rays(const or_camera *c, int W, int H, int frame, const int32_t *pixels, int n, float *rays7);
void or_primary_hits(const or_scene *s, const or_camera *c, int W, int H, int frame,
                     const int32_t *pixels, int n, float *t, int32_t *obj, float *u, float *v);
/* Renderer::Trace radiance averaged over spp for a pixel list (renderer.cpp:17-72, 222) */
void or_trace_pixels(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
                     const int32_t *pixels, int n, float *rgb, or_stats *st);
/* Traversal work of a pixel list (integrator 0 / 1): per pixel 8 counters -- closest-hit node
 * visits (interior + leaf) and primitive tests, any-hit node visits and primitive tests (shadow
 * rays counted in the library's farther-box-first order), closest-hit pops of interior / leaf
 * entries whose pushed entry distance is >= the ray's t at the pop, 0, 0 -- summed over the
 * pixel's samples */
/* the wave camera walk's exactness precondition per camera ray (see rt_oracle.c) */
void or_walk_need(const or_scene *s, const or_camera *c, int W, int H, int frame, const int32_t *pixels, int n,
                  int all, float *need, int32_t *obj);
void or_pixel_work(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
                   const int32_t *pixels, int n, uint32_t *work);
/* One Renderer::Tick over rows [y0,y1): trace, running average into acc (float4 per
 * pixel, renderer.cpp:235-241), RGB8 pack (template/precomp.h:432-448).  OpenMP. */
/* Renderer::Trace / WhittedTrace on caller rays with per-ray RNG states (updated in place) */
void or_trace_rays(const or_scene *s, const float *rays7, int n, const uint8_t *flags, int depth, uint32_t *seeds,
                   float *rgb, or_stats *st);
void or_tick(const or_scene *s, const or_camera *c, int W, int H, int spp, int depth, int frame,
             int y0, int y1, float *acc, uint32_t *rgb8, or_stats *st, int threads);
/* batched IntersectBVH / IsOccluded on explicit rays: ray = O.xyz D.xyz tmax */
void or_intersect(const or_scene *s, const float *rays7, int n, float *t, int32_t *obj, float *u, float *v, int brute);
/* Scene::IntersectBVHPacket on packets of 64 consecutive rays (the last may be partial) */
void or_intersect_packets(const or_scene *s, const float *rays7, int n, float *t, int32_t *obj, float *u, float *v);
void or_occluded(const or_scene *s, const float *rays7, int n, uint8_t *out);
/* reference probe with the shipped single global RNG (template/template.cpp:674-695),
 * sequence as SURVEY.md Appendix A's driver: coverage pass, then one mode pass. */
void or_probe(const or_scene *s, int W, int H, int mode, int depth, int spp, int brute, or_stats *st);

#ifdef __cplusplus
}
#endif
#endif
