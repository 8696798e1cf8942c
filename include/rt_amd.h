/*
 * rt_amd.h -- C-ABI of the MI355X-native ray-tracing hot path (librtamd.so).
 *
 * Drop-in boundary for the reference's Renderer::Tick / Renderer::Trace /
 * Scene::IntersectBVH / Scene::IsOccluded path (pmichels19/AdvancedGraphicsRayTracer).
 * The reference has no FFI of its own: its "boundary" is the in-process C++ class
 * surface cited on each entry point below.  A C++ host binds these functions
 * directly (see include/rt_compat.hpp); Python binds them with ctypes
 * (advancedgraphicsraytracer_amd/__init__.py).
 *
 * Conventions
 *   - every entry point is extern "C", returns int status (RT_OK = 0, < 0 error),
 *     and never throws; rt_last_error() returns a thread-local message;
 *   - scene/renderer handles are opaque; the library owns all device buffers it
 *     allocates; pointers named *_dev are caller-owned DEVICE memory, the rest are
 *     caller-owned host memory;
 *   - stream arguments are hipStream_t passed as void*; NULL is HIP's default (null)
 *     stream, as everywhere in HIP.  Handles create and finish their own setup work
 *     before returning; the *_host conveniences run on the handle's private stream
 *     and synchronize it;
 *   - primitive ids follow creation order exactly as the reference's
 *     Primitive::objIdx (Primitive.h:37-38); the light is primitive 0 and must be a
 *     sphere or a quad (Scene::GetRandomLight, template/scene.h:225-227).
 * No CPU fallback exists: without a usable gfx950 device every compute entry
 * point fails with RT_ERR_NO_DEVICE.
 */
#ifndef RT_AMD_H
#define RT_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 4

enum {
    RT_OK = 0,
    RT_ERR_INVALID = -1,    /* bad argument */
    RT_ERR_NO_DEVICE = -2,  /* no HIP device / kernel image not loadable */
    RT_ERR_HIP = -3,        /* HIP runtime error */
    RT_ERR_IO = -4,         /* file not found / parse error */
    RT_ERR_UNSUPPORTED = -5, /* scene outside the kernels' limits */
    RT_ERR_COMM = -6        /* RCCL missing or a collective failed */
};

/* Primitive kinds, Primitive.h:8-14. */
enum { RT_SPHERE = 0, RT_PLANE = 1, RT_CUBE = 2, RT_QUAD = 3, RT_TRIANGLE = 4 };
/* Materials: Diffuse.h, Mirror.h, Dielectric.h, Checkerboard.h, Light.h, DSMix.h,
 * TextureMaterial.h. */
enum { RT_DIFFUSE = 0, RT_MIRROR = 1, RT_DIELECTRIC = 2, RT_CHECKERBOARD = 3, RT_LIGHT = 4, RT_DSMIX = 5,
       RT_TEXTURE = 6 };
/* Integrators behind Renderer::Tick (renderer.cpp:227-231; the K key toggles them,
 * renderer.h:138): Trace (path tracer, default depth 10, renderer.h:9), WhittedTrace
 * (default depth 20, renderer.h:13), and the PACKET_TRAVERSAL build of Tick
 * (renderer.cpp:247-285): 8x8 tiles as 64-ray packets through IntersectBVHPacket, shaded
 * by TracePacket whose bounces are Trace(.., depth) -- depth 10 in the reference, 0 allowed.
 * depth <= 32 for all three. */
enum { RT_MODE_PATH = 0, RT_MODE_WHITTED = 1, RT_MODE_PACKET = 2 };

/* One primitive, Primitive::create* factories (Primitive.h:690-747):
 *   RT_SPHERE:   v[0..2] centre, v[3] radius
 *   RT_PLANE:    v[0..2] normal, v[3] distance
 *   RT_CUBE:     v[0..2] position, v[3..5] size; createCube(pos, size, material, T)
 *   RT_QUAD:     v[0] size; createQuad(size, material, T)
 *   RT_TRIANGLE: v[0..8] three world-space vertices (post Scene::LoadModel)
 * T (cube / quad only) comes from rt_scene_desc.transforms. */
typedef struct { int32_t type; int32_t material; float v[9]; } rt_prim;

/* One material.  color = Diffuse/Mirror/Light/DSMix colour or Dielectric absorption;
 * color2 = Checkerboard second colour; ior = Dielectric n; diffuse = the diffuse share
 * of Checkerboard / DSMix / TextureMaterial (clamped to [0, 1]; < 0 selects the short
 * Checkerboard / TextureMaterial constructor: diffuse 1, specular 0); texture = index
 * into rt_scene_desc.textures (RT_TEXTURE only). */
typedef struct {
    int32_t kind; float color[3]; float color2[3]; float ior; float diffuse; int32_t texture;
} rt_material;

/* A Surface (template/template.cpp:1571-1601): 0x00RRGGBB texels, row-major.
 * TextureMaterial indexes it as (u & (width-1)) + (v & (height-1)) * width. */
typedef struct { const uint32_t *pixels; uint32_t width, height; } rt_texture;

/* Scene description, the inputs of Scene::Scene (template/scene.h:40-128). */
typedef struct {
    const rt_prim *prims; uint32_t num_prims;
    const rt_material *materials; uint32_t num_materials;
    /* sky: power-of-two texture of 0x00RRGGBB (renderer.h:15-22); NULL = the
     * synthetic 1024x512 constant 0x406080 sky of SURVEY.md 8(d) */
    const uint32_t *sky_pixels; uint32_t sky_width, sky_height;
    /* optional prebuilt plain BVH: nodes in the 32-byte BVHNode layout
     * (BVHNode.h:5-14, root 0, node 1 unused) + primitiveIndices; NULL = build
     * here with the reference's binned SAH (template/scene.h:845-976) */
    const void *bvh_nodes; uint32_t bvh_num_nodes; const uint32_t *bvh_indices;
    int32_t device;
    /* per-primitive mat4 T (16 floats, row-major as rt_mat4_*), read for RT_CUBE and
     * RT_QUAD only; NULL = identity for all (the factories' default argument) */
    const float *transforms;
    const rt_texture *textures; uint32_t num_textures;
    /* RT_BVH_PLAIN (0): the reference's plain binned-SAH BVH (template/scene.h:845-976), the
     * parity tree; RT_BVH_SBVH: spatial splits (template/scene.h:521-840, built NaN-safe with a
     * growing pool) -- closest hits equal the plain tree's except exact-distance ties.
     * Ignored with a prebuilt BVH. */
    int32_t bvh_kind;
} rt_scene_desc;
enum { RT_BVH_PLAIN = 0, RT_BVH_SBVH = 1 };

/* num_refs = entries of the BVH's primitive-index array (= num_prims for the plain tree;
 * more for an SBVH, whose leaves may share primitives) */
typedef struct { uint32_t num_prims, nodes_used, depth, max_leaf, num_refs; } rt_scene_info;

/* Ray / hit records of the batched entry points (Ray.h:7-32). */
typedef struct { float ox, oy, oz, dx, dy, dz, tmax; } rt_ray;       /* 28 B */
typedef struct { float t; int32_t obj; float u, v; } rt_hit;           /* 16 B */

/* Camera state (camera.h:93-100): origin, virtual screen corners, lens radius. */
typedef struct { float pos[3], top_left[3], top_right[3], bottom_left[3]; float lens_radius; } rt_camera;

/* One frame.  spp samples per pixel per frame; depth = Trace depth (renderer.h:9
 * default 10; depth 1 = primary + NEE shadow ray); frame feeds the per-pixel seed
 * InitSeed(pixel + W*H*(sample + spp*frame)) (template/template.cpp:683-686);
 * reset = clear the accumulator first (renderer.cpp:237). */
typedef struct { uint32_t width, height, spp, depth, frame, mode, reset; } rt_frame_params;

/* Cumulative ray counters of a renderer. */
typedef struct { uint64_t primary, shadow, bounce, frames; } rt_counters;

typedef struct rt_scene rt_scene;
typedef struct rt_renderer rt_renderer;

/* ---- library ---------------------------------------------------------- */
int rt_abi_version(void);
const char *rt_last_error(void);
int rt_device_count(int *count);
void rt_free(void *p);

/* ---- host-side scene preparation (Scene::LoadModel, template/scene.h:156-201) ---- */
/* tinyobj-compatible OBJ read (template/tiny_obj_loader.h, triangulate=true):
 * vertices float[3*nv], faces int32[3*nt] in file order; free with rt_free. */
int rt_obj_load(const char *path, float **verts, uint32_t *nv, int32_t **faces, uint32_t *nt);
/* RTMESH1 container (parsed OBJ vertices + faces) used for the bundled scenes. */
int rt_mesh_load(const char *path, float **verts, uint32_t *nv, int32_t **faces, uint32_t *nt);
int rt_mesh_save(const char *path, const float *verts, uint32_t nv, const int32_t *faces, uint32_t nt);
/* mat4 helpers, template/precomp.h:1007-1039 and template/template.cpp:779-792 */
int rt_mat4_translate(float x, float y, float z, float out[16]);
int rt_mat4_scale(float s, float out[16]);
int rt_mat4_rotate(int axis, float angle, float out[16]);
int rt_mat4_mul(const float a[16], const float b[16], float out[16]);
/* append one triangle per face, vertices = TransformPosition(v, M)
 * (template/scene.h:185-191); out holds nt rt_prim records */
int rt_mesh_to_prims(const float *verts, uint32_t nv, const int32_t *faces, uint32_t nt,
                     const float M[16], int32_t material, rt_prim *out);
/* The SURVEY.md 8(d) scene recipes as descriptions: call once with prims == NULL to get
 * the counts, then with arrays of that size. */
int rt_recipe_describe(const char *name, const char *mesh_dir, rt_prim *prims, uint32_t *num_prims,
                       rt_material *materials, uint32_t *num_materials);
/* plain-BVH build only (no device): nodes (2N+2 x 32 B) and indices (N);
 * transforms as in rt_scene_desc (NULL = identity) */
int rt_bvh_build_host(const rt_prim *prims, const float *transforms, uint32_t n, void *nodes, uint32_t *indices,
                      rt_scene_info *info);
/* the opt-in spatial-split BVH (RT_BVH_SBVH) on the host: library-allocated nodes
 * (info->nodes_used x 32 B) and primitive-index array (info->num_refs; primitives may
 * repeat); free both with rt_free */
int rt_sbvh_build_host(const rt_prim *prims, const float *transforms, uint32_t n, void **nodes, uint32_t **indices,
                       rt_scene_info *info);
/* Surface::LoadImage (template/template.cpp:1579-1601) for PNG files (8/16-bit grey,
 * grey+alpha, RGB, RGBA, palette; not interlaced): pixels = 0x00RRGGBB; free with rt_free. */
int rt_image_load(const char *path, uint32_t **pixels, uint32_t *width, uint32_t *height);

/* ---- scene (Scene, template/scene.h:37-1014) ------------------------------ */
int rt_scene_create(const rt_scene_desc *desc, rt_scene **out);
/* the SURVEY.md 8(d) scenes: "teapotF", "teapot", "mig16", "cfg3", "cfg5"; and "default", the
 * reference's as-shipped Scene() (template/scene.h:40-128: light, glider, mig29 -- the other
 * models it names are not in its assets/).  mesh_dir holds <name>.rtmesh or the reference's
 * <name>.obj files. */
int rt_scene_create_recipe(const char *name, const char *mesh_dir, int32_t device, rt_scene **out);
/* the same with the BVH kind chosen (RT_BVH_PLAIN / RT_BVH_SBVH) */
int rt_scene_create_recipe_ex(const char *name, const char *mesh_dir, int32_t device, int32_t bvh_kind, rt_scene **out);
int rt_scene_destroy(rt_scene *s);
int rt_scene_get_info(const rt_scene *s, rt_scene_info *info);
/* How the primary+shadow frame kernel walks the BVH for camera rays (results identical):
 * RT_WALK_LANE -- one traversal per lane, the reference's order;
 * RT_WALK_WAVE -- the wave's 64 rays (an 8x8 tile) walk the union of their subtrees with
 *   a wave-uniform node and stack; lanes whose closest hit could depend on the visiting
 *   order (an exact distance tie, or a hit nearer than its leaf box's entry) are re-traced
 *   in the reference order.  Faster where rays share most of their walk (mig29 x16: 1.9x);
 *   slower where they split early (CFG3-sub);
 * RT_WALK_AUTO (default; LANE for scenes with cubes) -- each renderer times one frame of
 *   each after a warm-up frame and keeps the faster.
 * Only scenes whose nodes are not held in LDS use it.  RT_WAVE_PRIMARY=0/1 in the
 * environment forces LANE / WAVE at scene creation. */
enum { RT_WALK_LANE = 0, RT_WALK_WAVE = 1, RT_WALK_AUTO = 2 };
int rt_scene_set_camera_walk(rt_scene *s, int walk);
/* host copy of the BVH in use (nodes_used x 32 B, num_refs x u32), in the reference's node order */
int rt_scene_copy_bvh(const rt_scene *s, void *nodes, uint32_t *indices);

/* Batched Scene::IntersectBVH (template/scene.h:285-320): rays_dev[n] -> hits_dev[n]. */
int rt_intersect(rt_scene *s, const rt_ray *rays_dev, rt_hit *hits_dev, uint32_t n, void *stream);
/* Batched Scene::IsOccluded (template/scene.h:452-487): out_dev[i] = 1 if occluded. */
int rt_occluded(rt_scene *s, const rt_ray *rays_dev, uint8_t *out_dev, uint32_t n, void *stream);
/* Batched Scene::IntersectBVHPacket (template/scene.h:322-412, RayPacket Ray.h:34-64):
 * rays [64k, 64k + 64) form packet k (PACKET_SIZE 64) and share one first-active
 * traversal; the last packet may be partial (its missing slots take no part). */
int rt_intersect_packets(rt_scene *s, const rt_ray *rays_dev, rt_hit *hits_dev, uint32_t n, void *stream);
/* Host-pointer conveniences of the three above (copy in, launch, copy out, sync). */
int rt_intersect_host(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n);
int rt_occluded_host(rt_scene *s, const rt_ray *rays, uint8_t *out, uint32_t n);
int rt_intersect_packets_host(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n);

/* Batched Renderer::Trace(Ray&, bool lastSpecular, int depth) (renderer.h:9, renderer.cpp:17-72)
 * or, with mode RT_MODE_WHITTED, Renderer::WhittedTrace(Ray&, int depth) (renderer.h:13,
 * renderer.cpp:138-195); depth <= 32, 0 returns black as the reference does.
 *   rays_dev[n]        the rays (O, D, t);
 *   seeds_dev[n]       ray i's RNG state (the seed RandomFloat() advances,
 *                      template/template.cpp:673-704), updated in place to the state after
 *                      the call, so calls chain like the reference's global seed;
 *   flags_dev[n]       bit 0 = lastSpecular, bit 1 = Ray::inside; NULL = lastSpecular true,
 *                      outside (the reference's defaults);
 *   radiance_dev[3n]   the returned float3 per ray;
 *   hits_dev[n]        optional (NULL): the ray as the first Scene::IntersectBVH leaves it
 *                      (Trace takes Ray&, renderer.cpp:20);
 *   ray_counts_dev[2]  optional (NULL): shadow rays and bounce rays traced, added to. */
int rt_trace(rt_scene *s, int mode, const rt_ray *rays_dev, uint32_t *seeds_dev, const uint8_t *flags_dev,
             uint32_t depth, float *radiance_dev, rt_hit *hits_dev, uint64_t *ray_counts_dev, uint32_t n, void *stream);
/* Host-pointer convenience of rt_trace (all arrays in host memory; synchronous). */
int rt_trace_host(rt_scene *s, int mode, const rt_ray *rays, uint32_t *seeds, const uint8_t *flags, uint32_t depth,
                  float *radiance, rt_hit *hits, uint64_t *ray_counts, uint32_t n);

/* ---- renderer (Renderer, renderer.h:5-160) -------------------------------- */
/* Camera::Camera (camera.h:28-41) for a W x H target */
int rt_camera_default(uint32_t width, uint32_t height, rt_camera *out);
int rt_renderer_create(rt_scene *s, uint32_t width, uint32_t height, rt_renderer **out);
int rt_renderer_destroy(rt_renderer *r);
/* Renderer::Tick (renderer.cpp:200-309): trace every pixel, running average into
 * the float4 accumulator (235-241), RGBF32_to_RGB8 pack (template/precomp.h:432-448)
 * into rgb8_dev[W*H] (0x00RRGGBB).  One kernel launch. */
int rt_render_frame(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t *rgb8_dev, void *stream);
/* Same as rt_render_frame, RGB8 delivered to host memory (the reference's
 * screen->pixels, template/template.cpp:273-277); synchronous. */
int rt_render_frame_host(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t *rgb8_host);
/* Screen-tile shard of a frame: the 8x8 tiles t with t % num_shards == shard,
 * packed as [tile][64] pixels into tiles_dev (rt_shard_capacity pixels). */
int rt_shard_capacity(uint32_t width, uint32_t height, uint32_t num_shards, uint32_t *pixels);
int rt_render_shard(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard,
                    uint32_t num_shards, uint32_t *tiles_dev, void *stream);
/* Rank-0 side of the per-frame gather: gathered_dev = num_shards consecutive shard
 * buffers (each rt_shard_capacity pixels) -> rgb8_dev[W*H]. */
int rt_assemble_shards(rt_renderer *r, const uint32_t *gathered_dev, uint32_t num_shards, uint32_t *rgb8_dev,
                       void *stream);
/* Explicit tile deals (cost-balanced multi-GPU frames).  A deal lists every 8x8 tile of the
 * frame (row-major tile index t = ty * ceil(W/8) + tx) once: shard k owns
 * deal_tiles[deal_off[k] .. deal_off[k+1]).
 * rt_tile_deal: the Morton-ordered tiles cut into num_shards runs of equal summed cost
 *   (cost[t] per tile, e.g. rt_renderer_tile_costs of a full frame; NULL = equal costs):
 *   deal_tiles[ceil(W/8) * ceil(H/8)], deal_off[num_shards + 1].
 * rt_render_shard_tiles: the listed tiles (in that order) of one frame, packed as [i][64]
 *   into tiles_dev -- Renderer::Tick's pixel loop over those tiles only.
 * rt_assemble_tiles: rank 0's unshuffle; shard k's packed tiles at gathered_dev + k * stride_px. */
int rt_tile_deal(uint32_t width, uint32_t height, const uint32_t *cost, uint32_t num_shards, uint32_t *deal_tiles,
                 uint32_t *deal_off);
int rt_render_shard_tiles(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, const uint32_t *tiles,
                          uint32_t num_tiles, uint32_t *tiles_dev, void *stream);
int rt_assemble_tiles(rt_renderer *r, const uint32_t *gathered_dev, uint32_t stride_px, const uint32_t *deal_tiles,
                      const uint32_t *deal_off, uint32_t num_shards, uint32_t *rgb8_dev, void *stream);
/* ---- multi-GPU frames (one process per GPU) ---------------
 * Replaces the OpenMP pixel loop of Renderer::Tick (renderer.cpp:213-245) across the GPUs of
 * a node: rank k renders the 8x8 tiles t with t % world == k, then ONE RCCL gather per frame
 * (ncclSend / ncclRecv to rank 0 in one group) and rank 0's assembly.  Every rank keeps its
 * own scene replica and accumulator.  RCCL (librccl.so.1) is loaded at first use. */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
/* rank 0 makes the id (ncclGetUniqueId) and hands it to the other ranks out of band */
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
/* collective: every rank calls it with the same id (ncclCommInitRank); device = this rank's GPU */
int rt_comm_create(const uint8_t id[RT_COMM_ID_BYTES], int rank, int world, int device, rt_comm **out);
/* use a caller-owned ncclComm_t (from the same librccl.so.1; not destroyed by rt_comm_destroy) */
int rt_comm_wrap(void *nccl_comm, int device, rt_comm **out);
int rt_comm_info(const rt_comm *c, int *rank, int *world);
int rt_comm_destroy(rt_comm *c);
/* One frame on every rank (same camera and params everywhere).  flags 0: in stream order,
 * render this rank's tiles, gather, and on rank 0 assemble the frame into rgb8_dev (W*H;
 * ignored, may be NULL, on other ranks).  RT_MULTI_PIPELINED: the frame's gather runs on
 * the communicator's own stream beside the caller's next work, and the call completes the
 * PREVIOUS pipelined frame into rgb8_dev (nothing on the first call); rt_multi_flush
 * completes the last one.  Counters and the accumulator stay per rank. */
#define RT_MULTI_PIPELINED 1u
/* RT_MULTI_TIMING: HIP events around this rank's render and its gather, summed by rt_comm_timing */
#define RT_MULTI_TIMING 2u
/* RT_MULTI_BALANCED: the ranks render the cost-balanced compact deal of rt_tile_deal instead of
 * t % world.  Costs: the dry-run work map of each rank's tiles (rt_renderer_tile_work's node
 * visits + primitive tests, deterministic) for RT_MODE_PATH frames; the measured wave cycles
 * (rt_renderer_tile_costs) for the other modes, once every rank has them.  A parameter set
 * (camera, size, spp, depth, mode) tries on its 6th frame (then its 12th, 24th, ... while some
 * rank has no costs) -- one all-gather of [status, costs] blocks, after which every rank builds
 * the same deal -- and not again until a parameter changes; the deal in use is kept across
 * camera moves.  When tiles
 * change owner their accumulator values move to the new owner (point-to-point, in stream
 * order), except on frames with reset set, so accumulation goes on exactly.  Frames are
 * identical under any deal; every rank must pass the same flags. */
#define RT_MULTI_BALANCED 4u
int rt_render_frame_multi(rt_renderer *r, rt_comm *c, const rt_camera *cam, const rt_frame_params *p,
                          uint32_t *rgb8_dev, uint32_t flags, void *stream);
int rt_multi_flush(rt_renderer *r, rt_comm *c, uint32_t *rgb8_dev, void *stream);
/* Sum over the RT_MULTI_TIMING frames since the last call (waits for them): render_ms =
 * this rank's shard render, gather_ms = from the render's end to the gather's completion,
 * max(0, ...) per frame (exposed exchange latency; beside the next render in pipelined mode).
 * Pipelined rank 0 receives on the communicator's stream without waiting for its own render,
 * so its figure is how much later than its own tiles the peers' tiles arrived (0 when they
 * were there first); resets the sums. */
int rt_comm_timing(rt_comm *c, double *render_ms, double *gather_ms, uint64_t *frames);
/* The deal frames are rendered under now (every argument but c may be NULL): *balanced = 1 for a
 * cost-balanced deal, 0 for the interleaved one; *ntiles = this rank's tile count and tile_list
 * (room for *ntiles) its global tile indices in render order; stats: [0] balanced deals built,
 * [1] cost exchanges run, [2] accumulator moves run, [3] moves skipped on reset frames. */
int rt_comm_deal_info(const rt_comm *c, int *balanced, uint32_t *ntiles, uint32_t *tile_list, uint64_t stats[4]);
/* FNV-1a hash of the deal in use (every rank's tile lists and offsets): equal on every rank, and
 * in two runs that built the same deal -- every run of the same frames for RT_MODE_PATH deals,
 * whose costs are the deterministic work map.  (Cycle costs of the other modes are rounded to
 * 1/64 of the frame's mean tile cost first, so run-to-run noise rarely moves a cut.) */
int rt_comm_deal_hash(const rt_comm *c, uint64_t *hash);

int rt_renderer_counters(rt_renderer *r, rt_counters *out);
/* Overlapped primary+shadow frames (RT_PS_PIPELINE; no reference counterpart -- Renderer::Tick,
 * renderer.cpp:200-309, is one serial pass): *state = 1 this renderer's primary+shadow frames
 * run overlapped (frame kernel on a renderer stream, accumulate + RGB8 in a finishing pass on
 * the caller's stream), 0 serial, -1 not decided yet (RT_PS_PIPELINE=-1 times both modes on
 * the first eligible frames); ms (may be NULL) = the serial and 2-in-flight groups' milliseconds
 * (serial, overlapped, overlapped, serial) when decided by timing, else zeros. */
int rt_renderer_overlap(const rt_renderer *r, int *state, float ms[4]);
/* The same decision with its depth: *depth = primary+shadow frames in flight (1 serial, 2..6
 * overlapped on that many renderer streams; -1 not decided yet).  RT_PS_PIPELINE=-1 times groups
 * of eight frames in palindromic order -- serial, 2, 4, 6, 6, 4, 2, serial in flight for frames
 * of at most ~3 rounds of resident waves, serial, 2, 2, serial otherwise -- and keeps the
 * fastest; RT_PS_PIPELINE=1 forces RT_PS_DEPTH (default 2).  ms (may be NULL) = the groups' ms
 * (8 entries; unused ones 0). */
int rt_renderer_overlap_depth(const rt_renderer *r, int *depth, float ms[8]);
/* Device memory the renderer holds right now (diagnostics; INTEGRATION.md "Device memory per
 * renderer"): *bytes = accumulator, counters, RGB8, path-state slots, result and sample buffers,
 * tile orders and deal maps; *ps_buffers (may be NULL) = overlapped-frame result buffers allocated
 * (up to 7 while the frames-in-flight choice is timed, depth + 1 or 0 after it). */
int rt_renderer_device_bytes(const rt_renderer *r, uint64_t *bytes, uint32_t *ps_buffers);
/* The renderer's other timed choices for its current parameter set (diagnostics): *walk = the
 * camera-ray walk of primary+shadow frames (0 lane, 1 wave, -1 not decided); *split = the
 * half-tile split order of its costliest tiles (1 on, 0 off, -1 not decided / not applicable);
 * walk_ms / split_ms (may be NULL) = the four timed groups (A, B, B, A) in ms. */
int rt_renderer_choices(const rt_renderer *r, int *walk, int *split, float walk_ms[4], float split_ms[4]);
/* The measured cost map behind the longest-tile-first order of the renderer's current parameter
 * set (camera, size, spp, depth, mode, shard): costs[i] = wave cycles (s_memtime ticks) of
 * local tile i, recorded on one frame; *n_out = its tile count (0 until recorded: from the 2nd
 * frame of a parameter set on).  At most n entries are copied.  Diagnostics and cost-balanced
 * tile deals. */
int rt_renderer_tile_costs(const rt_renderer *r, uint32_t *costs, uint32_t n, uint32_t *n_out);
/* Deterministic work map of one whole frame (camera + params as rt_render_frame, RT_MODE_PATH
 * only): a dry run that traces the frame's rays -- same seeds, camera rays in the reference's
 * IntersectBVH order -- and writes nothing but counts; the accumulator, the frame count and the
 * ray counters are untouched.  work[t] (n >= ceil(W/8) * ceil(H/8), row-major tiles) = BVH node
 * visits + primitive tests of tile t's rays, summed over its pixels and samples.  pixel_work_dev
 * (device, may be NULL): 8 u32 per pixel -- [0] closest-hit node visits, [1] closest-hit primitive
 * tests, [2] any-hit (shadow) node visits, [3] any-hit primitive tests, [4] / [5] closest-hit
 * pops of an interior / leaf stack entry whose pushed entry distance is >= the ray's t at the pop
 * ([4]: pair loads an exact pop-time cull would skip; 0 for trees deeper than 28), [6] [7] 0.
 * Blocks on `stream`.  The multi-GPU deals (RT_MULTI_BALANCED) are cut on this map, so two runs
 * of a frame get the same deal. */
int rt_renderer_tile_work(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t *work, uint32_t n,
                          uint32_t *pixel_work_dev, void *stream);
/* Checks of the wave-coherent camera walk (RT_WALK_WAVE, or RT_WALK_AUTO once timed faster) of a
 * renderer's primary+shadow frames.  The walk always re-traces in the reference order every lane
 * whose result could depend on the visiting order (an exact-distance tie, or a hit nearer than
 * its leaf box's entry -- which covers every hit found in a box entered through the walk's 2^-18
 * cull margin).  Beyond that:
 *   RT_WALK_CHECK_OFF    (default) the production frame kernel, nothing counted;
 *   RT_WALK_CHECK_COUNT  a build of the frame kernel that counts camera rays walked, lanes
 *                        re-traced and boxes a lane entered only through the cull margin;
 *   RT_WALK_CHECK_VERIFY that build also re-traces EVERY walked lane in the reference order
 *                        (IntersectBVH, template/scene.h:285-320), keeps that result and counts the
 *                        lanes whose walk result (id, t, u, v bits) differed -- a diagnostic.
 * Frames are identical at every level. */
enum { RT_WALK_CHECK_OFF = 0, RT_WALK_CHECK_COUNT = 1, RT_WALK_CHECK_VERIFY = 2 };
int rt_renderer_set_walk_check(rt_renderer *r, int level);
/* Cumulative camera-walk counters of the frames rendered at RT_WALK_CHECK_COUNT / _VERIFY
 * (synchronises the device): out[0] camera rays the wave walk traced, out[1] boxes entered only
 * through its cull margin, out[2] lanes re-traced in the reference order, out[3]
 * RT_WALK_CHECK_VERIFY lanes whose walk result differed from the reference order's (0 expected). */
int rt_renderer_walk_stats(rt_renderer *r, uint64_t out[4]);
/* accumulator readback, W*H float4 */
int rt_renderer_read_accumulator(rt_renderer *r, float *host_out);
/* Name of the frame kernel rt_render_frame / rt_render_shard launch for these params
 * (as it appears in rocprofv3 kernel traces, template arguments abbreviated); for
 * profiling and the bench's roofline line.  NULL on a bad argument. */
const char *rt_frame_kernel_name(const rt_renderer *r, const rt_frame_params *p);
int rt_renderer_stream(rt_renderer *r, void **stream);
int rt_synchronize(rt_renderer *r);

#ifdef __cplusplus
}
#endif
#endif
