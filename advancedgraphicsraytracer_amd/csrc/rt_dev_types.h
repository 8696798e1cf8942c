// rt_dev_types.h -- the device scene / frame records shared by the host code
// (rt_device.hip) and the two kernel builds (rt_kern_core.hip, rt_kern_ext.hip), and the
// launchers each kernel build exports.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rt_amd.h"

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
    int wave_primary;                   // camera rays take the wave-coherent walk
    int walk_check;                     // RT_WALK_CHECK_*: what the walk counts / verifies
    float walk_margin;                  // the wave walk enters a box whose entry is below t * (1 + walk_margin)
    const float4 *__restrict__ quads;   // two-level node records (8 float4 each, build_quads) or null
    uint32_t quad_root;                 // the root's record word
    int quad_lanes;                     // the lane kernel walks the two-level records
    unsigned long long *walk_stats;     // the renderer's counter slots (kCounterSlots x 8 u64), set per
                                        // launch: the wave walk adds [2] boxes entered within its
                                        // cull margin, [3] lanes re-traced in the reference order,
                                        // [4] camera rays it walked, [5] RT_WALK_VERIFY mismatches
};

// Ray counters are spread over kCounterSlots 64-byte slots (wave w adds into slot
// w % kCounterSlots, the host sums them): device-scope atomics on ONE address serialise
// across the 8 XCDs -- one counter address cost 26 % of the primary+shadow frame.
constexpr uint32_t kCounterSlots = 1024;

// Launches size their dynamic LDS to at most 64 KB per workgroup (gfx950 allows 160 KB, but every
// launch here is sized for several workgroups per CU); the dry-run work map keeps 8 per-lane
// counters past the stacks.
constexpr size_t kLdsLaunchMax = 65536;
constexpr size_t kWorkCounterBytes = 8u * 256u * sizeof(uint32_t);

struct FrameArgs {
    float cam_pos[3], cam_tl[3], cam_tr[3], cam_bl[3];
    float lens, rw, rh;
    uint32_t W, H, spp, depth, frame, reset;
    uint32_t shard, nshards, tiles_x, ntiles_local;
    const uint32_t *tile_map;           // explicit deal: local tile -> global tile (nullptr: the
                                        // interleaved deal, local * nshards + shard)
    uint32_t nchunks, nunits;           // sample chunks per tile (1 = no split); ntiles_local * nchunks
    float4 *samples;                    // non-null: per-sample values [spp][ntiles_local][64] (sample
                                        // split, overlapped frames); k_pt_finish accumulates them
    int packed_out;
    const uint32_t *order;              // tile dispatch order: local tile of slot i (nullptr = identity); an
                                        // entry with bit 31 renders part (bits 28-30) of its tile only
    uint32_t part_shift;                // lanes per part of a split tile = 1 << part_shift (5: halves)
    uint32_t *tile_cost;                // if set: each tile's wave cycles (to build the order)
    float4 *acc;
    uint32_t *out;
    const uint32_t *fwd_src;            // if set (row-major frames only): each pixel's previous value is
    uint32_t *fwd_dst;                  // forwarded fwd_src[px] -> fwd_dst[px] as the pixel is stored --
                                        // the world-1 pipelined multi-GPU frame hands its previous frame
                                        // to the caller without a copy launch (rt_multi.cpp)
    unsigned long long *counters;       // kCounterSlots slots of 8 u64 (64 B): [0] shadow rays, [1] bounce rays
                                        // ([2..5] the camera walk's counters, SceneView::walk_stats)
};

// One launch of the frame kernel family (Renderer::Tick): integrator mode, Trace depth
// bucket, textured sky.
struct FrameLaunch {
    int mode;        // RT_MODE_*
    int md;          // depth bucket: 1, 4, 10 or 32
    bool tex;        // non-constant sky texture
    dim3 grid, block;
    size_t lds_bytes;
    hipStream_t stream;
    int waves;       // primary+shadow frames: 8 = the single-sample build (k_render_w8), else the plain one
};

// Wavefront path tracing (RT_MODE_PATH, Trace depth >= 2): the frame's paths advance one
// bounce per launch; between launches the paths still alive are compacted into a queue, so
// every wave of a deep level works on 64 live paths instead of a handful.  Per path (index
// p = (sample_in_batch * ntiles_local + local_tile) * 64 + lane):
//   state  : 2 float4 -- (O.xyz, seed bits), (D.xyz, meta bits: d | levels << 8 |
//            lastSpec << 16 | inside << 17)
//   rec    : [level][p] 2 float4 -- the fold record of a bounce (BRDF or albedo, dot;
//            Ld, diffuse flag), folded innermost-first when the path ends
//   result : float4, the path's Trace value
// queue_in / queue_out: path indices alive at this level / the next; qcount[level] their
// counts (level 0 = every path of the batch, no queue).  sum: the per-pixel running sum
// over the samples of earlier batches (sample order kept).
// The level queues are kQueueSegs segments of seg_cap entries, each with its own count
// (64 B apart): a wave appends its survivors to segment (chunk index % kQueueSegs), so
// the per-wave atomics spread over kQueueSegs addresses instead of serialising on one.
// qcount[(level * kQueueSegs + k) * 16] = entries of segment k at that level.
constexpr uint32_t kQueueSegs = 16;

struct PathArgs {
    uint32_t s0, batch_spp, npaths, level;
    uint32_t seg_cap;                    // entries per queue segment
    int dynamic;                         // levels >= 1 take their chunks from the qhead counters
    uint32_t *qhead;                     // [level][kQueueSegs] head counters, 64 B apart (k_pt_level uses 8)
    uint32_t drain_level, drain_below;   // drain (run every remaining level) from this level on /
                                         // at any level holding at most this many paths
    float4 *state;
    float4 *rec;
    float4 *result;
    uint32_t *queue_in, *queue_out;
    uint32_t *qcount;
    float4 *sum;
    uint32_t *tile_cost;                 // level 0: if set, each local tile's wave cycles (summed over its
                                         // samples) are added here -- a multi-GPU deal's cost map
};

// Batched Renderer::Trace / WhittedTrace on caller rays (rt_trace): one lane per ray.
struct TraceArgs {
    const rt_ray *rays;
    uint32_t *seeds;                     // per-ray RNG state, in / out
    const uint8_t *flags;                // bit 0 lastSpecular, bit 1 inside (nullptr: 1)
    float *radiance;                     // 3 floats per ray
    rt_hit *hits;                        // optional: the ray after the first IntersectBVH
    unsigned long long *counts;          // optional: [0] shadow rays, [1] bounce rays (added)
    uint32_t n, depth;
};

// Each kernel build provides the same launchers: `kcore` is compiled without the
// extension primitives and materials (cubes, quads, quad light, TextureMaterial,
// non-Light light materials), `kext` with them.  The host picks per scene.
#define RT_DECLARE_LAUNCHERS(NS)                                                                  \
    namespace NS {                                                                                \
    void launch_frame(const SceneView &S, const FrameArgs &F, const FrameLaunch &L);              \
    void launch_work(const SceneView &S, const FrameArgs &F, const FrameLaunch &L,               \
                     uint32_t *tile_work, uint32_t *pixel_work);                                  \
    void launch_intersect(const SceneView &S, const rt_ray *rays, rt_hit *hits, uint32_t n,       \
                          size_t lds, hipStream_t st);                                            \
    void launch_occluded(const SceneView &S, const rt_ray *rays, uint8_t *out, uint32_t n,        \
                         size_t lds, hipStream_t st);                                             \
    void launch_intersect_packet(const SceneView &S, const rt_ray *rays, rt_hit *hits,            \
                                 uint32_t n, hipStream_t st);                                     \
    int launch_pt_level(const SceneView &S, const FrameArgs &F, const PathArgs &P, bool tex,      \
                        size_t lds, uint32_t num_cus, hipStream_t st);                            \
    void launch_pt_lanes(const SceneView &S, const FrameArgs &F, const PathArgs &P, bool tex,     \
                         size_t lds, uint32_t num_cus, hipStream_t st);                           \
    void launch_pt_finish(const FrameArgs &F, const PathArgs &P, bool last, hipStream_t st);      \
    void launch_trace(const SceneView &S, const TraceArgs &A, int mode, int md, bool tex,         \
                      size_t lds, hipStream_t st);                                                \
    }
RT_DECLARE_LAUNCHERS(kcore)
RT_DECLARE_LAUNCHERS(kext)
#undef RT_DECLARE_LAUNCHERS
// where: per global tile (shard << 24 | local tile) of an explicit deal; nullptr = interleaved.
// first = 1: `gathered` holds shards 1.. only (rank 0's own tiles are already in `out`)
void launch_assemble(const uint32_t *gathered, uint32_t cap, uint32_t nshards, const uint32_t *where, uint32_t tiles_x,
                     uint32_t ntiles, uint32_t W, uint32_t H, uint32_t *out, hipStream_t st, uint32_t first = 0);

}  // namespace rt
