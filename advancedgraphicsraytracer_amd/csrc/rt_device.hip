// rt_device.hip -- the device half of the C-ABI: scene upload, renderer state, launches.
// The kernels live in rt_kernels.inc (built twice: rt_kern_core.hip / rt_kern_ext.hip).
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

#include "rt_dev_types.h"
#include "rt_internal.h"



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

// RT_PT_QUADS=1: the lane kernel walks two-level node records (build_quads).  Exact (the GPU suite
// passes with it on; test_wavefront_equals_one_kernel_path_tracer runs it), but measured slower,
// so off by default (tools/ab.py serial frames, profiles/r05/quadab): CFG3-sub 2.133 -> 2.385 ms,
// CFG5-sub 8.49 -> 9.41, TEAPOT-F depth 10 1.150 -> 1.253, mig29 x16 spp 4 depth 4 3.78 -> 4.40 --
// a record step costs four slab tests, two box unions and a 128-B load for every lane of the
// wave whichever branch (leaf, odd half, record) each lane is in, and the lanes' chains shrink less
// than the step grows.
#ifndef RT_PT_QUADS_DEFAULT
#define RT_PT_QUADS_DEFAULT 0
#endif
struct rt_scene {
    int device = 0;
    SceneView view{};
    Bvh bvh;
    uint32_t num_prims = 0;
    uint32_t stack_depth = 0;   // LDS stack entries per lane
    int frame_waves = 0;        // primary+shadow frame kernel build (frame_build): 0 = chosen, 7 = the
                                // plain build, 8 = the single-sample one wherever it applies (RT_FRAME_WAVES)
    uint32_t num_cus = 256;     // CUs of the device (resident grids, frames-in-flight rules)
    bool has_cubes = false;     // cube acceptance depends on the visiting order: no wave walk
    bool quads = false;         // two-level node records built (RT_PT_QUADS=1, build_quads)
    bool quad_lanes = false;    // ... and the lane kernel walks them
    void *d_quads = nullptr;
    bool walk_fits = true;      // the lane stacks + the wave walk's word stack fit one launch's LDS (kLdsLaunchMax)
    bool nested = true;         // every child box lies inside its parent's (as floats): the wave walk's
                                // exactness needs it (the builders' trees always; a caller's prebuilt one
                                // is checked at rt_scene_create)
    int walk = RT_WALK_LANE;    // camera-ray walk of the global-node primary+shadow kernel
    bool ext = false;           // needs the kext kernels (cubes, quads, textures, non-Light light)
    bool pt_lanes = true;           // levels >= 1 run the lane state machine (RT_PT_LANES=0: k_pt_level)
    bool pt_dynamic = true;         // wavefront levels >= 1 fetch chunks dynamically (RT_PT_DYNAMIC=0: static)
    bool pt_wavefront = true;   // depth >= 2 path tracing: wavefront (k_pt_level) vs one kernel (k_render)
    uint32_t pt_drain_level = 64;   // bounce level from which the wavefront always drains (64 = never forced)
    double pt_drain_rounds = 0.25;  // ... and it drains any level holding <= this many rounds of resident lanes
    // small batches (<= pt_small_rounds rounds of resident lanes, e.g. a 1/8 shard's): always drain
    // from level pt_drain_small (0 = off).  Config 5's 1/8 shard (4.1 M paths per batch, ~10 rounds):
    // 1.126 / 1.129 -> 1.055 / 1.059 ms forced from level 4 (1.095 / 1.068 from 3); whole frames
    // (33 M paths, ~84 rounds) lose with it (CFG5-sub 6.70 -> 6.85 ms), so they keep the threshold
    // alone (profiles/r05/c5drain)
    uint32_t pt_drain_small = 4;
    double pt_small_rounds = 16.0;
    // ... and drains any of its levels holding <= this many rounds (the whole frames' 0.25 above):
    // the 1/8 shard 1.084 / 1.077 -> 1.054 / 1.065 ms mean of three interleaved runs (0.0625: 1.058;
    // 0.5: 1.092; profiles/r05/c5drain/c5knobs*.jsonl)
    double pt_small_drain_rounds = 0.125;
    bool tile_order = true;         // measured-cost (longest first) tile order (RT_TILE_ORDER=0: off)
    uint32_t split_units = 40000;   // sample split below this many tiles (1080p = 32,400 tiles)
    bool xcd_order = false;         // measured order grouped by XCD: blocks b, b + 8, ... (one XCD) render
                                    // one compact screen region of 1/8 of the frame's cost (L2 locality)
    uint32_t split_parts = 2;       // ... each as this many waves of 64 / parts lanes (RT_SPLIT_PARTS: 2, 4, 8)
    int32_t heavy_split = -1;       // primary+shadow frames: the costliest tiles run as two half-tile
                                    // waves (RT_SPLIT_HEAVY = count; -1: ntiles / 32)
    uint64_t pt_mem_bytes = 12288ull << 20;   // path-state budget per slot (two when pipelined): 12 GB
                                              // of the 288 GB HBM holds all 16 spp of a 1080p depth-10 frame
    bool pt_pipeline = true;        // sample batches alternate path-state slots and streams
    uint32_t pt_slots = 0;          // path-state slots / streams of pipelined frames (RT_PT_SLOTS, 2-8;
                                    // 0 = 8 for batches of <= 8.4 M paths, else 4)
                                    // (RT_PT_PIPELINE=0: one slot, the caller's stream)
    uint32_t ps_buffers = 0;        // per-sample result buffers of overlapped frames (RT_PS_BUFFERS,
                                    // 2-7; 0 = frames in flight + 1)
    int32_t ps_pipeline = -1;       // primary+shadow frames overlap: -1 timed per renderer (auto),
                                    // 0 never, 1 always (RT_PS_PIPELINE)
    uint32_t ps_depth = 2;          // frames in flight when forced (RT_PS_DEPTH, 2-8)
    float tune_delay_ms = 100.0f;   // GPU time a parameter set runs before its timed choices start
                                    // (RT_TUNE_DELAY_MS): the clocks ramp over ~0.1 s, and choices
                                    // timed on the first frames at low clocks came out wrong
    void *d_nodes = nullptr, *d_prims = nullptr, *d_shade = nullptr, *d_mats = nullptr, *d_sky = nullptr;
    void *d_xprims = nullptr, *d_tex = nullptr;
    void *d_scratch = nullptr;  // staging for the host-pointer batched calls
    size_t scratch_bytes = 0;
    hipStream_t stream = nullptr;
};

// renderer streams: up to 8 -- frames in flight of overlapped primary+shadow frames (timed
// choice among 2 / 4 / 6, forced up to 8) and the path-state slots of pipelined path-traced
// frames (8 for small batches when the process has >= 8 hardware queues, else 4).  With the
// caller's stream and a communicator's a process may then drive 10 streams; HIP maps them onto
// GPU_MAX_HW_QUEUES hardware queues (default 4, bench.py sets 8 for the workloads that overlap).
constexpr int kPsMaxDepth = 8;   // renderer streams (frames in flight when forced: RT_PS_DEPTH)
constexpr int kPtMaxSlots = 8;    // path-state slots of pipelined path-traced frames (RT_PT_SLOTS; <= kPsMaxDepth streams)
// the process's hardware queues per device as HIP will use them (GPU_MAX_HW_QUEUES, default 4)
inline int hw_queues() {
    const char *e = std::getenv("GPU_MAX_HW_QUEUES");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 4;
}

struct rt_renderer {
    rt_scene *scene = nullptr;
    uint32_t W = 0, H = 0;
    float4 *d_acc = nullptr;
    unsigned long long *d_counters = nullptr;
    uint32_t *d_rgb = nullptr;   // staging frame for rt_render_frame_host
    uint64_t primary = 0, frames = 0;
    hipStream_t stream = nullptr;
    // RT_WALK_AUTO: the first eligible frames time the lane walk and the wave walk on the
    // caller's stream (one warm-up, one each), the fourth picks the faster for good
    // measured-cost tile order (tile_order_step): per-tile cycles of one frame (two cost
    // maps while the camera walk is being timed), longest tile first afterwards
    uint32_t *d_order = nullptr, *d_cost = nullptr;
    std::vector<uint32_t> host_cost;   // the cost map the active order was sorted from (local tiles)
    bool tail_bound = false;    // that map's costliest tile outlasts 2 x the frame's mean time per
                                // resident wave slot: frames in flight beyond 2 become candidates
    uint32_t order_n = 0;
    uint64_t order_key = 0;
    int order_state = 0;        // 0 idle, 1 costs recorded, 2 order active, 3 costs held without an
                                // order (path-traced frames)
    uint32_t order_split = 0;   // leading tiles of the split order that run as order_parts units each
    uint32_t order_parts = 2;
    int split_phase = -1;       // -1 decided / not tried; 0 .. 4 kTuneGroup - 1 timing frames in groups
                                // (plain, split, split, plain), 4 kTuneGroup decide
    bool use_split = false;     // the split order measured faster
    hipEvent_t sev[8] = {};     // split timing: events 2i, 2i+1 around timing frame i
    float split_ms[4] = {};
    int tune = 0;                   // camera walk: 0 warm-up, 1 .. kWalkTimed timed frames, kTuneDecide, kTuneDone
    hipEvent_t stall_ev = nullptr;  // after the previous frame while a timed group runs (kTuneRestarts)
    bool stall_armed = false;
    int walk_restarts = 0, split_restarts = 0, ps_restarts = 0;   // restarts of group *_rg
    int walk_rg = -1, split_rg = -1, ps_rg = -1;
    bool wave = false;
    uint64_t tune_key = 0;          // the parameter set whose frames the walk timing ran on
    int walk_check = RT_WALK_CHECK_OFF;     // rt_renderer_set_walk_check
    hipEvent_t tev[8] = {};         // walk timing: events 2g, 2g + 1 around group g
    // wavefront path tracer (PathArgs): two path-state slots (state, records, queues), grown on
    // demand, each owned by one of the renderer's two path streams.  Sample batches alternate
    // between them, so one batch's (or the next frame's) level 0 fills the CUs that the other
    // batch's thinning bounce levels leave idle.  The per-sample radiance goes to a frame-level
    // buffer (two, by frame parity); one finishing pass per frame on the caller's stream sums
    // it in sample order after every batch's levels (accumulator, RGB8).  d_pt[0] / the
    // caller's stream alone when pipelining is off or the results do not fit.
    void *d_pt[kPtMaxSlots] = {};
    size_t pt_bytes[kPtMaxSlots] = {};
    // [sample][pixel] radiance of a frame, frame n in buffer n % (slots + 1): frame n + slots + 1's
    // batches wait for frame n's finishing pass only (see launch_pt_frame)
    float4 *d_res[kPtMaxSlots + 1] = {};
    size_t res_bytes[kPtMaxSlots + 1] = {};
    float4 *d_sum = nullptr;        // the running sample sum across batches (serial path)
    // renderer streams: the path tracer's two path streams are 0 and 1; overlapped primary+
    // shadow frames use the first `depth` of them (frames in flight)
    hipStream_t pt_stream[kPsMaxDepth] = {};
    int nstreams = 0;               // pt_stream[0 .. nstreams) created (ensure_pipe_streams)

    hipEvent_t pt_lv[kPsMaxDepth] = {};   // a renderer stream's work of this frame is done
    hipEvent_t pt_fin[kPtMaxSlots + 1] = {};   // the finish that read d_res[b] is done
    bool pt_fin_set[kPtMaxSlots + 1] = {};
    int pt_slot = 0, pt_parity = 0;
    uint32_t pt_nslots = 0;         // slots in use, decided for path state of up to pt_need bytes
    size_t pt_need = 0;
    bool pt_serial_last = false;    // the last path-traced frame ran the serial path
    // overlapped primary+shadow frames (launch_render): with RT_PS_PIPELINE auto, eight groups
    // of kPsGroup eligible frames back to back -- serial, 2 in flight, 4, 6, 6, 4, 2, serial (or
    // four: serial, 2, 2, serial), so that a clock drift cancels -- are timed on the caller's
    // stream (events pev[2g], pev[2g + 1] around group g); the next frame keeps the fastest mode
    // for the parameter set, and the result buffers it does not use are freed
    int ps_phase = 0;               // 0 .. groups x G - 1 timing frames (G = kPsGroup, 2 kPsGroup for 8
                                    // groups), then decide; -1 decided
    int ps_groups = 0;              // timed groups of this decision (4: serial / 2; 8: serial / 2 / 4 / 6)
    uint32_t ps_use = 0;            // decided: frames in flight (0 = serial)
    uint64_t ps_last = 0;           // r->frames at the last timing frame (any other frame restarts)
    uint32_t ps_prev = 0;           // frames in flight of the previous eligible frame (0 serial)
    hipEvent_t pev[16] = {};
    hipEvent_t ps_join = nullptr;   // caller's stream -> overlap stream, on a switch to overlapped
    hipEvent_t cost_ev = nullptr;   // path-traced frames: the cost map was cleared (caller's stream)
    float ps_ms[8] = {};
    // the overlapped frames' per-sample results, frame n in buffer n % buffers (kernel on
    // renderer stream n % depth): frame n + buffers waits for the finishing pass of frame n only,
    // so a kernel never waits for the finish of a frame still running beside it
    float4 *ps_res[kPsMaxDepth + 1] = {};
    size_t ps_res_bytes[kPsMaxDepth + 1] = {};
    hipEvent_t ps_fin[kPsMaxDepth + 1] = {};
    bool ps_fin_set[kPsMaxDepth + 1] = {};
    uint32_t ps_count = 0;
    // tuning gate: the timed choices (camera walk, split order, frames in flight) of a parameter
    // set start once its frames have run tune_delay_ms of GPU time -- an event at its first frame
    // and a probe every 8 frames, read without blocking
    uint64_t gate_key = 0;
    int gate_state = 0;             // 0 start, 1 running, 2 probe recorded, 3 open
    uint32_t gate_frames = 0;
    hipEvent_t gate_ev[2] = {};
    // per-sample values of sample-split frames (FrameArgs::samples)
    void *d_samples = nullptr;
    size_t samples_bytes = 0;
    // explicit tile deal of rt_render_shard_tiles (FrameArgs::tile_map): local -> global tile,
    // uploaded when it changes; and rank 0's per-global-tile (shard << 24 | local) for assembly
    std::vector<uint32_t> map_host;
    // the tiles whose running averages the accumulator holds: those of the last frame (a frame
    // accumulates exactly its own tiles).  0 none yet, 1 every tile, 2 the interleaved shard
    // held_shard of held_nshards, 3 the explicit list held_list (renderer_held_tiles)
    int held_kind = 0;
    uint32_t held_shard = 0, held_nshards = 1;
    std::vector<uint32_t> held_list;
    uint64_t map_gen = 0, held_gen = 0;   // set_tile_map's changes; the one held_list was copied at
    uint32_t *d_work = nullptr;     // dry-run work frame: per local tile (work_frame)
    uint32_t work_cap = 0;
    uint32_t *d_map = nullptr;
    size_t map_cap = 0;
    uint64_t map_hash = 0;
    uint32_t *d_where = nullptr;
    size_t where_cap = 0;
    uint64_t where_hash = 0;
};

namespace {

inline float ubits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline float ibits(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

// The timed choices between two variants (camera walk, split order) time four groups of
// kTuneGroup frames in the order A, B, B, A (a clock drift over the groups cancels) and keep
// the faster -- single frames were too noisy to decide on (ranks with equal work came out 35 %
// apart in round-3 shard timings)
constexpr int kTuneGroup = 4;
// A timed choice between the default (groups 0 and 3) and an alternative (groups 1 and 2),
// groups run A, B, B, A: the alternative must win by kTuneMargin.  The palindrome cancels a
// linear clock drift, not a first group that still runs slow: TEAPOT-F 1080p timed its plain
// order at 0.4986 / 0.4195 ms per group against 0.4531 / 0.4551 for the half-tile split, whose
// sum looked 1 % faster -- and its frames then ran at 0.114 instead of 0.104 ms (bench config 2
// after a config-4 run on the same box, round 3).  The choices that pay win by 8-40 %.
constexpr float kTuneMargin = 0.03f;
inline bool tuned_alternative(const float ms[4]) {
    return ms[1] + ms[2] < (ms[0] + ms[3]) * (1.0f - kTuneMargin);
}
constexpr int kWalkTimed = 4 * kTuneGroup;
constexpr int kTuneDecide = 1 + kWalkTimed, kTuneDone = kTuneDecide + 1;
// A timed group assumes frames submitted back to back.  When the caller synchronises inside a
// group (bench.py's clock ramp every 20 frames, multi_overhead.py every 50), the GPU idles between
// two of its frames and the group times the host, not the frames: TEAPOT-F 1080p with 8 hardware
// queues timed its first serial group at 2.48 ms against 1.58 for the last, picked 2 frames in
// flight and ran at 0.0995 ms against 0.097 serial (round 5, profiles/r05/hwq/).  So while a group
// runs, an event after each frame is queried when the next frame is submitted: if the previous
// frame had already completed, the GPU ran dry in between and the group restarts (at most
// kTuneRestarts times per group, so a caller that syncs every frame still gets a decision).
constexpr int kTuneRestarts = 4;

// LDS stack entries per lane: a traversal pushes at most one entry per tree level, so the tree
// depth is enough.  Rounding it up to 8 cost occupancy where the stacks bound the workgroups
// per CU (mig29 x16: 26 levels, 32 KB per workgroup -> 5 per CU; exact: 26 KB -> 6): CFG3-sub
// 1.79 -> 1.65 ms, CFG5-sub 7.58 -> 7.47 ms, mig29 x16 0.330 -> 0.321 ms, TEAPOT-F unchanged
// (round 3, profiles/r03/ab_stack/).
#ifndef RT_STACK_ROUND
#define RT_STACK_ROUND 1u
#endif
// Two-level node records (the path tracer's lane kernel, k_pt_lanes<.., true>): one 128-B
// record per interior node x at even depth (the root at 0) holding the node entries of x's
// grandchildren -- slots 2h, 2h+1 = the children of x's child h -- or, for a leaf child h, that
// leaf's own entry in slot 2h (flag bit 0 in its .w word).  One load then serves two binary
// levels: the walk tests x's children on boxes rebuilt as the union of their children's (the
// reference's node bounds ARE that union -- each node's box is the min / max over its primitives'
// bounds, Scene::UpdateNodeBounds, template/scene.h:855-865 -- checked bit for bit here), then
// the nearer child's children on their own entries, in the reference's order and against the
// same r.t: the visits are the binary walk's exactly.  A popped odd-depth child is addressed by
// (its parent's record, half) and reads its children pair from that record.  Entry words: leaf
// (leftFirst << 8 | count) as in the binary array, even-depth interior node (record << 8), odd
// marker ((kQuadOdd | record << 1 | half) << 8).  false (no records) when a box is NaN, a parent is
// not the exact union of its children (a caller's prebuilt tree), or the tree is too large.
constexpr uint32_t kQuadOdd = 1u << 23;
bool build_quads(const Bvh &b, const std::vector<uint8_t> &sticky, std::vector<float4> &rec, uint32_t &root_word) {
    const Node *N = b.nodes.data();
    if (b.nodes_used < 3 || N[0].count > 0) return false;
    std::vector<int32_t> id(b.nodes_used, -1);
    std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};
    std::vector<uint32_t> order;
    while (!st.empty()) {   // pre-order, even-depth interior nodes numbered as met
        auto [k, d] = st.back();
        st.pop_back();
        const Node &nd = N[k];
        if (nd.count > 0) continue;
        if (!(d & 1u)) { id[k] = (int32_t)order.size(); order.push_back(k); }
        st.push_back({nd.leftFirst + 1, d + 1});
        st.push_back({nd.leftFirst, d + 1});
    }
    if (order.size() >= (kQuadOdd >> 1)) return false;
    auto bits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
    // the union of two floats as the device's fminf / fmaxf gives it, or fail on NaN / +-0 ties
    auto pick = [&](float a, float c, bool mn, float want) {
        if (a != a || c != c || want != want) return false;
        if (a == c && bits(a) != bits(c)) return false;
        const float u = mn ? (a < c ? a : c) : (a > c ? a : c);
        return bits(u) == bits(want);
    };
    auto entry = [&](uint32_t g, float4 *q) {
        const Node &nd = N[g];
        const uint32_t w = nd.count > 0 ? ((nd.leftFirst << 8) | nd.count) : ((uint32_t)id[g] << 8);
        q[0] = make_float4(nd.mn[0], nd.mn[1], nd.mn[2], nd.mx[0]);
        q[1] = make_float4(nd.mx[1], nd.mx[2], ubits(w), 0.0f);
    };
    // the .w word of each entry: bit 0 (first slot of a half) the child is a leaf and this its entry,
    // bit 1 this entry's node is sticky (mark_sticky), bit 2 (first slot) the child itself is sticky
    rec.assign(8 * order.size(), make_float4(0, 0, 0, 0));
    for (size_t r = 0; r < order.size(); ++r) {
        const Node &x = N[order[r]];
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t c = x.leftFirst + h;
            float4 *q = &rec[8 * r + 4 * h];
            const Node &cn = N[c];
            const uint32_t sc = sticky[c] ? 6u : 0u;
            if (cn.count > 0) {
                entry(c, q);
                q[1].w = ubits(1u | sc);
                continue;
            }
            const Node &g1 = N[cn.leftFirst], &g2 = N[cn.leftFirst + 1];
            for (int a = 0; a < 3; ++a)
                if (!pick(g1.mn[a], g2.mn[a], true, cn.mn[a]) || !pick(g1.mx[a], g2.mx[a], false, cn.mx[a])) return false;
            entry(cn.leftFirst, q);
            entry(cn.leftFirst + 1, q + 2);
            q[1].w = ubits((sticky[cn.leftFirst] ? 2u : 0u) | (sc & 4u));
            q[3].w = ubits(sticky[cn.leftFirst + 1] ? 2u : 0u);
        }
    }
    root_word = (uint32_t)id[0] << 8;
    return true;
}

uint32_t pick_stack(uint32_t depth) {   // entries needed <= tree depth (rounded up to RT_STACK_ROUND)
    uint32_t need = depth < 2 ? 2 : depth;
    return (need + RT_STACK_ROUND - 1u) / RT_STACK_ROUND * RT_STACK_ROUND;
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

constexpr uint32_t kMaxNodes = 1u << 24;   // the packed word's leftFirst field is 24 bits wide

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
    void *ptrs[] = {s->d_nodes, s->d_prims, s->d_shade, s->d_mats, s->d_sky, s->d_xprims, s->d_tex, s->d_scratch, s->d_quads};
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

// The wave camera walk's sticky boxes (rt_kernels.inc, wave_closest_hit_fast): a node with a
// primitive below it whose computed t can lie well before its leaf box's entry -- a sliver
// triangle (its smallest corner angle's sine under 2^RT_WALK_STICKY, default 2^-8: the common
// denominator of t, u, v is then mostly rounding, Primitive.h:255-273), a sphere (t = -b - sqrt(d)
// near a tangent, Primitive.h:150-177) or a quad -- gets b.w = 1, and the walk culls it only on a
// slab miss.  Computed in double on the float vertices.  b.w then holds the walk's cull margin per
// node: `margin` (SceneView::walk_margin), +inf for a sticky node; the lane traversals never read it.
void mark_sticky(const Bvh &b, const rt_scene_desc *d, std::vector<float4> &nodes, std::vector<uint8_t> &sticky,
                 float margin) {
    double lim = std::ldexp(1.0, -8);
    if (const char *e = std::getenv("RT_WALK_STICKY")) lim = std::atoi(e) >= 0 ? 0.0 : std::ldexp(1.0, std::atoi(e));
    bool spheres = true;   // RT_WALK_STICKY_SPHERES=0: A/B only
    if (const char *e = std::getenv("RT_WALK_STICKY_SPHERES")) spheres = std::atoi(e) != 0;
    auto prim_sticky = [&](const rt_prim &p) {
        if (p.type == RT_SPHERE || p.type == RT_QUAD) return spheres;
        if (p.type != RT_TRIANGLE) return false;   // planes: an unbounded box, entered from inside
        double v[3][3], e[3][3], len[3];
        for (int k = 0; k < 3; ++k)
            for (int a = 0; a < 3; ++a) v[k][a] = p.v[3 * k + a];
        for (int k = 0; k < 3; ++k) {
            for (int a = 0; a < 3; ++a) e[k][a] = v[(k + 1) % 3][a] - v[k][a];
            len[k] = std::sqrt(e[k][0] * e[k][0] + e[k][1] * e[k][1] + e[k][2] * e[k][2]);
        }
        const double cx = e[0][1] * e[2][2] - e[0][2] * e[2][1], cy = e[0][2] * e[2][0] - e[0][0] * e[2][2],
                     cz = e[0][0] * e[2][1] - e[0][1] * e[2][0];
        const double area2 = std::sqrt(cx * cx + cy * cy + cz * cz);
        std::sort(len, len + 3);
        return !(area2 >= lim * len[1] * len[2]);   // sine of the smallest angle = 2 area / (two longest edges)
    };
    const uint32_t used = b.nodes_used;
    std::vector<uint32_t> parent(used, ~0u);
    for (uint32_t i = 0; i < used; ++i)
        if (i != 1 && b.nodes[i].count == 0)
            for (uint32_t c = b.nodes[i].leftFirst; c < b.nodes[i].leftFirst + 2; ++c) parent[c] = i;
    for (uint32_t i = 0; i < used; ++i) {
        const Node &nd = b.nodes[i];
        if (i == 1 || nd.count == 0 || nodes[2 * i + 1].w != 0.0f) continue;
        bool st = false;
        for (uint32_t k = nd.leftFirst; k < nd.leftFirst + nd.count && !st; ++k) st = prim_sticky(d->prims[b.indices[k]]);
        for (uint32_t j = i; st && j != ~0u && nodes[2 * j + 1].w == 0.0f; j = parent[j]) nodes[2 * j + 1].w = 1.0f;
    }
    sticky.assign(used, 0);
    for (uint32_t i = 0; i < used; ++i) {
        sticky[i] = nodes[2 * i + 1].w != 0.0f;
        nodes[2 * i + 1].w = sticky[i] ? HUGE_VALF : margin;
    }
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
    bool ext = d->prims[0].type == RT_QUAD;
    {
        const int lk = d->materials[d->prims[0].material].kind;
        ext = ext || !(lk == RT_LIGHT || lk == RT_DIFFUSE || lk == RT_MIRROR || lk == RT_DSMIX);
    }
    for (uint32_t i = 0; i < n && !ext; ++i) ext = d->prims[i].type == RT_CUBE || d->prims[i].type == RT_QUAD;
    for (uint32_t i = 0; i < d->num_materials && !ext; ++i) ext = d->materials[i].kind == RT_TEXTURE;
    if (d->sky_pixels) {
        uint32_t w = d->sky_width, h = d->sky_height;
        if (!w || !h || (w & (w - 1)) || (h & (h - 1)))
            return fail(RT_ERR_INVALID, "sky texture must have power-of-two sides (renderer.h:18)");
    }
    // interior nodes store a node index in the 24-bit leftFirst field of the packed device
    // word (leftFirst << 8 | count): trees with more than 2^24 nodes cannot be addressed
    if (d->bvh_nodes && d->bvh_num_nodes > kMaxNodes)
        return fail(RT_ERR_UNSUPPORTED, "prebuilt BVH with more than 2^24 nodes (24-bit child index)");
    int32_t bvh_kind = d->bvh_kind;
    if (bvh_kind != RT_BVH_PLAIN && bvh_kind != RT_BVH_SBVH) return fail(RT_ERR_INVALID, "unknown bvh_kind");
    // RT_BVH (plain / sbvh) picks the tree only where the caller left the default
    if (const char *e = std::getenv("RT_BVH")) {
        if (std::strcmp(e, "sbvh") != 0 && std::strcmp(e, "plain") != 0)
            return fail(RT_ERR_INVALID, std::string("RT_BVH must be 'plain' or 'sbvh', not '") + e + "'");
        if (bvh_kind == RT_BVH_PLAIN) bvh_kind = std::strcmp(e, "sbvh") == 0 ? RT_BVH_SBVH : RT_BVH_PLAIN;
    }
    int rc = ensure_device(d->device);
    if (rc != RT_OK) return rc;

    rt_scene *s = new rt_scene();
    s->device = d->device;
    s->ext = ext;
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
    } else if ((rc = (bvh_kind == RT_BVH_SBVH ? build_sbvh : build_bvh)(d->prims, d->transforms, n, s->bvh)) != RT_OK) {
        delete s;
        return rc;
    }
    if (s->bvh.nodes_used > kMaxNodes) { delete s; return fail(RT_ERR_UNSUPPORTED, "BVH with more than 2^24 nodes (24-bit child index)"); }
    if (s->bvh.max_leaf > 255) { delete s; return fail(RT_ERR_UNSUPPORTED, "BVH leaf with more than 255 primitives"); }
    if (s->bvh.depth > 64) { delete s; return fail(RT_ERR_UNSUPPORTED, "BVH deeper than 64 (the reference's stack[64])"); }
    s->stack_depth = pick_stack(s->bvh.depth);
    // trees deeper than 60: the lane stacks (depth x 1 KB) leave no room for the walk's words
    s->walk_fits = (size_t)s->stack_depth * (256u + 4u) * sizeof(uint32_t) <= kLdsLaunchMax;

    // ---- device node array: packed (leftFirst << 8 | count) word in b.z
    std::vector<float4> nodes(2 * (size_t)s->bvh.nodes_used);
    for (uint32_t i = 0; i < s->bvh.nodes_used; ++i) {
        const Node &nd = s->bvh.nodes[i];
        uint32_t word = (nd.leftFirst << 8) | nd.count;
        nodes[2 * i] = make_float4(nd.mn[0], nd.mn[1], nd.mn[2], nd.mx[0]);
        nodes[2 * i + 1] = make_float4(nd.mx[1], nd.mx[2], ubits(word), 0.0f);
    }
    std::vector<uint8_t> sticky;
    // the wave walk's cull margin: RT_WALK_MARGIN = its base-2 exponent
    s->view.walk_margin = 0x1p-12f;
    if (const char *e = std::getenv("RT_WALK_MARGIN"))
        s->view.walk_margin = std::ldexp(1.0f, std::max(-40, std::min(-1, std::atoi(e))));
    mark_sticky(s->bvh, d, nodes, sticky, s->view.walk_margin);
    std::vector<float4> quads;
    uint32_t quad_root = 0;
    {
        bool lanes = RT_PT_QUADS_DEFAULT != 0;
        if (const char *e = std::getenv("RT_PT_QUADS")) lanes = std::atoi(e) != 0;
        s->quads = lanes && build_quads(s->bvh, sticky, quads, quad_root);
        s->quad_lanes = s->quads;
    }
    // ---- leaf-order primitive records and per-id shading records; cubes and quads keep
    // their matrices and data in a side table (8 float4 each)
    static const float I16[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const uint32_t nrefs = (uint32_t)s->bvh.indices.size();   // leaf slots (an SBVH repeats primitives)
    std::vector<float4> prims(3 * (size_t)nrefs), shade(2 * (size_t)n), xprims;
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
    for (uint32_t k = 0; k < nrefs; ++k) {
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
    if (rc == RT_OK && s->quads) rc = upload(&s->d_quads, quads);
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
    v.quads = s->quads ? (const float4 *)s->d_quads : nullptr;
    v.quad_root = quad_root;
    v.quad_lanes = 0;
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
    // Primary+shadow frames read the nodes from global memory (L1/L2-resident, 256-thread
    // workgroups).  The LDS-node kernels of rounds 1-3 (48-B pairs + u16 stacks in two 512-thread
    // workgroups per CU, or 64-B pairs in one 1024-thread group) lost by 12 % once the ray
    // counters were spread over slots (TEAPOT-F 0.169 vs 0.192 ms, profiles/r01/ab_kernel_choice_*;
    // LDS occupancy caps them at 4 waves/SIMD) and were removed in round 4.
    // RT_PT_WAVEFRONT=0 selects the one-kernel path tracer (k_render<path, MAXD>) for A/B runs
    if (const char *e = std::getenv("RT_PT_WAVEFRONT")) s->pt_wavefront = std::atoi(e) != 0;
    if (const char *e = std::getenv("RT_PT_DYNAMIC")) s->pt_dynamic = std::atoi(e) != 0;
    if (const char *e = std::getenv("RT_PT_LANES")) s->pt_lanes = std::atoi(e) != 0;
    // RT_PT_DRAIN_LEVEL / RT_PT_MEM_MB: wavefront drain level and path-state budget (A/B runs)
    if (const char *e = std::getenv("RT_PT_DRAIN_LEVEL")) s->pt_drain_level = (uint32_t)std::max(1, std::atoi(e));
    if (const char *e = std::getenv("RT_PT_DRAIN_ROUNDS")) s->pt_drain_rounds = std::max(0.0, std::atof(e));
    if (const char *e = std::getenv("RT_PT_DRAIN_SMALL")) s->pt_drain_small = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = std::getenv("RT_PT_SMALL_ROUNDS")) s->pt_small_rounds = std::max(0.0, std::atof(e));
    if (const char *e = std::getenv("RT_PT_SMALL_DRAIN_ROUNDS")) s->pt_small_drain_rounds = std::max(0.0, std::atof(e));
    if (const char *e = std::getenv("RT_TILE_ORDER")) s->tile_order = std::atoi(e) != 0;
    // RT_SPLIT_UNITS: sample-split target units (0 = never split)
    if (const char *e = std::getenv("RT_SPLIT_UNITS")) s->split_units = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = std::getenv("RT_FRAME_WAVES")) {
        const int w = std::atoi(e);
        s->frame_waves = w == 7 || w == 8 ? w : 0;
    }
    if (const char *e = std::getenv("RT_SPLIT_HEAVY")) s->heavy_split = std::max(-1, std::atoi(e));
    if (const char *e = std::getenv("RT_SPLIT_PARTS")) {
        const int k = std::atoi(e);
        s->split_parts = k >= 8 ? 8u : k >= 4 ? 4u : 2u;
    }
    // XCD-grouped tile order for scenes whose nodes + primitive slots exceed one XCD's 4 MB L2:
    // mig29 x16 (11.6 MB) 0.449 -> 0.406 ms; a cache-resident TEAPOT-F loses with it (4K
    // 0.377 -> 0.441 ms, 720p neutral) -- profiles/r02/ab_xcd_*.json.  RT_XCD_ORDER=0/1 forces it.
    s->xcd_order = (size_t)s->bvh.nodes_used * 32u + (size_t)n * 48u > (4u << 20);
    if (const char *e = std::getenv("RT_XCD_ORDER")) s->xcd_order = std::atoi(e) != 0;
    if (const char *e = std::getenv("RT_PT_PIPELINE")) s->pt_pipeline = std::atoi(e) != 0;
    if (const char *e = std::getenv("RT_PT_SLOTS")) s->pt_slots = (uint32_t)std::max(2, std::min((int)kPtMaxSlots, std::atoi(e)));
    if (const char *e = std::getenv("RT_PS_PIPELINE")) s->ps_pipeline = std::max(-1, std::min(1, std::atoi(e)));
    if (const char *e = std::getenv("RT_PS_BUFFERS")) s->ps_buffers = (uint32_t)std::max(2, std::min(kPsMaxDepth + 1, std::atoi(e)));
    if (const char *e = std::getenv("RT_PS_DEPTH")) s->ps_depth = (uint32_t)std::max(2, std::min(kPsMaxDepth, std::atoi(e)));
    if (const char *e = std::getenv("RT_TUNE_DELAY_MS")) s->tune_delay_ms = (float)std::max(0.0, std::atof(e));
    if (const char *e = std::getenv("RT_PT_MEM_MB"))
        s->pt_mem_bytes = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20;
    // every child box inside its parent's, compared as floats (the wave walk's pops and its leaf
    // check rely on it: a child's slab entry is then never below its parent's)
    for (uint32_t i = 0; i < s->bvh.nodes_used && s->nested; ++i) {
        if (i == 1) continue;
        const Node &nd = s->bvh.nodes[i];
        if (nd.count > 0) continue;
        for (uint32_t c = nd.leftFirst; c < nd.leftFirst + 2 && s->nested; ++c) {
            const Node &ch = s->bvh.nodes[c];
            for (int a = 0; a < 3; ++a)
                if (!(ch.mn[a] >= nd.mn[a]) || !(ch.mx[a] <= nd.mx[a])) s->nested = false;
        }
    }
    // camera-ray walk: wave-coherent vs per-lane (RT_WAVE_PRIMARY=0/1 overrides the policy)
    v.wave_primary = 0;
    const bool wave_ok = !s->has_cubes && s->nested && s->walk_fits;
    s->walk = wave_ok ? RT_WALK_AUTO : RT_WALK_LANE;
    if (const char *e = std::getenv("RT_WAVE_PRIMARY")) s->walk = std::atoi(e) != 0 && wave_ok ? RT_WALK_WAVE : RT_WALK_LANE;
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
// launches whose camera rays may take the wave walk (SceneView::wave_primary) also hold each wave's
// uniform stack of node words past the lane stacks (walk_words in rt_kernels.inc): 4 waves x depth
size_t walk_bytes(const rt_scene *s, const SceneView &v) {
    return v.wave_primary ? (size_t)s->stack_depth * 4u * sizeof(uint32_t) : 0u;
}
// the compiled MAXD class a Trace depth runs in
int max_depth_class(uint32_t depth) { return depth <= 1 ? 1 : depth <= 4 ? 4 : depth <= 10 ? 10 : 32; }
// pixels covered by a frame / shard launch (primary rays per sample)
uint64_t frame_pixels(const rt_renderer *r, const FrameArgs &F, uint32_t shard, uint32_t nshards, uint32_t tiles_x,
                      uint32_t ntiles) {
    uint64_t px = (uint64_t)F.ntiles_local * 64u;
    if ((r->W & 7u) || (r->H & 7u)) {
        px = 0;
        auto add = [&](uint32_t t) {
            uint32_t tx = t % tiles_x, ty = t / tiles_x;
            px += (uint64_t)std::min(8u, r->W - tx * 8) * std::min(8u, r->H - ty * 8);
        };
        if (F.tile_map)
            for (uint32_t t : r->map_host) add(t);
        else
            for (uint32_t t = shard; t < ntiles; t += nshards) add(t);
    }
    return px;
}

uint64_t fnv1a(const void *d, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char *c = static_cast<const unsigned char *>(d);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
    return h;
}

// an explicit deal's tile list on the device (FrameArgs::tile_map); a changed list waits for
// every frame still reading the old one.  The list in use is compared element by element (a
// memcmp of at most ntiles words, the same O(n) as hashing it): a caller-supplied identity of
// the list could repeat after its owner was freed and reallocated, and the range /
// duplicate checks below must see every list that differs.
int set_tile_map(rt_renderer *r, const uint32_t *tiles, uint32_t n, uint32_t ntiles) {
    if (r->d_map && r->map_host.size() == n && (n == 0 || std::memcmp(r->map_host.data(), tiles, sizeof(uint32_t) * n) == 0))
        return RT_OK;
    const uint64_t h = fnv1a(tiles, sizeof(uint32_t) * n, fnv1a(&n, sizeof(n)));
    std::vector<uint8_t> seen(ntiles, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (tiles[i] >= ntiles || seen[tiles[i]]) return fail(RT_ERR_INVALID, "tile list: index out of range or repeated");
        seen[tiles[i]] = 1;
    }
    HIP_TRY(hipDeviceSynchronize());
    if (n > r->map_cap || !r->d_map) {
        if (r->d_map) HIP_TRY(hipFree(r->d_map));
        r->d_map = nullptr;
        r->map_cap = 0;
        HIP_TRY(hipMalloc(&r->d_map, sizeof(uint32_t) * std::max<size_t>(n, 1)));
        r->map_cap = std::max<size_t>(n, 1);
    }
    if (n) HIP_TRY(hipMemcpy(r->d_map, tiles, sizeof(uint32_t) * n, hipMemcpyHostToDevice));
    r->map_host.assign(tiles, tiles + n);
    r->map_hash = h;
    r->map_gen += 1;
    return RT_OK;
}


// Per-sample result buffers of pipelined path-traced frames: with two slots and two buffers
// (by frame parity), frame n + 2's batches waited for frame n's finishing pass, which itself
// follows frame n + 1's levels on the caller's stream; slots + 1 buffers let a frame start
// behind the finish of the frame `slots` back.

// The renderer's overlap streams 0 .. n-1 and their ordering events, created as first needed.
// Only as many as a mode uses: each stream becomes a hardware queue of its own (up to
// GPU_MAX_HW_QUEUES), and with 8 queues, creating all 8 streams for a timing that used 2 left
// TEAPOT-F's frames slow for the next ~50 frames -- the first two frames-in-flight groups timed
// 2.5-3.1 / 2.2 ms against 1.5 / 1.6 for the last two (round 5, profiles/r05/hwq).
int ensure_pipe_streams(rt_renderer *r, int n) {
    n = std::min(n, kPsMaxDepth);
    if (!r->pt_fin[0])
        for (int k = 0; k <= kPtMaxSlots; ++k)
            HIP_TRY(hipEventCreateWithFlags(&r->pt_fin[k], hipEventDisableTiming | hipEventReleaseToDevice));
    for (int k = r->nstreams; k < n; ++k) {
        HIP_TRY(hipStreamCreateWithFlags(&r->pt_stream[k], hipStreamNonBlocking));
        // ordering between streams of this device only: a device-scope release
        HIP_TRY(hipEventCreateWithFlags(&r->pt_lv[k], hipEventDisableTiming | hipEventReleaseToDevice));
        r->nstreams = k + 1;
    }
    return RT_OK;
}

// The frame-level per-sample result buffer of parity `par`, grown to `bytes`.
int ensure_res(rt_renderer *r, int par, uint64_t bytes) {
    if (bytes <= r->res_bytes[par]) return RT_OK;
    HIP_TRY(hipDeviceSynchronize());   // every pending use of the old buffer
    if (r->d_res[par]) HIP_TRY(hipFree(r->d_res[par]));
    r->d_res[par] = nullptr;
    r->res_bytes[par] = 0;
    r->pt_fin_set[par] = false;
    HIP_TRY(hipMalloc(&r->d_res[par], bytes));
    r->res_bytes[par] = bytes;
    return RT_OK;
}

// Overlapped primary+shadow frames' result buffer b, grown to `bytes` (launch_render).
int ensure_ps_res(rt_renderer *r, uint32_t b, uint64_t bytes) {
    if (!r->ps_fin[b]) HIP_TRY(hipEventCreateWithFlags(&r->ps_fin[b], hipEventDisableTiming | hipEventReleaseToDevice));
    if (bytes <= r->ps_res_bytes[b]) return RT_OK;
    HIP_TRY(hipDeviceSynchronize());   // every pending use of the old buffer
    if (r->ps_res[b]) HIP_TRY(hipFree(r->ps_res[b]));
    r->ps_res[b] = nullptr;
    r->ps_res_bytes[b] = 0;
    r->ps_fin_set[b] = false;
    HIP_TRY(hipMalloc(&r->ps_res[b], bytes));
    r->ps_res_bytes[b] = bytes;
    return RT_OK;
}

// Wavefront path tracing of one frame / shard (PathArgs, rt_dev_types.h): the samples are
// processed in batches that fit RT_PT_MEM_MB (default 12288 MB) of path state; per batch
// one k_pt_level launch per bounce level, then k_pt_finish.
int launch_pt_frame(rt_renderer *r, const FrameArgs &F, SceneView view, bool tex, hipStream_t st,
                    uint32_t *tile_cost = nullptr) {
    rt_scene *s = r->scene;
    // camera rays of level 0 take the wave-coherent walk when the scene forces it, or when
    // the renderer's primary+shadow frames timed it faster (RT_WALK_AUTO)
    view.wave_primary = !s->has_cubes && s->nested && s->walk_fits &&
                        (s->walk == RT_WALK_WAVE || (s->walk == RT_WALK_AUTO && r->tune == kTuneDone && r->wave));
    view.walk_stats = r->d_counters;
    view.walk_check = r->walk_check;
    view.quad_lanes = s->quad_lanes ? 1 : 0;
    const uint64_t npix = (uint64_t)F.ntiles_local * 64u;
    // pipelined: per-sample results of the whole frame in a frame-level buffer (two by frame
    // parity, up to 2 GB each); the serial path keeps them per batch with a running sum
    const uint64_t res_need = (uint64_t)F.spp * npix * 16u;
    const bool pipe = s->pt_pipeline && res_need <= (2ull << 30);
    const uint64_t per_path = 32u + 16u + 8u + (uint64_t)(F.depth - 1) * 32u;
    // per slot: two slots of up to RT_PT_MEM_MB each when pipelined (fewer, larger batches and
    // frame-to-frame overlap beat more batches: CFG5-sub 8.85 ms with half the budget per slot
    // -- two batches a frame -- vs 8.51 ms with one batch a frame, profiles/r02/bench_pipe_*)
    const uint64_t budget = s->pt_mem_bytes;
    uint64_t batch = std::max<uint64_t>(1, budget / (per_path * npix));
    batch = std::min<uint64_t>(batch, F.spp);
    if (batch * npix > 0xffffffffull / 2) batch = std::max<uint64_t>(1, (0xffffffffull / 2) / npix);
    const uint64_t np = batch * npix;
    // queue segment k takes the survivors of chunks j = k (mod kQueueSegs); the grid's
    // wave count is a multiple of kQueueSegs, so a segment never gets more than this
    const uint64_t seg_cap = ((np / 64u + kQueueSegs - 1) / kQueueSegs + 1) * 64u;
    const size_t qbytes = (size_t)seg_cap * kQueueSegs * 4u;
    const size_t cbytes = (size_t)(F.depth + 1) * (2u * kQueueSegs) * 64u;   // queue counts + head counters
    const size_t need = (size_t)(np * (per_path - 8u) + 2 * qbytes + cbytes + 4096u);
    if (!r->d_sum) {   // one float4 per pixel of the whole frame (a shard uses its first npix)
        const size_t tiles = (size_t)((r->W + 7) / 8) * ((r->H + 7) / 8);
        HIP_TRY(hipMalloc(&r->d_sum, tiles * 64u * sizeof(float4)));
    }
    int par = 0;
    // slot 0 was last written on the caller's stream (a serial frame): that work is done before
    // a path stream takes the slot over (a rare switch: frames whose results exceed the buffer)
    if (pipe && r->pt_serial_last) HIP_TRY(hipStreamSynchronize(st));
    r->pt_serial_last = !pipe;
    if (pipe) {
        int rc = RT_OK;
        if (need > r->pt_need) {
            // as many slots as fit beside 8 GB of headroom (at least 2), decided again whenever a
            // frame needs larger slots: every pending frame is done, slots past the count freed
            HIP_TRY(hipDeviceSynchronize());
            size_t free_b = 0, total_b = 0;
            HIP_TRY(hipMemGetInfo(&free_b, &total_b));
            double avail = (double)free_b;
            for (size_t b : r->pt_bytes) avail += (double)b;
            // a frame of a few M paths (a multi-GPU rank's 1/8 of config 5: 4.1 M) is as long as
            // its deep paths' latency chain, and 8 frames in flight overlap more of it (1/8 shard
            // 1.24 -> 1.16-1.18 ms); whole 1080p x 16 spp frames lose with more than 4 (7.51 ->
            // 7.61 / 7.72 ms with 6 / 8; profiles/r04/slots)
            // (measured with GPU_MAX_HW_QUEUES=8, as bench.py runs path-traced and multi-GPU
            // workloads; with HIP's default of 4 queues eight slot streams share them and the
            // measurement does not carry over, so the small-batch default is 8 only when the
            // process has at least 8 hardware queues -- ADVICE r4)
            uint32_t k = s->pt_slots ? s->pt_slots : (np <= (8400u << 10) && hw_queues() >= 8 ? 8u : 4u);
            while (k > 2 && (double)k * need + (8ull << 30) > avail) --k;
            for (uint32_t j = k; j < (uint32_t)kPtMaxSlots; ++j) {
                if (r->d_pt[j]) HIP_TRY(hipFree(r->d_pt[j]));
                r->d_pt[j] = nullptr;
                r->pt_bytes[j] = 0;
            }
            for (uint32_t j = k + 1; j <= (uint32_t)kPtMaxSlots; ++j) {
                if (r->d_res[j]) HIP_TRY(hipFree(r->d_res[j]));
                r->d_res[j] = nullptr;
                r->res_bytes[j] = 0;
            }
            r->pt_nslots = k;
            r->pt_need = need;
            r->pt_slot = r->pt_parity = 0;
            for (bool &f : r->pt_fin_set) f = false;
        }
        par = r->pt_parity;
        r->pt_parity = (par + 1) % (int)(r->pt_nslots + 1);
        if ((rc = ensure_pipe_streams(r, (int)r->pt_nslots)) != RT_OK) return rc;
        if ((rc = ensure_res(r, par, res_need)) != RT_OK) return rc;
    }
    bool used[kPtMaxSlots] = {};
    const size_t lds = stack_bytes(s);
    // levels are compacted level by level until one is small enough to drain (k_pt_level)
    const uint32_t drain_level = s->pt_drain_level;
    for (uint32_t s0 = 0; s0 < F.spp; s0 += (uint32_t)batch) {
        const int k = pipe ? r->pt_slot : 0;
        if (pipe) r->pt_slot = (r->pt_slot + 1) % (int)r->pt_nslots;
        hipStream_t X = pipe ? r->pt_stream[k] : st;
        const size_t slot_need = need + (pipe ? 0 : (size_t)np * 16u + 256u);   // serial: + the results
        if (slot_need > r->pt_bytes[k]) {
            HIP_TRY(hipStreamSynchronize(X));   // the slot's previous batch is done with it
            if (r->d_pt[k]) HIP_TRY(hipFree(r->d_pt[k]));
            r->d_pt[k] = nullptr;
            r->pt_bytes[k] = 0;
            HIP_TRY(hipMalloc(&r->d_pt[k], slot_need));
            r->pt_bytes[k] = slot_need;
        }
        // this frame's results buffer was last read by the finish of two frames ago
        if (pipe && !used[k] && r->pt_fin_set[par]) HIP_TRY(hipStreamWaitEvent(X, r->pt_fin[par], 0));
        if (pipe && !used[k] && tile_cost) HIP_TRY(hipStreamWaitEvent(X, r->cost_ev, 0));   // the cleared cost map
        used[k] = true;
        char *b = static_cast<char *>(r->d_pt[k]);
        auto take = [&](size_t bytes) { char *q = b; b += (bytes + 255u) & ~(size_t)255u; return q; };
        PathArgs P{};
        P.state = reinterpret_cast<float4 *>(take(np * 32u));
        uint32_t *q0 = reinterpret_cast<uint32_t *>(take(qbytes));
        uint32_t *q1 = reinterpret_cast<uint32_t *>(take(qbytes));
        P.qcount = reinterpret_cast<uint32_t *>(take(cbytes));
        P.seg_cap = (uint32_t)seg_cap;
        P.qhead = P.qcount + (size_t)(F.depth + 1) * kQueueSegs * 16u;
        P.dynamic = s->pt_dynamic ? 1 : 0;
        P.rec = reinterpret_cast<float4 *>(take((size_t)(F.depth - 1) * np * 32u));
        // per-path radiance, indexed (sample - s0) * npix + pixel
        P.result = pipe ? r->d_res[par] + (size_t)s0 * npix : reinterpret_cast<float4 *>(take(np * 16u));
        P.sum = r->d_sum;
        P.tile_cost = tile_cost;
        uint32_t dlevel = drain_level;   // this batch's (a small batch drains from pt_drain_small on)
        P.drain_level = dlevel;
        P.drain_below = 0;
        P.s0 = s0;
        P.batch_spp = std::min<uint32_t>((uint32_t)batch, F.spp - s0);
        P.npaths = (uint32_t)(P.batch_spp * npix);
        HIP_TRY(hipMemsetAsync(P.qcount, 0, cbytes, X));
        for (uint32_t level = 0; level < F.depth; ++level) {
            P.level = level;
            P.queue_in = (level & 1u) ? q1 : q0;
            P.queue_out = (level & 1u) ? q0 : q1;
            int resident = 0;
            if (level > 0 && s->pt_lanes) {             // incoherent levels: the lane state machine
                if (s->ext) kext::launch_pt_lanes(view, F, P, tex, lds, s->num_cus, X);
                else kcore::launch_pt_lanes(view, F, P, tex, lds, s->num_cus, X);
            } else {
                const size_t lv = level == 0 ? lds + walk_bytes(s, view) : lds;   // camera rays: the walk's words
                resident = s->ext ? kext::launch_pt_level(view, F, P, tex, lv, s->num_cus, X)
                                  : kcore::launch_pt_level(view, F, P, tex, lv, s->num_cus, X);
            }
            if (level >= dlevel) break;                // that launch finished every remaining level
            if (level == 0) {
                const bool small = s->pt_drain_small && (double)P.npaths <= s->pt_small_rounds * resident;
                P.drain_below = (uint32_t)std::min<double>(4e9, (small ? s->pt_small_drain_rounds : s->pt_drain_rounds) * resident);
                if (small) P.drain_level = dlevel = std::min(dlevel, s->pt_drain_small);
            }
        }
        if (!pipe) {   // serial: this batch's samples onto the running sum (the last: accumulate, RGB8)
            const bool last = s0 + P.batch_spp >= F.spp;
            if (s->ext) kext::launch_pt_finish(F, P, last, st);
            else kcore::launch_pt_finish(F, P, last, st);
        }
    }
    if (pipe) {
        // one finishing pass on the caller's stream: every sample of the frame in sample order
        // (the same float sums as the batched running sum), after every batch's levels
        for (int k = 0; k < (int)r->pt_nslots; ++k)
            if (used[k]) {
                HIP_TRY(hipEventRecord(r->pt_lv[k], r->pt_stream[k]));
                HIP_TRY(hipStreamWaitEvent(st, r->pt_lv[k], 0));
            }
        PathArgs P{};
        P.result = r->d_res[par];
        P.sum = r->d_sum;
        P.s0 = 0;
        P.batch_spp = F.spp;
        if (s->ext) kext::launch_pt_finish(F, P, true, st);
        else kcore::launch_pt_finish(F, P, true, st);
        HIP_TRY(hipEventRecord(r->pt_fin[par], st));
        r->pt_fin_set[par] = true;
    }
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

// Longest-tile-first dispatch (LPT): tiles differ in cost by an order of magnitude (sky vs
// mesh), and the dispatcher hands out workgroups in index order, so expensive tiles that come
// last leave most CUs idle at the end of the frame.  Each tile's wave cycles are recorded on
// one frame, sorted on the host once, and from the next frame on slot i renders the i-th most
// expensive tile -- for as long as camera, size, spp, depth, mode and shard stay the same.
// With the RT_WALK_AUTO camera walk still being timed, the two timed frames record the costs
// under each walk and the frame that picks the walk applies the matching order (active from
// the 4th frame); otherwise frame 1 records and frame 2 applies.  Pixel values do not depend
// on the order.  walk_phase: -1 no walk timing pending, 0 / 1 this frame times the lane /
// wave walk, 2 the walk was picked on this frame, 3 the timing has not started yet.
// XCD-grouped measured order (RT_XCD_ORDER=1): the frame kernel's block b (4 waves = slots
// 4b .. 4b+3) runs on the XCD of blocks b % 8 (blocks are dealt round-robin over the 8 XCDs,
// MI355X_MICROARCH.md), so group g = b % 8 gets one compact screen region -- a run of the
// tiles in Morton order holding 1/8 of the measured cost -- costliest tile first.  Each XCD's
// L2 then holds the nodes of its region only, not of the whole frame.  A group whose region
// ran out takes tiles from the region with the most cost left.
std::vector<uint32_t> xcd_grouped_order(const FrameArgs &F, const uint32_t *map, const std::vector<uint32_t> &entries,
                                        const std::vector<uint32_t> &cost, uint32_t parts) {
    // entries: order entries (local tile | split bits); an entry's cost is its tile's, divided
    // by the parts of a split tile (bit 31)
    const uint32_t n = (uint32_t)entries.size();
    auto morton = [](uint32_t x, uint32_t y) {
        uint64_t m = 0;
        for (int b = 0; b < 16; ++b) m |= (uint64_t)((x >> b) & 1u) << (2 * b) | (uint64_t)((y >> b) & 1u) << (2 * b + 1);
        return m;
    };
    std::vector<uint32_t> z(n);
    std::vector<uint64_t> code(n);
    std::vector<double> ec(n);
    double total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t e = entries[i], lt = e & 0x0fffffffu;
        const uint32_t tile = map ? map[lt] : lt * F.nshards + F.shard;
        code[i] = morton(tile % F.tiles_x, tile / F.tiles_x) * 16u + (e >> 28);
        ec[i] = (e >> 31) ? cost[lt] / (double)parts : (double)cost[lt];
        z[i] = i;
        total += ec[i];
    }
    std::stable_sort(z.begin(), z.end(), [&](uint32_t a, uint32_t b) { return code[a] < code[b]; });
    std::vector<std::vector<uint32_t>> region(8);
    std::vector<double> left(8, 0.0);
    double acc = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t g = std::min<uint32_t>(7u, (uint32_t)(acc * 8.0 / std::max(total, 1.0)));
        region[g].push_back(z[i]);
        left[g] += ec[z[i]];
        acc += ec[z[i]];
    }
    for (auto &rg : region)   // costliest first within a region (sorted ascending: taken from the back)
        std::stable_sort(rg.begin(), rg.end(), [&](uint32_t a, uint32_t b) { return ec[a] < ec[b]; });
    std::vector<uint32_t> out;
    out.reserve(n);
    for (uint32_t b = 0; out.size() < n; ++b) {
        for (uint32_t w = 0; w < 4 && out.size() < n; ++w) {
            uint32_t g = b % 8u;
            if (region[g].empty()) {   // out.size() < n: some region still holds entries
                int best = -1;
                for (uint32_t h = 0; h < 8; ++h)
                    if (!region[h].empty() && (best < 0 || left[h] > left[best])) best = (int)h;
                g = (uint32_t)best;
            }
            const uint32_t i = region[g].back();
            region[g].pop_back();
            left[g] -= ec[i];
            out.push_back(entries[i]);
        }
    }
    return out;
}

// The primary+shadow frame kernel's build (FrameLaunch::waves): frames of one sample per work
// unit run k_render_w8 (render_tile ONE: no sample loop, 51 VGPRs, 8 waves/SIMD where the LDS
// stacks allow), others the plain k_render (71 VGPRs, 7 waves).
void frame_build(const rt_renderer *r, const SceneView &view, const FrameArgs &F, FrameLaunch &L, bool overlapped) {
    const rt_scene *s = r->scene;
    L.waves = 7;
    if (L.mode != RT_MODE_PATH || L.md != 1 || s->frame_waves == 7) return;
    if (F.nchunks != std::max(1u, F.spp)) return;   // the single-sample build: one sample per unit
    if (view.wave_primary && view.walk_check != RT_WALK_CHECK_OFF) return;   // the walk-check build
    // small overlapped frames (<= 3 rounds of resident waves: TEAPOT-F 720p with 4 in flight
    // 0.059 -> 0.062 ms) keep the plain build; everywhere else the single-sample build won or
    // tied (TEAPOT-F 1080p serial 0.1025 -> 0.096, 2 in flight 0.108 -> 0.099; mig29 x16 1080p 4 in
    // flight 0.223 -> 0.215, serial 0.466 -> 0.471; profiles/r04/frame_build/one_*.log)
    if (overlapped && F.nunits <= 3u * 4u * 5u * s->num_cus && s->frame_waves != 8) return;
    L.waves = 8;
}

int tile_order_step(rt_renderer *r, FrameArgs &F, uint64_t key, int walk_phase, bool split_ok, bool gate_open,
                    bool stalled, int &split_ev0, int &split_ev1) {
    split_ev0 = split_ev1 = -1;
    const uint32_t n = F.ntiles_local;
    if (key != r->order_key || n != r->order_n) {
        r->order_key = key;
        r->order_state = 0;
        r->host_cost.clear();
        r->tail_bound = false;
        r->ps_phase = 0;   // the overlap decision belongs to the parameter set too
        r->ps_restarts = 0;
        r->ps_rg = -1;
        if (n != r->order_n) {
            HIP_TRY(hipDeviceSynchronize());                             // frames may still read them
            if (r->d_order) HIP_TRY(hipFree(r->d_order));
            if (r->d_cost) HIP_TRY(hipFree(r->d_cost));
            r->d_order = r->d_cost = nullptr;
            r->order_n = 0;
            // plain order (n) | split order: n + (parts - 1) x the split tiles -- up to 9 n with 8 parts
            // and every tile split (RT_SPLIT_PARTS / RT_SPLIT_HEAVY; 3 n overflowed a balanced rank's
            // short tile list with 4 parts and 500 split tiles, round 5)
            HIP_TRY(hipMalloc(&r->d_order, 9u * n * sizeof(uint32_t)));
            HIP_TRY(hipMalloc(&r->d_cost, 2u * n * sizeof(uint32_t)));   // one cost map per camera walk
            r->order_n = n;
        }
    }
    int use = -1;                                                      // cost map to sort this frame
    if (walk_phase == 3) {
        // walk timing not started yet: record nothing
    } else if (r->order_state == 0) {
        if (walk_phase == 0 || walk_phase == 1) F.tile_cost = r->d_cost + (size_t)walk_phase * n;
        else if (walk_phase == 2) use = r->wave ? 1 : 0;              // recorded on the timed frames
        else { F.tile_cost = r->d_cost; r->order_state = 1; }
    } else if (r->order_state == 1) {
        use = 0;
    }
    if (use >= 0) {
        // once per parameter set: a device-wide sync orders the cost read after the recording
        // frame and the order write after every frame still reading the previous order,
        // whatever streams the caller used
        HIP_TRY(hipDeviceSynchronize());
        std::vector<uint32_t> cost(n), ord(n);
        HIP_TRY(hipMemcpy(cost.data(), r->d_cost + (size_t)use * n, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
        r->host_cost = cost;
        {   // a tile's cost is its wave's residence time, so sum / slots is the frame's throughput
            // time and the costliest tile its latency floor (mig29 x16 1080p: 3.6x, its 1/2 shard
            // 7x; TEAPOT-F 1080p 1.2-1.3x).  A sample-split frame's map holds one chunk's cycles
            // per tile (the last unit of the tile to finish writes it): nchunks of them run.
            double sum = 0, mx = 0;
            for (uint32_t c : cost) { sum += c; mx = std::max<double>(mx, c); }
            const double slots = (double)r->scene->num_cus * 4.0 * 7.0;
            r->tail_bound = sum > 0 && mx * slots > 2.0 * sum * std::max(1u, F.nchunks);
        }
        for (uint32_t i = 0; i < n; ++i) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });

        // The costliest tiles can bound the frame's tail (one wave's latency chain): the split
        // order runs the first k of them as two waves of half a tile each (entry bit 31 =
        // split, bit 30 = which half).  It shortens tail-bound frames (mig29 x16 -10 %, 720p
        // TEAPOT-F -9 %) and lengthens throughput-bound ones (1080p TEAPOT-F +9 %: the half-
        // empty waves cost issue slots), so with RT_SPLIT_HEAVY = -1 (default) both orders are
        // timed on two frames each and the faster one is kept; frames are identical either way.
        uint32_t k = 0;
        if (split_ok) {
            const int32_t hs = r->scene->heavy_split;
            k = std::min<uint32_t>(n, hs < 0 ? n / 32u : (uint32_t)hs);
        }
        // RT_SPLIT_PARTS: a split tile runs as 2 (rows 0-3 / 4-7), 4 or 8 waves of a part each
        const uint32_t parts = r->scene->split_parts;
        std::vector<uint32_t> ent(ord), sp;
        for (uint32_t i = 0; i < k; ++i)
            for (uint32_t q = 0; q < parts; ++q) sp.push_back(ord[i] | 0x80000000u | (q << 28));
        for (uint32_t i = k; i < n; ++i) sp.push_back(ord[i]);
        if (r->scene->xcd_order && split_ok) {   // both orders grouped by XCD (global-node frame kernel)
            const uint32_t *map = F.tile_map ? r->map_host.data() : nullptr;
            ent = xcd_grouped_order(F, map, ord, cost, parts);
            sp = xcd_grouped_order(F, map, sp, cost, parts);
        }
        ent.insert(ent.end(), sp.begin(), sp.end());
        HIP_TRY(hipMemcpy(r->d_order, ent.data(), ent.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        r->order_split = k;
        r->order_parts = parts;
        r->order_state = 2;
        r->use_split = k > 0 && r->scene->heavy_split > 0;            // a forced count: no timing
        r->split_phase = (k > 0 && r->scene->heavy_split < 0) ? 0 : -1;
        r->split_restarts = 0;
        r->split_rg = -1;
        if (r->split_phase == 0 && !r->sev[0])
            for (auto &e : r->sev) HIP_TRY(hipEventCreate(&e));
    }
    if (r->order_state == 2) {
        bool split = r->use_split;
        if (r->split_phase == 4 * kTuneGroup) {                        // decide after the timed groups
            HIP_TRY(hipEventSynchronize(r->sev[7]));
            for (int i = 0; i < 4; ++i) HIP_TRY(hipEventElapsedTime(&r->split_ms[i], r->sev[2 * i], r->sev[2 * i + 1]));
            r->use_split = split = tuned_alternative(r->split_ms);
            r->split_phase = -1;
        } else if (r->split_phase >= 0 && gate_open) {
            if (r->split_phase / kTuneGroup != r->split_rg) {
                r->split_rg = r->split_phase / kTuneGroup;
                r->split_restarts = 0;
            }
            if (stalled && r->split_phase % kTuneGroup != 0 && r->split_restarts < kTuneRestarts) {
                r->split_phase -= r->split_phase % kTuneGroup;                 // redo the group
                ++r->split_restarts;
            }
            const int g = r->split_phase / kTuneGroup, i = r->split_phase % kTuneGroup;   // plain, split, split, plain
            split = g == 1 || g == 2;
            split_ev0 = i == 0 ? 2 * g : -1;
            split_ev1 = i == kTuneGroup - 1 ? 2 * g + 1 : -1;
            ++r->split_phase;
        }
        F.order = split ? r->d_order + n : r->d_order;
        F.nunits = F.ntiles_local * F.nchunks + (split ? r->order_split * (r->order_parts - 1u) : 0u);   // split only with nchunks 1
        F.part_shift = r->order_parts == 8 ? 3u : r->order_parts == 4 ? 4u : 5u;
    }
    return RT_OK;
}

constexpr int kPsGroup = 16;  // frames per timed group of the overlap decision (8 in round 3)

// the parameter set a frame belongs to (the tuned choices and the tile order are per set)
uint64_t param_key(const rt_renderer *r, const FrameArgs &F, const rt_camera *cam, const rt_frame_params *p) {
    uint64_t key = fnv1a(cam, sizeof(*cam));
    key = fnv1a(&p->width, sizeof(uint32_t) * 4, key);   // width height spp depth
    key = fnv1a(&p->mode, sizeof(uint32_t), key);
    key = fnv1a(&F.shard, sizeof(uint32_t) * 2, key);    // shard nshards
    if (F.tile_map) key = fnv1a(&r->map_hash, sizeof(r->map_hash), key);   // an explicit deal's tile list
    return key;
}

// true once this parameter set's frames have run tune_delay_ms of GPU time (never blocks)
int tune_gate(rt_renderer *r, uint64_t key, hipStream_t st, bool &open) {
    const float delay = r->scene->tune_delay_ms;
    if (key != r->gate_key) {
        r->gate_key = key;
        r->gate_state = 0;
    }
    if (delay <= 0.0f) r->gate_state = 3;
    if (r->gate_state == 3) { open = true; return RT_OK; }
    open = false;
    if (!r->gate_ev[0])
        for (auto &e : r->gate_ev) HIP_TRY(hipEventCreate(&e));
    if (r->gate_state == 0) {
        HIP_TRY(hipEventRecord(r->gate_ev[0], st));
        r->gate_state = 1;
        r->gate_frames = 0;
    } else if (r->gate_state == 1) {
        if (++r->gate_frames % 8 == 0) {
            HIP_TRY(hipEventRecord(r->gate_ev[1], st));
            r->gate_state = 2;
        }
    } else if (hipEventQuery(r->gate_ev[1]) == hipSuccess) {   // state 2: the probe has run
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, r->gate_ev[0], r->gate_ev[1]));
        r->gate_state = ms >= delay ? 3 : 1;
        open = r->gate_state == 3;
    }
    return RT_OK;
}

// The frame record of one rank's part of a frame (camera, size, the interleaved shard or the
// explicit tile list) -- shared by the frame launch and the dry-run work frame.
int frame_args(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
               const uint32_t *tiles, uint32_t ntiles_map, FrameArgs &F) {
    if (p->width != r->W || p->height != r->H)
        return fail(RT_ERR_INVALID, "frame size differs from the renderer's accumulator");
    if (p->spp == 0) return fail(RT_ERR_INVALID, "spp must be >= 1");
    if (p->mode > RT_MODE_PACKET) return fail(RT_ERR_INVALID, "unknown integrator mode");
    if (nshards == 0 || shard >= nshards) return fail(RT_ERR_INVALID, "bad shard index");
    HIP_TRY(hipSetDevice(r->scene->device));
    F = FrameArgs{};
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
    if (tiles) {   // an explicit deal (rt_render_shard_tiles)
        int rc = set_tile_map(r, tiles, ntiles_map, ntiles);
        if (rc != RT_OK) return rc;
        F.ntiles_local = ntiles_map;
        F.tile_map = r->d_map;
    }
    F.acc = r->d_acc;
    F.counters = r->d_counters;
    F.nchunks = 1;
    F.nunits = F.ntiles_local;
    return RT_OK;
}

// Dry-run work map (k_render_work) of one rank's part of a frame: per local tile, node visits +
// primitive tests of its rays summed over lanes and samples, read back to the host (blocking on
// `st`).  The camera rays take the reference-order lane walk whatever walk the renderer timed,
// so the map depends on the frame alone.  Path-traced / primary+shadow frames (RT_MODE_PATH) only.
int work_frame(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
               const uint32_t *tiles, uint32_t ntiles_map, std::vector<uint32_t> &work, uint32_t *pixel_work,
               hipStream_t st) {
    if (!r || !cam || !p) return fail(RT_ERR_INVALID, "work frame: null argument");
    if (p->mode != RT_MODE_PATH) return fail(RT_ERR_UNSUPPORTED, "work frame: RT_MODE_PATH frames only");
    if (p->depth > 32) return fail(RT_ERR_UNSUPPORTED, "Trace depth above 32");
    // the counting build keeps 8 per-lane counters past the stacks (launch_work): a tree deeper than
    // 56 leaves no room -- UNSUPPORTED, so rebalance() falls back to the measured cycle costs
    if (stack_bytes(r->scene) + kWorkCounterBytes > kLdsLaunchMax)
        return fail(RT_ERR_UNSUPPORTED, "work frame: this tree's stacks leave no LDS for the counters");
    FrameArgs F;
    int rc = frame_args(r, cam, p, shard, nshards, tiles, ntiles_map, F);
    if (rc != RT_OK) return rc;
    const uint32_t n = F.ntiles_local;
    work.assign(n, 0u);
    if (n == 0) return RT_OK;
    rt_scene *s = r->scene;
    if (n > r->work_cap) {
        HIP_TRY(hipDeviceSynchronize());
        if (r->d_work) HIP_TRY(hipFree(r->d_work));
        r->d_work = nullptr;
        r->work_cap = 0;
        HIP_TRY(hipMalloc(&r->d_work, sizeof(uint32_t) * n));
        r->work_cap = n;
    }
    HIP_TRY(hipMemsetAsync(r->d_work, 0, sizeof(uint32_t) * n, st));
    SceneView view = s->view;
    view.wave_primary = 0;
    view.walk_check = RT_WALK_CHECK_OFF;
    view.walk_stats = nullptr;
    const int md = p->depth <= 1 ? 1 : 32;
    FrameLaunch L{RT_MODE_PATH, md, !s->view.sky_const, dim3((n + 3) / 4), dim3(256), stack_bytes(s), st, 0};
    if (s->ext) kext::launch_work(view, F, L, r->d_work, pixel_work);
    else kcore::launch_work(view, F, L, r->d_work, pixel_work);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(work.data(), r->d_work, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return RT_OK;
}

int launch_render(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                  uint32_t *out, int packed, void *stream, const uint32_t *tiles = nullptr, uint32_t ntiles_map = 0,
                  const uint32_t *fwd_src = nullptr, uint32_t *fwd_dst = nullptr) {
    if (!r || !cam || !p || !out) return fail(RT_ERR_INVALID, "rt_render: null argument");
    if ((fwd_src || fwd_dst) && (packed || !fwd_src || !fwd_dst)) return fail(RT_ERR_INVALID, "rt_render: bad forward");
    rt_scene *s = r->scene;
    FrameArgs F;
    if (int rc = frame_args(r, cam, p, shard, nshards, tiles, ntiles_map, F); rc != RT_OK) return rc;
    const uint32_t tiles_x = F.tiles_x, tiles_y = (r->H + 7) / 8, ntiles = tiles_x * tiles_y;
    if (tiles) {   // (copied only when the map changed: frames of one deal keep the same list)
        if (r->held_kind != 3 || r->held_gen != r->map_gen) {
            r->held_list = r->map_host;
            r->held_gen = r->map_gen;
        }
        r->held_kind = 3;
    } else {
        r->held_kind = nshards == 1 ? 1 : 2;
        r->held_shard = shard;
        r->held_nshards = nshards;
    }
    F.packed_out = packed;
    F.out = out;
    F.fwd_src = fwd_src;
    F.fwd_dst = fwd_dst;
    if (F.ntiles_local == 0) return RT_OK;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t depth = p->depth;
    if (depth > 32) return fail(RT_ERR_UNSUPPORTED, "Trace depth above 32");   // = kWHITTED_MAX
    const int md = max_depth_class(depth);
    const bool tex = !s->view.sky_const;
    const int mode = (int)p->mode;
    // sample split: a frame (or a shard of one) with few tiles and several samples per
    // pixel is cut into (tile, sample chunk) units, so the dispatcher still balances about
    // s->split_units waves of uneven cost (a 1/8 shard at spp 8 would otherwise be one
    // round of whole-tile waves, as long as its slowest tile)
    F.nchunks = 1;
    const bool wavefront = mode == RT_MODE_PATH && depth >= 2 && s->pt_wavefront;
    // (first measured on TEAPOT-F shards, tools/shard_time.py: split below ~5 rounds of
    // waves, until ~10 rounds, chunks of equal sample counts.  Round 3: whole 1080p frames at
    // spp > 1 gain from it too -- CFG5-sub scene spp 16 2.41 -> 1.44 ms, mig29 x16 spp 4 1.49
    // -> 0.76 ms, TEAPOT-F spp 4 0.390 -> 0.386 ms, frames identical (profiles/r03/split_ab/) --
    // so the threshold is 40,000 tiles instead of 20,000; 80,000 measured the same or slower)
    if (p->spp > 1 && mode != RT_MODE_PACKET && !wavefront && F.ntiles_local < s->split_units)
        while (F.ntiles_local * F.nchunks < 2u * s->split_units && F.nchunks < p->spp) {
            uint32_t d = F.nchunks + 1;                  // next divisor of spp: equal chunks
            while (p->spp % d) ++d;
            F.nchunks = d;
        }
    F.nunits = F.ntiles_local * F.nchunks;
    if (F.nchunks > 1) {
        const size_t need = sizeof(float4) * (size_t)p->spp * F.ntiles_local * 64u;
        if (need > r->samples_bytes) {
            if (r->d_samples) HIP_TRY(hipFree(r->d_samples));
            r->d_samples = nullptr;
            r->samples_bytes = 0;
            HIP_TRY(hipMalloc(&r->d_samples, need));
            r->samples_bytes = need;
        }
        F.samples = static_cast<float4 *>(r->d_samples);
    }
    const dim3 grid((F.nunits + 3) / 4), block(256);
    const size_t lds = stack_bytes(s);
    if (wavefront) {
        // per-tile cost map of a path-traced parameter set (rt_renderer_tile_costs, the multi-GPU
        // deal's input): each tile's level-0 wave cycles -- its camera rays, their shading and
        // NEE, summed over the samples -- recorded on the set's first frame, read on its second
        // (one device synchronisation per set); the bounce levels follow the camera level's
        // hits, so a sky tile is cheap at every level.  No tile order is built from it.
        uint32_t *rec_cost = nullptr;
        if (s->tile_order) {
            const uint64_t pkey = param_key(r, F, cam, p);
            const uint32_t n = F.ntiles_local;
            if (pkey != r->order_key || n != r->order_n) {
                r->order_key = pkey;
                r->order_state = 0;
                r->host_cost.clear();
                if (n != r->order_n) {
                    HIP_TRY(hipDeviceSynchronize());                             // frames may still read them
                    if (r->d_order) HIP_TRY(hipFree(r->d_order));
                    if (r->d_cost) HIP_TRY(hipFree(r->d_cost));
                    r->d_order = r->d_cost = nullptr;
                    r->order_n = 0;
                    HIP_TRY(hipMalloc(&r->d_order, 9u * n * sizeof(uint32_t)));
                    HIP_TRY(hipMalloc(&r->d_cost, 2u * n * sizeof(uint32_t)));
                    r->order_n = n;
                }
            }
            if (r->order_state == 0) {
                if (!r->cost_ev) HIP_TRY(hipEventCreateWithFlags(&r->cost_ev, hipEventDisableTiming | hipEventReleaseToDevice));
                HIP_TRY(hipMemsetAsync(r->d_cost, 0, n * sizeof(uint32_t), st));
                HIP_TRY(hipEventRecord(r->cost_ev, st));
                rec_cost = r->d_cost;
                r->order_state = 1;
            } else if (r->order_state == 1) {
                HIP_TRY(hipDeviceSynchronize());                                 // the recording frame is done
                r->host_cost.resize(n);
                HIP_TRY(hipMemcpy(r->host_cost.data(), r->d_cost, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
                r->order_state = 3;                                              // costs held, no order
            }
        }
        int rc = launch_pt_frame(r, F, s->view, tex, st, rec_cost);
        if (rc != RT_OK) return rc;
        r->primary += frame_pixels(r, F, shard, nshards, tiles_x, ntiles) * p->spp;
        r->frames += 1;
        return RT_OK;
    }
    FrameLaunch L{mode, md, tex, grid, block, lds, st, s->frame_waves};
    SceneView view = s->view;
    view.walk_stats = r->d_counters;
    view.walk_check = r->walk_check;
    const uint64_t pkey = param_key(r, F, cam, p);
    bool gate_open = false;
    if (int rc = tune_gate(r, pkey, st, gate_open); rc != RT_OK) return rc;
    // did the GPU run dry since the previous frame?  (a timed group then restarts: kTuneRestarts)
    bool stalled = false;
    if (r->stall_armed) {
        stalled = hipEventQuery(r->stall_ev) == hipSuccess;
        r->stall_armed = false;
    }
    // camera-ray walk (only the global-node primary+shadow kernel has both)
    const bool walk_kernel = mode == RT_MODE_PATH && md == 1 && !s->ext;
    int walk_ev0 = -1, walk_ev1 = -1;   // tev recorded before / after this launch
    int cost_map = -1;                  // this frame records the tile costs under walk 0 / 1
    bool walk_decided = false;
    // the walk's timed groups (lane, wave, wave, lane) must all run on one parameter set's
    // frames: a set change in the middle (a multi-GPU deal switch, a camera move) restarts them
    if (walk_kernel && s->walk == RT_WALK_AUTO && r->tune >= 1 && r->tune < kTuneDecide && pkey != r->tune_key)
        r->tune = 0;
    if (r->tune == 0) {
        r->tune_key = pkey;
        r->walk_restarts = 0;
        r->walk_rg = -1;
    }
    const bool walk_pending = walk_kernel && s->walk == RT_WALK_AUTO && r->tune < kTuneDone;
    if (walk_kernel) {
        if (s->walk == RT_WALK_WAVE) view.wave_primary = 1;
        else if (s->walk == RT_WALK_AUTO && (gate_open || r->tune >= kTuneDecide)) {
            if (r->tune < kTuneDecide) {
                if (!r->tev[0])
                    for (auto &e : r->tev) HIP_TRY(hipEventCreate(&e));
                if (r->tune >= 1) {   // groups lane, wave, wave, lane
                    if ((r->tune - 1) / kTuneGroup != r->walk_rg) {
                        r->walk_rg = (r->tune - 1) / kTuneGroup;
                        r->walk_restarts = 0;
                    }
                    if (stalled && (r->tune - 1) % kTuneGroup != 0 && r->walk_restarts < kTuneRestarts) {
                        r->tune -= (r->tune - 1) % kTuneGroup;             // redo the group from its first frame
                        ++r->walk_restarts;
                    }
                    const int g = (r->tune - 1) / kTuneGroup, i = (r->tune - 1) % kTuneGroup;
                    view.wave_primary = (g == 1 || g == 2) ? 1 : 0;
                    if (i == 0) walk_ev0 = 2 * g;
                    if (i == kTuneGroup - 1) walk_ev1 = 2 * g + 1;
                    if (i == 0 && g < 2) cost_map = g;   // each walk's tile costs, on its first frame
                }
                ++r->tune;
            } else if (r->tune == kTuneDecide) {                   // decide once, after the timed groups
                float t[4] = {};
                HIP_TRY(hipEventSynchronize(r->tev[7]));
                for (int g = 0; g < 4; ++g) HIP_TRY(hipEventElapsedTime(&t[g], r->tev[2 * g], r->tev[2 * g + 1]));
                r->wave = tuned_alternative(t);
                r->tune = kTuneDone;
                walk_decided = true;
            }
            if (r->tune == kTuneDone) view.wave_primary = r->wave ? 1 : 0;
        }
    }
    int split_ev0 = -1, split_ev1 = -1;   // sev recorded before / after this launch
    if (s->tile_order) {
        // half-tile units: primary+shadow frames of the global-node kernel, whole-tile units only
        const bool split_ok = mode == RT_MODE_PATH && md == 1 && F.nchunks <= 1;
        const int rc = tile_order_step(r, F, pkey, cost_map >= 0 ? cost_map : walk_decided ? 2 : walk_pending ? 3 : -1,
                                       split_ok, gate_open, stalled, split_ev0, split_ev1);
        if (rc != RT_OK) return rc;
        L.grid = dim3((F.nunits + 3) / 4);
    }
    // Overlapped primary+shadow frames: each pixel's accumulator update has to follow the
    // previous frame's, but its traversal does not.  Once the frame is in its steady state
    // (no timing events, no cost recording) the frame kernel runs on one of the renderer's
    // two overlap streams (by frame parity) and stores its samples in the frame-level result
    // buffer of that parity; a finishing pass on the caller's stream then does the running
    // average + RGB8 (k_pt_finish, the same float operations as the kernel's own epilogue).
    // Frame f+1's waves so fill the CUs that frame f's tail leaves idle.  The kernel touches
    // only renderer-private memory; a stream waits only for the finishing pass that last read
    // its result buffer (two frames back).
    // Three result buffers (RT_PS_BUFFERS): with two, frame f + 2's kernel waited for frame f's
    // finishing pass while frame f + 1's kernel shared the CUs, which put the finishing pass and
    // two cross-stream waits on the critical path (TEAPOT-F 1080p 0.119 ms per frame vs 0.1055
    // with three; four measure the same as three; profiles/r02/ps_window*.log).
    // It pays where a frame is latency- or tail-bound (mig29 x16 1080p 0.41 -> 0.33 ms, 720p
    // 0.385 -> 0.255 ms) and costs where it is issue-bound (TEAPOT-F 1080p 0.1024 -> 0.1055 ms:
    // the finishing pass's extra 66 MB of sample traffic is not hidden there), and only
    // when the caller submits frames back to back.  A small frame -- a multi-GPU rank's 1/N
    // shard, about one round of resident waves -- is one latency chain long, and more frames
    // in flight keep filling its idle issue slots: up to 6 renderer streams (round 3).  So by
    // default each renderer times serial, 2, 4 and 6 frames in flight on its own frames and
    // keeps the fastest (RT_PS_PIPELINE: -1 auto, 0 off, 1 on with RT_PS_DEPTH frames in flight).
    const uint64_t ps_bytes = (uint64_t)p->spp * F.ntiles_local * 64u * 16u;
    // (sample-split frames -- a multi-GPU rank's shard at spp N -- store their samples anyway;
    // overlapped, they go to the result buffers instead of d_samples)
    const bool ps_ok = s->ps_pipeline != 0 && mode == RT_MODE_PATH && md == 1 &&
                       split_ev0 < 0 && split_ev1 < 0 && r->split_phase < 0 && !F.tile_cost && !walk_pending &&
                       ps_bytes <= (2ull << 30);
    // frames in flight for this frame: 0 = serial, else 2..6 renderer streams
    uint32_t depth_k = (ps_ok && s->ps_pipeline == 1) ? s->ps_depth : 0u;
    // pev recorded on the caller's stream after this frame: ps_ev0 after a timed group's frame
    // SKIP, ps_ev1 after its last -- the group is timed from one frame's completion to another's,
    // G - 1 - SKIP frame periods at its depth in steady state.  (Events before the first frame timed a
    // deeper group short: its first kernels start on their streams while the caller's stream still
    // finishes earlier frames; TEAPOT-F shards then picked 4-6 in flight, 0.125-0.144 ms against
    // 0.092 with 2.  Round 4.)
    int ps_ev0 = -1, ps_ev1 = -1;
    // More than 2 frames in flight are candidates only for frames of a few rounds of resident
    // waves (a multi-GPU rank's small shard, 720p) or whose costliest tile outlasts twice the
    // frame's throughput time (tail_bound, from the tile-order cost map: mig29 x16 1080p and its
    // 1/2 shard, 16,200 tiles, 0.222 -> 0.167 ms with 4 in flight; round 4, depth_exp_*.jsonl);
    // a throughput-bound frame (TEAPOT-F 1080p, 8 rounds) lost with 4 (0.1035 -> 0.114 ms) and
    // the timing only risked picking them.  Groups in palindromic order: serial, 2, 4, 6, 6, 4,
    // 2, serial -- or serial, 2, 2, serial.
    const bool deep_ok = F.nunits <= 3u * 4u * 5u * s->num_cus || r->tail_bound;
    static const uint32_t kDeep[8] = {0, 2, 4, 6, 6, 4, 2, 0}, kShallow[4] = {0, 2, 2, 0};
    if (ps_ok && s->ps_pipeline < 0 && !gate_open) depth_k = 0;   // timing not started: serial
    if (ps_ok && s->ps_pipeline < 0 && gate_open) {
        if (r->ps_phase == 0) r->ps_groups = deep_ok ? 8 : 4;
        const int NG = r->ps_groups;
        // a group's first frames fill its pipeline (every renderer stream starts behind the previous
        // group), and their completions bunch up: timed from the first frame's completion, a 6-deep
        // group of 16 frames measured 0.23-0.25 ms per frame on mig29 x16 whose 6-deep frames then
        // ran at 0.272 ms against 0.256 with 4 (round 5).  Deep timings run 32-frame groups and time
        // them from the completion of frame 8 (23 periods), shallow ones 16 frames from frame 2.
        const int G = NG == 8 ? 2 * kPsGroup : kPsGroup, SKIP = NG == 8 ? 8 : 2;
        const uint32_t *depths = NG == 8 ? kDeep : kShallow;
        if (r->ps_phase > 0 && r->ps_phase < NG * G && r->frames != r->ps_last + 1) {   // interrupted
            r->ps_phase = 0;
            r->ps_restarts = 0;
        r->ps_rg = -1;
        }
        if (r->ps_phase > 0 && r->ps_phase == NG * G) {
            HIP_TRY(hipEventSynchronize(r->pev[2 * NG - 1]));
            for (int g = 0; g < NG; ++g) HIP_TRY(hipEventElapsedTime(&r->ps_ms[g], r->pev[2 * g], r->pev[2 * g + 1]));
            // group g and its mirror NG - 1 - g ran the same depth.  Shallow candidates (serial,
            // 2): 2 in flight replaces serial only when it beats it by kTuneMargin, so noise does not
            // buy frames in flight.  Deep candidates (tail-bound or small frames: serial, 2, 4, 6):
            // 4 in flight is the default, which another depth replaces only when it beats it by
            // kTuneMargin -- the deep groups time a deeper pipeline's gain short (mig29 x16: 4 in
            // flight 1.9 % ahead of 2 in its groups, 3.5 % ahead in steady state, 0.236-0.238
            // against 0.246 ms; profiles/r05/c4depth), so with serial as the default the choice
            // between 2 and 4 was a coin toss
            const int pref = NG == 8 ? 2 : 0;
            float best = r->ps_ms[pref] + r->ps_ms[NG - 1 - pref];
            r->ps_use = depths[pref];
            for (int g = 0; g < NG / 2; ++g) {
                if (g == pref) continue;
                const float t = r->ps_ms[g] + r->ps_ms[NG - 1 - g];
                if (t < best * (1.0f - kTuneMargin)) { best = t; r->ps_use = depths[g]; }
            }
            r->ps_phase = -1;
            // every timed frame's finishing pass preceded pev[2 NG - 1]: no buffer is in use, and
            // the ones the chosen depth never touches are released (a 1080p spp-1 buffer is 33 MB)
            const uint32_t keep = r->ps_use == 0 ? 0u : (s->ps_buffers ? s->ps_buffers : r->ps_use + 1u);
            for (uint32_t b = keep; b <= (uint32_t)kPsMaxDepth; ++b) {
                if (r->ps_res[b]) HIP_TRY(hipFree(r->ps_res[b]));
                r->ps_res[b] = nullptr;
                r->ps_res_bytes[b] = 0;
                r->ps_fin_set[b] = false;
            }
        }
        if (r->ps_phase >= 0) {
            if (r->ps_phase == 0) {   // streams, events and every result buffer before the timing
                if (!r->pev[0])
                    for (auto &e : r->pev) HIP_TRY(hipEventCreate(&e));
                const uint32_t maxd = NG == 8 ? 6u : 2u;
                int rc = ensure_pipe_streams(r, (int)maxd);
                const uint32_t nb = s->ps_buffers ? s->ps_buffers : maxd + 1u;
                for (uint32_t k = 0; k < nb && rc == RT_OK; ++k) rc = ensure_ps_res(r, k, ps_bytes);
                if (rc != RT_OK) return rc;
            }
            if (r->ps_phase / G != r->ps_rg) {
                r->ps_rg = r->ps_phase / G;
                r->ps_restarts = 0;
            }
            if (stalled && r->ps_phase % G != 0 && r->ps_restarts < kTuneRestarts) {
                r->ps_phase -= r->ps_phase % G;                                // redo the group
                ++r->ps_restarts;
            }
            const int g = r->ps_phase / G;
            depth_k = depths[g];
            if (r->ps_phase % G == SKIP) ps_ev0 = 2 * g;
            if (r->ps_phase % G == G - 1) ps_ev1 = 2 * g + 1;
            r->ps_last = r->frames;
            ++r->ps_phase;
        } else {
            depth_k = r->ps_use;
        }
    }
    const bool ps_pipe = depth_k > 0;

    uint32_t buf = 0;
    int lane_st = 0;
    if (ps_pipe) {
        int rc = ensure_pipe_streams(r, (int)depth_k);
        if (rc != RT_OK) return rc;
        // frame n's kernel on renderer stream n % depth, its samples in buffer n % buffers: with
        // depth + 1 buffers frame n + depth + 1 waits for frame n's finishing pass only, which
        // follows frame n's kernel alone -- never a kernel still running beside it
        const uint32_t buffers = s->ps_buffers ? s->ps_buffers : depth_k + 1u;
        buf = r->ps_count % buffers;
        lane_st = (int)(r->ps_count % depth_k);
        ++r->ps_count;
        if ((rc = ensure_ps_res(r, buf, ps_bytes)) != RT_OK) return rc;
        L.stream = r->pt_stream[lane_st];
        if (r->ps_fin_set[buf]) HIP_TRY(hipStreamWaitEvent(L.stream, r->ps_fin[buf], 0));
        if (!r->ps_prev || ps_ev0 >= 0) {
            // switching from serial frames: start behind the caller's stream; a timed group's first
            // frame: every renderer stream starts behind everything before it, so that no frame of
            // the group runs beside the previous group's (whose depth differs)
            if (!r->ps_join) HIP_TRY(hipEventCreateWithFlags(&r->ps_join, hipEventDisableTiming | hipEventReleaseToDevice));
            HIP_TRY(hipEventRecord(r->ps_join, st));
            if (ps_ev0 >= 0)
                for (int k = 0; k < r->nstreams; ++k) HIP_TRY(hipStreamWaitEvent(r->pt_stream[k], r->ps_join, 0));
            else
                HIP_TRY(hipStreamWaitEvent(L.stream, r->ps_join, 0));
        }
        F.samples = r->ps_res[buf];
    }
    if (ps_ok) r->ps_prev = depth_k;
    L.lds_bytes = stack_bytes(s) + walk_bytes(s, view);   // the camera walk's word stack when it runs
    frame_build(r, view, F, L, ps_pipe);
    if (walk_ev0 >= 0) HIP_TRY(hipEventRecord(r->tev[walk_ev0], st));
    if (split_ev0 >= 0) HIP_TRY(hipEventRecord(r->sev[split_ev0], st));
    if (s->ext) kext::launch_frame(view, F, L);
    else kcore::launch_frame(view, F, L);
    HIP_TRY(hipGetLastError());
    if (walk_ev1 >= 0) HIP_TRY(hipEventRecord(r->tev[walk_ev1], st));
    if (split_ev1 >= 0) HIP_TRY(hipEventRecord(r->sev[split_ev1], st));
    if (ps_pipe) {
        HIP_TRY(hipEventRecord(r->pt_lv[lane_st], L.stream));
        HIP_TRY(hipStreamWaitEvent(st, r->pt_lv[lane_st], 0));
    }
    if (F.samples) {   // the pixels' samples in sample order, running average, RGB8
        PathArgs P{};
        P.batch_spp = p->spp;
        P.result = F.samples;
        if (s->ext) kext::launch_pt_finish(F, P, true, st);
        else kcore::launch_pt_finish(F, P, true, st);
        HIP_TRY(hipGetLastError());
        if (ps_pipe) {
            HIP_TRY(hipEventRecord(r->ps_fin[buf], st));
            r->ps_fin_set[buf] = true;
        }
    }
    if (ps_ev0 >= 0) HIP_TRY(hipEventRecord(r->pev[ps_ev0], st));
    if (ps_ev1 >= 0) HIP_TRY(hipEventRecord(r->pev[ps_ev1], st));
    // a timed group is running: mark this frame's completion for the next submission's stall check
    if ((r->tune >= 1 && r->tune < kTuneDecide) || r->split_phase >= 0 || (s->ps_pipeline < 0 && r->ps_phase > 0)) {
        if (!r->stall_ev) HIP_TRY(hipEventCreateWithFlags(&r->stall_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(r->stall_ev, st));
        r->stall_armed = true;
    }
    (void)tiles_y;
    r->primary += frame_pixels(r, F, shard, nshards, tiles_x, ntiles) * p->spp;
    r->frames += 1;
    return RT_OK;
}

}  // namespace

// accumulator <-> packed [tile][64] float4 of listed tiles: one wave per tile, one lane per pixel
__global__ __launch_bounds__(256) void k_acc_tiles(float4 *__restrict__ acc, float4 *__restrict__ buf,
                                                   const uint32_t *__restrict__ tiles, uint32_t n, uint32_t tiles_x,
                                                   uint32_t W, uint32_t H, int unpack) {
    const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (i >= n) return;
    const uint32_t t = tiles[i];
    const uint32_t x = (t % tiles_x) * 8u + (lane & 7u), y = (t / tiles_x) * 8u + (lane >> 3);
    const bool on = x < W && y < H;
    if (unpack) {
        if (on) acc[x + (size_t)y * W] = buf[(size_t)i * 64u + lane];
    } else {
        buf[(size_t)i * 64u + lane] = on ? acc[x + (size_t)y * W] : make_float4(0, 0, 0, 0);
    }
}

int rt::renderer_accumulator(rt_renderer *r, void **acc_dev, size_t *bytes) {
    if (!r || !acc_dev || !bytes) return fail(RT_ERR_INVALID, "null argument");
    *acc_dev = r->d_acc;
    *bytes = sizeof(float4) * (size_t)r->W * r->H;
    return RT_OK;
}

static int acc_tiles(rt_renderer *r, const uint32_t *d_tiles, uint32_t n, void *buf, void *stream, int unpack) {
    if (!r || (n && (!d_tiles || !buf))) return fail(RT_ERR_INVALID, "null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(r->scene->device));
    const uint32_t tiles_x = (r->W + 7) / 8;
    hipLaunchKernelGGL(k_acc_tiles, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, r->d_acc,
                       static_cast<float4 *>(buf), d_tiles, n, tiles_x, r->W, r->H, unpack);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt::accumulator_pack(rt_renderer *r, const uint32_t *tiles_dev, uint32_t n, void *buf_dev, void *stream) {
    return acc_tiles(r, tiles_dev, n, buf_dev, stream, 0);
}

int rt::accumulator_unpack(rt_renderer *r, const uint32_t *tiles_dev, uint32_t n, const void *buf_dev, void *stream) {
    return acc_tiles(r, tiles_dev, n, const_cast<void *>(buf_dev), stream, 1);
}

int rt::render_part(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                    const uint32_t *tiles, uint32_t n, int packed, uint32_t *out_dev, void *stream,
                    const uint32_t *fwd_src, uint32_t *fwd_dst) {
    if (!r) return fail(RT_ERR_INVALID, "render_part: null renderer");
    if (tiles || n)
        return launch_render(r, cam, p, 0, 1, out_dev, packed, stream, tiles ? tiles : reinterpret_cast<const uint32_t *>(r), n,
                             fwd_src, fwd_dst);
    return launch_render(r, cam, p, shard, nshards, out_dev, packed, stream, nullptr, 0, fwd_src, fwd_dst);
}

int rt::render_work(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t shard, uint32_t nshards,
                    const uint32_t *tiles, uint32_t n, std::vector<uint32_t> &work, void *stream) {
    if (!r) return fail(RT_ERR_INVALID, "render_work: null renderer");
    if (tiles || n)
        return work_frame(r, cam, p, 0, 1, tiles ? tiles : reinterpret_cast<const uint32_t *>(r), n, work, nullptr, (hipStream_t)stream);
    return work_frame(r, cam, p, shard, nshards, nullptr, 0, work, nullptr, (hipStream_t)stream);
}

bool rt::renderer_held_tiles(const rt_renderer *r, std::vector<uint32_t> &tiles) {
    tiles.clear();
    const uint32_t ntiles = ((r->W + 7) / 8) * ((r->H + 7) / 8);
    switch (r->held_kind) {
    case 1:
        for (uint32_t t = 0; t < ntiles; ++t) tiles.push_back(t);
        return true;
    case 2:
        for (uint32_t t = r->held_shard; t < ntiles; t += r->held_nshards) tiles.push_back(t);
        return true;
    case 3:
        tiles = r->held_list;
        return true;
    default:
        return false;
    }
}

int rt::renderer_geometry(const rt_renderer *r, uint32_t *W, uint32_t *H, int *device) {
    if (!r) return fail(RT_ERR_INVALID, "null renderer");
    *W = r->W;
    *H = r->H;
    *device = r->scene->device;
    return RT_OK;
}

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
    return rt_scene_create_recipe_ex(name, mesh_dir, device, RT_BVH_PLAIN, out);
}

int rt_scene_create_recipe_ex(const char *name, const char *mesh_dir, int32_t device, int32_t bvh_kind, rt_scene **out) {
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
        d.bvh_kind = bvh_kind;
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
    info->num_refs = (uint32_t)s->bvh.indices.size();
    return RT_OK;
}

int rt_scene_set_camera_walk(rt_scene *s, int walk) {
    if (!s) return fail(RT_ERR_INVALID, "null argument");
    if (walk != RT_WALK_LANE && walk != RT_WALK_WAVE && walk != RT_WALK_AUTO)
        return fail(RT_ERR_INVALID, "unknown camera walk");
    if (walk != RT_WALK_LANE && s->has_cubes)
        return fail(RT_ERR_UNSUPPORTED, "the wave walk needs order-independent hits; cubes accept on tmax (Primitive.h:221-233)");
    if (walk != RT_WALK_LANE && !s->nested)
        return fail(RT_ERR_UNSUPPORTED, "the wave walk needs every child box inside its parent's (this prebuilt BVH has one outside)");
    if (walk != RT_WALK_LANE && !s->walk_fits)
        return fail(RT_ERR_UNSUPPORTED, "the wave walk's word stack does not fit beside this tree's lane stacks (64 KB of LDS)");
    s->walk = walk;
    return RT_OK;
}

int rt_scene_copy_bvh(const rt_scene *s, void *nodes, uint32_t *indices) {
    if (!s || !nodes || !indices) return fail(RT_ERR_INVALID, "null argument");
    std::memcpy(nodes, s->bvh.nodes.data(), sizeof(Node) * s->bvh.nodes_used);
    std::memcpy(indices, s->bvh.indices.data(), sizeof(uint32_t) * s->bvh.indices.size());
    return RT_OK;
}

int rt_intersect(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !hits))) return fail(RT_ERR_INVALID, "rt_intersect: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    if (s->ext) kext::launch_intersect(s->view, rays, hits, n, stack_bytes(s), st);
    else kcore::launch_intersect(s->view, rays, hits, n, stack_bytes(s), st);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_occluded(rt_scene *s, const rt_ray *rays, uint8_t *out, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !out))) return fail(RT_ERR_INVALID, "rt_occluded: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    if (s->ext) kext::launch_occluded(s->view, rays, out, n, stack_bytes(s), st);
    else kcore::launch_occluded(s->view, rays, out, n, stack_bytes(s), st);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_intersect_packets(rt_scene *s, const rt_ray *rays, rt_hit *hits, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !hits))) return fail(RT_ERR_INVALID, "rt_intersect_packets: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    if (s->ext) kext::launch_intersect_packet(s->view, rays, hits, n, st);
    else kcore::launch_intersect_packet(s->view, rays, hits, n, st);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}
int rt_trace(rt_scene *s, int mode, const rt_ray *rays, uint32_t *seeds, const uint8_t *flags, uint32_t depth,
             float *radiance, rt_hit *hits, uint64_t *ray_counts, uint32_t n, void *stream) {
    if (!s || (n && (!rays || !seeds || !radiance))) return fail(RT_ERR_INVALID, "rt_trace: null argument");
    if (mode != RT_MODE_PATH && mode != RT_MODE_WHITTED) return fail(RT_ERR_INVALID, "rt_trace: mode must be PATH or WHITTED");
    if (depth > 32) return fail(RT_ERR_UNSUPPORTED, "Trace depth above 32");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    TraceArgs A{};
    A.rays = rays; A.seeds = seeds; A.flags = flags; A.radiance = radiance; A.hits = hits;
    A.counts = reinterpret_cast<unsigned long long *>(ray_counts);
    A.n = n; A.depth = depth;
    const bool tex = !s->view.sky_const;
    hipStream_t st = (hipStream_t)stream;
    if (s->ext) kext::launch_trace(s->view, A, mode, max_depth_class(depth), tex, stack_bytes(s), st);
    else kcore::launch_trace(s->view, A, mode, max_depth_class(depth), tex, stack_bytes(s), st);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_trace_host(rt_scene *s, int mode, const rt_ray *rays, uint32_t *seeds, const uint8_t *flags, uint32_t depth,
                  float *radiance, rt_hit *hits, uint64_t *ray_counts, uint32_t n) {
    if (!s || (n && (!rays || !seeds || !radiance))) return fail(RT_ERR_INVALID, "rt_trace_host: null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    // staging: rays | seeds | flags | radiance | hits | counts, 256-B aligned pieces
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_seed = up(sizeof(rt_ray) * (size_t)n), o_flag = o_seed + up(4 * (size_t)n),
                 o_rad = o_flag + up((size_t)n), o_hit = o_rad + up(12 * (size_t)n),
                 o_cnt = o_hit + up(sizeof(rt_hit) * (size_t)n), need = o_cnt + 256;
    if (need > s->scratch_bytes) {
        if (s->d_scratch) HIP_TRY(hipFree(s->d_scratch));
        s->d_scratch = nullptr;
        s->scratch_bytes = 0;
        HIP_TRY(hipMalloc(&s->d_scratch, need));
        s->scratch_bytes = need;
    }
    char *b = (char *)s->d_scratch;
    HIP_TRY(hipMemcpyAsync(b, rays, sizeof(rt_ray) * n, hipMemcpyHostToDevice, s->stream));
    HIP_TRY(hipMemcpyAsync(b + o_seed, seeds, 4 * (size_t)n, hipMemcpyHostToDevice, s->stream));
    if (flags) HIP_TRY(hipMemcpyAsync(b + o_flag, flags, n, hipMemcpyHostToDevice, s->stream));
    if (ray_counts) HIP_TRY(hipMemcpyAsync(b + o_cnt, ray_counts, 16, hipMemcpyHostToDevice, s->stream));
    int rc = rt_trace(s, mode, (const rt_ray *)b, (uint32_t *)(b + o_seed), flags ? (const uint8_t *)(b + o_flag) : nullptr,
                      depth, (float *)(b + o_rad), hits ? (rt_hit *)(b + o_hit) : nullptr,
                      ray_counts ? (uint64_t *)(b + o_cnt) : nullptr, n, s->stream);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(radiance, b + o_rad, 12 * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipMemcpyAsync(seeds, b + o_seed, 4 * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    if (hits) HIP_TRY(hipMemcpyAsync(hits, b + o_hit, sizeof(rt_hit) * n, hipMemcpyDeviceToHost, s->stream));
    if (ray_counts) HIP_TRY(hipMemcpyAsync(ray_counts, b + o_cnt, 16, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
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
    if (e == hipSuccess) e = hipMalloc(&r->d_counters, kCounterSlots * 8 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemsetAsync(r->d_counters, 0, kCounterSlots * 8 * sizeof(unsigned long long), r->stream);
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
    for (int k = 0; k < kPtMaxSlots; ++k)
        if (r->d_pt[k]) (void)hipFree(r->d_pt[k]);
    for (int k = 0; k < kPsMaxDepth; ++k) {
        if (r->pt_stream[k]) (void)hipStreamDestroy(r->pt_stream[k]);
        if (r->pt_lv[k]) (void)hipEventDestroy(r->pt_lv[k]);
    }
    for (int k = 0; k <= kPtMaxSlots; ++k) {
        if (r->d_res[k]) (void)hipFree(r->d_res[k]);
        if (r->pt_fin[k]) (void)hipEventDestroy(r->pt_fin[k]);
    }
    if (r->d_sum) (void)hipFree(r->d_sum);
    if (r->d_samples) (void)hipFree(r->d_samples);
    if (r->d_order) (void)hipFree(r->d_order);
    if (r->d_cost) (void)hipFree(r->d_cost);
    if (r->d_map) (void)hipFree(r->d_map);
    if (r->d_work) (void)hipFree(r->d_work);
    if (r->d_where) (void)hipFree(r->d_where);
    for (auto &e : r->tev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : r->sev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : r->pev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : r->gate_ev)
        if (e) (void)hipEventDestroy(e);
    if (r->ps_join) (void)hipEventDestroy(r->ps_join);
    if (r->cost_ev) (void)hipEventDestroy(r->cost_ev);
    if (r->stall_ev) (void)hipEventDestroy(r->stall_ev);
    for (int b = 0; b < kPsMaxDepth + 1; ++b) {
        if (r->ps_res[b]) (void)hipFree(r->ps_res[b]);
        if (r->ps_fin[b]) (void)hipEventDestroy(r->ps_fin[b]);
    }
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
    launch_assemble(gathered, cap, nshards, nullptr, tiles_x, ntiles, r->W, r->H, rgb8, st);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_render_shard_tiles(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, const uint32_t *tiles,
                          uint32_t ntiles, uint32_t *tiles_dev, void *stream) {
    if (!r || (ntiles && !tiles)) return fail(RT_ERR_INVALID, "rt_render_shard_tiles: null argument");
    return launch_render(r, cam, p, 0, 1, tiles_dev, 1, stream, tiles ? tiles : reinterpret_cast<const uint32_t *>(r), ntiles);
}

int rt_assemble_tiles(rt_renderer *r, const uint32_t *gathered, uint32_t stride_px, const uint32_t *deal_tiles,
                      const uint32_t *deal_off, uint32_t nshards, uint32_t *rgb8, void *stream) {
    if (!r || !gathered || !deal_tiles || !deal_off || !rgb8 || !nshards || nshards > 255)
        return fail(RT_ERR_INVALID, "rt_assemble_tiles: bad argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    const uint32_t tiles_x = (r->W + 7) / 8, ntiles = tiles_x * ((r->H + 7) / 8);
    if (deal_off[0] != 0 || deal_off[nshards] != ntiles) return fail(RT_ERR_INVALID, "rt_assemble_tiles: the deal must cover every tile once");
    uint64_t h = fnv1a(deal_off, sizeof(uint32_t) * (nshards + 1u), fnv1a(deal_tiles, sizeof(uint32_t) * ntiles));
    if (!r->d_where || h != r->where_hash) {
        std::vector<uint32_t> where(ntiles, 0xffffffffu);
        for (uint32_t k = 0; k < nshards; ++k) {
            if (deal_off[k + 1] < deal_off[k] || (size_t)(deal_off[k + 1] - deal_off[k]) * 64u > stride_px)
                return fail(RT_ERR_INVALID, "rt_assemble_tiles: a shard's tiles exceed the stride");
            for (uint32_t i = deal_off[k]; i < deal_off[k + 1]; ++i) {
                const uint32_t t = deal_tiles[i];
                if (t >= ntiles || where[t] != 0xffffffffu) return fail(RT_ERR_INVALID, "rt_assemble_tiles: tile out of range or repeated");
                where[t] = (k << 24) | (i - deal_off[k]);
            }
        }
        HIP_TRY(hipDeviceSynchronize());   // an assembly may still read the previous map
        if (!r->d_where || r->where_cap < ntiles) {
            if (r->d_where) HIP_TRY(hipFree(r->d_where));
            r->d_where = nullptr;
            HIP_TRY(hipMalloc(&r->d_where, sizeof(uint32_t) * ntiles));
            r->where_cap = ntiles;
        }
        HIP_TRY(hipMemcpy(r->d_where, where.data(), sizeof(uint32_t) * ntiles, hipMemcpyHostToDevice));
        r->where_hash = h;
    }
    launch_assemble(gathered, stride_px, nshards, r->d_where, tiles_x, ntiles, r->W, r->H, rgb8, (hipStream_t)stream);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_renderer_counters(rt_renderer *r, rt_counters *out) {
    if (!r || !out) return fail(RT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    HIP_TRY(hipDeviceSynchronize());
    std::vector<unsigned long long> c((size_t)kCounterSlots * 8);
    HIP_TRY(hipMemcpy(c.data(), r->d_counters, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    out->primary = r->primary;
    out->shadow = 0;
    out->bounce = 0;
    for (uint32_t k = 0; k < kCounterSlots; ++k) {
        out->shadow += c[(size_t)k * 8];
        out->bounce += c[(size_t)k * 8 + 1];
    }
    out->frames = r->frames;
    return RT_OK;
}

int rt_renderer_set_walk_check(rt_renderer *r, int level) {
    if (!r || level < RT_WALK_CHECK_OFF || level > RT_WALK_CHECK_VERIFY)
        return fail(RT_ERR_INVALID, "rt_renderer_set_walk_check: bad argument");
    r->walk_check = level;
    return RT_OK;
}

int rt_renderer_walk_stats(rt_renderer *r, uint64_t out[4]) {
    if (!r || !out) return fail(RT_ERR_INVALID, "rt_renderer_walk_stats: null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    HIP_TRY(hipDeviceSynchronize());
    std::vector<unsigned long long> c((size_t)kCounterSlots * 8);
    HIP_TRY(hipMemcpy(c.data(), r->d_counters, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out[i] = 0;
    for (uint32_t k = 0; k < kCounterSlots; ++k) {
        out[0] += c[(size_t)k * 8 + 4];   // camera rays walked
        out[1] += c[(size_t)k * 8 + 2];   // boxes entered through the margin
        out[2] += c[(size_t)k * 8 + 3];   // lanes re-traced (tie / odd)
        out[3] += c[(size_t)k * 8 + 5];   // verify: walk result differed
    }
    return RT_OK;
}

int rt_renderer_overlap(const rt_renderer *r, int *state, float ms[4]) {
    if (!r || !state) return fail(RT_ERR_INVALID, "rt_renderer_overlap: null argument");
    int depth = 0;
    float all[8];
    rt_renderer_overlap_depth(r, &depth, all);
    *state = depth < 0 ? -1 : (depth > 1 ? 1 : 0);
    if (ms) {   // serial, 2 in flight, 2 in flight, serial
        const int n = r->ps_groups == 8 ? 8 : 4;
        const int g[4] = {0, 1, n - 2, n - 1};
        for (int k = 0; k < 4; ++k) ms[k] = all[g[k]];
    }
    return RT_OK;
}

int rt_renderer_choices(const rt_renderer *r, int *walk, int *split, float walk_ms[4], float split_ms[4]) {
    if (!r || !walk || !split) return fail(RT_ERR_INVALID, "rt_renderer_choices: null argument");
    const rt_scene *s = r->scene;
    *walk = s->walk == RT_WALK_WAVE ? 1 : s->walk == RT_WALK_LANE ? 0 : (r->tune == kTuneDone ? (r->wave ? 1 : 0) : -1);
    *split = r->order_state == 2 && r->split_phase < 0 ? (r->use_split ? 1 : 0) : -1;
    for (int g = 0; g < 4; ++g) {
        float t = 0.0f;
        if (walk_ms) {
            if (r->tune == kTuneDone && s->walk == RT_WALK_AUTO && r->tev[2 * g]) (void)hipEventElapsedTime(&t, r->tev[2 * g], r->tev[2 * g + 1]);
            walk_ms[g] = t;
        }
        if (split_ms) split_ms[g] = (r->split_phase < 0 && r->order_state == 2) ? r->split_ms[g] : 0.0f;
    }
    return RT_OK;
}

int rt_renderer_overlap_depth(const rt_renderer *r, int *depth, float ms[8]) {
    if (!r || !depth) return fail(RT_ERR_INVALID, "rt_renderer_overlap_depth: null argument");
    const int32_t mode = r->scene->ps_pipeline;
    const bool decided = mode < 0 && r->ps_phase == -1;
    if (mode == 0) *depth = 1;
    else if (mode == 1) *depth = (int)r->scene->ps_depth;
    else *depth = decided ? (r->ps_use ? (int)r->ps_use : 1) : -1;
    if (ms)
        for (int g = 0; g < 8; ++g) ms[g] = (decided && g < r->ps_groups) ? r->ps_ms[g] : 0.0f;
    return RT_OK;
}

int rt_renderer_device_bytes(const rt_renderer *r, uint64_t *bytes, uint32_t *ps_buffers) {
    if (!r || !bytes) return fail(RT_ERR_INVALID, "rt_renderer_device_bytes: null argument");
    const uint64_t pix = (uint64_t)r->W * r->H;
    const uint64_t tiles = (uint64_t)((r->W + 7) / 8) * ((r->H + 7) / 8);
    uint64_t b = 16u * pix + kCounterSlots * 8u * sizeof(unsigned long long);   // accumulator, counters
    if (r->d_rgb) b += 4u * pix;
    for (size_t k : r->pt_bytes) b += k;
    for (size_t k : r->res_bytes) b += k;
    if (r->d_sum) b += tiles * 64u * sizeof(float4);
    b += r->samples_bytes;
    b += 5u * (uint64_t)r->order_n * sizeof(uint32_t);   // plain + split order, two cost maps
    b += (r->d_map ? r->map_cap : 0) * sizeof(uint32_t) + (r->d_where ? r->where_cap : 0) * sizeof(uint32_t);
    uint32_t nps = 0;
    for (int k = 0; k <= kPsMaxDepth; ++k) {
        b += r->ps_res_bytes[k];
        nps += r->ps_res[k] != nullptr;
    }
    *bytes = b;
    if (ps_buffers) *ps_buffers = nps;
    return RT_OK;
}

int rt_renderer_tile_work(rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, uint32_t *work, uint32_t n,
                          uint32_t *pixel_work_dev, void *stream) {
    if (!r || !cam || !p || (n && !work)) return fail(RT_ERR_INVALID, "rt_renderer_tile_work: null argument");
    const uint32_t ntiles = ((r->W + 7) / 8) * ((r->H + 7) / 8);
    if (n < ntiles) return fail(RT_ERR_INVALID, "rt_renderer_tile_work: room for every tile needed");
    std::vector<uint32_t> w;
    int rc = work_frame(r, cam, p, 0, 1, nullptr, 0, w, pixel_work_dev, (hipStream_t)stream);
    if (rc != RT_OK) return rc;
    std::memcpy(work, w.data(), sizeof(uint32_t) * w.size());
    return RT_OK;
}

int rt_renderer_tile_costs(const rt_renderer *r, uint32_t *costs, uint32_t n, uint32_t *n_out) {
    if (!r || !n_out || (n && !costs)) return fail(RT_ERR_INVALID, "rt_renderer_tile_costs: null argument");
    *n_out = (uint32_t)r->host_cost.size();
    if (n && !r->host_cost.empty()) std::memcpy(costs, r->host_cost.data(), sizeof(uint32_t) * std::min<size_t>(n, r->host_cost.size()));
    return RT_OK;
}

int rt_renderer_read_accumulator(rt_renderer *r, float *host) {
    if (!r || !host) return fail(RT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->scene->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(host, r->d_acc, sizeof(float4) * (size_t)r->W * r->H, hipMemcpyDeviceToHost));
    return RT_OK;
}

const char *rt_frame_kernel_name(const rt_renderer *r, const rt_frame_params *p) {
    if (!r || !p || p->mode > RT_MODE_PACKET || p->depth > 32) {
        fail(RT_ERR_INVALID, "rt_frame_kernel_name: bad argument");
        return nullptr;
    }
    const rt_scene *s = r->scene;
    if (p->mode == RT_MODE_PATH && p->depth >= 2 && s->pt_wavefront) return "k_pt_level";
    const int md = max_depth_class(p->depth);
    static const char *names[3][4] = {
        {"k_render<path,1>", "k_render<path,4>", "k_render<path,10>", "k_render<path,32>"},
        {"k_render<whitted,1>", "k_render<whitted,1>", "k_render<whitted,1>", "k_render<whitted,1>"},
        {"k_render<packet,1>", "k_render<packet,10>", "k_render<packet,10>", "k_render<packet,32>"}};
    const int col = md == 1 ? 0 : md == 4 ? 1 : md == 10 ? 2 : 3;
    return names[p->mode][col];
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
