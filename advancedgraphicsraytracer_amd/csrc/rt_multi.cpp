// rt_multi.cpp -- multi-GPU frames behind the C-ABI: every rank renders the
// 8x8 screen tiles t with t % world == rank (rt_render_shard), ONE RCCL gather per frame
// brings the packed tiles to rank 0 (ncclSend / ncclRecv inside one group: each rank's xGMI
// link to rank 0 carries 1/world of the frame, not the world-fold bytes of a ring
// all-gather), and rank 0 unshuffles them (rt_assemble_shards).  This is the multi-GPU
// split of Renderer::Tick's pixel loop (renderer.cpp:213-245, an OpenMP row loop in the
// reference); nothing else crosses ranks, since pixels are independent.
//
// RCCL is resolved at run time (dlopen "librccl.so.1"), so librtamd.so loads on hosts
// without it and a process that already holds an RCCL (e.g. PyTorch's) shares that copy.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <array>
#include <vector>

#include "rt_internal.h"

using namespace rt;

namespace {

struct Rccl {
    void *h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;
};

const Rccl &rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        // RT_RCCL_LIB: a library with RCCL's point-to-point API to use instead -- the tests'
        // in-process stand-in (tests/cpp/inproc_rccl.cpp) that runs several ranks as threads of
        // one process on one GPU, which RCCL itself refuses
        if (const char *e = std::getenv("RT_RCCL_LIB")) {
            R.h = dlopen(e, RTLD_NOW | RTLD_LOCAL);
            if (!R.h) {
                const char *d = dlerror();
                R.error = std::string("RT_RCCL_LIB not loadable: ") + (d ? d : e);
                return;
            }
        }
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            if (R.h) break;
            R.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
        }
        if (!R.h) {
            const char *e = dlerror();
            R.error = std::string("RCCL not loadable: ") + (e ? e : "librccl.so.1");
            return;
        }
        bool ok = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(R.h, name));
            ok = ok && fn != nullptr;
        };
        sym(R.get_unique_id, "ncclGetUniqueId");
        sym(R.comm_init_rank, "ncclCommInitRank");
        sym(R.comm_destroy, "ncclCommDestroy");
        sym(R.comm_count, "ncclCommCount");
        sym(R.comm_user_rank, "ncclCommUserRank");
        sym(R.group_start, "ncclGroupStart");
        sym(R.group_end, "ncclGroupEnd");
        sym(R.send, "ncclSend");
        sym(R.recv, "ncclRecv");
        sym(R.error_string, "ncclGetErrorString");
        if (!ok) R.error = "RCCL library lacks a required symbol";
    });
    return R;
}

int comm_fail(const Rccl &R, ncclResult_t e, const char *what) {
    return fail(RT_ERR_COMM, std::string(what) + ": " + (R.error_string ? R.error_string(e) : "RCCL error"));
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define NCCL_TRY(R, call, what)                        \
    do {                                               \
        ncclResult_t e_ = (call);                      \
        if (e_ != ncclSuccess) return comm_fail(R, e_, what); \
    } while (0)

}  // namespace

// One communicator + the per-renderer exchange buffers (double-buffered for the pipelined mode).
// A frame is rendered under a deal (which rank owns which 8x8 tiles): the interleaved deal
// t % world == rank, or with RT_MULTI_BALANCED -- from the kDealAfter-th frame of a parameter
// set on -- the cost-balanced compact deal of rt_tile_deal, built once per parameter set from
// the ranks' measured tile costs (one exchange: costs to rank 0, the deal back to every rank).
struct Deal {
    std::vector<uint32_t> tiles, off;      // rt_tile_deal layout
    uint32_t count(int k) const { return off[k + 1] - off[k]; }
};

struct rt_comm {
    ncclComm_t comm = nullptr;
    bool owned = false;
    int rank = 0, world = 1, device = 0;
    hipStream_t comm_stream = nullptr;     // pipelined gathers run here, beside the next render
    hipStream_t setup_stream = nullptr;    // the one-time deal exchange
    const rt_renderer *renderer = nullptr; // buffers below belong to this renderer's frame size
    uint32_t W = 0, H = 0, ntiles = 0;
    uint32_t stride = 0;                   // packed pixels per shard slot (room for any deal)
    uint32_t *tiles[2] = {nullptr, nullptr};      // this rank's packed tiles (rank 0: unused)
    uint32_t *gathered[2] = {nullptr, nullptr};   // rank 0: world x stride, slot 0 rendered in place
    hipEvent_t ev_render[2] = {nullptr, nullptr}, ev_gather[2] = {nullptr, nullptr};
    hipEvent_t ev_asm[2] = {nullptr, nullptr};   // rank 0, pipelined: frame assembled (comm stream)
    hipEvent_t ev_caller = nullptr;        // rank 0, pipelined: the caller's stream at the call, so the
                                           // unshuffle into rgb8_dev follows the caller's reads of it
    int slot = 0;
    int pending = -1;                      // slot whose gather is in flight (pipelined mode)
    int slot_deal[2] = {0, 0};             // the deal a slot's frame was rendered under: 0 interleaved, 1 balanced
    uint64_t frames = 0;
    Deal interleaved, balanced;
    Deal last_balanced;                    // the balanced deal the last balanced frame used
    int last_deal = -1;                    // deal of the previous frame (-1 none yet)
    uint64_t deal_version = 0, last_version = 0;   // balanced deals built / the one last used
    uint64_t deal_key = 0;                 // parameter set the balanced deal belongs to
    uint32_t key_calls = 0;                // frames of that parameter set so far
    bool deal_on = false;
    bool deal_moot = false;                // no costs measured (path-traced frames): keep interleaving
    uint32_t *d_setup = nullptr;           // staging of the exchange
    // RT_MULTI_TIMING: per frame (render start, render end, gather end) events, summed by rt_comm_timing
    std::vector<std::array<hipEvent_t, 3>> tev;
    size_t tev_used = 0;
};

namespace {

// frames of a parameter set rendered under the interleaved deal before the balanced one is built:
// the renderer records its tile costs and sorts them within its first four frames
constexpr uint32_t kDealAfter = 6;

void free_buffers(rt_comm *c) {
    for (int k = 0; k < 2; ++k) {
        if (c->tiles[k]) (void)hipFree(c->tiles[k]);
        if (c->gathered[k]) (void)hipFree(c->gathered[k]);
        c->tiles[k] = c->gathered[k] = nullptr;
    }
    if (c->d_setup) (void)hipFree(c->d_setup);
    c->d_setup = nullptr;
    c->renderer = nullptr;
    c->stride = 0;
    c->pending = -1;
    c->deal_on = false;
    c->deal_key = 0;
    c->key_calls = 0;
    c->last_deal = -1;
}

int bind_renderer(rt_comm *c, rt_renderer *r) {
    uint32_t W = 0, H = 0;
    int dev = 0;
    int rc = renderer_geometry(r, &W, &H, &dev);
    if (rc != RT_OK) return rc;
    if (dev != c->device) return fail(RT_ERR_INVALID, "renderer and communicator are on different devices");
    if (c->renderer == r && c->W == W && c->H == H) return RT_OK;
    if (c->pending >= 0) return fail(RT_ERR_INVALID, "rt_render_frame_multi: flush the pipelined frame before switching renderers");
    free_buffers(c);
    const uint32_t ntiles = ((W + 7) / 8) * ((H + 7) / 8);
    // every deal fits: a shard holds at most all tiles (a balanced deal's region may hold many cheap ones)
    const uint32_t stride = ntiles * 64u;
    for (int k = 0; k < 2; ++k) {
        if (c->rank == 0) HIP_TRY(hipMalloc(&c->gathered[k], sizeof(uint32_t) * (size_t)stride * c->world));
        else HIP_TRY(hipMalloc(&c->tiles[k], sizeof(uint32_t) * (size_t)stride));
    }
    HIP_TRY(hipMalloc(&c->d_setup, sizeof(uint32_t) * ((size_t)ntiles + c->world + 1)));
    Deal &d = c->interleaved;   // t % world == rank, in tile order (rt_render_shard's packing)
    d.tiles.clear();
    d.off.assign(1, 0);
    for (int k = 0; k < c->world; ++k) {
        for (uint32_t t = (uint32_t)k; t < ntiles; t += (uint32_t)c->world) d.tiles.push_back(t);
        d.off.push_back((uint32_t)d.tiles.size());
    }
    c->renderer = r;
    c->W = W;
    c->H = H;
    c->ntiles = ntiles;
    c->stride = stride;
    c->slot = 0;
    return RT_OK;
}

// the frame's one collective: every rank's packed tiles to rank 0 (rank 0's own shard was
// rendered in place into slot 0 of the gather buffer); each peer sends its deal's tile count
int gather(rt_comm *c, int k, const Deal &d, hipStream_t st) {
    const Rccl &R = rccl();
    NCCL_TRY(R, R.group_start(), "ncclGroupStart");
    if (c->rank == 0) {
        for (int peer = 1; peer < c->world; ++peer) {
            const size_t bytes = sizeof(uint32_t) * 64u * d.count(peer);
            ncclResult_t e = R.recv(c->gathered[k] + (size_t)peer * c->stride, bytes, ncclUint8, peer, c->comm, st);
            if (e != ncclSuccess) {
                (void)R.group_end();
                return comm_fail(R, e, "ncclRecv");
            }
        }
    } else {
        const size_t bytes = sizeof(uint32_t) * 64u * d.count(c->rank);
        ncclResult_t e = R.send(c->tiles[k], bytes, ncclUint8, 0, c->comm, st);
        if (e != ncclSuccess) {
            (void)R.group_end();
            return comm_fail(R, e, "ncclSend");
        }
    }
    NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
    return RT_OK;
}

// The per-frame ordering events order work between streams of ONE device (render -> gather ->
// unshuffle): a device-scope release is enough and cheaper than the default system-scope one
// (world-1 pipelined frame 0.1205 -> 0.1181 ms, profiles/r02/multi_overhead_events.json);
// RT_EVENT_SCOPE=system restores the default.
unsigned sync_event_flags() {
    const char *e = std::getenv("RT_EVENT_SCOPE");
    return hipEventDisableTiming | (e && std::strcmp(e, "system") == 0 ? 0u : (unsigned)hipEventReleaseToDevice);
}

int assemble(rt_comm *c, rt_renderer *r, int k, uint32_t *rgb8, hipStream_t st) {
    if (c->rank != 0) return RT_OK;
    if (!rgb8) return fail(RT_ERR_INVALID, "rt_render_frame_multi: rank 0 needs an output frame");
    const Deal &d = c->slot_deal[k] ? c->balanced : c->interleaved;
    return rt_assemble_tiles(r, c->gathered[k], c->stride, d.tiles.data(), d.off.data(), (uint32_t)c->world, rgb8, st);
}

uint64_t params_key(const rt_camera *cam, const rt_frame_params *p) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void *d, size_t n) {
        const unsigned char *q = static_cast<const unsigned char *>(d);
        for (size_t i = 0; i < n; ++i) h = (h ^ q[i]) * 1099511628211ull;
    };
    mix(cam, sizeof(*cam));
    mix(&p->width, sizeof(uint32_t) * 4);   // width height spp depth
    mix(&p->mode, sizeof(uint32_t));
    return h;
}

// The one-time exchange behind the balanced deal (every rank, the same call): each rank's
// measured costs of its interleaved tiles to rank 0, rank 0 builds rt_tile_deal over the whole
// frame (equal costs when any rank has none, e.g. path-traced frames), the deal back to every
// rank.  Blocking: it runs once per parameter set.
int exchange_deal(rt_comm *c, rt_renderer *r) {
    const Rccl &R = rccl();
    if (!c->setup_stream) HIP_TRY(hipStreamCreateWithFlags(&c->setup_stream, hipStreamNonBlocking));
    const Deal &il = c->interleaved;
    const uint32_t mine = il.count(c->rank);
    std::vector<uint32_t> cost(mine, 0u);
    uint32_t have = 0;
    int rc = rt_renderer_tile_costs(r, cost.data(), mine, &have);
    if (rc != RT_OK) return rc;
    if (have != mine) std::fill(cost.begin(), cost.end(), 0u);   // none recorded: 0 = "no costs"
    hipStream_t st = c->setup_stream;
    std::vector<uint32_t> all(c->ntiles, 0u);
    if (c->rank == 0) {
        std::copy(cost.begin(), cost.end(), all.begin());
        if (c->world > 1) {
            NCCL_TRY(R, R.group_start(), "ncclGroupStart");
            for (int peer = 1; peer < c->world; ++peer)
                NCCL_TRY(R, R.recv(c->d_setup + il.off[peer], sizeof(uint32_t) * il.count(peer), ncclUint8, peer, c->comm, st), "ncclRecv");
            NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipMemcpy(all.data() + il.off[1], c->d_setup + il.off[1], sizeof(uint32_t) * (c->ntiles - il.off[1]),
                              hipMemcpyDeviceToHost));
        }
        // local order -> global tile; a rank without costs (zeros) makes the deal count-balanced
        std::vector<uint32_t> global(c->ntiles, 0u);
        bool complete = true;
        for (int k = 0; k < c->world; ++k) {
            bool any = false;
            for (uint32_t i = il.off[k]; i < il.off[k + 1]; ++i) {
                global[il.tiles[i]] = all[i];
                any = any || all[i] != 0;
            }
            complete = complete && (any || il.count(k) == 0);
        }
        // without measured costs (path-traced frames record none) equal-count regions measured
        // worse than interleaving (CFG5-sub 1/4 shards 3.36 vs 2.54 ms): keep the interleaved deal
        Deal &d = c->balanced;
        if (complete) {
            d.tiles.assign(c->ntiles, 0u);
            d.off.assign((size_t)c->world + 1, 0u);
            if ((rc = rt_tile_deal(c->W, c->H, global.data(), (uint32_t)c->world, d.tiles.data(), d.off.data())) != RT_OK)
                return rc;
        } else {
            d = c->interleaved;
        }
        if (c->world > 1) {
            std::vector<uint32_t> msg(d.off);
            msg.insert(msg.end(), d.tiles.begin(), d.tiles.end());
            HIP_TRY(hipMemcpy(c->d_setup, msg.data(), sizeof(uint32_t) * msg.size(), hipMemcpyHostToDevice));
            NCCL_TRY(R, R.group_start(), "ncclGroupStart");
            for (int peer = 1; peer < c->world; ++peer)
                NCCL_TRY(R, R.send(c->d_setup, sizeof(uint32_t) * msg.size(), ncclUint8, peer, c->comm, st), "ncclSend");
            NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
            HIP_TRY(hipStreamSynchronize(st));
        }
    } else {
        HIP_TRY(hipMemcpy(c->d_setup, cost.data(), sizeof(uint32_t) * mine, hipMemcpyHostToDevice));
        NCCL_TRY(R, R.send(c->d_setup, sizeof(uint32_t) * mine, ncclUint8, 0, c->comm, st), "ncclSend");
        HIP_TRY(hipStreamSynchronize(st));
        const size_t words = (size_t)c->world + 1 + c->ntiles;
        NCCL_TRY(R, R.recv(c->d_setup, sizeof(uint32_t) * words, ncclUint8, 0, c->comm, st), "ncclRecv");
        HIP_TRY(hipStreamSynchronize(st));
        std::vector<uint32_t> msg(words);
        HIP_TRY(hipMemcpy(msg.data(), c->d_setup, sizeof(uint32_t) * words, hipMemcpyDeviceToHost));
        c->balanced.off.assign(msg.begin(), msg.begin() + c->world + 1);
        c->balanced.tiles.assign(msg.begin() + c->world + 1, msg.end());
    }
    c->deal_on = true;
    c->deal_moot = c->balanced.tiles == c->interleaved.tiles && c->balanced.off == c->interleaved.off;
    c->deal_version += 1;
    return RT_OK;
}

// Tiles change owner between two frames (interleaved <-> balanced deal): a pixel's running
// average (renderer.cpp:235-241) must go on from the frames its previous owner accumulated.
// Every rank packs its accumulator values of the tiles it owned under the old deal, rank 0
// writes them into its accumulator (now the whole frame's) and hands that to every rank.
// Collective and blocking; once per deal switch.
int migrate_accumulators(rt_comm *c, rt_renderer *r, const Deal &old) {
    const Rccl &R = rccl();
    if (!c->setup_stream) HIP_TRY(hipStreamCreateWithFlags(&c->setup_stream, hipStreamNonBlocking));
    hipStream_t st = c->setup_stream;
    HIP_TRY(hipDeviceSynchronize());   // every frame so far has updated its accumulator
    void *acc = nullptr;
    size_t bytes = 0;
    int rc = renderer_accumulator(r, &acc, &bytes);
    if (rc != RT_OK) return rc;
    uint32_t most = 0;
    for (int k = 0; k < c->world; ++k) most = std::max(most, old.count(k));
    void *staging = nullptr;
    HIP_TRY(hipMalloc(&staging, std::max<size_t>(16, (size_t)most * 64u * 16u)));
    auto run = [&]() -> int {
        if (c->rank == 0) {
            for (int peer = 1; peer < c->world; ++peer) {
                const uint32_t n = old.count(peer);
                if (!n) continue;
                NCCL_TRY(R, R.recv(staging, (size_t)n * 64u * 16u, ncclUint8, peer, c->comm, st), "ncclRecv");
                HIP_TRY(hipStreamSynchronize(st));
                int e = accumulator_unpack(r, old.tiles.data() + old.off[peer], n, staging, st);
                if (e != RT_OK) return e;
            }
            NCCL_TRY(R, R.group_start(), "ncclGroupStart");
            for (int peer = 1; peer < c->world; ++peer)
                NCCL_TRY(R, R.send(acc, bytes, ncclUint8, peer, c->comm, st), "ncclSend");
            NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
            HIP_TRY(hipStreamSynchronize(st));
        } else {
            const uint32_t n = old.count(c->rank);
            if (n) {
                int e = accumulator_pack(r, old.tiles.data() + old.off[c->rank], n, staging, st);
                if (e != RT_OK) return e;
                NCCL_TRY(R, R.send(staging, (size_t)n * 64u * 16u, ncclUint8, 0, c->comm, st), "ncclSend");
                HIP_TRY(hipStreamSynchronize(st));
            }
            NCCL_TRY(R, R.recv(acc, bytes, ncclUint8, 0, c->comm, st), "ncclRecv");
            HIP_TRY(hipStreamSynchronize(st));
        }
        return RT_OK;
    };
    rc = run();
    (void)hipFree(staging);
    return rc;
}

}  // namespace

extern "C" {

// Cost-balanced, spatially compact tile deal: the frame's 8x8 tiles in Morton (Z) order of
// their (x, y), cut into nshards runs of equal summed cost (cost == NULL: one per tile).  A
// rank then renders one compact screen region -- its GPU's caches hold the nodes of that
// region only -- whose measured cost is 1/nshards of the frame's, where the interleaved deal
// (t % nshards) spreads every rank over the whole screen.
int rt_tile_deal(uint32_t width, uint32_t height, const uint32_t *cost, uint32_t nshards, uint32_t *deal_tiles,
                 uint32_t *deal_off) {
    if (!width || !height || !nshards || nshards > 255 || !deal_tiles || !deal_off)
        return fail(RT_ERR_INVALID, "rt_tile_deal: bad argument");
    const uint32_t tx = (width + 7) / 8, ty = (height + 7) / 8, n = tx * ty;
    auto morton = [](uint32_t x, uint32_t y) {
        uint64_t m = 0;
        for (int b = 0; b < 16; ++b) m |= (uint64_t)((x >> b) & 1u) << (2 * b) | (uint64_t)((y >> b) & 1u) << (2 * b + 1);
        return m;
    };
    std::vector<uint64_t> key(n);
    for (uint32_t t = 0; t < n; ++t) {
        key[t] = morton(t % tx, t / tx);
        deal_tiles[t] = t;
    }
    std::sort(deal_tiles, deal_tiles + n, [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    std::vector<double> prefix(n + 1, 0.0);
    for (uint32_t i = 0; i < n; ++i) prefix[i + 1] = prefix[i] + (cost ? (double)cost[deal_tiles[i]] : 1.0);
    const double total = prefix[n];
    deal_off[0] = 0;
    for (uint32_t k = 1; k < nshards; ++k) {
        // first index whose prefix reaches k / nshards of the cost (ties: the nearer boundary)
        const double target = total * k / nshards;
        uint32_t b = (uint32_t)(std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin());
        if (b > 0 && b <= n && target - prefix[b - 1] < prefix[b] - target) --b;
        deal_off[k] = std::min(n, std::max(b, deal_off[k - 1]));
    }
    deal_off[nshards] = n;
    return RT_OK;
}

int rt_comm_unique_id(uint8_t *id) {
    if (!id) return fail(RT_ERR_INVALID, "rt_comm_unique_id: null argument");
    const Rccl &R = rccl();
    if (!R.h || !R.error.empty()) return fail(RT_ERR_COMM, R.error);
    ncclUniqueId u;
    NCCL_TRY(R, R.get_unique_id(&u), "ncclGetUniqueId");
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "unique id size");
    std::memcpy(id, &u, sizeof(u));
    return RT_OK;
}

int rt_comm_create(const uint8_t *id, int rank, int world, int device, rt_comm **out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return fail(RT_ERR_INVALID, "rt_comm_create: bad argument");
    *out = nullptr;
    const Rccl &R = rccl();
    if (!R.h || !R.error.empty()) return fail(RT_ERR_COMM, R.error);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= count) return fail(RT_ERR_INVALID, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    NCCL_TRY(R, R.comm_init_rank(&comm, world, u, rank), "ncclCommInitRank");   // collective over the ranks
    rt_comm *c = new rt_comm();
    c->comm = comm;
    c->owned = true;
    c->rank = rank;
    c->world = world;
    c->device = device;
    *out = c;
    return RT_OK;
}

int rt_comm_wrap(void *nccl_comm, int device, rt_comm **out) {
    if (!nccl_comm || !out) return fail(RT_ERR_INVALID, "rt_comm_wrap: null argument");
    *out = nullptr;
    const Rccl &R = rccl();
    if (!R.h || !R.error.empty()) return fail(RT_ERR_COMM, R.error);
    ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
    int world = 0, rank = 0;
    NCCL_TRY(R, R.comm_count(comm, &world), "ncclCommCount");
    NCCL_TRY(R, R.comm_user_rank(comm, &rank), "ncclCommUserRank");
    rt_comm *c = new rt_comm();
    c->comm = comm;
    c->owned = false;
    c->rank = rank;
    c->world = world;
    c->device = device;
    *out = c;
    return RT_OK;
}

int rt_comm_info(const rt_comm *c, int *rank, int *world) {
    if (!c) return fail(RT_ERR_INVALID, "rt_comm_info: null argument");
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    return RT_OK;
}

int rt_comm_destroy(rt_comm *c) {
    if (!c) return RT_OK;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    free_buffers(c);
    for (int k = 0; k < 2; ++k) {
        if (c->ev_render[k]) (void)hipEventDestroy(c->ev_render[k]);
        if (c->ev_gather[k]) (void)hipEventDestroy(c->ev_gather[k]);
        if (c->ev_asm[k]) (void)hipEventDestroy(c->ev_asm[k]);
    }
    if (c->ev_caller) (void)hipEventDestroy(c->ev_caller);
    for (auto &e : c->tev)
        for (auto &x : e) (void)hipEventDestroy(x);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->setup_stream) (void)hipStreamDestroy(c->setup_stream);
    if (c->owned && c->comm) (void)rccl().comm_destroy(c->comm);
    delete c;
    return RT_OK;
}

int rt_render_frame_multi(rt_renderer *r, rt_comm *c, const rt_camera *cam, const rt_frame_params *p,
                          uint32_t *rgb8_dev, uint32_t flags, void *stream) {
    if (!r || !c || !cam || !p) return fail(RT_ERR_INVALID, "rt_render_frame_multi: null argument");
    if (flags & ~(uint32_t)(RT_MULTI_PIPELINED | RT_MULTI_TIMING | RT_MULTI_BALANCED))
        return fail(RT_ERR_INVALID, "rt_render_frame_multi: unknown flags");
    const bool pipelined = (flags & RT_MULTI_PIPELINED) != 0;
    // every check before the first side effect: a rejected call leaves the accumulator, the
    // frame count and the communicator as they were
    if (!pipelined && c->pending >= 0)
        return fail(RT_ERR_INVALID, "rt_render_frame_multi: a pipelined frame is pending (rt_multi_flush)");
    if (c->rank == 0 && !rgb8_dev && (!pipelined || c->pending >= 0))
        return fail(RT_ERR_INVALID, "rt_render_frame_multi: rank 0 needs an output frame");
    HIP_TRY(hipSetDevice(c->device));
    int rc = bind_renderer(c, r);
    if (rc != RT_OK) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (pipelined && !c->comm_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        for (int j = 0; j < 2; ++j) {
            HIP_TRY(hipEventCreateWithFlags(&c->ev_render[j], sync_event_flags()));
            HIP_TRY(hipEventCreateWithFlags(&c->ev_gather[j], sync_event_flags()));
            HIP_TRY(hipEventCreateWithFlags(&c->ev_asm[j], sync_event_flags()));
        }
        HIP_TRY(hipEventCreateWithFlags(&c->ev_caller, sync_event_flags()));
    }
    // rank 0, pipelined: this call unshuffles the previous frame into rgb8_dev on the
    // communicator's stream; whatever the caller queued on its stream before this call (a copy
    // or display of the frame before) must be done with rgb8_dev first
    const bool assemble_prev = pipelined && c->rank == 0 && c->pending >= 0;
    if (assemble_prev) HIP_TRY(hipEventRecord(c->ev_caller, st));
    // the deal of this frame: interleaved, or (RT_MULTI_BALANCED) the balanced deal of this
    // parameter set, exchanged once on its kDealAfter-th frame
    const uint64_t key = params_key(cam, p);
    if (key != c->deal_key) {
        c->deal_key = key;
        c->key_calls = 0;
        c->deal_on = false;
    }
    if ((flags & RT_MULTI_BALANCED) && !c->deal_on && c->key_calls >= kDealAfter && (rc = exchange_deal(c, r)) != RT_OK)
        return rc;
    c->key_calls += 1;
    const bool use_balanced = (flags & RT_MULTI_BALANCED) && c->deal_on && !c->deal_moot;
    const Deal &deal = use_balanced ? c->balanced : c->interleaved;
    const int deal_id = use_balanced ? 1 : 0;
    if (c->world > 1 && c->last_deal >= 0 && (c->last_deal != deal_id || (deal_id == 1 && c->last_version != c->deal_version))) {
        // the frames before were rendered under another deal: move the accumulators first
        // (pending pipelined work is finished by the device-wide sync inside)
        if ((rc = migrate_accumulators(c, r, c->last_deal == 1 ? c->last_balanced : c->interleaved)) != RT_OK) return rc;
    }
    if (deal_id == 1 && c->last_version != c->deal_version) c->last_balanced = c->balanced;
    c->last_deal = deal_id;
    c->last_version = c->deal_version;
    const int k = c->slot;
    c->slot_deal[k] = deal_id;
    uint32_t *mine = c->rank == 0 ? c->gathered[k] : c->tiles[k];
    std::array<hipEvent_t, 3> *tv = nullptr;
    if (flags & RT_MULTI_TIMING) {
        if (c->tev_used == c->tev.size()) {
            std::array<hipEvent_t, 3> e{};
            for (auto &x : e) HIP_TRY(hipEventCreate(&x));
            c->tev.push_back(e);
        }
        tv = &c->tev[c->tev_used++];
        HIP_TRY(hipEventRecord((*tv)[0], st));
    }
    if (use_balanced)
        rc = rt_render_shard_tiles(r, cam, p, deal.tiles.data() + deal.off[c->rank], deal.count(c->rank), mine, st);
    else
        rc = rt_render_shard(r, cam, p, (uint32_t)c->rank, (uint32_t)c->world, mine, st);
    if (rc != RT_OK) return rc;
    if (tv) HIP_TRY(hipEventRecord((*tv)[1], st));
    if (!pipelined) {
        if ((rc = gather(c, k, deal, st)) != RT_OK) return rc;   // in stream order after the render
        if (tv) HIP_TRY(hipEventRecord((*tv)[2], st));
        if ((rc = assemble(c, r, k, rgb8_dev, st)) != RT_OK) return rc;
        c->frames += 1;
        return RT_OK;
    }
    // pipelined: this frame's gather runs on the communicator's stream while the caller's
    // stream goes on (the next frame's render).  The previous frame is completed here: on rank
    // 0 its unshuffle also runs on the communicator's stream, right behind its gather, so the
    // render stream does not wait for it (only the render into its slot, one frame later, does)
    if (c->pending >= 0) {
        // frame i-1: assembled after its gather (stream order on the comm stream) and after the
        // caller's earlier work on rgb8_dev; its buffers are rendered into again by the next
        // call, which the render stream reaches only after this wait
        const int j = c->pending;
        if (c->rank == 0) {
            HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_caller, 0));
            if ((rc = assemble(c, r, j, rgb8_dev, c->comm_stream)) != RT_OK) return rc;
            HIP_TRY(hipEventRecord(c->ev_asm[j], c->comm_stream));
            HIP_TRY(hipStreamWaitEvent(st, c->ev_asm[j], 0));
        } else {
            HIP_TRY(hipStreamWaitEvent(st, c->ev_gather[j], 0));
        }
        c->frames += 1;
    }
    HIP_TRY(hipEventRecord(c->ev_render[k], st));
    HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_render[k], 0));
    if ((rc = gather(c, k, deal, c->comm_stream)) != RT_OK) return rc;
    HIP_TRY(hipEventRecord(c->ev_gather[k], c->comm_stream));
    if (tv) HIP_TRY(hipEventRecord((*tv)[2], c->comm_stream));
    c->pending = k;
    c->slot = k ^ 1;
    return RT_OK;
}

int rt_comm_timing(rt_comm *c, double *render_ms, double *gather_ms, uint64_t *frames) {
    if (!c || !render_ms || !gather_ms || !frames) return fail(RT_ERR_INVALID, "rt_comm_timing: null argument");
    HIP_TRY(hipSetDevice(c->device));
    double a = 0, b = 0;
    for (size_t i = 0; i < c->tev_used; ++i) {
        auto &e = c->tev[i];
        HIP_TRY(hipEventSynchronize(e[2]));
        float x = 0, y = 0;
        HIP_TRY(hipEventElapsedTime(&x, e[0], e[1]));
        HIP_TRY(hipEventElapsedTime(&y, e[1], e[2]));
        a += x;
        b += y;
    }
    *render_ms = a;
    *gather_ms = b;
    *frames = c->tev_used;
    c->tev_used = 0;
    return RT_OK;
}

int rt_multi_flush(rt_renderer *r, rt_comm *c, uint32_t *rgb8_dev, void *stream) {
    if (!r || !c) return fail(RT_ERR_INVALID, "rt_multi_flush: null argument");
    if (c->pending < 0) return RT_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    const int j = c->pending;
    HIP_TRY(hipStreamWaitEvent(st, c->ev_gather[j], 0));
    int rc = assemble(c, r, j, rgb8_dev, st);
    if (rc != RT_OK) return rc;
    c->pending = -1;
    c->frames += 1;
    return RT_OK;
}

}  // extern "C"
