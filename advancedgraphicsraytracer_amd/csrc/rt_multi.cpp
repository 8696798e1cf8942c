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
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <array>
#include <memory>
#include <vector>

#include "rt_dev_types.h"
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

// A deal: which rank renders which 8x8 tiles (the rt_tile_deal layout: rank k owns
// tiles[off[k] .. off[k+1])).  The interleaved deal t % world == rank has id 0; cost-balanced
// deals (RT_MULTI_BALANCED) take ids from one process-wide counter, so an id never repeats --
// not even for a communicator allocated where a destroyed one lived.  Rank 0 keeps a device map
// for the assembly of a balanced deal: (shard << 24 | local index) per global tile.  `hash`
// (FNV-1a of tiles and offsets) is the same on every rank and in every run that builds the
// same deal (rt_comm_deal_hash).
struct Deal {
    std::vector<uint32_t> tiles, off;
    std::vector<uint8_t> owner;            // rank of every global tile
    uint64_t id = 0, hash = 0;
    uint32_t *d_where = nullptr;
    int device = 0;
    uint32_t count(int k) const { return off[k + 1] - off[k]; }
    ~Deal() {
        if (d_where) {
            (void)hipSetDevice(device);
            (void)hipFree(d_where);
        }
    }
};
using DealP = std::shared_ptr<const Deal>;

// One communicator + the per-renderer exchange buffers (double-buffered for the pipelined mode).
// Every collective after set-up -- the per-frame gathers, the cost exchange and the accumulator
// moves of a deal change -- runs on the communicator's own stream, so the communicator's
// operations are serialised in issue order on every rank whatever streams the caller uses.
// Rank 0 renders its own tiles straight into a row-major frame (the caller's in flags-0 mode,
// its own frame[k] when pipelined): the gather brings only the peers' packed tiles and the
// assembly scatters only those (round 5; at world 1 there is no gather, no assembly and no
// cross-stream event at all).
struct rt_comm {
    ncclComm_t comm = nullptr;
    bool owned = false;
    int rank = 0, world = 1, device = 0;
    hipStream_t comm_stream = nullptr;
    const rt_renderer *renderer = nullptr; // buffers below belong to this renderer's frame size
    uint32_t W = 0, H = 0, ntiles = 0;
    uint32_t stride = 0;                   // packed pixels per shard slot (room for any deal)
    uint32_t *tiles[2] = {nullptr, nullptr};      // rank > 0: this rank's packed tiles
    uint32_t *gathered[2] = {nullptr, nullptr};   // rank 0: (world - 1) x stride, peer p at (p - 1) x stride
    uint32_t *frame[2] = {nullptr, nullptr};      // rank 0, pipelined: slot k's row-major frame
    hipEvent_t ev_render[2] = {nullptr, nullptr}; // rank > 0: render done (caller's stream)
    hipEvent_t ev_gather[2] = {nullptr, nullptr}; // gather / send done (communicator's stream)
    hipEvent_t ev_asm[2] = {nullptr, nullptr};    // rank 0, pipelined: peers' tiles scattered into frame[k]
    hipEvent_t ev_copy[2] = {nullptr, nullptr};   // rank 0, pipelined: frame[k] copied out (caller's stream)
    bool sent[2] = {false, false}, copied[2] = {false, false};   // ev_gather / ev_copy recorded
    hipEvent_t ev_caller = nullptr;        // rank 0, flags 0: the caller's stream at the call
    hipEvent_t ev_mig[2] = {nullptr, nullptr};   // accumulator move: caller -> comm stream -> caller
    int slot = 0;
    int pending = -1;                      // slot whose gather is in flight (pipelined mode)
    DealP slot_deal[2];                    // the deal a slot's frame was rendered under
    uint64_t frames = 0;
    DealP interleaved, cur;                // cur: the deal frames are rendered under now
    uint64_t deals_built = 0;              // balanced deals built by this communicator
    // RT_MULTI_BALANCED: a parameter set (camera, size, spp, depth, mode) tries to balance the
    // deal on its kDealAfter-th frame, then after 2x, 4x, ... as many frames until every rank has
    // measured tile costs (a renderer records them once its own timed choices are done), and not
    // again until the parameters change.  The deal in use is kept across parameter changes.
    uint64_t pkey = 0;
    uint32_t pcalls = 0, next_try = 0;
    bool settled = false;
    // staging, allocated with the renderer binding (nothing is allocated between collectives)
    uint32_t *d_setup = nullptr;           // cost exchange: world blocks of (2 + ntiles) words
    void *d_mig_send = nullptr, *d_mig_recv = nullptr;   // accumulator moves: ntiles x 64 float4 each
    uint32_t *d_mig_list = nullptr;        // ... their tile lists (2 x ntiles)
    uint32_t *h_mig_list = nullptr;        // pinned host staging of those lists
    uint32_t *d_status = nullptr;          // accumulator moves: world status words (own at [rank])
    uint32_t *h_status = nullptr;          // ... read back (pinned)
    bool mig_pending = false;              // ev_mig[1] marks a move whose list upload may still run
    bool adopted = false;                  // the bound renderers' accumulators are on this deal
    uint64_t n_exchanges = 0, n_migrations = 0, n_mig_skipped = 0;
    // RT_MULTI_TIMING: per frame (render start, render end, gather end) events, summed by rt_comm_timing
    std::vector<std::array<hipEvent_t, 3>> tev;
    size_t tev_used = 0;
};

namespace {

// frames of a parameter set rendered before its first balancing attempt: the renderer records
// its tile costs within its first frames unless a timed camera walk holds them back
constexpr uint32_t kDealAfter = 6;

// balanced deal ids: one counter for the process (never reused, see Deal)
std::atomic<uint64_t> g_deal_serial{0};

// Test-only fault injection (RT_MULTI_FAULT=<site>:<rank>): the named local step fails on that
// rank, so the tests can check that every rank of a per-frame collective returns an error and
// none is left waiting in it.  Sites: cost_upload (rebalance's block upload), mig_pack
// (migrate's accumulator_pack).  Unset in production.
bool injected(const rt_comm *c, const char *site) {
    const char *e = std::getenv("RT_MULTI_FAULT");
    if (!e) return false;
    const size_t n = std::strlen(site);
    return std::strncmp(e, site, n) == 0 && e[n] == ':' && std::atoi(e + n + 1) == c->rank;
}

void free_buffers(rt_comm *c) {
    for (int k = 0; k < 2; ++k) {
        for (uint32_t **q : {&c->tiles[k], &c->gathered[k], &c->frame[k]}) {
            if (*q) (void)hipFree(*q);
            *q = nullptr;
        }
        c->slot_deal[k].reset();
        c->sent[k] = c->copied[k] = false;
    }
    for (void *p : {(void *)c->d_setup, c->d_mig_send, c->d_mig_recv, (void *)c->d_mig_list, (void *)c->d_status})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)c->h_mig_list, (void *)c->h_status})
        if (p) (void)hipHostFree(p);
    c->h_mig_list = c->h_status = nullptr;
    c->mig_pending = false;
    c->d_setup = c->d_mig_list = c->d_status = nullptr;
    c->d_mig_send = c->d_mig_recv = nullptr;
    c->interleaved.reset();
    c->cur.reset();
    c->renderer = nullptr;
    c->stride = 0;
    c->pending = -1;
    c->pkey = 0;
    c->pcalls = 0;
    c->settled = false;
    c->adopted = false;
}

uint64_t deal_hash(const std::vector<uint32_t> &tiles, const std::vector<uint32_t> &off) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const std::vector<uint32_t> &v) {
        for (uint32_t x : v)
            for (int b = 0; b < 4; ++b) h = (h ^ ((x >> (8 * b)) & 0xffu)) * 1099511628211ull;
    };
    mix(tiles);
    mix(off);
    return h;
}

// a deal from its tile lists; rank 0 uploads the assembly map of a balanced one
int make_deal(rt_comm *c, std::vector<uint32_t> tiles, std::vector<uint32_t> off, uint64_t id, DealP &out) {
    auto d = std::make_shared<Deal>();
    d->tiles = std::move(tiles);
    d->off = std::move(off);
    d->id = id;
    d->hash = deal_hash(d->tiles, d->off);
    d->device = c->device;
    d->owner.assign(c->ntiles, 0);
    std::vector<uint32_t> where(c->ntiles, 0);
    for (int k = 0; k < c->world; ++k)
        for (uint32_t i = d->off[k]; i < d->off[k + 1]; ++i) {
            d->owner[d->tiles[i]] = (uint8_t)k;
            where[d->tiles[i]] = ((uint32_t)k << 24) | (i - d->off[k]);
        }
    if (c->rank == 0 && id != 0 && c->world > 1) {
        HIP_TRY(hipMalloc(&d->d_where, sizeof(uint32_t) * c->ntiles));
        HIP_TRY(hipMemcpy(d->d_where, where.data(), sizeof(uint32_t) * c->ntiles, hipMemcpyHostToDevice));
    }
    out = d;
    return RT_OK;
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
        if (c->rank == 0) {
            HIP_TRY(hipMalloc(&c->frame[k], sizeof(uint32_t) * (size_t)W * H));
            if (c->world > 1) HIP_TRY(hipMalloc(&c->gathered[k], sizeof(uint32_t) * (size_t)stride * (c->world - 1)));
        } else {
            HIP_TRY(hipMalloc(&c->tiles[k], sizeof(uint32_t) * (size_t)stride));
        }
    }
    if (c->world > 1) {
        HIP_TRY(hipMalloc(&c->d_setup, sizeof(uint32_t) * ((size_t)ntiles + 2) * c->world));
        HIP_TRY(hipMalloc(&c->d_mig_send, (size_t)stride * 16u));
        HIP_TRY(hipMalloc(&c->d_mig_recv, (size_t)stride * 16u));
        HIP_TRY(hipMalloc(&c->d_mig_list, sizeof(uint32_t) * 2u * ntiles));
        HIP_TRY(hipHostMalloc(&c->h_mig_list, sizeof(uint32_t) * 2u * ntiles, hipHostMallocDefault));
        HIP_TRY(hipMalloc(&c->d_status, sizeof(uint32_t) * (size_t)c->world));
        HIP_TRY(hipHostMalloc(&c->h_status, sizeof(uint32_t) * (size_t)c->world, hipHostMallocDefault));
    }
    c->W = W;
    c->H = H;
    c->ntiles = ntiles;
    c->stride = stride;
    std::vector<uint32_t> tl, off(1, 0);   // t % world == rank, in tile order (rt_render_shard's packing)
    for (int k = 0; k < c->world; ++k) {
        for (uint32_t t = (uint32_t)k; t < ntiles; t += (uint32_t)c->world) tl.push_back(t);
        off.push_back((uint32_t)tl.size());
    }
    if ((rc = make_deal(c, std::move(tl), std::move(off), 0, c->interleaved)) != RT_OK) return rc;
    c->cur = c->interleaved;
    c->renderer = r;
    c->slot = 0;
    return RT_OK;
}

// the frame's one collective: every peer's packed tiles to rank 0 (rank 0's own tiles are in
// its frame already); each peer sends its deal's tile count
int gather(rt_comm *c, int k, const Deal &d, hipStream_t st) {
    const Rccl &R = rccl();
    NCCL_TRY(R, R.group_start(), "ncclGroupStart");
    if (c->rank == 0) {
        for (int peer = 1; peer < c->world; ++peer) {
            const size_t bytes = sizeof(uint32_t) * 64u * d.count(peer);
            ncclResult_t e = R.recv(c->gathered[k] + (size_t)(peer - 1) * c->stride, bytes, ncclUint8, peer, c->comm, st);
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

// rank 0: slot k's gathered peer tiles -> their pixels of the row-major frame `out`, under the
// deal that slot was rendered with (rank 0's own tiles are already there)
int scatter_peers(rt_comm *c, int k, uint32_t *out, hipStream_t st) {
    const Deal &d = *c->slot_deal[k];
    launch_assemble(c->gathered[k], c->stride, (uint32_t)c->world, d.id ? d.d_where : nullptr, (c->W + 7) / 8,
                    c->ntiles, c->W, c->H, out, st, 1u);
    HIP_TRY(hipGetLastError());
    return RT_OK;
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

// The exchanged tile costs (wave cycles) move by a few percent between runs of the same frame;
// the deal is cut on costs rounded to 1/kCostQuant of the frame's mean tile cost, so that such
// noise rarely moves a cut (rt_comm_deal_hash reports the deal actually built).
constexpr double kCostQuant = 64.0;

// One balancing attempt (every rank, the same call): an all-gather of the ranks' measured tile
// costs under the current deal -- each rank sends one block [status, count, costs] to every
// peer inside one group -- then every rank builds the same rt_tile_deal over the whole frame
// (deterministic host code on identical inputs).  The status words make the outcome collective:
// a rank that could not read its costs, or could not upload its block, still enters the group
// (its status word says so) and the call then fails on every rank; the deal changes only when
// every rank measured its tiles (`complete`).  Blocking: O(log frames) calls per parameter set.
int rebalance(rt_comm *c, rt_renderer *r, const rt_camera *cam, const rt_frame_params *p, DealP &next, bool &complete) {
    const Rccl &R = rccl();
    const Deal &cur = *c->cur;
    uint32_t most = 0;
    for (int k = 0; k < c->world; ++k) most = std::max(most, cur.count(k));
    const uint32_t B = 2 + most;
    const uint32_t mine = cur.count(c->rank);
    std::vector<uint32_t> block(B, 0u);
    uint32_t have = 0;
    // this rank's tile costs under the current deal: the dry-run work map (deterministic; on the
    // communicator's stream -- it reads only the scene), else the renderer's measured cycles
    std::vector<uint32_t> work;
    int lrc = mine == 0 ? RT_OK
              : cur.id != 0 ? render_work(r, cam, p, 0, 1, cur.tiles.data() + cur.off[c->rank], mine, work, c->comm_stream)
                            : render_work(r, cam, p, (uint32_t)c->rank, (uint32_t)c->world, nullptr, 0, work, c->comm_stream);
    if (lrc == RT_OK && work.size() == mine) {
        std::copy(work.begin(), work.end(), block.begin() + 2);
        have = mine;
    } else if (lrc == RT_ERR_UNSUPPORTED) {
        lrc = rt_renderer_tile_costs(r, block.data() + 2, mine, &have);
    }
    bool any = mine == 0;
    for (uint32_t i = 0; i < mine && lrc == RT_OK && have == mine; ++i) any = any || block[2 + i] != 0;
    block[0] = (lrc != RT_OK ? 2u : 0u) | (lrc == RT_OK && have == mine && any ? 1u : 0u);
    block[1] = mine;
    hipStream_t st = c->comm_stream;
    uint32_t *own = c->d_setup + (size_t)c->rank * B;
    int local = lrc;
    hipError_t up = injected(c, "cost_upload") ? hipErrorInvalidValue
                                               : hipMemcpyAsync(own, block.data(), sizeof(uint32_t) * B, hipMemcpyHostToDevice, st);
    if (up != hipSuccess) {   // the peers learn it from the status word; the group runs anyway
        local = fail(RT_ERR_HIP, std::string("cost upload: ") + hipGetErrorString(up));
        (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(own), 2u, 1, st);
    }
    NCCL_TRY(R, R.group_start(), "ncclGroupStart");
    for (int q = 0; q < c->world; ++q) {
        if (q == c->rank) continue;
        ncclResult_t e = R.send(own, sizeof(uint32_t) * B, ncclUint8, q, c->comm, st);
        if (e == ncclSuccess) e = R.recv(c->d_setup + (size_t)q * B, sizeof(uint32_t) * B, ncclUint8, q, c->comm, st);
        if (e != ncclSuccess) {
            (void)R.group_end();
            return comm_fail(R, e, "cost exchange");
        }
    }
    NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
    std::vector<uint32_t> all((size_t)B * c->world);
    HIP_TRY(hipMemcpyAsync(all.data(), c->d_setup, sizeof(uint32_t) * all.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    c->n_exchanges += 1;
    if (local != RT_OK) return local;
    complete = true;
    for (int k = 0; k < c->world; ++k) {
        const uint32_t status = all[(size_t)k * B];
        if (status & 2u) return fail(RT_ERR_COMM, "rt_render_frame_multi: rank " + std::to_string(k) + " failed before the cost exchange");
        if (all[(size_t)k * B + 1] != cur.count(k)) return fail(RT_ERR_COMM, "rt_render_frame_multi: ranks disagree on the deal");
        complete = complete && (status & 1u);
    }
    next = c->cur;
    if (!complete) return RT_OK;   // e.g. a renderer still timing its camera walk: try again later
    std::vector<uint32_t> global(c->ntiles, 0u);
    double total = 0.0;
    for (int k = 0; k < c->world; ++k)
        for (uint32_t i = 0; i < cur.count(k); ++i) {
            global[cur.tiles[cur.off[k] + i]] = all[(size_t)k * B + 2 + i];
            total += all[(size_t)k * B + 2 + i];
        }
    const double q = std::max(1.0, total / c->ntiles / kCostQuant);
    for (uint32_t &x : global) x = (uint32_t)std::min(4294967295.0, std::floor(x / q + 0.5));
    std::vector<uint32_t> tiles(c->ntiles), off((size_t)c->world + 1);
    int rc = rt_tile_deal(c->W, c->H, global.data(), (uint32_t)c->world, tiles.data(), off.data());
    if (rc != RT_OK) return rc;
    if (tiles == cur.tiles && off == cur.off) return RT_OK;
    c->deals_built += 1;
    return make_deal(c, std::move(tiles), std::move(off), ++g_deal_serial, next);
}

// Tiles change owner between two frames: a pixel's running average (renderer.cpp:235-241) must
// go on from the frames its previous owner accumulated.  Each rank sends the accumulator values
// of every tile it owned under `from` and owns no longer straight to the tile's owner under
// `to` (one group of point-to-point transfers, each pair's tiles in `from` order) and writes the
// ones it receives into its accumulator.  In stream order: the caller's stream's earlier frames
// have updated the accumulator before the pack, and its next frame renders after the unpack --
// no whole-frame broadcast.  Frames that reset the accumulator skip it.
// Failure is collective: a rank whose local steps (the staging wait, the list upload, the pack)
// fail still enters the group, and every rank's status word travels with the data; the ranks
// read the statuses back (one host synchronisation per deal change) and unpack only when all
// are clean -- otherwise every rank returns RT_ERR_COMM, keeps the old deal and its accumulator.
int migrate(rt_comm *c, rt_renderer *r, const Deal &from, const Deal &to, hipStream_t st) {
    const Rccl &R = rccl();
    std::vector<uint32_t> L;
    std::vector<uint32_t> send_off(c->world + 1, 0), recv_off(c->world + 1, 0);
    for (int q = 0; q < c->world; ++q) {   // mine under `from`, q's under `to`
        for (uint32_t i = from.off[c->rank]; i < from.off[c->rank + 1]; ++i)
            if (q != c->rank && to.owner[from.tiles[i]] == q) L.push_back(from.tiles[i]);
        send_off[q + 1] = (uint32_t)L.size();
    }
    const uint32_t nsend = (uint32_t)L.size();
    for (int q = 0; q < c->world; ++q) {   // q's under `from`, mine under `to`
        for (uint32_t i = from.off[q]; i < from.off[q + 1]; ++i)
            if (q != c->rank && to.owner[from.tiles[i]] == c->rank) L.push_back(from.tiles[i]);
        recv_off[q + 1] = (uint32_t)L.size() - nsend;
    }
    const uint32_t nrecv = (uint32_t)L.size() - nsend;
    hipStream_t cs = c->comm_stream;
    int local = RT_OK;
    auto step = [&](hipError_t e, const char *what) {
        if (local == RT_OK && e != hipSuccess) local = fail(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    step(hipEventRecord(c->ev_mig[0], st), "hipEventRecord");
    step(hipStreamWaitEvent(cs, c->ev_mig[0], 0), "hipStreamWaitEvent");
    if (local == RT_OK && c->mig_pending) step(hipEventSynchronize(c->ev_mig[1]), "staging wait");   // the previous move read it
    if (local == RT_OK) {
        std::copy(L.begin(), L.end(), c->h_mig_list);
        if (!L.empty())
            step(hipMemcpyAsync(c->d_mig_list, c->h_mig_list, sizeof(uint32_t) * L.size(), hipMemcpyHostToDevice, cs), "move list upload");
    }
    if (local == RT_OK) {
        local = injected(c, "mig_pack") ? fail(RT_ERR_HIP, "accumulator_pack: injected fault (RT_MULTI_FAULT)")
                                        : accumulator_pack(r, c->d_mig_list, nsend, c->d_mig_send, cs);
    }
    // this rank's status word (a memset on the stream, so it follows whatever ran before)
    (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->d_status + c->rank), local == RT_OK ? 0u : 1u, 1, cs);
    const size_t tile_bytes = 64u * 16u;
    char *sb = static_cast<char *>(c->d_mig_send), *rb = static_cast<char *>(c->d_mig_recv);
    NCCL_TRY(R, R.group_start(), "ncclGroupStart");
    for (int q = 0; q < c->world; ++q) {
        if (q == c->rank) continue;
        ncclResult_t e = ncclSuccess;
        if (send_off[q + 1] > send_off[q])
            e = R.send(sb + send_off[q] * tile_bytes, (send_off[q + 1] - send_off[q]) * tile_bytes, ncclUint8, q, c->comm, cs);
        if (e == ncclSuccess && recv_off[q + 1] > recv_off[q])
            e = R.recv(rb + recv_off[q] * tile_bytes, (recv_off[q + 1] - recv_off[q]) * tile_bytes, ncclUint8, q, c->comm, cs);
        if (e == ncclSuccess) e = R.send(c->d_status + c->rank, sizeof(uint32_t), ncclUint8, q, c->comm, cs);
        if (e == ncclSuccess) e = R.recv(c->d_status + q, sizeof(uint32_t), ncclUint8, q, c->comm, cs);
        if (e != ncclSuccess) {
            (void)R.group_end();
            return comm_fail(R, e, "accumulator move");
        }
    }
    NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
    HIP_TRY(hipMemcpyAsync(c->h_status, c->d_status, sizeof(uint32_t) * c->world, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    c->mig_pending = false;   // the stream is drained: the staging is free again
    if (local != RT_OK) return local;
    for (int q = 0; q < c->world; ++q)
        if (c->h_status[q] != 0u)
            return fail(RT_ERR_COMM, "rt_render_frame_multi: rank " + std::to_string(q) + " failed its part of the accumulator move");
    int rc = accumulator_unpack(r, c->d_mig_list + nsend, nrecv, c->d_mig_recv, cs);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipEventRecord(c->ev_mig[1], cs));
    HIP_TRY(hipStreamWaitEvent(st, c->ev_mig[1], 0));
    c->mig_pending = true;
    c->n_migrations += 1;
    return RT_OK;
}

// The first frame of a communicator on its renderers (a new communicator, or another renderer
// bound) that does not reset the accumulation: the renderers' accumulators hold the tiles of
// their last frames -- another communicator's deal, whole frames, or nothing yet -- and not
// necessarily this communicator's deal (a communicator destroyed and created again
// around the same renderer).  One exchange of every rank's held tile list; each tile's running
// average then moves from a rank that holds it (its new owner if that one does, else the lowest
// rank that does) to its owner under the current deal, through migrate().  Tiles no rank holds
// stay as they are (fresh renderers: every accumulator starts from zero, as the plain renderer's).
// Collective failure as in rebalance: the status word travels in the exchange.
int adopt(rt_comm *c, rt_renderer *r, hipStream_t st) {
    const Rccl &R = rccl();
    const uint32_t B = 2 + c->ntiles;       // d_setup holds world blocks of (2 + ntiles) words
    std::vector<uint32_t> held;
    const bool known = renderer_held_tiles(r, held);
    std::vector<uint32_t> block(2 + held.size(), 0u);
    block[0] = known ? 1u : 0u;
    block[1] = (uint32_t)held.size();
    std::copy(held.begin(), held.end(), block.begin() + 2);
    hipStream_t cs = c->comm_stream;
    uint32_t *own = c->d_setup + (size_t)c->rank * B;
    // local steps before the group collect their error: the rank still enters the group (with
    // status bit 2) so that no peer is left waiting in it
    hipError_t e = hipEventRecord(c->ev_mig[0], st);   // the caller's earlier frames, then the exchange
    if (e == hipSuccess) e = hipStreamWaitEvent(cs, c->ev_mig[0], 0);
    if (e == hipSuccess) e = hipMemcpyAsync(own, block.data(), sizeof(uint32_t) * block.size(), hipMemcpyHostToDevice, cs);
    int local = RT_OK;
    if (e != hipSuccess) {
        local = fail(RT_ERR_HIP, std::string("held tile upload: ") + hipGetErrorString(e));
        (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(own), 2u, 1, cs);
    }
    NCCL_TRY(R, R.group_start(), "ncclGroupStart");
    for (int q = 0; q < c->world; ++q) {
        if (q == c->rank) continue;
        ncclResult_t ne = R.send(own, sizeof(uint32_t) * B, ncclUint8, q, c->comm, cs);
        if (ne == ncclSuccess) ne = R.recv(c->d_setup + (size_t)q * B, sizeof(uint32_t) * B, ncclUint8, q, c->comm, cs);
        if (ne != ncclSuccess) {
            (void)R.group_end();
            return comm_fail(R, ne, "held tile exchange");
        }
    }
    NCCL_TRY(R, R.group_end(), "ncclGroupEnd");
    std::vector<uint32_t> all((size_t)B * c->world);
    HIP_TRY(hipMemcpyAsync(all.data(), c->d_setup, sizeof(uint32_t) * all.size(), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    if (local != RT_OK) return local;
    // (the own block was written before the copy back: `all` holds it too)
    std::vector<uint32_t> src(c->ntiles, 0xffffffffu);   // the rank each tile's average comes from
    const Deal &cur = *c->cur;
    for (int q = 0; q < c->world; ++q) {
        const uint32_t *b = all.data() + (size_t)q * B;
        if (b[0] & 2u) return fail(RT_ERR_COMM, "rt_render_frame_multi: rank " + std::to_string(q) + " failed before the held tile exchange");
        if (b[1] > c->ntiles) return fail(RT_ERR_COMM, "rt_render_frame_multi: bad held tile list");
        for (uint32_t i = 0; i < b[1]; ++i) {
            const uint32_t t = b[2 + i];
            if (t >= c->ntiles) return fail(RT_ERR_COMM, "rt_render_frame_multi: bad held tile list");
            if (src[t] == 0xffffffffu || (int)cur.owner[t] == q) src[t] = (uint32_t)q;   // lowest holder, or the owner
        }
    }
    bool moves = false;
    std::vector<uint32_t> tiles, off(1, 0);
    for (int q = 0; q < c->world; ++q) {
        for (uint32_t t = 0; t < c->ntiles; ++t) {
            const uint32_t from = src[t] == 0xffffffffu ? cur.owner[t] : src[t];
            if ((int)from != q) continue;
            tiles.push_back(t);
            moves = moves || from != cur.owner[t];
        }
        off.push_back((uint32_t)tiles.size());
    }
    if (!moves) return RT_OK;
    DealP from;
    int rc = make_deal(c, std::move(tiles), std::move(off), 0, from);
    if (rc != RT_OK) return rc;
    return migrate(c, r, *from, cur, st);
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
    for (int k = 0; k < 2; ++k)
        for (hipEvent_t e : {c->ev_render[k], c->ev_gather[k], c->ev_asm[k], c->ev_copy[k], c->ev_mig[k]})
            if (e) (void)hipEventDestroy(e);
    if (c->ev_caller) (void)hipEventDestroy(c->ev_caller);
    for (auto &e : c->tev)
        for (auto &x : e) (void)hipEventDestroy(x);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->owned && c->comm) (void)rccl().comm_destroy(c->comm);
    delete c;
    return RT_OK;
}

int rt_comm_deal_info(const rt_comm *c, int *balanced, uint32_t *ntiles, uint32_t *tile_list, uint64_t stats[4]) {
    if (!c) return fail(RT_ERR_INVALID, "rt_comm_deal_info: null argument");
    const bool bal = c->cur && c->cur->id != 0;
    if (balanced) *balanced = bal ? 1 : 0;
    const uint32_t n = c->cur ? c->cur->count(c->rank) : 0u;
    if (ntiles) *ntiles = n;
    if (tile_list && n) std::memcpy(tile_list, c->cur->tiles.data() + c->cur->off[c->rank], sizeof(uint32_t) * n);
    if (stats) {
        stats[0] = c->deals_built;
        stats[1] = c->n_exchanges;
        stats[2] = c->n_migrations;
        stats[3] = c->n_mig_skipped;
    }
    return RT_OK;
}

int rt_comm_deal_hash(const rt_comm *c, uint64_t *hash) {
    if (!c || !hash) return fail(RT_ERR_INVALID, "rt_comm_deal_hash: null argument");
    *hash = c->cur ? c->cur->hash : 0u;
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
    {
        uint32_t W = 0, H = 0;
        int dev = 0;
        if (renderer_geometry(r, &W, &H, &dev) == RT_OK && (p->width != W || p->height != H))
            return fail(RT_ERR_INVALID, "frame size differs from the renderer's accumulator");
    }
    HIP_TRY(hipSetDevice(c->device));
    if (!c->comm_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        for (int j = 0; j < 2; ++j)
            for (hipEvent_t *e : {&c->ev_render[j], &c->ev_gather[j], &c->ev_asm[j], &c->ev_copy[j], &c->ev_mig[j]})
                HIP_TRY(hipEventCreateWithFlags(e, sync_event_flags()));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_caller, sync_event_flags()));
    }
    int rc = bind_renderer(c, r);
    if (rc != RT_OK) return rc;
    hipStream_t st = (hipStream_t)stream;
    // the deal of this frame: the interleaved one, or with RT_MULTI_BALANCED the last deal
    // balanced on measured tile costs -- kept across camera moves; each parameter set tries to
    // rebalance on its kDealAfter-th frame (then 2x, 4x, ... until every rank has costs).  Every
    // rank takes the same decisions: same frames, same parameters, same flags.
    if (c->world > 1 && !c->adopted) {   // the renderers' accumulators onto this communicator's deal
        if (!p->reset && (rc = adopt(c, r, st)) != RT_OK) return rc;
        c->adopted = true;
    }
    DealP next = c->cur;
    if (c->world > 1) {
        if (!(flags & RT_MULTI_BALANCED)) {
            next = c->interleaved;
            // re-enabling the flag later starts the balancing schedule again
            c->pkey = 0;
            c->settled = false;
        } else {
            const uint64_t key = params_key(cam, p);
            if (key != c->pkey) {
                c->pkey = key;
                c->pcalls = 0;
                c->next_try = kDealAfter;
                c->settled = false;
            }
            if (!c->settled && c->pcalls == c->next_try) {
                bool complete = false;
                // the attempt's dry-run work map runs on the communicator's stream: behind the
                // caller's frames in flight, not beside them (ADVICE r5 -- it would share the CUs
                // with them and skew the renderer's timed groups)
                HIP_TRY(hipEventRecord(c->ev_caller, st));
                HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_caller, 0));
                if ((rc = rebalance(c, r, cam, p, next, complete)) != RT_OK) {
                    // failed on every rank alike (the status words): the parameter set settles on
                    // the deal in use instead of retrying a failure every later frame
                    c->settled = true;
                    c->pcalls += 1;
                    return rc;
                }
                if (complete) c->settled = true;
                else c->next_try = c->next_try < (1u << 30) ? 2u * c->next_try : c->next_try;
            }
            c->pcalls += 1;
        }
        if (next != c->cur) {
            // tiles change owner: their running averages move along, unless this frame starts the
            // accumulation over (the reference resets it on camera motion, renderer.cpp:204-208, 237)
            if (p->reset) c->n_mig_skipped += 1;
            else if ((rc = migrate(c, r, *c->cur, *next, st)) != RT_OK) return rc;
            c->cur = next;
        }
    }
    const Deal &deal = *c->cur;
    const int k = c->slot;
    const bool peers = c->world > 1;
    std::array<hipEvent_t, 3> *tv = nullptr;
    if (flags & RT_MULTI_TIMING) {
        if (c->tev_used == c->tev.size()) {
            std::array<hipEvent_t, 3> e{};
            for (auto &x : e) HIP_TRY(hipEventCreate(&x));
            c->tev.push_back(e);
        }
        tv = &c->tev[c->tev_used++];
    }
    auto render = [&](uint32_t *out, int packed, const uint32_t *fwd_src = nullptr, uint32_t *fwd_dst = nullptr) -> int {
        if (tv) HIP_TRY(hipEventRecord((*tv)[0], st));
        int e = deal.id != 0
                    ? render_part(r, cam, p, 0, 1, deal.tiles.data() + deal.off[c->rank], deal.count(c->rank), packed, out, st,
                                  fwd_src, fwd_dst)
                    : render_part(r, cam, p, (uint32_t)c->rank, (uint32_t)c->world, nullptr, 0, packed, out, st, fwd_src,
                                  fwd_dst);
        if (e != RT_OK) return e;
        if (tv) HIP_TRY(hipEventRecord((*tv)[1], st));
        return RT_OK;
    };

    if (c->rank != 0) {
        // peers: packed tiles into slot k, then the send on the communicator's stream.  The slot
        // was last read by the send of two frames back (pipelined) -- wait for that one only.
        if (c->sent[k]) HIP_TRY(hipStreamWaitEvent(st, c->ev_gather[k], 0));
        c->slot_deal[k] = c->cur;
        if ((rc = render(c->tiles[k], 1)) != RT_OK) return rc;
        HIP_TRY(hipEventRecord(c->ev_render[k], st));
        HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_render[k], 0));
        if ((rc = gather(c, k, deal, c->comm_stream)) != RT_OK) return rc;
        HIP_TRY(hipEventRecord(c->ev_gather[k], c->comm_stream));
        c->sent[k] = true;
        if (tv) HIP_TRY(hipEventRecord((*tv)[2], c->comm_stream));
        if (!pipelined) {   // in stream order: the call's work includes the send
            HIP_TRY(hipStreamWaitEvent(st, c->ev_gather[k], 0));
            c->frames += 1;
            return RT_OK;
        }
        if (c->pending >= 0) c->frames += 1;
        c->pending = k;
        c->slot = k ^ 1;
        return RT_OK;
    }

    if (!pipelined) {
        // rank 0, flags 0: its tiles straight into rgb8_dev; the gather waits only for the caller's
        // earlier work (the previous frame's scatter read gathered[k] on the caller's stream),
        // and the peers' tiles are scattered on the caller's stream behind it
        c->slot_deal[k] = c->cur;
        if (peers) {
            HIP_TRY(hipEventRecord(c->ev_caller, st));
            HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_caller, 0));
            if ((rc = gather(c, k, deal, c->comm_stream)) != RT_OK) return rc;
            HIP_TRY(hipEventRecord(c->ev_gather[k], c->comm_stream));
        }
        if ((rc = render(rgb8_dev, 0)) != RT_OK) return rc;
        if (peers) {
            HIP_TRY(hipStreamWaitEvent(st, c->ev_gather[k], 0));
            if (tv) HIP_TRY(hipEventRecord((*tv)[2], st));
            if ((rc = scatter_peers(c, k, rgb8_dev, st)) != RT_OK) return rc;
            HIP_TRY(hipEventRecord(c->ev_copy[k], st));   // the caller's stream is done with slot k
            c->copied[k] = true;
        } else if (tv) {
            HIP_TRY(hipEventRecord((*tv)[2], st));
        }
        c->frames += 1;
        return RT_OK;
    }

    // rank 0, pipelined.  On the caller's stream: this frame's own tiles into frame[k] (which the
    // copy of two frames back read, earlier on this same stream), then the completion of the
    // previous frame (slot j: wait for its peers' scatter, copy it to rgb8_dev) -- behind the render,
    // so the render never waits for the peers.  On the communicator's stream: this frame's gather
    // and the scatter of its peers' tiles into frame[k] (after that old copy, ev_copy[k]).  At
    // world 1 the previous frame is complete when rendered and covers every pixel: the render stores
    // each pixel of frame[k] after forwarding the same pixel of frame[j] to rgb8_dev
    // (FrameArgs::fwd_*) -- no copy launch, one launch per frame as in Tick (a separate 8 MB copy
    // cost ~8 us per 1080p frame, profiles/r05/session1).
    const int j = c->pending;
    c->slot_deal[k] = c->cur;
    if (!peers && j >= 0) {
        if ((rc = render(c->frame[k], 0, c->frame[j], rgb8_dev)) != RT_OK) return rc;
        if (tv) HIP_TRY(hipEventRecord((*tv)[2], st));
        c->frames += 1;
        c->pending = k;
        c->slot = k ^ 1;
        return RT_OK;
    }
    if ((rc = render(c->frame[k], 0)) != RT_OK) return rc;
    if (peers) {
        if (c->copied[k]) HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_copy[k], 0));
        if ((rc = gather(c, k, deal, c->comm_stream)) != RT_OK) return rc;
        if (tv) HIP_TRY(hipEventRecord((*tv)[2], c->comm_stream));
        if ((rc = scatter_peers(c, k, c->frame[k], c->comm_stream)) != RT_OK) return rc;
        HIP_TRY(hipEventRecord(c->ev_asm[k], c->comm_stream));
    } else if (tv) {
        HIP_TRY(hipEventRecord((*tv)[2], st));
    }
    if (j >= 0) {
        if (peers) HIP_TRY(hipStreamWaitEvent(st, c->ev_asm[j], 0));
        HIP_TRY(hipMemcpyAsync(rgb8_dev, c->frame[j], sizeof(uint32_t) * (size_t)c->W * c->H, hipMemcpyDeviceToDevice, st));
        if (peers) {
            HIP_TRY(hipEventRecord(c->ev_copy[j], st));
            c->copied[j] = true;
        }
        c->frames += 1;
    }
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
        b += std::max(0.0f, y);
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
    if (c->rank == 0 && !rgb8_dev) return fail(RT_ERR_INVALID, "rt_multi_flush: rank 0 needs an output frame");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    const int j = c->pending;
    if (c->rank == 0) {
        if (c->world > 1) HIP_TRY(hipStreamWaitEvent(st, c->ev_asm[j], 0));
        HIP_TRY(hipMemcpyAsync(rgb8_dev, c->frame[j], sizeof(uint32_t) * (size_t)c->W * c->H, hipMemcpyDeviceToDevice, st));
        if (c->world > 1) {
            HIP_TRY(hipEventRecord(c->ev_copy[j], st));
            c->copied[j] = true;
        }
    } else {
        HIP_TRY(hipStreamWaitEvent(st, c->ev_gather[j], 0));
    }
    c->pending = -1;
    c->frames += 1;
    return RT_OK;
}

}  // extern "C"
