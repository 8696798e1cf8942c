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
struct rt_comm {
    ncclComm_t comm = nullptr;
    bool owned = false;
    int rank = 0, world = 1, device = 0;
    hipStream_t comm_stream = nullptr;     // pipelined gathers run here, beside the next render
    const rt_renderer *renderer = nullptr; // buffers below belong to this renderer's frame size
    uint32_t cap = 0;                      // packed pixels per shard
    uint32_t *tiles[2] = {nullptr, nullptr};      // this rank's packed tiles (rank 0: unused)
    uint32_t *gathered[2] = {nullptr, nullptr};   // rank 0: world x cap, slot 0 rendered in place
    hipEvent_t ev_render[2] = {nullptr, nullptr}, ev_gather[2] = {nullptr, nullptr};
    hipEvent_t ev_asm[2] = {nullptr, nullptr};   // rank 0, pipelined: frame assembled (comm stream)
    hipEvent_t ev_caller = nullptr;        // rank 0, pipelined: the caller's stream at the call, so the
                                           // unshuffle into rgb8_dev follows the caller's reads of it
    int slot = 0;
    int pending = -1;                      // slot whose gather is in flight (pipelined mode)
    uint64_t frames = 0;
    // RT_MULTI_TIMING: per frame (render start, render end, gather end) events, summed by rt_comm_timing
    std::vector<std::array<hipEvent_t, 3>> tev;
    size_t tev_used = 0;
};

namespace {

void free_buffers(rt_comm *c) {
    for (int k = 0; k < 2; ++k) {
        if (c->tiles[k]) (void)hipFree(c->tiles[k]);
        if (c->gathered[k]) (void)hipFree(c->gathered[k]);
        c->tiles[k] = c->gathered[k] = nullptr;
    }
    c->renderer = nullptr;
    c->cap = 0;
    c->pending = -1;
}

int bind_renderer(rt_comm *c, rt_renderer *r) {
    uint32_t W = 0, H = 0;
    int dev = 0;
    int rc = renderer_geometry(r, &W, &H, &dev);
    if (rc != RT_OK) return rc;
    if (dev != c->device) return fail(RT_ERR_INVALID, "renderer and communicator are on different devices");
    uint32_t cap = 0;
    rc = rt_shard_capacity(W, H, (uint32_t)c->world, &cap);
    if (rc != RT_OK) return rc;
    if (c->renderer == r && c->cap == cap) return RT_OK;
    if (c->pending >= 0) return fail(RT_ERR_INVALID, "rt_render_frame_multi: flush the pipelined frame before switching renderers");
    free_buffers(c);
    for (int k = 0; k < 2; ++k) {
        if (c->rank == 0) HIP_TRY(hipMalloc(&c->gathered[k], sizeof(uint32_t) * (size_t)cap * c->world));
        else HIP_TRY(hipMalloc(&c->tiles[k], sizeof(uint32_t) * (size_t)cap));
    }
    c->renderer = r;
    c->cap = cap;
    c->slot = 0;
    return RT_OK;
}

// the frame's one collective: every rank's packed tiles to rank 0 (rank 0's own shard was
// rendered in place into slot 0 of the gather buffer)
int gather(rt_comm *c, int k, hipStream_t st) {
    const Rccl &R = rccl();
    const size_t bytes = sizeof(uint32_t) * (size_t)c->cap;
    NCCL_TRY(R, R.group_start(), "ncclGroupStart");
    if (c->rank == 0) {
        for (int peer = 1; peer < c->world; ++peer) {
            ncclResult_t e = R.recv(c->gathered[k] + (size_t)peer * c->cap, bytes, ncclUint8, peer, c->comm, st);
            if (e != ncclSuccess) {
                (void)R.group_end();
                return comm_fail(R, e, "ncclRecv");
            }
        }
    } else {
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
    return rt_assemble_shards(r, c->gathered[k], (uint32_t)c->world, rgb8, st);
}

}  // namespace

extern "C" {

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
    if (c->owned && c->comm) (void)rccl().comm_destroy(c->comm);
    delete c;
    return RT_OK;
}

int rt_render_frame_multi(rt_renderer *r, rt_comm *c, const rt_camera *cam, const rt_frame_params *p,
                          uint32_t *rgb8_dev, uint32_t flags, void *stream) {
    if (!r || !c || !cam || !p) return fail(RT_ERR_INVALID, "rt_render_frame_multi: null argument");
    if (flags & ~(uint32_t)(RT_MULTI_PIPELINED | RT_MULTI_TIMING)) return fail(RT_ERR_INVALID, "rt_render_frame_multi: unknown flags");
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
    const int k = c->slot;
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
    rc = rt_render_shard(r, cam, p, (uint32_t)c->rank, (uint32_t)c->world, mine, st);
    if (rc != RT_OK) return rc;
    if (tv) HIP_TRY(hipEventRecord((*tv)[1], st));
    if (!pipelined) {
        if ((rc = gather(c, k, st)) != RT_OK) return rc;   // in stream order after the render
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
    if ((rc = gather(c, k, c->comm_stream)) != RT_OK) return rc;
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
