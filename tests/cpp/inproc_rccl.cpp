// inproc_rccl.cpp -- TEST-ONLY stand-in for librccl.so.1 that lets several ranks of
// rt_render_frame_multi live as threads of ONE process on ONE GPU (real RCCL refuses two ranks
// on one device), so the rank != 0 branches of csrc/rt_multi.cpp (the send, rank 0's peer
// receive loop, the double-buffered tiles, the pipelined waits) run under `-m gpu`.
// Selected with RT_RCCL_LIB=<path of this library> (csrc/rt_multi.cpp tries it first); never
// shipped or loaded by the product.
//
// Semantics, the subset rt_multi.cpp uses: ncclGetUniqueId / ncclCommInitRank (a rendezvous
// of `nranks` threads on the id) / ncclCommDestroy / ncclCommCount / ncclCommUserRank,
// ncclGroupStart / ncclGroupEnd and ncclSend / ncclRecv inside or outside a group.  At
// ncclGroupEnd a thread first posts its sends (an event recorded on the send stream after the
// caller's earlier work), then serves its receives in order -- the receive stream waits for
// the matching send's event and copies device-to-device -- and finally makes each send stream
// wait for its receiver's copy, as NCCL completes a send only once the data left the buffer.
// Matching is FIFO per (sender, receiver) pair, as NCCL's point-to-point ordering.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct SendRec {
    const void *buf = nullptr;
    size_t bytes = 0;
    hipEvent_t sent = nullptr;     // recorded on the sender's stream: the data is ready
    hipEvent_t copied = nullptr;   // recorded on the receiver's stream: the data has left
    bool done = false;
};

struct Group {
    int nranks = 0, joined = 0;
    std::mutex m;
    std::condition_variable cv;
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<SendRec>>> chan;   // (src, dst) -> sends
};

std::mutex g_reg;
std::map<std::string, std::shared_ptr<Group>> g_groups;
constexpr auto kTimeout = std::chrono::seconds(60);

struct Op {
    bool send;
    void *buf;
    size_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

}  // namespace

struct ncclComm {
    std::shared_ptr<Group> g;
    std::string key;
    int rank = 0, nranks = 1;
    std::vector<hipEvent_t> events;   // kept until the communicator is destroyed
};

namespace {

hipEvent_t new_event(ncclComm *c) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    c->events.push_back(e);
    return e;
}

ncclResult_t run_ops(std::vector<Op> &ops) {
    std::vector<std::shared_ptr<SendRec>> posted;
    for (const Op &o : ops) {   // 1. post every send
        if (!o.send) continue;
        auto rec = std::make_shared<SendRec>();
        rec->buf = o.buf;
        rec->bytes = o.bytes;
        rec->sent = new_event(o.comm);
        if (!rec->sent || hipEventRecord(rec->sent, o.stream) != hipSuccess) return ncclUnhandledCudaError;
        Group &g = *o.comm->g;
        {
            std::lock_guard<std::mutex> lk(g.m);
            g.chan[{o.comm->rank, o.peer}].push_back(rec);
        }
        g.cv.notify_all();
        posted.push_back(rec);
    }
    for (const Op &o : ops) {   // 2. serve the receives, in order
        if (o.send) continue;
        Group &g = *o.comm->g;
        std::shared_ptr<SendRec> rec;
        {
            std::unique_lock<std::mutex> lk(g.m);
            auto &q = g.chan[{o.peer, o.comm->rank}];
            if (!g.cv.wait_for(lk, kTimeout, [&] { return !q.empty(); })) return ncclSystemError;
            rec = q.front();
            q.pop_front();
        }
        if (rec->bytes != o.bytes) return ncclInvalidUsage;
        if (hipStreamWaitEvent(o.stream, rec->sent, 0) != hipSuccess) return ncclUnhandledCudaError;
        if (o.bytes && hipMemcpyAsync(o.buf, rec->buf, o.bytes, hipMemcpyDeviceToDevice, o.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        hipEvent_t done = new_event(o.comm);
        if (!done || hipEventRecord(done, o.stream) != hipSuccess) return ncclUnhandledCudaError;
        {
            std::lock_guard<std::mutex> lk(g.m);
            rec->copied = done;
            rec->done = true;
        }
        g.cv.notify_all();
    }
    size_t i = 0;
    for (const Op &o : ops) {   // 3. a send completes once its data has been copied out
        if (!o.send) continue;
        std::shared_ptr<SendRec> rec = posted[i++];
        Group &g = *o.comm->g;
        {
            std::unique_lock<std::mutex> lk(g.m);
            if (!g.cv.wait_for(lk, kTimeout, [&] { return rec->done; })) return ncclSystemError;
        }
        if (hipStreamWaitEvent(o.stream, rec->copied, 0) != hipSuccess) return ncclUnhandledCudaError;
    }
    return ncclSuccess;
}

ncclResult_t enqueue(Op o) {
    if (!o.comm || o.peer < 0 || o.peer >= o.comm->nranks || o.peer == o.comm->rank) return ncclInvalidArgument;
    if (t_depth > 0) {
        t_ops.push_back(o);
        return ncclSuccess;
    }
    std::vector<Op> one{o};
    return run_ops(one);
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    static std::atomic<unsigned> n{0};
    std::memset(id->internal, 0, sizeof(id->internal));
    std::snprintf(id->internal, sizeof(id->internal), "inproc-%p-%u", (void *)&n, n.fetch_add(1));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    std::shared_ptr<Group> g;
    {
        std::lock_guard<std::mutex> lk(g_reg);
        auto &slot = g_groups[key];
        if (!slot) {
            slot = std::make_shared<Group>();
            slot->nranks = nranks;
        }
        g = slot;
    }
    if (g->nranks != nranks) return ncclInvalidUsage;
    {
        std::unique_lock<std::mutex> lk(g->m);
        g->joined += 1;
        g->cv.notify_all();
        if (!g->cv.wait_for(lk, kTimeout, [&] { return g->joined >= g->nranks; })) return ncclSystemError;
    }
    ncclComm *c = new ncclComm();
    c->g = g;
    c->key = key;
    c->rank = rank;
    c->nranks = nranks;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : comm->events) (void)hipEventDestroy(e);
    {
        std::lock_guard<std::mutex> lk(g_reg);
        auto it = g_groups.find(comm->key);
        if (it != g_groups.end() && it->second == comm->g && comm->g.use_count() <= 2) g_groups.erase(it);
    }
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int *count) {
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->nranks;
    return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int *rank) {
    if (!comm || !rank) return ncclInvalidArgument;
    *rank = comm->rank;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    t_depth += 1;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_ops(ops);
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream) {
    const size_t tb = type_bytes(type);
    if (!tb) return ncclInvalidArgument;
    return enqueue(Op{true, const_cast<void *>(buf), count * tb, peer, comm, stream});
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream) {
    const size_t tb = type_bytes(type);
    if (!tb) return ncclInvalidArgument;
    return enqueue(Op{false, buf, count * tb, peer, comm, stream});
}

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "no error (in-process stand-in)";
    case ncclInvalidArgument: return "invalid argument (in-process stand-in)";
    case ncclInvalidUsage: return "invalid usage: size mismatch or bad group (in-process stand-in)";
    case ncclSystemError: return "rendezvous / matching timed out (in-process stand-in)";
    default: return "HIP error (in-process stand-in)";
    }
}

}  // extern "C"
