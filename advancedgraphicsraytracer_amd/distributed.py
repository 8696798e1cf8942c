"""Multi-GPU frame rendering: screen-tile shards + one gather per frame.

One process per GPU.  Every rank holds a full replica of the scene (<= 11 MB for the
largest benchmark scene) and renders the 8x8 tiles t with t % world == rank into a packed
buffer; the frame's single collective gathers those packed buffers to rank 0 (each rank's
xGMI link to rank 0 carries 1/world of the RGB8 frame; SURVEY.md 5: gather-to-root, not a
ring), after which rank 0 unshuffles them into the row-major image.  Nothing else crosses
ranks: pixels are independent in the reference's Tick (renderer.cpp:215-244).

Two front-ends with the same render / submit / flush interface:

* NativeShardedFrame -- the product path on GPUs: librtamd.so's rt_render_frame_multi, the
  RCCL gather issued from C++ on the renderer's stream (rt_comm, include/rt_amd.h); the
  process group only hands the RCCL unique id from rank 0 to the others;
* ShardedFrame -- the same shard / gather / assemble through torch.distributed, for any
  renderer with the shard interface (the gloo CPU tests run it with an oracle-backed one).
"""
import ctypes as C

import torch
import torch.distributed as dist


def _exchange_for(group, tensor):
    """The gather this backend runs, chosen once: dist.gather to rank 0 (NCCL/RCCL, and gloo
    on CPU tensors); gloo holding device tensors stages through host memory.  Errors are
    never caught here: a failed collective must fail on every rank, not turn into a
    different collective its peers never enter."""
    backend = dist.get_backend(group)
    if backend == "gloo" and tensor.device.type != "cpu":
        return "gloo_staged"
    return "gather"


def gather_into(gathered, tiles, group=None, async_op=False, how="gather"):
    """Gather of equal-size packed tile buffers to rank 0, into one flat tensor [world * cap]
    there (other ranks only send: 1/world of the frame each over its link to rank 0).  With
    async_op the work handle is returned (wait() orders the caller's current stream after
    the collective, as ProcessGroupNCCL does)."""
    rank = dist.get_rank(group)
    dst = dist.get_global_rank(group, 0) if group is not None else 0
    if how == "gloo_staged":   # gloo gathers host tensors only: stage through host memory
        host = tiles.cpu()
        parts = list(torch.empty((dist.get_world_size(group), host.numel()), dtype=host.dtype).unbind(0)) \
            if rank == 0 else None
        dist.gather(host, gather_list=parts, dst=dst, group=group)
        if rank == 0:
            gathered.copy_(torch.cat(parts).to(gathered.device))
        return None
    parts = list(gathered.view(-1, tiles.numel()).unbind(0)) if rank == 0 else None
    return dist.gather(tiles, gather_list=parts, dst=dst, group=group, async_op=async_op)


class ShardedFrame:
    """Renders frames of `renderer` tile-sharded across the ranks of `group` (torch.distributed).

    renderer must provide shard_capacity(world), render_shard(out, shard, world, ...),
    assemble(gathered, world, out, ...), width and height (advancedgraphicsraytracer_amd.Renderer).
    """

    def __init__(self, renderer, group=None, device=None):
        self.r = renderer
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.cap = renderer.shard_capacity(self.world)
        dev = device if device is not None else torch.device("cpu")
        # two packed-tile / gathered buffers: the pipelined path (submit) renders frame i+1
        # into one while frame i's gather still reads the other
        self._tiles = [torch.zeros(self.cap, dtype=torch.int32, device=dev) for _ in range(2)]
        self._gathered = [torch.zeros(self.world * self.cap, dtype=torch.int32, device=dev) for _ in range(2)]
        self.tiles, self.gathered = self._tiles[0], self._gathered[0]
        self.frame = torch.zeros(renderer.width * renderer.height, dtype=torch.int32, device=dev)
        self._how = _exchange_for(group, self.tiles)
        self._slot = 0
        self._pending = None      # (work, slot) of the frame whose gather is in flight

    def render_local(self, spp=1, depth=10, frame=0, stream=None):
        self.r.render_shard(self.tiles, self.rank, self.world, spp=spp, depth=depth, frame=frame, stream=stream)

    def exchange(self, stream=None):
        gather_into(self.gathered, self.tiles, self.group, how=self._how)
        if self.rank == 0:
            self.r.assemble(self.gathered, self.world, self.frame, stream=stream)
            return self.frame
        return None

    def render(self, spp=1, depth=10, frame=0, stream=None):
        """One frame: local tiles, one gather, rank-0 assembly.  Returns the frame on rank 0."""
        self.flush(stream)
        self.render_local(spp, depth, frame, stream)
        return self.exchange(stream)

    def submit(self, spp=1, depth=10, frame=0, stream=None, events=None):
        """Pipelined frame: render this frame's tiles, start its gather asynchronously and
        complete the previous frame (wait for its gather, rank-0 assembly).  The gather of
        frame i overlaps the rendering of frame i+1; every frame still gets exactly one
        collective.  Returns the completed previous frame on rank 0 (None before the
        first completion, and on other ranks); flush() completes the last one.
        GPU tensors: call under torch.cuda.stream(s) with stream = s.cuda_stream, so the
        collective is ordered after the render.  events = (start, end) torch.cuda.Events
        recorded around the render launch."""
        k = self._slot
        if events is not None:
            events[0].record()
        self.r.render_shard(self._tiles[k], self.rank, self.world, spp=spp, depth=depth, frame=frame, stream=stream)
        if events is not None:
            events[1].record()
        work = gather_into(self._gathered[k], self._tiles[k], self.group, async_op=True, how=self._how)
        done = self.flush(stream)
        self._pending = (work, k)
        self._slot = k ^ 1
        return done

    def flush(self, stream=None):
        """Complete the frame whose gather is in flight (if any): the caller's stream waits
        for the collective, rank 0 assembles.  Returns the frame on rank 0."""
        if self._pending is None:
            return None
        work, k = self._pending
        self._pending = None
        if work is not None:
            work.wait()
        if self.rank == 0:
            self.r.assemble(self._gathered[k], self.world, self.frame, stream=stream)
            return self.frame
        return None

    def set_timing(self, on):
        pass

    def timing(self):
        return None

    def close(self):
        pass


class NativeCommUnavailable(RuntimeError):
    """The C++ RCCL communicator could not be set up; raised on every rank of the group
    together, so the caller can fall back to ShardedFrame (the same gather through
    torch.distributed) without any rank being left inside a collective."""


class NativeShardedFrame:
    """Multi-GPU frames through the C-ABI: rt_render_frame_multi renders this rank's tiles and
    runs the frame's RCCL gather from C++ (rt_multi.cpp); rank 0 assembles.  Same interface
    as ShardedFrame.  The process group (any backend) carries only the RCCL unique id."""

    def __init__(self, renderer, group=None, device=None, timing=False, balanced=False):
        from . import RT_COMM_ID_BYTES, MULTI_BALANCED, MULTI_PIPELINED, MULTI_TIMING, _check, lib
        self.L, self._check = lib(), _check
        self.r = renderer
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device("cuda", renderer.scene.device) if device is None else torch.device(device)
        # Set-up fails on every rank together (NativeCommUnavailable), never on one rank while
        # its peers wait in a collective: rank 0's unique-id failure is broadcast as None, and
        # every rank's rt_comm_create result is min-reduced before anyone goes on.
        uid = (C.c_uint8 * RT_COMM_ID_BYTES)()
        box = [None]
        if self.rank == 0:
            rc = self.L.rt_comm_unique_id(uid)
            box = [bytes(uid) if rc == 0 else None]
            err = "" if rc == 0 else self.L.rt_last_error().decode(errors="replace")
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if box[0] is None:
            raise NativeCommUnavailable("rt_comm_unique_id failed on rank 0" + (f": {err}" if self.rank == 0 else ""))
        uid = (C.c_uint8 * RT_COMM_ID_BYTES).from_buffer_copy(box[0])
        self.h = C.c_void_p()
        rc = self.L.rt_comm_create(uid, self.rank, self.world, self.device.index or 0, C.byref(self.h))
        err = "" if rc == 0 else self.L.rt_last_error().decode(errors="replace")
        ok = torch.tensor([1 if rc == 0 else 0], device=self.device if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if not int(ok.item()):
            if rc == 0:
                self.L.rt_comm_destroy(self.h)
            self.h = None
            raise NativeCommUnavailable(f"rt_comm_create failed on some rank (this rank: {err or 'ok'})")
        self.frame = torch.zeros(renderer.width * renderer.height, dtype=torch.int32, device=self.device)
        self._pipelined, self._timing_flag = MULTI_PIPELINED, (MULTI_TIMING if timing else 0)
        # RT_MULTI_BALANCED: the cost-balanced compact tile deal from a parameter set's 7th frame on
        self._deal_flag = MULTI_BALANCED if balanced else 0
        self._pending = False

    def _stream(self, stream):
        return stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream

    def _call(self, spp, depth, frame, stream, flags):
        p = self.r.params(spp, depth, frame)
        out = C.c_void_p(self.frame.data_ptr()) if self.rank == 0 else None
        self._check(self.L.rt_render_frame_multi(self.r.h, self.h, C.byref(self.r.camera), C.byref(p), out,
                                                 flags | self._timing_flag | self._deal_flag,
                                                 C.c_void_p(self._stream(stream))))

    def render(self, spp=1, depth=10, frame=0, stream=None):
        """One frame, in stream order: render, gather, rank-0 assembly.  The frame on rank 0."""
        self.flush(stream)
        self._call(spp, depth, frame, stream, 0)
        return self.frame if self.rank == 0 else None

    def submit(self, spp=1, depth=10, frame=0, stream=None, events=None):
        """Pipelined: this frame's gather runs on the communicator's stream beside the next
        render; returns the previous frame on rank 0 (None on the first call / other ranks)."""
        if events is not None:
            events[0].record()
        self._call(spp, depth, frame, stream, self._pipelined)
        if events is not None:
            events[1].record()
        had, self._pending = self._pending, True
        return self.frame if (had and self.rank == 0) else None

    def flush(self, stream=None):
        if not self._pending:
            return None
        out = C.c_void_p(self.frame.data_ptr()) if self.rank == 0 else None
        self._check(self.L.rt_multi_flush(self.r.h, self.h, out, C.c_void_p(self._stream(stream))))
        self._pending = False
        return self.frame if self.rank == 0 else None

    def set_timing(self, on):
        """Record HIP events around every following frame's render and gather (RT_MULTI_TIMING)."""
        from . import MULTI_TIMING
        self._timing_flag = MULTI_TIMING if on else 0

    def timing(self):
        """(render ms, gather ms, frames) summed over the timed frames since the last call."""
        a, b, n = C.c_double(), C.c_double(), C.c_uint64()
        self._check(self.L.rt_comm_timing(self.h, C.byref(a), C.byref(b), C.byref(n)))
        return a.value, b.value, n.value

    def deal_info(self):
        """The deal frames are rendered under now (rt_comm_deal_info): {balanced, tiles, deals_built,
        exchanges, moves, moves_skipped_on_reset}."""
        b, t, st, h = C.c_int(), C.c_uint32(), (C.c_uint64 * 4)(), C.c_uint64()
        self._check(self.L.rt_comm_deal_info(self.h, C.byref(b), C.byref(t), None, st))
        self._check(self.L.rt_comm_deal_hash(self.h, C.byref(h)))
        return {"balanced": b.value, "tiles": t.value, "deals_built": int(st[0]), "exchanges": int(st[1]),
                "moves": int(st[2]), "moves_skipped_on_reset": int(st[3]), "hash": f"{h.value:016x}"}

    def close(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.L.rt_comm_destroy(h)
            self.h = None

    __del__ = close
