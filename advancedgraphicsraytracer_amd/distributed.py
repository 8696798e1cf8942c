"""Multi-GPU frame rendering: screen-tile shards + one gather per frame.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Every rank
holds a full replica of the scene (<= 11 MB for the largest benchmark scene) and renders
the 8x8 tiles t with t % world == rank into a packed buffer; the frame's single
collective gathers those packed buffers to rank 0 (each rank's xGMI link to rank 0 carries
1/world of the RGB8 frame; SURVEY.md 5: gather-to-root, not a ring), after which rank 0
unshuffles them into the row-major image.  Nothing else crosses ranks: pixels are independent in the reference's Tick
(renderer.cpp:215-244).
"""
import torch
import torch.distributed as dist


def gather_into(gathered, tiles, group=None, async_op=False):
    """Gather of equal-size packed tile buffers to rank 0, into one flat tensor [world * cap]
    there (other ranks only send: 1/world of the frame each over its xGMI link to rank 0,
    instead of the world-fold traffic of an all-gather).  With async_op the work handle is
    returned (wait() orders the caller's current stream after the collective, as
    ProcessGroupNCCL does).  Backends without gather fall back to an all-gather."""
    rank = dist.get_rank(group)
    dst = dist.get_global_rank(group, 0) if group is not None else 0
    parts = list(gathered.view(-1, tiles.numel()).unbind(0)) if rank == 0 else None
    try:
        return dist.gather(tiles, gather_list=parts, dst=dst, group=group, async_op=async_op)
    except (RuntimeError, NotImplementedError, AttributeError, ValueError):
        try:
            return dist.all_gather_into_tensor(gathered, tiles, group=group, async_op=async_op)
        except (RuntimeError, NotImplementedError, AttributeError, ValueError):
            parts = list(gathered.view(-1, tiles.numel()).unbind(0))
            return dist.all_gather(parts, tiles, group=group, async_op=async_op)


class ShardedFrame:
    """Renders frames of `renderer` tile-sharded across the ranks of `group`.

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
        self._slot = 0
        self._pending = None      # (work, slot, stream) of the frame whose gather is in flight

    def render_local(self, spp=1, depth=10, frame=0, stream=None):
        self.r.render_shard(self.tiles, self.rank, self.world, spp=spp, depth=depth, frame=frame, stream=stream)

    def exchange(self, stream=None):
        gather_into(self.gathered, self.tiles, self.group)
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
        work = gather_into(self._gathered[k], self._tiles[k], self.group, async_op=True)
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
