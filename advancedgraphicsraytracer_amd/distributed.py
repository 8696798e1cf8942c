"""Multi-GPU frame rendering: screen-tile shards + one gather per frame.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Every rank
holds a full replica of the scene (<= 11 MB for the largest benchmark scene) and renders
the 8x8 tiles t with t % world == rank into a packed buffer; the frame's single
collective is an all-gather of those packed buffers (xGMI point-to-point links carry
1/world of the RGB8 frame each), after which rank 0 unshuffles them into the row-major
image.  Nothing else crosses ranks: pixels are independent in the reference's Tick
(renderer.cpp:215-244).
"""
import torch
import torch.distributed as dist


def gather_into(gathered, tiles, group=None):
    """all_gather of equal-size packed tile buffers into one flat tensor [world * cap]."""
    try:
        dist.all_gather_into_tensor(gathered, tiles, group=group)
    except (RuntimeError, NotImplementedError, AttributeError):   # backends without the fused form
        parts = list(gathered.view(-1, tiles.numel()).unbind(0))
        dist.all_gather(parts, tiles, group=group)


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
        self.tiles = torch.zeros(self.cap, dtype=torch.int32, device=dev)
        self.gathered = torch.zeros(self.world * self.cap, dtype=torch.int32, device=dev)
        self.frame = torch.zeros(renderer.width * renderer.height, dtype=torch.int32, device=dev)

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
        self.render_local(spp, depth, frame, stream)
        return self.exchange(stream)
