"""Screen-tile sharding of a frame across ranks.

The frame is cut into 8x8 tiles (one wave64 each, the reference's 64-ray packet,
Ray.h:3-5); tile t belongs to rank t % world_size (round-robin interleave keeps the
centre-heavy teapot scenes balanced).  A rank renders its tiles into a packed buffer
[local_tile][64]; one collective per frame gathers the packed buffers and rank 0
unshuffles them (rt_assemble_shards on the GPU, assemble_host below for CPU checks).
"""
import numpy as np

TILE = 8


def tile_grid(width, height):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def shard_capacity(width, height, world):
    tx, ty = tile_grid(width, height)
    return -(-(tx * ty) // world) * TILE * TILE


def shard_pixels(width, height, shard, world):
    """Pixel index (x + y*W) of every packed slot of a shard, -1 for slots outside the frame."""
    tx, ty = tile_grid(width, height)
    tiles = np.arange(shard, tx * ty, world)
    lane = np.arange(TILE * TILE)
    x = (tiles[:, None] % tx) * TILE + (lane[None, :] & 7)
    y = (tiles[:, None] // tx) * TILE + (lane[None, :] >> 3)
    px = np.where((x < width) & (y < height), x + y * width, -1).reshape(-1)
    out = np.full(shard_capacity(width, height, world), -1, np.int64)
    out[:px.size] = px
    return out


def assemble_host(gathered, width, height, world):
    """gathered: [world, capacity] packed shard buffers -> [H*W] frame."""
    cap = shard_capacity(width, height, world)
    gathered = np.asarray(gathered).reshape(world, cap)
    frame = np.zeros(width * height, gathered.dtype)
    for s in range(world):
        px = shard_pixels(width, height, s, world)
        ok = px >= 0
        frame[px[ok]] = gathered[s][ok]
    return frame


# ---- explicit deals (rt_tile_deal / rt_render_shard_tiles / rt_assemble_tiles)
def _morton(x, y):
    m = np.zeros_like(x, dtype=np.uint64)
    for b in range(16):
        m |= ((x >> b) & 1).astype(np.uint64) << np.uint64(2 * b)
        m |= ((y >> b) & 1).astype(np.uint64) << np.uint64(2 * b + 1)
    return m


def tile_deal_host(width, height, num_shards, cost=None):
    """Host mirror of rt_tile_deal: the tiles in Morton order of (tx, ty), cut into num_shards
    runs of equal summed cost (boundary at the prefix nearest to k/num_shards of the total)."""
    tx, ty = tile_grid(width, height)
    n = tx * ty
    t = np.arange(n)
    tiles = t[np.argsort(_morton(t % tx, t // tx), kind="stable")].astype(np.uint32)
    c = np.ones(n) if cost is None else np.asarray(cost, np.float64)[tiles]
    prefix = np.concatenate([[0.0], np.cumsum(c)])
    total = prefix[-1]
    off = [0]
    for k in range(1, num_shards):
        target = total * k / num_shards
        b = int(np.searchsorted(prefix, target, side="left"))
        if 0 < b <= n and target - prefix[b - 1] < prefix[b] - target:
            b -= 1
        off.append(min(n, max(b, off[-1])))
    off.append(n)
    return tiles, np.asarray(off, np.uint32)


def assemble_host_deal(gathered, width, height, stride, deal_tiles, deal_off):
    """gathered: [num_shards * stride] packed shards of an explicit deal -> [H*W] frame."""
    tx, _ = tile_grid(width, height)
    frame = np.zeros(width * height, np.asarray(gathered).dtype)
    g = np.asarray(gathered).reshape(-1)
    lane = np.arange(TILE * TILE)
    for k in range(len(deal_off) - 1):
        for i, t in enumerate(deal_tiles[deal_off[k]:deal_off[k + 1]]):
            x = (t % tx) * TILE + (lane & 7)
            y = (t // tx) * TILE + (lane >> 3)
            ok = (x < width) & (y < height)
            frame[(x + y * width)[ok]] = g[k * stride + i * 64 + lane[ok]]
    return frame
