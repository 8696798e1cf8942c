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
