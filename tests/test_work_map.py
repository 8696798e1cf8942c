"""The dry-run work map (rt_renderer_tile_work, csrc k_render_work): per-pixel traversal counters
of a frame's rays -- closest-hit node visits / primitive tests, any-hit node visits / primitive
tests -- equal to the oracle's counts of the same rays (or_pixel_work), pixel for pixel.  The
closest-hit counters follow the reference's IntersectBVH order (template/scene.h:285-320), so
this pins the GPU's visiting ORDER, not only its answers; the any-hit counters follow the
library's farther-box-first order for IsOccluded (template/scene.h:452-487: same bool in any
order).  The map is what the balanced multi-GPU deals are cut on, so it must be deterministic
and must not touch the renderer's accumulator, frame count or ray counters."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def tile_sums(px_work, W, H):
    tx, ty = (W + 7) // 8, (H + 7) // 8
    tot = px_work[:, :4].astype(np.int64).sum(axis=1).reshape(H, W)
    pad = np.zeros((ty * 8, tx * 8), np.int64)
    pad[:H, :W] = tot
    return pad.reshape(ty, 8, tx, 8).sum(axis=(1, 3)).reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("recipe,W,H,spp,depth", [
    ("teapotF", 160, 96, 1, 1),      # config 2's workload, primary + shadow
    ("mig16", 200, 120, 1, 1),       # config 4's scene (deep tree, heavy shadow rays)
    ("cfg3", 136, 80, 2, 4),         # Mirror + Dielectric bounces
    ("cfg5", 96, 64, 4, 10),         # path tracing depth 10
])
def test_work_map_equals_oracle_counts(rt, oracle, torch, recipe, W, H, spp, depth):
    g = rt.Scene.recipe(recipe)
    o = oracle.Scene(recipe, rt.DATA_DIR)
    r = rt.Renderer(g, W, H)
    work, px = r.tile_work(spp=spp, depth=depth, frame=3, pixels=True)
    want = o.pixel_work(W, H, np.arange(W * H, dtype=np.int32), spp=spp, depth=depth, frame=3)
    bad = np.nonzero((px != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} pixels differ, first {bad[:5]}: gpu {px[bad[:3]]} oracle {want[bad[:3]]}"
    assert np.array_equal(work.astype(np.int64), tile_sums(want, W, H))
    assert want[:, 0].min() >= spp            # every sample visits the root
    # the exact pop-time cull's ceiling (counters [4] / [5]): printed for DESIGN.md
    print(f"{recipe}: pops of interior entries beyond t = {want[:, 4].sum() / max(1, want[:, 0].sum()):.4f} of "
          f"closest-hit node visits, leaf entries {want[:, 5].sum() / max(1, want[:, 0].sum()):.4f}")
    r.close()


@pytest.mark.gpu
def test_work_map_is_a_deterministic_dry_run(rt, torch):
    g = rt.Scene.recipe("mig16")
    W, H = 256, 144
    r, ref = rt.Renderer(g, W, H), rt.Renderer(g, W, H)
    for f in range(3):
        r.tick_host(spp=1, depth=1, frame=f)
        ref.tick_host(spp=1, depth=1, frame=f)
    c0, a0 = r.counters(), r.accumulator()
    w1 = r.tile_work(spp=1, depth=1, frame=3)
    w2 = r.tile_work(spp=1, depth=1, frame=3)
    assert np.array_equal(w1, w2) and w1.sum() > 0
    assert r.counters() == c0
    assert np.array_equal(r.accumulator().view(np.uint32), a0.view(np.uint32))
    # the next frame goes on exactly as if the dry run had not happened
    assert np.array_equal(r.tick_host(spp=1, depth=1, frame=3), ref.tick_host(spp=1, depth=1, frame=3))
    assert np.array_equal(r.accumulator().view(np.uint32), ref.accumulator().view(np.uint32))
    # the wave camera walk (a timed choice) does not change the map: camera rays are counted in
    # the reference order
    g.set_camera_walk(rt.WALK_WAVE)
    assert np.array_equal(r.tile_work(spp=1, depth=1, frame=3), w1)
    r.close()
    ref.close()


def test_oracle_pixel_work_counts(oracle, rt):
    """CPU: the oracle's counters -- every sample visits the root; a pixel that sees only sky
    tests the root and nothing below it; two calls agree."""
    o = oracle.Scene("teapotF", rt.DATA_DIR)
    W, H = 64, 36
    px = np.arange(W * H, dtype=np.int32)
    a = o.pixel_work(W, H, px, spp=2, depth=1, frame=0)
    b = o.pixel_work(W, H, px, spp=2, depth=1, frame=0)
    assert np.array_equal(a, b)
    assert a[:, 0].min() >= 2
    assert (a[:, 2] > 0).any()                # some shadow rays
    assert (a[:, 4] > 0).any() and not a[:, 6:].any()
