"""Batched Renderer::Trace / WhittedTrace through the C-ABI (rt_trace, renderer.cpp:17-72,
138-195) against the oracle's trace on the same rays, RNG states and flags: radiance and
the RNG state after the call bit for bit, shadow / bounce ray counts exact."""
import numpy as np
import pytest

from test_gpu_parity import glass_scene, random_rays, shapes_scene, sky_scene, twin_scene  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def trace_rays(o, W=320, H=180, n_random=3000, seed=5):
    cam = o.camera_rays(W, H, np.arange(0, W * H, 7, dtype=np.int32))
    rnd = random_rays(n_random, seed, origin_box=1.5)
    rays = np.concatenate([cam, rnd], 0).astype(np.float32)
    rng = np.random.default_rng(seed)
    seeds = rng.integers(1, 1 << 32, len(rays), dtype=np.uint64).astype(np.uint32)   # xorshift32: never 0
    flags = rng.integers(0, 4, len(rays)).astype(np.uint8)                             # lastSpecular, inside
    flags[: len(cam)] = 1                                                             # camera rays: defaults
    return rays, seeds, flags


def check_trace(g, o, rays, seeds, flags, depth, mode):
    import advancedgraphicsraytracer_amd as rt
    o.set_integrator(mode)
    want, wseeds, st = o.trace_rays(rays, seeds, depth=depth, flags=flags)
    rad, sd, counts, hits = g.trace(rays, seeds, depth=depth, last_specular=(flags & 1) != 0,
                                    inside=(flags & 2) != 0, mode=mode, hits=True)
    got = rad.cpu().numpy()
    bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)).any(1))[0]
    assert len(bad) == 0, (f"depth {depth} mode {mode}: {len(bad)} rays differ, max |d| "
                           f"{np.abs(got - want).max()}, first {bad[:3]}: {got[bad[:3]]} vs {want[bad[:3]]}")
    assert np.array_equal(sd.cpu().numpy().view(np.uint32), wseeds), "RNG state after the call"
    c = counts.cpu().numpy()
    assert c[0] == st["shadow"], (c, st)
    n_primary = len(rays) if depth > 0 else 0
    assert c[1] == st["isect"] - n_primary, (c, st)
    # the ray after Trace's first IntersectBVH (renderer.cpp:20)
    t, obj, u, v = (x.cpu().numpy() for x in hits)
    if depth > 0:
        wt, wobj, _, _ = o.intersect(rays)
        assert np.array_equal(obj, wobj) and np.array_equal(t.view(np.uint32), wt.view(np.uint32))
    else:
        assert (obj == -1).all() and np.array_equal(t, rays[:, 6])
    o.set_integrator(rt.MODE_PATH)


@pytest.mark.parametrize("name,depth", [("teapotF", 1), ("teapotF", 10), ("cfg3", 4), ("cfg3", 32), ("cfg5", 0),
                                        ("mig16", 3)])
def test_trace_matches_oracle(rt, oracle, torch, name, depth):
    g, o = rt.Scene.recipe(name), oracle.Scene(name, rt.DATA_DIR)
    rays, seeds, flags = trace_rays(o)
    check_trace(g, o, rays, seeds, flags, depth, rt.MODE_PATH)


@pytest.mark.parametrize("depth", [1, 20])
def test_whitted_trace_matches_oracle(rt, oracle, torch, depth):
    g, o = glass_scene(rt, oracle)
    rays, seeds, flags = trace_rays(o, 160, 120)
    check_trace(g, o, rays, seeds, flags, depth, rt.MODE_WHITTED)


@pytest.mark.parametrize("make", [sky_scene, shapes_scene])
def test_trace_textured_sky_and_extension_build(rt, oracle, torch, make):
    g, o = make(rt, oracle)
    rays, seeds, flags = trace_rays(o, 160, 100, 1500)
    check_trace(g, o, rays, seeds, flags, 6, rt.MODE_PATH)
    check_trace(g, o, rays, seeds, flags, 12, rt.MODE_WHITTED)


def test_trace_chains_like_the_global_seed(rt, oracle, torch):
    """Two calls with the returned seeds equal the oracle's two consecutive calls (the
    reference's global seed keeps advancing across Trace calls)."""
    g, o = rt.Scene.recipe("teapotF"), oracle.Scene("teapotF", rt.DATA_DIR)
    rays, seeds, _ = trace_rays(o, 64, 36, 100)
    r1, s1, _ = g.trace(rays, seeds, depth=5)
    r2, s2, _ = g.trace(rays, s1, depth=5)
    w1, ws1, _ = o.trace_rays(rays, seeds, depth=5)
    w2, ws2, _ = o.trace_rays(rays, ws1, depth=5)
    assert np.array_equal(r2.cpu().numpy(), w2) and np.array_equal(s2.cpu().numpy().view(np.uint32), ws2)
    rad, sd = rt.Renderer(g, 64, 36).Trace(rays, seeds, depth=5)
    assert np.array_equal(rad.cpu().numpy(), w1)


def test_trace_rejects_bad_arguments(rt, torch):
    g = rt.Scene.recipe("teapotF")
    with pytest.raises(rt.RTError):
        g.trace(np.zeros((4, 7), np.float32), np.ones(4, np.uint32), depth=33)
    with pytest.raises(rt.RTError):
        g.trace(np.zeros((4, 7), np.float32), np.ones(4, np.uint32), mode=rt.MODE_PACKET)
    rad, sd, c = g.trace(np.zeros((0, 7), np.float32), np.zeros(0, np.uint32))
    assert rad.shape == (0, 3)
