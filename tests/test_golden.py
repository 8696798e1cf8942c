"""Committed golden fixtures (tests/golden/, made by tests/golden/make_fixtures.py from the
pinned oracle): the oracle must keep reproducing them (CPU), and the HIP kernels must match
them (GPU) -- bit-exact ids/t/u/v, RGB8 frame CRCs and ray counts."""
import json
import os
import zlib

import numpy as np
import pytest

from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")


def load_hits():
    return np.load(os.path.join(GOLD, "teapotF_1080p_hits.npz"))


def frames():
    with open(os.path.join(GOLD, "frames.json")) as f:
        return json.load(f)


MODES = {"path": 0, "whitted": 1, "packet": 2}


def parse_key(key):
    """'{recipe}_{W}x{H}_spp{n}_d{depth}[_whitted|_packet]' -> (recipe, W, H, spp, depth, mode)"""
    parts = key.split("_")
    mode = MODES[parts[4]] if len(parts) > 4 else 0
    recipe, size, spp, depth = parts[:4]
    W, H = map(int, size.split("x"))
    return recipe, W, H, int(spp[3:]), int(depth[1:]), mode


def test_oracle_reproduces_golden_hits(oracle, rt):
    g = load_hits()
    s = oracle.Scene("teapotF", rt.DATA_DIR)
    rays = s.camera_rays(1920, 1080, g["pixels"])
    assert np.array_equal(rays.view(np.uint32), g["rays"].view(np.uint32))
    t, obj, u, v = s.intersect(rays)
    assert np.array_equal(obj, g["obj"]) and np.array_equal(t.view(np.uint32), g["t"].view(np.uint32))
    assert np.array_equal(s.occluded(g["occl_rays"]), g["occluded"])


@pytest.mark.parametrize("key", ["teapotF_320x180_spp1_d10", "cfg3_256x144_spp4_d4", "mig16_480x270_spp1_d1",
                                 "cfg3_256x144_spp1_d20_whitted", "teapotF_320x180_spp1_d20_whitted",
                                 "teapotF_320x180_spp1_d10_packet", "cfg3_250x140_spp2_d4_packet"])
def test_oracle_reproduces_golden_frames(oracle, rt, key):
    recipe, W, H, spp, depth, mode = parse_key(key)
    want = frames()[key]
    s = oracle.Scene(recipe, rt.DATA_DIR)
    s.set_integrator(mode)
    acc = np.zeros((W * H, 4), np.float32)
    rgb, st = s.tick(W, H, acc, spp=spp, depth=depth, frame=0)
    assert zlib.crc32(rgb.astype("<u4").tobytes()) == want["rgb8_crc32"]
    assert st["shadow"] == want["shadow"]


@pytest.mark.gpu
def test_gpu_matches_golden_hits(rt):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = load_hits()
    sc = rt.Scene.recipe("teapotF")
    t, obj, u, v = (x.cpu().numpy() for x in sc.IntersectBVH(g["rays"]))
    assert np.array_equal(obj, g["obj"])
    assert np.array_equal(t.view(np.uint32), g["t"].view(np.uint32))
    hit = g["obj"] >= 0
    assert np.array_equal(u[hit].view(np.uint32), g["u"][hit].view(np.uint32))
    assert np.array_equal(sc.IsOccluded(g["occl_rays"]).cpu().numpy(), g["occluded"].astype(bool))


@pytest.mark.gpu
@pytest.mark.parametrize("key", sorted(json.load(open(os.path.join(GOLD, "frames.json")))))
def test_gpu_matches_golden_frames(rt, key):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    recipe, W, H, spp, depth, mode = parse_key(key)
    want = frames()[key]
    sc = rt.Scene.recipe(recipe)
    r = rt.Renderer(sc, W, H)
    r.mode = mode
    rgb = r.tick_host(spp=spp, depth=depth, frame=0)
    c = r.counters()
    assert c["shadow"] == want["shadow"] and c["bounce"] == want["bounce"]
    assert zlib.crc32(rgb.astype("<u4").tobytes()) == want["rgb8_crc32"]
    acc = r.accumulator()
    assert abs(float(acc[:, :3].astype(np.float64).sum()) - want["acc_sum"]) <= 1e-4 * W * H


def load_kat():
    return np.load(os.path.join(GOLD, "prim_kat.npz"))


def test_oracle_reproduces_prim_kat(oracle, rt):
    """Primitive known answers (tests/scenes_util.py: vertices, shared edges, exact ties,
    grazing / in-plane rays, t ~ EPS, inside / tangent spheres, planes, NaN slabs)."""
    from scenes_util import kat_rays, kat_scene, oracle_scene
    g = load_kat()
    rays = kat_rays()
    assert np.array_equal(rays.view(np.uint32), g["rays"].view(np.uint32))
    o = oracle_scene(rt, oracle, *kat_scene(rt))
    t, obj, u, v = o.intersect(rays)
    assert np.array_equal(obj, g["obj"])
    for a, k in ((t, "t"), (u, "u"), (v, "v")):
        assert np.array_equal(a.view(np.uint32), g[k].view(np.uint32)), k
    assert np.array_equal(o.occluded(rays), g["occluded"])
    # the set exercises the tie rules: brute force (id order) and the BVH order disagree
    _, ob, _, _ = o.intersect(rays, brute=True)
    assert (ob != obj).sum() > 0


@pytest.mark.gpu
def test_gpu_matches_prim_kat(rt):
    from scenes_util import kat_scene
    g = load_kat()
    s = rt.Scene(*kat_scene(rt))
    t, obj, u, v = (x.cpu().numpy() for x in s.IntersectBVH(g["rays"]))
    assert np.array_equal(obj, g["obj"]), f"{(obj != g['obj']).sum()} objIdx mismatches"
    assert np.array_equal(t.view(np.uint32), g["t"].view(np.uint32))
    hit = g["obj"] >= 0
    assert np.array_equal(u[hit].view(np.uint32), g["u"][hit].view(np.uint32))
    assert np.array_equal(v[hit].view(np.uint32), g["v"][hit].view(np.uint32))
    occ = s.IsOccluded(g["rays"]).cpu().numpy()
    assert np.array_equal(occ, g["occluded"].astype(bool))
    hh = s.intersect_host(g["rays"])
    assert np.array_equal(hh["obj"], g["obj"])
