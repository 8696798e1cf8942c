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


# ---- path-traced radiance subsets and geometry digests
def load_pt():
    return np.load(os.path.join(GOLD, "pt_subsets.npz"))


def geometry():
    with open(os.path.join(GOLD, "geometry.json")) as f:
        return json.load(f)


PT_KEYS = ["teapotF_spp1_d10", "cfg3_spp4_d4", "cfg5_spp16_d10"]


def parse_pt(key):
    recipe, spp, depth = key.split("_")
    return recipe, int(spp[3:]), int(depth[1:])


@pytest.mark.parametrize("recipe", ["teapotF", "cfg3", "cfg5", "mig16", "default"])
def test_geometry_digests(rt, oracle, recipe):
    """The recipe's primitive records after the OBJ load, and the plain BVH (library host build
    and oracle) hash to the committed digests."""
    import sys
    sys.path.insert(0, GOLD)
    from make_fixtures import bvh_digest, prims_digest
    want = geometry()[recipe]
    prims, _ = rt.recipe_describe(recipe)
    assert len(prims) == want["prims"] and prims_digest(prims) == want["prims_sha256"]
    nodes, idx, info = rt.build_bvh_host(prims)
    nodes = nodes.copy()
    nodes[1] = 0
    assert info["nodes_used"] == want["nodes_used"] and info["depth"] == want["depth"]
    assert bvh_digest(nodes[:want["nodes_used"]], idx) == want["bvh_sha256"]
    o = oracle.Scene(recipe, rt.DATA_DIR)
    on = o.nodes().copy()
    on[1] = 0
    assert bvh_digest(on, o.indices()) == want["bvh_sha256"]


@pytest.mark.parametrize("key", PT_KEYS)
def test_oracle_reproduces_pt_subsets(oracle, rt, key):
    recipe, spp, depth = parse_pt(key)
    g = load_pt()
    px = g[key + "_pixels"]
    s = oracle.Scene(recipe, rt.DATA_DIR)
    rgb, _ = s.trace_pixels(1920, 1080, px, spp=spp, depth=depth, frame=0)
    assert np.array_equal(rgb.view(np.uint32), g[key + "_rgb"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("key", PT_KEYS)
def test_gpu_matches_golden_pt_subsets(rt, key):
    """Full 1920x1080 frame 0 on the GPU (wavefront path tracer): the accumulator at the subset's
    pixels equals the committed Renderer::Trace radiance bit for bit (the first frame's running
    average is the frame's sample mean itself)."""
    recipe, spp, depth = parse_pt(key)
    g = load_pt()
    px, want = g[key + "_pixels"], g[key + "_rgb"]
    r = rt.Renderer(rt.Scene.recipe(recipe), 1920, 1080)
    r.tick_host(spp=spp, depth=depth, frame=0, reset=True)
    acc = r.accumulator()
    got = acc[px, :3]
    bad = np.flatnonzero((got.view(np.uint32) != want.view(np.uint32)).any(axis=1))
    assert bad.size == 0, f"{bad.size} of {px.size} pixels differ, first {px[bad[:5]]}"
    assert np.array_equal(acc[px, 3], np.ones(px.size, np.float32))
