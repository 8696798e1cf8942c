"""The opt-in spatial-split BVH (rt_sbvh.cpp, RT_BVH_SBVH; reference template/scene.h:521-840)
on the CPU: structure (every primitive referenced, boxes nested, no NaN bounds, bounded
duplication) and traversal results through the oracle's IntersectBVH / IsOccluded restatement
loaded with the SBVH: closest-hit distances identical to the plain BVH's for every ray and
primitive ids identical except exact-distance ties; occlusion identical."""
import numpy as np
import pytest

from scenes_util import oracle_scene


def node_fields(nodes):
    f = nodes.view(np.float32).reshape(-1, 8)
    u = nodes.view(np.uint32).reshape(-1, 8)
    return f[:, 0:3], f[:, 3:6], u[:, 6], u[:, 7]


def check_structure(nodes, idx, n):
    mn, mx, lf, cnt = node_fields(nodes)
    assert not np.isnan(mn).any() and not np.isnan(mx).any()
    seen = np.zeros(n, bool)
    stack = [0]
    while stack:
        k = stack.pop()
        if cnt[k] > 0:
            ids = idx[lf[k]:lf[k] + cnt[k]]
            assert len(ids) == cnt[k] and (ids < n).all()
            seen[ids] = True
            continue
        for c in (lf[k], lf[k] + 1):
            if k != 0:   # the root's own box is never tested; children lie inside their parent
                assert (mn[c] >= mn[k]).all() and (mx[c] <= mx[k]).all(), (k, c)
            stack.append(c)
    assert seen.all(), "a primitive is in no leaf"
    assert len(idx) <= 2 * n


@pytest.mark.parametrize("name", ["teapotF", "cfg3"])
def test_sbvh_hits_equal_plain_bvh_except_ties(rt, oracle, name):
    prims, mats = rt.recipe_describe(name)
    nodes, idx, info = rt.build_sbvh_host(prims)
    assert info["num_refs"] == len(idx) and info["num_refs"] >= len(prims)
    check_structure(nodes, idx, len(prims))
    o_plain = oracle_scene(rt, oracle, prims, mats)
    o_sbvh = oracle_scene(rt, oracle, prims, mats, bvh=(nodes, idx))
    W, H = 480, 270
    cam = o_plain.camera_rays(W, H, np.arange(W * H, dtype=np.int32))
    rng = np.random.default_rng(4)
    O = rng.uniform(-3, 3, (20000, 3)).astype(np.float32)
    D = rng.normal(size=(20000, 3)).astype(np.float32)
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    rnd = np.concatenate([O, D, np.full((20000, 1), 1e34, np.float32)], 1).astype(np.float32)
    for rays in (cam, rnd):
        tp, op, _, _ = o_plain.intersect(rays)
        ts, os_, _, _ = o_sbvh.intersect(rays)
        assert np.array_equal(tp.view(np.uint32), ts.view(np.uint32)), "closest-hit distance differs"
        diff = op != os_
        assert diff.mean() < 1e-3, diff.sum()        # only exact ties (same t) may pick another primitive
        short = rays.copy()
        short[:, 6] = rng.uniform(0, 4, len(rays)).astype(np.float32)
        assert np.array_equal(o_plain.occluded(short), o_sbvh.occluded(short))


def test_sbvh_splits_references_on_the_big_scene(rt):
    """mig29 x16: spatial splits happen (references duplicated) within the 2N budget, and the
    tree stays within the kernels' limits (depth <= 64, leaves <= 255, nodes < 2^24)."""
    prims, _ = rt.recipe_describe("mig16")
    nodes, idx, info = rt.build_sbvh_host(prims)
    assert len(prims) < info["num_refs"] <= 2 * len(prims)
    assert info["depth"] <= 64 and info["max_leaf"] <= 255 and info["nodes_used"] < (1 << 24)
    check_structure(nodes, idx, len(prims))


def test_sbvh_splits_coincident_triangles_into_bounded_leaves(rt):
    """300 copies of one triangle share one centroid, so no SAH plane separates them: the
    builder halves such sets by index (leaves stay within the kernels' 255-primitive word,
    above 64 references a split is forced) instead of failing the scene."""
    light = rt.sphere((0, 4, -2), 0.5, 0)
    tris = [rt.triangle((0, 0, 1), (1, 0, 1), (0, 1, 1), 0) for _ in range(300)]
    nodes, idx, info = rt.build_sbvh_host([light] + tris)
    check_structure(nodes, idx, 301)
    assert info["max_leaf"] <= 64


def test_rt_bvh_environment_value_is_checked(rt, monkeypatch):
    """RT_BVH takes 'plain' or 'sbvh' only (a typo is an error, not a silent plain tree)."""
    monkeypatch.setenv("RT_BVH", "SBVH")
    with pytest.raises(rt.RTError) as e:   # refused before any device call
        rt.Scene.recipe("teapotF")
    assert e.value.code == rt.RT_ERR_INVALID and "RT_BVH" in str(e.value)
