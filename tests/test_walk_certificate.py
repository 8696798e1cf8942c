"""The wave camera walk's exactness precondition, checked exhaustively with the oracle (CPU).

DESIGN 2.3: the walk (rt_kernels.inc wave_closest_hit_fast) returns IntersectBVH's answer R for a
camera ray -- or flags the lane and re-traces it in the reference order -- unless R lies in a box the
walk culled; and that needs R's computed t to lie more than the cull margin (2^-12) before its own
leaf box's computed entry, with R in a box that is not sticky (sticky boxes -- those above a sphere,
a quad or a sliver triangle, sine of its smallest angle under 2^-8 -- are culled only on a slab miss).  or_walk_need computes, for every
camera ray of a frame, (entry of R's leaf - t_R) / t_R from the reference traversal itself; here
every ray of every checked frame must have need < 2^-16 (16x under the margin) or a sticky R.  Frames: the BASELINE
cameras at 1080p (three frames of lens jitter each; config 4's mig29 x16 included) and the grazing
cameras aimed at the case (tests/scenes_util.grazing_cameras)."""
import numpy as np
import pytest

from scenes_util import grazing_cameras, sticky_prims

MARGIN = 2.0 ** -12    # rt_device.hip: SceneView::walk_margin (RT_WALK_MARGIN)
HEADROOM = 2.0 ** -16  # what the non-sticky answers of the checked frames stay under (4 bits below)


def _cases(rt):
    W, H = 1920, 1080
    out = [(rec, None, f"{rec}_default") for rec in ("teapotF", "mig16", "cfg3", "cfg5")]
    out += [(rec, cam, name) for name, (rec, cam) in grazing_cameras(rt, W, H).items()]
    return W, H, out


@pytest.mark.slow
def test_every_camera_ray_meets_the_walk_precondition(rt, oracle):
    W, H, cases = _cases(rt)
    report = {}
    for rec, cam, name in cases:
        prims, _ = rt.recipe_describe(rec)
        sticky = sticky_prims(rt, prims)
        o = oracle.Scene(rec, rt.DATA_DIR)
        worst = 0.0
        for frame in range(3):
            need, obj = o.walk_need(W, H, frame=frame, cam=cam, with_obj=True)
            bad = (need >= HEADROOM) & ~((obj >= 0) & sticky[np.maximum(obj, 0)])
            assert not bad.any(), (name, frame, np.flatnonzero(bad)[:5], need[bad][:5], obj[bad][:5])
            plain = (obj >= 0) & ~sticky[np.maximum(obj, 0)]
            worst = max(worst, float(need[plain].max()) if plain.any() else 0.0)
        report[name] = round(float(np.log2(worst)), 2) if worst > 0 else None
    print("log2 of the largest need over non-sticky answers:", report)


def test_sliver_answers_exist_and_are_sticky(rt, oracle):
    """The case that motivated sticky boxes: a camera ray in the plane of a mig29 wing whose
    reference answer is a sliver triangle (two corners 2e-7 apart) reported 2^-8 before its leaf
    box's entry -- past the 2^-12 margin; its primitive is classed sticky."""
    W, H = 1920, 1080
    rec, cam = grazing_cameras(rt, W, H)["mig16_wing_plane"]
    prims, _ = rt.recipe_describe(rec)
    sticky = sticky_prims(rt, prims)
    o = oracle.Scene(rec, rt.DATA_DIR)
    need, obj = o.walk_need(W, H, frame=0, cam=cam, with_obj=True)
    hot = np.flatnonzero(need >= MARGIN)
    assert len(hot) >= 1
    assert sticky[obj[hot]].all()
    assert int(sticky.sum()) > 800   # the mig29 mesh's slivers, 16 copies
