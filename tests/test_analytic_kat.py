"""Analytic known answers (tests/kat_analytic.py), independent of the oracle: the oracle
(CPU) and the HIP kernels (GPU) must both reproduce the closed-form t / objIdx / u / v of
Primitive.h:150-194,248-275 and the slab semantics of template/scene.h:414-450 bit for bit."""
import numpy as np
import pytest

import kat_analytic as K
from scenes_util import oracle_scene


@pytest.fixture(scope="module")
def vectors():
    v = K.vectors()
    return v


def test_vector_set_is_substantial(vectors):
    rays, T, OBJ, U, V, OCC = vectors
    assert len(rays) >= 400, len(rays)
    for pid in range(1, 5):                   # both triangles, the sphere and the plane are hit
        assert (OBJ == pid).sum() >= 10, (pid, (OBJ == pid).sum())
    assert (OBJ == -1).sum() >= 50            # misses, including the NaN-slab rays
    assert (~np.isnan(U[OBJ == 3])).sum() >= 2    # sphere hits with exactly known u, v
    assert OCC.sum() > 0 and (~OCC).sum() > 0


def test_nan_slab_rays_miss(vectors):
    """An axis-parallel ray starting on a face of TRI1's box computes (face - O) * inf = NaN,
    which std::min / std::max carry to the end: the box (and the triangle) are missed even
    though the ray runs along the triangle's edge."""
    rays, T, OBJ, *_ = vectors
    on_face = (rays[:, 0] == 0) & (rays[:, 1] == 0.5) & (rays[:, 3] == 0) & (rays[:, 4] == 0)
    assert on_face.sum() >= 2 and (OBJ[on_face] == -1).all()
    inside = (rays[:, 0] == 0.5) & (rays[:, 1] == 0.5) & (rays[:, 2] == 0) & (rays[:, 3] == 0) & (rays[:, 4] == 0) & (rays[:, 6] > 1e30)
    assert inside.sum() >= 1 and (OBJ[inside] == 1).all()


def test_oracle_matches_analytic(rt, oracle, vectors):
    prims, mats = K.scene(rt)
    o = oracle_scene(rt, oracle, prims, mats, bvh=K.bvh())
    rays, T, OBJ, U, V, OCC = vectors
    t, obj, u, v = o.intersect(rays)
    bad = K.check(t, obj, u, v, vectors)
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:3]}"
    assert np.array_equal(o.occluded(rays).astype(bool), OCC)


@pytest.mark.gpu
def test_gpu_matches_analytic(rt, vectors):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    prims, mats = K.scene(rt)
    g = rt.Scene(prims, mats, bvh=K.bvh())
    rays, T, OBJ, U, V, OCC = vectors
    t, obj, u, v = (x.cpu().numpy() for x in g.IntersectBVH(rays))
    bad = K.check(t, obj, u, v, vectors)
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:3]}"
    assert np.array_equal(g.IsOccluded(rays).cpu().numpy(), OCC)
