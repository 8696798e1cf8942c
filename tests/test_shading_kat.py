"""Closed-form known answers for Renderer::Trace / WhittedTrace (renderer.cpp:17-72, 138-195),
independent of the oracle: rays whose whole path draws no random number -- the sky, the light
seen directly, a mirror at normal incidence -- so the radiance is one float product per channel:

    sky     = float3(0x40, 0x60, 0x80) * SKYDOME_CORRECTION        (renderer.h:15-22, precomp.h:1657)
    light   = (24, 24, 22) if lastSpecular else 0                  (renderer.cpp:63-66); Whitted:
              clamp(color, 0, 1) * GetLightColor() = (24, 24, 22)  (renderer.cpp:151-153, Light.h)
    mirror  = albedo * Trace(reflected, depth - 1)                 (renderer.cpp:45-47, Mirror.h)
    depth 0 = 0                                                    (renderer.cpp:18, 140)

The RNG state must come back unchanged (no draws on these paths).  The oracle (CPU) and the
batched GPU Trace (rt_trace) are both held to these values bit for bit."""
import numpy as np
import pytest

from scenes_util import oracle_scene

SKY = np.float32(0.00392156862745)
SKY_RGB = np.array([0x40, 0x60, 0x80], np.float32) * SKY
ALBEDO = np.array([0.9, 0.75, 0.0], np.float32)
LIGHT = np.array([24, 24, 22], np.float32)


def scene(rt):
    mats = [rt.material(rt.LIGHT, tuple(LIGHT)), rt.material(rt.MIRROR, tuple(ALBEDO))]
    prims = [rt.sphere((0, 8, 0), 1.0, 0),
             rt.triangle((-64, -64, 16), (64, -64, 16), (0, 64, 16), 1)]   # mirror, plane z = 16
    return prims, mats


def cases():
    """(ray (7), depth, lastSpecular, whitted, expected rgb, expected first hit (obj, t))"""
    sky_ray = [0, 0, 0, 0, 0, -1, 1e34]
    light_ray = [0, 0, 0, 0, 1, 0, 1e34]
    mirror_ray = [0, 0, 0, 0, 0, 1, 1e34]
    C = []
    for w in (False, True):
        for d in (1, 2, 10, 32):
            C.append((sky_ray, d, True, w, SKY_RGB, (-1, None)))
            C.append((mirror_ray, d, True, w, np.zeros(3, np.float32) if d == 1 else ALBEDO * SKY_RGB, (1, 16.0)))
        C.append((light_ray, 3, True, w, LIGHT, (0, 7.0)))
        C.append((sky_ray, 0, True, w, np.zeros(3, np.float32), (-1, None)))
        C.append((mirror_ray, 0, True, w, np.zeros(3, np.float32), (-1, None)))
    C.append((sky_ray, 5, False, False, SKY_RGB, (-1, None)))
    C.append((light_ray, 3, False, False, np.zeros(3, np.float32), (0, 7.0)))       # lastSpecular false
    C.append((mirror_ray, 4, False, False, ALBEDO * SKY_RGB, (1, 16.0)))
    return C


def run(trace, whitted_flag):
    """trace(rays, seeds, depth, flags, whitted) -> (rgb, seeds_out); groups the cases by call"""
    bad = []
    for ray, d, ls, w, want, _ in cases():
        if w != whitted_flag:
            continue
        rays = np.array([ray], np.float32)
        seeds = np.array([0x2545F491], np.uint32)
        rgb, s_out = trace(rays, seeds, d, np.array([1 if ls else 0], np.uint8), w)
        if rgb[0].tobytes() != np.asarray(want, np.float32).tobytes() or s_out[0] != seeds[0]:
            bad.append((ray, d, ls, w, rgb[0].tolist(), np.asarray(want).tolist(), int(s_out[0])))
    return bad


@pytest.mark.parametrize("whitted", [False, True])
def test_oracle_trace_closed_form(rt, oracle, whitted):
    prims, mats = scene(rt)
    o = oracle_scene(rt, oracle, prims, mats)

    def trace(rays, seeds, d, flags, w):
        o.set_integrator(rt.MODE_WHITTED if w else rt.MODE_PATH)
        rgb, s_out, _ = o.trace_rays(rays, seeds, depth=d, flags=flags)
        return rgb, s_out
    bad = run(trace, whitted)
    assert not bad, bad[:3]


@pytest.mark.gpu
@pytest.mark.parametrize("whitted", [False, True])
def test_gpu_trace_closed_form(rt, whitted):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    prims, mats = scene(rt)
    g = rt.Scene(prims, mats)

    def trace(rays, seeds, d, flags, w):
        rad, sd, _ = g.trace(rays, seeds, depth=d, last_specular=(flags & 1) != 0,
                             mode=rt.MODE_WHITTED if w else rt.MODE_PATH)
        return rad.cpu().numpy(), sd.cpu().numpy().view(np.uint32)
    bad = run(trace, whitted)
    assert not bad, bad[:3]
    # the first hit record (Trace takes Ray&): light at t = 7, mirror at t = 16, sky: none
    for ray, d, ls, w, want, (obj, t) in cases():
        if w or d == 0:
            continue
        _, _, _, (ht, hobj, _, _) = g.trace(np.array([ray], np.float32), np.array([7], np.uint32), depth=d, hits=True)
        assert int(hobj.cpu()[0]) == obj
        if t is not None:
            assert float(ht.cpu()[0]) == t
