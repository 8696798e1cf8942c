#!/usr/bin/env python3
"""How fast are the batched traversal kernels (k_intersect 66 VGPRs, k_occluded) on
diffuse-bounce-like rays?  Camera rays of a 1080p frame -> hit points -> random
hemisphere directions (away from the camera), traced with rt_intersect / rt_occluded,
compared with the camera rays themselves.  Isolates traversal cost from shading."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / reps


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    W, H = 1920, 1080
    s = rt.Scene.recipe(scene_name)
    cam = rt.Camera.default(W, H)
    pos, tl, tr, bl = (np.array(getattr(cam, k), np.float32) for k in ("pos", "top_left", "top_right", "bottom_left"))
    ys, xs = (a.reshape(-1) for a in np.mgrid[0:H, 0:W])
    # tile order (8x8 tiles, lane-major) like the frame kernels
    order = np.lexsort(((xs % 8) + 8 * (ys % 8), xs // 8 + (W // 8) * (ys // 8)))
    u = ((xs + 0.5) / W)[order].astype(np.float32)
    v = ((ys + 0.5) / H)[order].astype(np.float32)
    P = tl[None] + u[:, None] * (tr - tl)[None] + v[:, None] * (bl - tl)[None]
    D = P - pos[None]
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    rays = np.concatenate([np.repeat(pos[None], len(D), 0), D, np.full((len(D), 1), 1e34, np.float32)], 1).astype(np.float32)
    dr = torch.from_numpy(rays).cuda()
    t, obj, _, _ = s.IntersectBVH(dr)
    torch.cuda.synchronize()
    hit = (obj != -1).cpu().numpy()
    tt = t.cpu().numpy()
    O = rays[hit, :3] + (tt[hit, None] - 1e-3) * rays[hit, 3:6]
    rng = np.random.default_rng(1)
    R = rng.normal(size=(len(O), 3)).astype(np.float32)
    R /= np.linalg.norm(R, axis=1, keepdims=True)
    R = np.where((R * rays[hit, 3:6]).sum(1, keepdims=True) > 0, -R, R)   # back toward the camera side
    b = np.concatenate([O, R, np.full((len(O), 1), 1e34, np.float32)], 1).astype(np.float32)
    db = torch.from_numpy(b).cuda()
    light = np.array([0, 4, -2], np.float32) if scene_name != "mig16" else np.array([0, 6, 5], np.float32)
    L = light[None] - O
    dist = np.linalg.norm(L, axis=1, keepdims=True)
    sh = np.concatenate([O, L / dist, dist - 2e-4], 1).astype(np.float32)
    dsh = torch.from_numpy(sh).cuda()
    res = {"scene": scene_name,
           "camera_rays": len(rays), "camera_ms": timed(lambda: s.IntersectBVH(dr)),
           "bounce_rays": len(b), "bounce_ms": timed(lambda: s.IntersectBVH(db)),
           "shadow_rays": len(sh), "shadow_ms": timed(lambda: s.IsOccluded(dsh))}
    for k in ("camera", "bounce", "shadow"):
        res[f"{k}_grays_s"] = round(res[f"{k}_rays"] / (res[f"{k}_ms"] * 1e-3) / 1e9, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
