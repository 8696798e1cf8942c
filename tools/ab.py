#!/usr/bin/env python3
"""Interleaved A/B timing of librtamd.so builds in ONE process (cdna_hip_programming.md
5.4 rule 24).  Each build is loaded RTLD_LOCAL through raw ctypes; rounds alternate
between builds; the per-build median and min of the per-frame kernel time are printed.

usage: ab.py LIB[@mode=M,depth=D] [...] [--scene teapotF] [--w 1920] [--h 1080] [--spp 1]
             [--depth 1] [--rounds 7] [--frames 20] [--check] [--ramp-seconds 1]
A LIB may carry its own integrator mode (0 path, 1 Whitted, 2 packet) and depth, so one
build can be timed against itself in another mode.
--check compares every entry's RGB8 frame with the first entry's (bit-exact).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402  (structs only)


def load(path):
    L = C.CDLL(os.path.abspath(path), mode=C.RTLD_LOCAL)
    vp, u32 = C.c_void_p, C.c_uint32
    L.rt_scene_create_recipe.argtypes = [C.c_char_p, C.c_char_p, C.c_int32, C.POINTER(vp)]
    L.rt_renderer_create.argtypes = [vp, u32, u32, C.POINTER(vp)]
    L.rt_render_frame.argtypes = [vp, C.POINTER(rt.Camera), C.POINTER(rt.FrameParams), vp, vp]
    L.rt_camera_default.argtypes = [u32, u32, C.POINTER(rt.Camera)]
    L.rt_renderer_counters.argtypes = [vp, C.POINTER(rt.Counters)]
    L.rt_last_error.restype = C.c_char_p
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--scene", default="teapotF")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--ramp-seconds", type=float, default=1.0, help="untimed frames of every build first (clock ramp)")
    a = ap.parse_args()
    builds = []      # (key, spec, lib, scene, renderer, camera, out, mode, depth) per entry
    loaded = {}
    for i, p in enumerate(a.libs):
        path, _, opts = p.partition("@")
        kv = dict(o.split("=") for o in opts.split(",") if o)
        L = loaded.get(path) or load(path)
        loaded[path] = L
        for k, v in kv.items():              # upper-case options are environment knobs read at scene creation
            if k.isupper():
                os.environ[k] = v
            elif k not in ("mode", "depth"):
                raise SystemExit(f"unknown option {k}")
        sc, r = C.c_void_p(), C.c_void_p()
        assert L.rt_scene_create_recipe(a.scene.encode(), rt.DATA_DIR.encode(), 0, C.byref(sc)) == 0, L.rt_last_error()
        assert L.rt_renderer_create(sc, a.w, a.h, C.byref(r)) == 0, L.rt_last_error()
        cam = rt.Camera()
        L.rt_camera_default(a.w, a.h, C.byref(cam))
        out = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
        key = os.path.basename(p)
        if key in [bd[0] for bd in builds]:   # the same entry listed twice (position-bias checks)
            key = f"{key}#{i}"
        builds.append((key, p, L, sc, r, cam, out, int(kv.get("mode", 0)), int(kv.get("depth", a.depth))))
        for k in kv:
            if k.isupper():
                del os.environ[k]
    times = [[] for _ in builds]
    frame = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.ramp_seconds:
        for key, p, L, sc, r, cam, out, mode, depth in builds:
            fp = rt.FrameParams(a.w, a.h, a.spp, depth, frame, mode, 0)
            L.rt_render_frame(r, C.byref(cam), C.byref(fp), C.c_void_p(out.data_ptr()), None)
        torch.cuda.synchronize()
        frame += 1
    for rnd in range(a.rounds):
        for i, (key, p, L, sc, r, cam, out, mode, depth) in enumerate(builds):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            # warm + timed frames on the default stream
            fp = rt.FrameParams(a.w, a.h, a.spp, depth, frame, mode, 0)
            L.rt_render_frame(r, C.byref(cam), C.byref(fp), C.c_void_p(out.data_ptr()), None)
            # idle GPU before the first event: pipelined path-traced frames start their levels on
            # the renderer's streams without waiting for the caller's stream, so an event recorded
            # behind a running frame would miss the next frame's early work
            torch.cuda.synchronize()
            ev[0].record()
            for k in range(a.frames):
                fp = rt.FrameParams(a.w, a.h, a.spp, depth, frame + 1 + k, mode, 0)
                rc = L.rt_render_frame(r, C.byref(cam), C.byref(fp), C.c_void_p(out.data_ptr()), None)
                assert rc == 0, L.rt_last_error()
            ev[1].record()
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]) / a.frames)
        frame += a.frames + 1
    res = {}
    for i, (key, p, L, sc, r, cam, out, mode, depth) in enumerate(builds):
        c = rt.Counters()
        L.rt_renderer_counters(r, C.byref(c))
        t = np.array(times[i])
        rays_per_frame = (c.primary + c.shadow + c.bounce) / max(1, c.frames)
        res[key] = {"mode": mode, "depth": depth, "median_ms": round(float(np.median(t)), 4),
                    "min_ms": round(float(t.min()), 4), "mrays_s": round(rays_per_frame / (np.median(t) * 1e-3) / 1e6, 1)}
    if a.check:
        ref = None
        for key, p, L, sc, r, cam, out, mode, depth in builds:
            fr = rt.FrameParams(a.w, a.h, a.spp, depth, 12345, mode, 1)
            L.rt_render_frame(r, C.byref(cam), C.byref(fr), C.c_void_p(out.data_ptr()), None)
            torch.cuda.synchronize()
            img = out.cpu().numpy().copy()
            if ref is None:
                ref = img
            res[key]["same_image_as_first"] = bool(np.array_equal(img, ref))
    print(json.dumps({"scene": a.scene, "w": a.w, "h": a.h, "spp": a.spp, "depth": a.depth, "results": res}, indent=1))


if __name__ == "__main__":
    main()
