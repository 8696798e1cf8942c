#!/usr/bin/env python3
"""Where the lane state machine (k_pt_lanes) spends its wave cycles, per bounce level, from a
diagnostic build (tools/build_variant.sh NAME -DRT_PT_PROFILE=1): s_memtime around the
queue refill, the bounded traversal steps and the shading / hand-on of every loop
iteration, plus the lanes still traversing in each step (lane utilisation of the steps).

usage: pt_profile.py variants/NAME.so [--scene cfg5] [--spp 16] [--depth 10] [--frames 4]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--scene", default="cfg5")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--frames", type=int, default=4)
    a = ap.parse_args()
    os.environ["RTAMD_LIB"] = os.path.abspath(a.lib)
    import advancedgraphicsraytracer_amd as rt
    L = rt.lib()
    L.rt_debug_pt_profile.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    g = rt.Scene.recipe(a.scene)
    r = rt.Renderer(g, a.w, a.h)
    out = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
    t0 = time.perf_counter()
    f = 0
    while time.perf_counter() - t0 < 0.5:
        r.Tick(out, spp=a.spp, depth=a.depth, frame=f)
        f += 1
        torch.cuda.synchronize()
    buf = (C.c_ulonglong * 128)()
    L.rt_debug_pt_profile(buf, 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for k in range(a.frames):
        r.Tick(out, spp=a.spp, depth=a.depth, frame=f + k)
    ev[1].record()
    torch.cuda.synchronize()
    L.rt_debug_pt_profile(buf, 1)
    res = {"scene": a.scene, "spp": a.spp, "depth": a.depth, "frame_ms": ev[0].elapsed_time(ev[1]) / a.frames,
           "levels": {}}
    for lv in range(16):
        q = [buf[lv * 8 + i] for i in range(8)]
        if q[7] == 0:
            continue
        tot = q[0] + q[1] + q[2]
        res["levels"][lv] = {"wave_cycles": q[7] / a.frames, "fetch_frac": round(q[0] / tot, 4),
                             "step_frac": round(q[1] / tot, 4), "shade_frac": round(q[2] / tot, 4),
                             "iterations_per_wave_frame": q[3], "fetches": q[4] / a.frames, "steps": q[5] / a.frames,
                             "step_lane_util": round(q[6] / max(1, q[5]) / 64, 4),
                             "cycles_per_step": round(q[1] / max(1, q[5]), 1),
                             "cycles_per_fetch": round(q[0] / max(1, q[4]), 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
