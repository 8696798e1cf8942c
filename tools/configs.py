#!/usr/bin/env python3
"""Per-config GPU throughput of every BASELINE.json workload that fits one GPU.

Each config is one Renderer::Tick equivalent (rt_render_frame) per frame on a dedicated
stream; frames are timed with HIP events around the launch, rays come from the library's
counters (primary + shadow + bounce = closest-hit + any-hit rays actually traced).

usage: configs.py [--frames 20] [--warmup 5] [--only cfg3,cfg5] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402

# BASELINE.json configs[1..4] (configs[0] is the reference's CPU run); SURVEY.md 8(d) recipes
CONFIGS = {
    "cfg2_teapotF_ps": dict(scene="teapotF", w=1920, h=1080, spp=1, depth=1),
    "cfg3_shiba_glider_pt4": dict(scene="cfg3", w=1920, h=1080, spp=4, depth=4),
    "cfg4_mig16_ps": dict(scene="mig16", w=1920, h=1080, spp=1, depth=1),
    "cfg5_shiba_pt16": dict(scene="cfg5", w=1920, h=1080, spp=16, depth=10),
    "teapotF_pt_d10": dict(scene="teapotF", w=1920, h=1080, spp=1, depth=10),
}


def run(cfg, frames, warmup, ramp_s=0.5):
    scene = rt.Scene.recipe(cfg["scene"], device=0)
    r = rt.Renderer(scene, cfg["w"], cfg["h"])
    out = torch.zeros(cfg["w"] * cfg["h"], dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    nf, t_ramp = 0, time.perf_counter()
    while time.perf_counter() - t_ramp < ramp_s:     # GPU clock ramp (untimed), as bench.py
        for _ in range(4):
            r.Tick(out, spp=cfg["spp"], depth=cfg["depth"], frame=nf, stream=st.cuda_stream)
            nf += 1
        torch.cuda.synchronize()
    for i in range(warmup):
        r.Tick(out, spp=cfg["spp"], depth=cfg["depth"], frame=nf, stream=st.cuda_stream)
        nf += 1
    torch.cuda.synchronize()
    c0 = r.counters()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(frames)]
    t0 = time.perf_counter()
    with torch.cuda.stream(st):
        for k in range(frames):
            ev[k][0].record(st)
            r.Tick(out, spp=cfg["spp"], depth=cfg["depth"], frame=nf + k, stream=st.cuda_stream)
            ev[k][1].record(st)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    c1 = r.counters()
    ms = [a.elapsed_time(b) for a, b in ev]
    rays = {k: c1[k] - c0[k] for k in ("primary", "shadow", "bounce")}
    tot = sum(rays.values())
    med = float(np.median(ms))
    res = dict(cfg, median_ms=round(med, 4), min_ms=round(min(ms), 4), wall_ms_per_frame=round(wall / frames * 1e3, 4),
               rays_per_frame={k: v / frames for k, v in rays.items()},
               mrays_s=round(tot / frames / (med * 1e-3) / 1e6, 1),
               msamples_s=round(cfg["w"] * cfg["h"] * cfg["spp"] / (med * 1e-3) / 1e6, 1))
    r.close()
    scene.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)   # walk timing + tile-order recording settle in 4 frames
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--custom", action="append", default=[], help="scene,w,h,spp,depth (repeatable)")
    a = ap.parse_args()
    for c in a.custom:
        sc, w, h, spp, depth = c.split(",")
        CONFIGS[f"custom_{sc}_{w}x{h}_spp{spp}_d{depth}"] = dict(scene=sc, w=int(w), h=int(h), spp=int(spp), depth=int(depth))
    names = [n for n in CONFIGS if (not a.only and not a.custom) or (a.only and any(o in n for o in a.only.split(",")))
             or (a.custom and n.startswith("custom_"))]
    out = {}
    for n in names:
        out[n] = run(CONFIGS[n], a.frames, a.warmup)
        print(n, json.dumps(out[n]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
