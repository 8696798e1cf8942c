#!/usr/bin/env python3
"""Per-rank frame time of bench.py's N > 1 workload, measured on one GPU: the 1/N screen
shard at spp = N (weak scaling), render + (rank-0) assembly, for N = 1, 2, 4, 8.
Predicts the driver's scaling efficiency up to the gather.
usage: shard_time.py [--scene teapotF] [--depth 1] [--spp S] [--strong] [--frames 30] [--out file.jsonl]
(RT_SPLIT_UNITS=U: split threshold; RT_PS_PIPELINE / RT_PS_DEPTH: frames in flight)"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="teapotF")
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--warm", type=int, default=80, help="untimed frames per renderer (walk, tile order and "
                    "frames-in-flight timing: ~60 frames)")
    ap.add_argument("--strong", action="store_true", help="the config's spp per shard (one frame split N ways)")
    ap.add_argument("--spp", type=int, default=1, help="samples per pixel of the whole frame (strong) / per GPU (weak)")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--out", default=None, help="append the summary line to this jsonl file")
    a = ap.parse_args()
    scene = rt.Scene.recipe(a.scene)
    out = {}
    r0 = rt.Renderer(scene, a.w, a.h)                  # GPU clock ramp (untimed), as bench.py
    o0 = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
    t0, f = time.perf_counter(), 0
    while time.perf_counter() - t0 < 0.5:
        r0.Tick(o0, spp=1, depth=a.depth, frame=f)
        f += 1
        if f % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    r0.close()
    for n in [int(x) for x in a.ns.split(",")]:   # warm-up frames: walk timing, tile order, overlap timing settle first
        r = rt.Renderer(scene, a.w, a.h)
        cap = r.shard_capacity(n)
        tiles = torch.zeros(cap, dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        spp = a.spp if a.strong else a.spp * n
        for f in range(a.warm):
            r.render_shard(tiles, n - 1, n, spp=spp, depth=a.depth, frame=f, stream=st.cuda_stream)
        torch.cuda.synchronize()
        c0 = r.counters()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        with torch.cuda.stream(st):
            ev[0].record()
            for f in range(a.frames):
                r.render_shard(tiles, n - 1, n, spp=spp, depth=a.depth, frame=a.warm + f, stream=st.cuda_stream)
            ev[1].record()
        torch.cuda.synchronize()
        c1 = r.counters()
        ms = ev[0].elapsed_time(ev[1]) / a.frames
        rays = sum(c1[k] - c0[k] for k in ("primary", "shadow", "bounce")) / a.frames
        out[n] = {"ms_per_frame": round(ms, 4), "mrays_s_per_gpu": round(rays / (ms * 1e-3) / 1e6, 1),
                  "in_flight": r.overlap_depth()[0], "groups_ms": r.overlap_depth()[1]}
        cost = r.tile_costs().astype(np.float64)
        if cost.size:   # the shard's per-tile wave cycles (s_memtime ticks) behind its tile order
            out[n]["tile_cycles"] = {"tiles": int(cost.size), "max": int(cost.max()), "p99": int(np.percentile(cost, 99)),
                                     "mean": round(float(cost.mean()), 1), "sum": int(cost.sum())}
        print(n, json.dumps(out[n]), flush=True)
        r.close()
    base = out[1]["mrays_s_per_gpu"]
    line = json.dumps({"scene": a.scene, "depth": a.depth, "spp": a.spp, "strong": a.strong, "ps": os.environ.get("RT_PS_PIPELINE", "-1"),
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "per_rank": out,
                       "predicted_efficiency_without_gather": {n: round(v["mrays_s_per_gpu"] / base, 3) for n, v in out.items()}})
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
