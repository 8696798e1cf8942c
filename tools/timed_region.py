#!/usr/bin/env python3
"""Where the bench's wall clock goes beyond the frames' GPU time (config 2, the driver's
--steps 20 region): repeats the timed region R times per variant and reports the median
wall ms/step, HIP-event ms/step and their gap per region.

  bench   -- bench.py's region: sync, t0, event, 20 x Tick under torch.cuda.stream, event,
             torch.cuda.synchronize, t1
  spin    -- the same, t1 taken when the end event is observed complete by polling
             (event.query() loop) instead of a blocking device synchronize
  noctx   -- spin, Tick called without the per-step torch.cuda.stream context manager
  host    -- host time of one Tick submission (no GPU wait), median

usage: timed_region.py [--steps 20] [--reps 40] [--scene teapotF]"""
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--scene", default="teapotF")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    W, H = 1920, 1080
    scene = rt.Scene.recipe(a.scene)
    r = rt.Renderer(scene, W, H)
    st = torch.cuda.Stream()
    sptr = st.cuda_stream
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    f = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.6:          # ramp + tuning (walk, tile order, overlap decision)
        with torch.cuda.stream(st):
            for _ in range(20):
                r.Tick(out, spp=1, depth=1, frame=f, stream=sptr)
                f += 1
        torch.cuda.synchronize()
    res = {}
    for variant in ("bench", "spin", "noctx", "bench", "spin", "noctx"):
        walls, evs = [], []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            for k in range(a.steps):
                if variant == "noctx":
                    r.Tick(out, spp=1, depth=1, frame=f, stream=sptr)
                else:
                    with torch.cuda.stream(st):
                        r.Tick(out, spp=1, depth=1, frame=f, stream=sptr)
                f += 1
            e1.record(st)
            if variant == "bench":
                torch.cuda.synchronize()
            else:
                while not e1.query():
                    pass
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            walls.append((t1 - t0) * 1e3 / a.steps)
            evs.append(e0.elapsed_time(e1) / a.steps)
        w, e = float(np.median(walls)), float(np.median(evs))
        res.setdefault(variant, []).append({"wall_ms_step": round(w, 4), "event_ms_step": round(e, 4),
                                             "gap_us_region": round((w - e) * a.steps * 1e3, 1),
                                             "wall_p10_p90": [round(float(np.percentile(walls, 10)), 4),
                                                              round(float(np.percentile(walls, 90)), 4)]})
        print(variant, res[variant][-1], flush=True)
    hs = []
    for _ in range(200):
        h0 = time.perf_counter()
        r.Tick(out, spp=1, depth=1, frame=f, stream=sptr)
        hs.append((time.perf_counter() - h0) * 1e6)
        f += 1
        if len(hs) % 20 == 0:
            torch.cuda.synchronize()
    res["host_submit_us_median"] = round(float(np.median(hs)), 2)
    res["overlap"] = r.overlap_depth()[0]
    line = json.dumps({"scene": a.scene, "steps": a.steps, "reps": a.reps, **res})
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as fo:
            fo.write(line + "\n")


if __name__ == "__main__":
    main()
