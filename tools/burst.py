#!/usr/bin/env python3
"""Per-frame time of back-to-back frames as a function of the burst length (frames submitted
between two synchronisations): a diagnostic for stream overlap and submission effects.

usage: burst.py [--scene cfg5] [--spp 16] [--depth 10] [--bursts 4,8,16,32] [--repeat 3] [--null-stream] [--extra-renderers K]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cfg5")
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--bursts", default="2,4,8,16,32")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--null-stream", action="store_true")
    ap.add_argument("--extra-renderers", type=int, default=0, help="idle renderers created first (one frame each)")
    a = ap.parse_args()
    scene = rt.Scene.recipe(a.scene)
    out0 = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
    extra = [rt.Renderer(scene, a.w, a.h) for _ in range(a.extra_renderers)]
    for x in extra:
        x.Tick(out0, spp=a.spp, depth=a.depth, frame=0)
    torch.cuda.synchronize()
    r = rt.Renderer(scene, a.w, a.h)
    out = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
    st = torch.cuda.default_stream() if a.null_stream else torch.cuda.Stream()
    f = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:      # clock ramp + the renderer's first frames
        r.Tick(out, spp=a.spp, depth=a.depth, frame=f, stream=st.cuda_stream)
        f += 1
        torch.cuda.synchronize()
    res = {}
    for rep in range(a.repeat):
        for n in [int(x) for x in a.bursts.split(",")]:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            h0 = time.perf_counter()
            e0.record(st)
            for k in range(n):
                r.Tick(out, spp=a.spp, depth=a.depth, frame=f, stream=st.cuda_stream)
                f += 1
            e1.record(st)
            h1 = time.perf_counter()
            torch.cuda.synchronize()
            res.setdefault(n, []).append((round(e0.elapsed_time(e1) / n, 4), round((h1 - h0) * 1e3 / n, 4)))
            print(n, res[n][-1], flush=True)
    print(json.dumps({"scene": a.scene, "spp": a.spp, "depth": a.depth, "null_stream": a.null_stream, "extra_renderers": a.extra_renderers,
                      "pt_pipeline": os.environ.get("RT_PT_PIPELINE", "1"),
                      "ms_per_frame_gpu_host": {n: v for n, v in res.items()}}))


if __name__ == "__main__":
    main()
