#!/usr/bin/env python3
"""Interleaved A/B of scene-creation environment knobs in ONE process: one scene + renderer
per variant (each created with its variables set), rounds alternate between the variants,
each round `--frames` back-to-back frames between two HIP events on one stream; prints the
per-variant median and min ms/frame, and (--check) asserts every variant's last frame equals
the first variant's bit for bit.

usage: knob_ab.py --scene cfg5 --spp 16 --depth 10 --var RT_PT_DRAIN_ROUNDS=1 --var RT_PT_DRAIN_ROUNDS=0.25 [--var A=1,B=2]
                  [--w 1920 --h 1080] [--rounds 7] [--frames 4] [--warm 6] [--check] [--out f.jsonl]"""
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
    ap.add_argument("--scene", default="cfg5")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--var", action="append", required=True, help="NAME=V[,NAME=V...] set while creating the scene")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--warm", type=int, default=6)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    variants = []
    for v in a.var:
        kv = dict(x.split("=", 1) for x in v.split(","))
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        s = rt.Scene.recipe(a.scene)
        for k, o in old.items():
            if o is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = o
        r = rt.Renderer(s, a.w, a.h)
        out = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
        variants.append({"name": v, "scene": s, "r": r, "out": out, "ms": [], "frame": 0})
    st = torch.cuda.Stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5 or variants[-1]["frame"] < a.warm:   # clock ramp + tuning
        for v in variants:
            v["r"].Tick(v["out"], spp=a.spp, depth=a.depth, frame=v["frame"], stream=st.cuda_stream)
            v["frame"] += 1
        torch.cuda.synchronize()
    for _ in range(a.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.frames):
                v["r"].Tick(v["out"], spp=a.spp, depth=a.depth, frame=v["frame"], stream=st.cuda_stream)
                v["frame"] += 1
            e1.record(st)
            torch.cuda.synchronize()
            v["ms"].append(e0.elapsed_time(e1) / a.frames)
    res = {"scene": a.scene, "spp": a.spp, "depth": a.depth, "size": [a.w, a.h], "variants": {}}
    for v in variants:
        res["variants"][v["name"]] = {"median_ms": round(float(np.median(v["ms"])), 4), "min_ms": round(float(np.min(v["ms"])), 4)}
    if a.check:   # same frame index on every variant: render one more aligned frame each
        f = max(v["frame"] for v in variants)
        ref = None
        for v in variants:
            o = v["r"].Tick(v["out"], spp=a.spp, depth=a.depth, frame=f, stream=st.cuda_stream)
            torch.cuda.synchronize()
            x = o.cpu().numpy()
            if ref is None:
                ref = x
            res["variants"][v["name"]]["frame_equal_first"] = bool(np.array_equal(x, ref))
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as fo:
            fo.write(line + "\n")


if __name__ == "__main__":
    main()
