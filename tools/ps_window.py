#!/usr/bin/env python3
"""Per-window frame times of back-to-back primary+shadow frames (caller-stream events every
`win` frames), serial vs overlapped (RT_PS_PIPELINE=0 / 1): does the overlapped mode's rate
change over a long run?  usage: ps_window.py [--scene teapotF] [--frames 400] [--win 16]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(rt, torch, scene, W, H, frames, win, mode):
    os.environ["RT_PS_PIPELINE"] = mode
    s = rt.Scene.recipe(scene)
    r = rt.Renderer(s, W, H)
    st = torch.cuda.Stream()
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    with torch.cuda.stream(st):
        for f in range(40):
            r.Tick(out, spp=1, depth=1, frame=f, stream=st.cuda_stream)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(frames // win + 1)]
        ev[0].record(st)
        for f in range(frames):
            r.Tick(out, spp=1, depth=1, frame=40 + f, stream=st.cuda_stream)
            if (f + 1) % win == 0:
                ev[(f + 1) // win].record(st)
        torch.cuda.synchronize()
    ms = [round(ev[i].elapsed_time(ev[i + 1]) / win, 4) for i in range(len(ev) - 1)]
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="teapotF")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--win", type=int, default=16)
    a = ap.parse_args()
    import torch
    import advancedgraphicsraytracer_amd as rt
    for mode in ("0", "1", "0", "1"):
        ms = run(rt, torch, a.scene, 1920, 1080, a.frames, a.win, mode)
        print(json.dumps({"scene": a.scene, "mode": mode, "window_ms": ms}), flush=True)


if __name__ == "__main__":
    main()
