#!/usr/bin/env python3
"""Per-tile cost of the two camera walks (lane / wave) on one frame: each walk forced on a
renderer of its own, the renderer's measured tile-cost map (wave cycles per tile, the map behind
its longest-tile-first order) read back after its order is built; prints the totals, the
costliest tiles, and what a per-tile choice (the cheaper walk per tile) would sum to.

usage: walk_tiles.py [--scene mig16] [--w 1920 --h 1080] [--frames 8] [--out f.json]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402


def costs(scene, walk, W, H, frames):
    g = rt.Scene.recipe(scene)
    g.set_camera_walk(walk)
    r = rt.Renderer(g, W, H)
    out = []
    for f in range(frames):
        r.tick_host(spp=1, depth=1, frame=f)
    c = r.tile_costs().astype(np.float64)
    r.close()
    g.close()
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="mig16")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.environ.setdefault("RT_TUNE_DELAY_MS", "0")
    res = {}
    for rep in range(a.reps):
        lane = costs(a.scene, rt.WALK_LANE, a.w, a.h, a.frames)
        wave = costs(a.scene, rt.WALK_WAVE, a.w, a.h, a.frames)
        best = np.minimum(lane, wave)
        rec = {"sum_lane": lane.sum(), "sum_wave": wave.sum(), "sum_min": best.sum(),
               "max_lane": lane.max(), "max_wave": wave.max(), "max_min": best.max(),
               "tiles_lane_cheaper": int((lane < wave).sum()), "tiles": int(lane.size),
               "tiles_lane_cheaper_by_10pct": int((lane < 0.9 * wave).sum())}
        top = np.argsort(-wave)[:10]
        rec["top_wave_tiles"] = [[int(t), float(wave[t]), float(lane[t])] for t in top]
        print(json.dumps({"rep": rep, **{k: (round(v) if isinstance(v, float) else v) for k, v in rec.items()}}), flush=True)
        res[rep] = rec
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, default=float)


if __name__ == "__main__":
    main()
