#!/usr/bin/env python3
"""Certify frames for the wave camera walk with the oracle, CPU only: for every
camera ray of each frame in [--first, --last), the reference's answer R must lie less than the
walk's cull margin (2^--margin) before its own leaf box's entry, or be sticky (a sphere, a quad or a
sliver triangle -- boxes above it are culled only on a slab miss).  A certified frame is rendered
by the walk exactly as by IntersectBVH.  One JSON line per frame block, then a summary.

usage: walk_certify.py --scene mig16 [--w 1920 --h 1080] [--first 0 --last 6000] [--block 100]
                       [--margin -12] [--sticky -8] [--cam NAME]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import advancedgraphicsraytracer_amd as rt  # noqa: E402
import pyoracle  # noqa: E402
from scenes_util import sticky_prims  # noqa: E402



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="mig16")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--last", type=int, default=6000)
    ap.add_argument("--block", type=int, default=100)
    ap.add_argument("--margin", type=int, default=-12, help="base-2 exponent of the walk's cull margin (RT_WALK_MARGIN)")
    ap.add_argument("--sticky", type=int, default=-8, help="sliver threshold exponent (RT_WALK_STICKY)")
    ap.add_argument("--cam", default=None, help="a tests/scenes_util.grazing_cameras name instead of the default camera")
    a = ap.parse_args()
    MARGIN = 2.0 ** a.margin
    pyoracle.build()
    prims, _ = rt.recipe_describe(a.scene)
    sticky = sticky_prims(rt, prims, a.sticky)
    o = pyoracle.Scene(a.scene, rt.DATA_DIR)
    cam = None
    if a.cam:
        from scenes_util import grazing_cameras
        rec, cam = grazing_cameras(rt, a.w, a.h)[a.cam]
        assert rec == a.scene
    t0, worst, bad_total, rays = time.time(), 0.0, 0, 0
    sticky_hot = 0
    for b0 in range(a.first, a.last, a.block):
        bw, bb, bs = 0.0, 0, 0
        for f in range(b0, min(a.last, b0 + a.block)):
            need, obj = o.walk_need(a.w, a.h, frame=f, cam=cam, with_obj=True)
            st = (obj >= 0) & sticky[np.maximum(obj, 0)]
            hot = need >= MARGIN
            bb += int((hot & ~st).sum())
            bs += int((hot & st).sum())
            plain = (obj >= 0) & ~st
            if plain.any():
                bw = max(bw, float(need[plain].max()))
            rays += need.size
        worst, bad_total, sticky_hot = max(worst, bw), bad_total + bb, sticky_hot + bs
        print(json.dumps({"frames": [b0, min(a.last, b0 + a.block)], "violations": bb, "sticky_answers_past_margin": bs,
                          "log2_worst_plain_need": round(float(np.log2(bw)), 2) if bw > 0 else None,
                          "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"summary": True, "scene": a.scene, "size": [a.w, a.h], "frames": [a.first, a.last], "rays": rays,
                      "violations": bad_total, "sticky_answers_past_margin": sticky_hot,
                      "log2_worst_plain_need": round(float(np.log2(worst)), 2) if worst > 0 else None,
                      "margin_log2": a.margin, "sticky_log2": a.sticky, "camera": a.cam or "default",
                      "certified": bad_total == 0}), flush=True)


if __name__ == "__main__":
    main()
