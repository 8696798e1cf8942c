#!/usr/bin/env python3
"""The wave camera walk's counters under scene-creation knobs (RT_WALK_STICKY, RT_WALK_MARGIN):
for each variant and camera (the recipe's default and tests/scenes_util.grazing_cameras), frames
with the walk forced and RT_WALK_CHECK_VERIFY (every walked lane re-traced in the reference order):
rays walked, boxes entered through the margin / a sticky mark, lanes re-traced, mismatches.

usage: walk_verify.py --var RT_WALK_STICKY=0 --var RT_WALK_STICKY=-10 [--frames 3] [--w 1920 --h 1080]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import advancedgraphicsraytracer_amd as rt  # noqa: E402
from scenes_util import grazing_cameras  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", action="append", required=True)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    a = ap.parse_args()
    W, H = a.w, a.h
    cams = [("mig16", None, "mig16_default"), ("teapotF", None, "teapotF_default")]
    cams += [(rec, cam, name) for name, (rec, cam) in grazing_cameras(rt, W, H).items()]
    for v in a.var:
        kv = dict(x.split("=", 1) for x in v.split(","))
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        scenes = {rec: rt.Scene.recipe(rec) for rec in ("mig16", "teapotF")}
        for k, o in old.items():
            if o is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = o
        for rec, cam, name in cams:
            g = scenes[rec]
            g.set_camera_walk(rt.WALK_WAVE)
            r = rt.Renderer(g, W, H)
            if cam is not None:
                r.camera = cam
            r.set_walk_check(rt.WALK_CHECK_VERIFY)
            for f in range(a.frames):
                r.tick_host(spp=1, depth=1, frame=f)
            print(json.dumps({"variant": v, "camera": name, "frames": a.frames, **r.walk_stats()}), flush=True)
            r.close()
        for g in scenes.values():
            g.close()


if __name__ == "__main__":
    main()
