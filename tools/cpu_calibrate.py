#!/usr/bin/env python3
"""Cross-calibrate the CPU restatement (oracle/, the bench's cpu_baseline) against the
reference's own CPU path, both timed in the build container (the reference,
plain BVH, thread-local RNG, clang -O2 -mavx2, 8 threads best of 3, 1 thread single run).

Writes profiles/cpu_calibration.json: per config the restatement's Mrays/s at 8 threads
(best of 3 frames) and 1 thread (one frame) and its ratio to the reference numbers, which
bench.py reports beside the GPU box's cpu_baseline.  Run it here (not on the GPU box: the
reference numbers are this container's).

The same-moment control (`gcc_control`): the restatement also built with gcc -O3 -mavx2 (the
round-1 build) and timed in the same run, so that a ratio change between runs can be split
into compiler gain and host variance (this VM type is not one machine: the same gcc build
measured 30.9 Mrays/s at 8 threads on one instance and 23-26 on another).

usage: cpu_calibrate.py [--threads 8] [--no-gcc-control]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402
from advancedgraphicsraytracer_amd import DATA_DIR  # noqa: E402

# BASELINE.md 2, TL variant: (8 threads, 1 thread) Mrays/s, primary + shadow at 1080p
REFERENCE = {"config2": ("teapotF", 55.76, 7.03), "config4": ("mig16", 24.98, 3.70)}


def rate(s, threads, frames, W=1920, H=1080):
    acc = np.zeros((W * H, 4), np.float32)
    s.tick(W, H, acc, spp=1, depth=1, frame=0, threads=threads)
    best = 0.0
    for f in range(frames):
        t0 = time.perf_counter()
        _, st = s.tick(W, H, acc, spp=1, depth=1, frame=f + 1, threads=threads)
        best = max(best, (st["isect"] + st["occl"]) / (time.perf_counter() - t0) / 1e6)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--no-gcc-control", action="store_true")
    args = ap.parse_args()
    out = {"host": {"cpus": os.cpu_count(), "threads": args.threads},
           "oracle_build": "oracle/Makefile (ROCm clang -O2 -mavx2 -ffp-contract=off, libomp)",
           "reference": "BASELINE.md 2 (plain BVH, TL RNG, clang -O2 -mavx2)"}
    for key, (scene, ref8, ref1) in REFERENCE.items():
        s = pyoracle.Scene(scene, DATA_DIR)
        r8, r1 = rate(s, args.threads, 3), rate(s, 1, 1)
        out[key] = {"scene": scene, "restatement_threads": round(r8, 2), "restatement_1core": round(r1, 2),
                    "reference_threads": ref8, "reference_1core": ref1,
                    "ratio_threads": round(r8 / ref8, 3), "ratio_1core": round(r1 / ref1, 3)}
        print(key, out[key], flush=True)
    if not args.no_gcc_control:
        so = os.path.join(tempfile.mkdtemp(), "liboracle_gcc.so")
        subprocess.run(["gcc", "-O3", "-mavx2", "-std=gnu11", "-fPIC", "-fopenmp", "-ffp-contract=off", "-shared",
                        "-o", so, os.path.join(ROOT, "oracle", "rt_oracle.c"), "-lm"], check=True)
        pyoracle.LIB_PATH, pyoracle._lib = so, None
        ctl = {"build": "gcc -O3 -mavx2 -ffp-contract=off (libgomp)"}
        for key, (scene, _, _) in REFERENCE.items():
            s = pyoracle.Scene(scene, DATA_DIR)
            r8, r1 = rate(s, args.threads, 3), rate(s, 1, 1)
            ctl[key] = {"restatement_threads": round(r8, 2), "restatement_1core": round(r1, 2),
                        "clang_over_gcc_threads": round(out[key]["restatement_threads"] / r8, 3),
                        "clang_over_gcc_1core": round(out[key]["restatement_1core"] / r1, 3)}
        out["gcc_control"] = ctl
        print("gcc_control", ctl, flush=True)
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
