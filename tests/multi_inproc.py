#!/usr/bin/env python3
"""Several ranks of the C-ABI multi-GPU frame (rt_comm_create + rt_render_frame_multi +
rt_multi_flush, csrc/rt_multi.cpp) as THREADS of this process sharing GPU 0, exchanging
through the in-process RCCL stand-in (tests/cpp/libinproc_rccl.so, selected by RT_RCCL_LIB;
real RCCL refuses two ranks on one device).  Run by tests/test_multi_inproc.py in a child
process (the stand-in must be the process's first RCCL).

Every rank renders its t % world tiles of the same frames; rank 0's assembled frames must equal
a plain renderer's Tick frames bit for bit, every rank's accumulator must equal the plain
accumulator on the pixels of its tiles, and the ranks' ray counts must add up to the plain
renderer's.  In pipelined mode rank 0 copies each returned frame on its own stream WITHOUT a
host sync before the next call (the next call's unshuffle must wait for that copy).

usage: multi_inproc.py WORLD {sync|pipelined|balanced} RECIPE WIDTH HEIGHT   -> exit 0 and a JSON line
(balanced = pipelined + RT_MULTI_BALANCED: the cost-balanced deal from a parameter set's 7th frame)"""
import ctypes as C
import json
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402
from advancedgraphicsraytracer_amd.shard import shard_pixels  # noqa: E402

# (spp, Trace depth) per frame: primary+shadow frames (past the tile-order tuning), a sample-
# split frame, path-traced frames, primary+shadow again
PLAN = [(1, 1)] * 6 + [(2, 1), (1, 3), (2, 4), (1, 1), (1, 1)]
# balanced mode: the deal switches on the 7th frame of a parameter set (kDealAfter), so runs of
# equal parameters: primary+shadow (measured costs), path-traced (equal costs), primary+shadow
PLAN_BALANCED = [(1, 1)] * 10 + [(1, 3)] * 8 + [(2, 1)] * 3


def rank_main(rank, world, uid, recipe, W, H, mode, results, errors):
    try:
        L = rt.lib()
        torch.cuda.set_device(0)
        scene = rt.Scene.recipe(recipe)          # every rank holds its own replica
        r = rt.Renderer(scene, W, H)
        h = C.c_void_p()
        rt._check(L.rt_comm_create(uid, rank, world, 0, C.byref(h)))
        st = torch.cuda.Stream()
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda:0") if rank == 0 else None
        optr = C.c_void_p(out.data_ptr()) if rank == 0 else None
        pipelined = mode != "sync"
        flags = (rt.MULTI_PIPELINED if pipelined else 0) | (rt.MULTI_BALANCED if mode == "balanced" else 0)
        plan = PLAN_BALANCED if mode == "balanced" else PLAN
        copies = []
        with torch.cuda.stream(st):
            for f, (spp, depth) in enumerate(plan):
                p = r.params(spp, depth, f)
                rt._check(L.rt_render_frame_multi(r.h, h, C.byref(r.camera), C.byref(p), optr, flags,
                                                  C.c_void_p(st.cuda_stream)))
                if rank == 0 and (not pipelined or f > 0):
                    copies.append(out.clone())       # on st: no host sync before the next call
            if pipelined:
                rt._check(L.rt_multi_flush(r.h, h, optr, C.c_void_p(st.cuda_stream)))
                if rank == 0:
                    copies.append(out.clone())
        st.synchronize()
        results[rank] = {"frames": [c.cpu().numpy() for c in copies], "acc": r.accumulator(), "counters": r.counters()}
        rt._check(L.rt_comm_destroy(h))
        r.close()
        scene.close()
    except Exception as e:   # reported by the main thread
        errors.append(f"rank {rank}: {type(e).__name__}: {e}")


def main():
    world, mode, recipe, W, H = int(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    L = rt.lib()
    uid = (C.c_uint8 * rt.RT_COMM_ID_BYTES)()
    rt._check(L.rt_comm_unique_id(uid))
    results, errors = [None] * world, []
    threads = [threading.Thread(target=rank_main, args=(k, world, uid, recipe, W, H, mode, results, errors))
               for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    if errors or any(t.is_alive() for t in threads):
        print(json.dumps({"ok": False, "errors": errors, "alive": [t.is_alive() for t in threads]}), flush=True)
        sys.exit(1)
    plan = PLAN_BALANCED if mode == "balanced" else PLAN
    ref = rt.Renderer(rt.Scene.recipe(recipe), W, H)
    want = [ref.tick_host(spp=spp, depth=depth, frame=f).view(np.int32) for f, (spp, depth) in enumerate(plan)]
    got = results[0]["frames"]
    bad_frames = [f for f in range(len(plan)) if not np.array_equal(got[f], want[f])]
    acc = ref.accumulator()
    bad_acc = []
    if mode != "balanced":   # (under a deal switch a pixel's accumulator lives on two ranks)
        for k in range(world):
            px = shard_pixels(W, H, k, world)
            px = px[px >= 0]
            if not np.array_equal(results[k]["acc"][px].view(np.uint32), acc[px].view(np.uint32)):
                bad_acc.append(k)
    c = ref.counters()
    sums = {key: sum(results[k]["counters"][key] for k in range(world)) for key in ("primary", "shadow", "bounce")}
    ok = len(got) == len(plan) and not bad_frames and not bad_acc and all(sums[key] == c[key] for key in sums)
    print(json.dumps({"ok": ok, "world": world, "mode": mode, "frames": len(got), "bad_frames": bad_frames,
                      "bad_acc_ranks": bad_acc, "counters": sums, "want_counters": {k: c[k] for k in sums}}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
