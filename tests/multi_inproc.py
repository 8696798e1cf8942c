#!/usr/bin/env python3
"""Several ranks of the C-ABI multi-GPU frame (rt_comm_create + rt_render_frame_multi +
rt_multi_flush, csrc/rt_multi.cpp) as THREADS of this process sharing GPU 0, exchanging
through the in-process RCCL stand-in (tests/cpp/libinproc_rccl.so, selected by RT_RCCL_LIB;
real RCCL refuses two ranks on one device).  Run by tests/test_multi_inproc.py in a child
process (the stand-in must be the process's first RCCL).

Every rank renders its share of the same frames; rank 0's assembled frames must equal a plain
renderer's Tick frames bit for bit (same cameras, same resets), every rank's accumulator must
equal the plain accumulator on the pixels of its tiles (interleaved modes), and the ranks' ray
counts must add up to the plain renderer's.  In pipelined mode rank 0 copies each returned frame
on its own stream WITHOUT a host sync before the next call (the next call's unshuffle must wait
for that copy).

usage: multi_inproc.py WORLD MODE RECIPE WIDTH HEIGHT   -> exit 0 and a JSON line
MODE: sync | pipelined -- the interleaved deal;
      balanced -- pipelined + RT_MULTI_BALANCED: primary+shadow frames until the cost-balanced
                  deal is on (each rank's renderer times its camera walk first), path-traced
                  frames (level-0 costs: a second balanced deal), primary+shadow again;
      moving   -- balanced, then the camera moves every frame with the accumulator reset (the
                  deal is kept), then a new static camera (rebalanced; the switch frame resets);
      ptbal    -- path-traced frames only (spp 16, depth 10), balanced on the dry-run work map;
      pt       -- path-traced frames only (spp 16, depth 10), pipelined, interleaved deal (the
                  bench's config 5 split: BASELINE config 5 is 1080p x 16 spp on 8 GPUs);
      after_tick -- every rank's renderer first renders the first 5 frames whole (Tick), then the
                  communicator takes over (balanced): each rank holds every tile, nothing moves;
      recreate -- balanced; after 20 frames every rank destroys its communicator and creates a
                  new one (a second unique id) around the SAME renderer, which must take the new
                  communicator's deals (a reused communicator address must not revive
                  the old tile map);
      fault:<site>:<rank> -- balanced, with RT_MULTI_FAULT=<site>:<rank> (csrc/rt_multi.cpp): that
                  rank's local step of a per-frame collective fails; every rank must return an
                  error from the same call and none may be left waiting in the collective; the
                  frames after it render (the failed attempt is not retried) and equal
                  Tick's frames with the failed one left out.
RECIPE: a bench recipe, or chain64 (tests/scenes_util.chain_scene: a 64-level prebuilt tree whose
        dry-run work map is unsupported, so balancing falls back to measured cycle costs).
The balanced modes print the communicator's deal_info and deal hash (equal on every rank) and
require the balanced deal at the end."""
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

sys.path.insert(0, os.path.join(ROOT, "tests"))


def make_scene(recipe):
    if recipe == "chain64":
        from scenes_util import chain_scene
        prims, mats, bvh = chain_scene(rt, 64)
        return rt.Scene(prims, mats, bvh=bvh)
    return rt.Scene.recipe(recipe)

BALANCED_MODES = ("balanced", "moving", "ptbal", "recreate", "after_tick")


def plan_for(mode):
    """[(spp, depth, camera shift, reset)] per frame"""
    if mode in ("sync", "pipelined"):
        # primary+shadow frames (past the tile-order tuning), a sample-split frame, path-traced
        # frames, primary+shadow again
        return [(s, d, 0, False) for s, d in [(1, 1)] * 6 + [(2, 1), (1, 3), (2, 4), (1, 1), (1, 1)]]
    if mode == "balanced":
        # the first balancing attempt (frame 6) builds the deal from the dry-run work map
        # (INPROC_PS_FRAMES: more primary+shadow frames, for runs with a tuning delay)
        n = int(os.environ.get("INPROC_PS_FRAMES", "30"))
        return [(1, 1, 0, False)] * n + [(1, 3, 0, False)] * 10 + [(2, 1, 0, False)] * 3
    if mode == "moving":
        static = [(1, 1, 0, False)] * 30
        moving = [(1, 1, k, True) for k in range(1, 11)]             # every frame a new camera, reset
        settle = [(1, 1, 11, f == 0 or f == 6) for f in range(20)]   # new static camera; its 6th frame
        return static + moving + settle                              # (the rebalancing one) resets
    if mode == "ptbal":
        return [(16, 10, 0, False)] * 10
    if mode == "pt":
        return [(16, 10, 0, False)] * 6
    if mode in ("recreate", "after_tick"):
        return [(1, 1, 0, False)] * 40
    if mode.startswith("fault:"):
        return [(1, 1, 0, False)] * 40
    raise SystemExit(f"unknown mode {mode}")


def tile_pixels(W, H, tiles):
    """pixel indices of the listed 8x8 tiles (on screen only)"""
    tx = (W + 7) // 8
    lane = np.arange(64)
    t = np.asarray(tiles, np.int64)[:, None]
    x, y = (t % tx) * 8 + lane % 8, (t // tx) * 8 + lane // 8
    return (y * W + x)[(x < W) & (y < H)]


def camera_for(W, H, shift):
    cam = rt.Camera.default(W, H)
    if shift:   # a sideways move, as Camera::AdjustCamera does for the arrow keys (camera.h:54-86)
        d = 0.01 * shift
        for f in ("pos", "top_left", "top_right", "bottom_left"):
            getattr(cam, f)[0] += d
    return cam


RECREATE_AT = 20
TICK_FRAMES = 5


def rank_main(rank, world, uid, recipe, W, H, mode, plan, results, errors, uid2=None):
    try:
        L = rt.lib()
        torch.cuda.set_device(0)
        scene = make_scene(recipe)               # every rank holds its own replica
        r = rt.Renderer(scene, W, H)
        h = C.c_void_p()
        rt._check(L.rt_comm_create(uid, rank, world, 0, C.byref(h)))
        st = torch.cuda.Stream()
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda:0") if rank == 0 else None
        optr = C.c_void_p(out.data_ptr()) if rank == 0 else None
        pipelined = mode != "sync"   # every other mode, "pt" included
        fault = mode.startswith("fault:")
        flags = (rt.MULTI_PIPELINED if pipelined else 0) | (rt.MULTI_BALANCED if mode in BALANCED_MODES or fault else 0)
        copies, deals, exch = [], [], []
        failed_at = None
        first = 0
        if mode == "after_tick":   # whole frames first, on this rank's own renderer
            first = TICK_FRAMES
            for f in range(first):
                spp, depth, shift, reset = plan[f]
                r.camera = camera_for(W, H, shift)
                frame = r.tick_host(spp=spp, depth=depth, frame=f, reset=reset)
                if rank == 0:
                    copies.append(torch.from_numpy(frame.view(np.int32).copy()))
        with torch.cuda.stream(st):
            for f, (spp, depth, shift, reset) in enumerate(plan):
                if f < first:
                    continue
                if mode == "recreate" and f == RECREATE_AT:   # a new communicator, the same renderer
                    rt._check(L.rt_multi_flush(r.h, h, optr, C.c_void_p(st.cuda_stream)))
                    if rank == 0:
                        copies.append(out.clone())
                    st.synchronize()
                    rt._check(L.rt_comm_destroy(h))
                    h = C.c_void_p()
                    rt._check(L.rt_comm_create(uid2, rank, world, 0, C.byref(h)))
                cam = camera_for(W, H, shift)
                p = r.params(spp, depth, f, reset)
                rc = L.rt_render_frame_multi(r.h, h, C.byref(cam), C.byref(p), optr, flags, C.c_void_p(st.cuda_stream))
                if fault and rc != 0:   # the injected failure: every rank must see it on this call,
                    if failed_at is None:   # and only on this one
                        failed_at = (f, rc, L.rt_last_error().decode(errors="replace"))
                        continue
                    raise RuntimeError(f"frame {f} failed again after the failure at {failed_at[0]}: "
                                       + L.rt_last_error().decode(errors="replace"))
                rt._check(rc)
                if rank == 0 and (not pipelined or (f > first and not (mode == "recreate" and f == RECREATE_AT))):
                    copies.append(out.clone())       # on st: no host sync before the next call
                b, stats = C.c_int(), (C.c_uint64 * 4)()
                rt._check(L.rt_comm_deal_info(h, C.byref(b), None, None, stats))
                deals.append(b.value)
                exch.append(int(stats[1]))
            if pipelined:
                rt._check(L.rt_multi_flush(r.h, h, optr, C.c_void_p(st.cuda_stream)))
                if rank == 0:
                    copies.append(out.clone())
        st.synchronize()
        b, t, stats, dh = C.c_int(), C.c_uint32(), (C.c_uint64 * 4)(), C.c_uint64()
        rt._check(L.rt_comm_deal_info(h, C.byref(b), C.byref(t), None, stats))
        rt._check(L.rt_comm_deal_hash(h, C.byref(dh)))
        mine = np.zeros(t.value, np.uint32)
        rt._check(L.rt_comm_deal_info(h, None, C.byref(t), mine.ctypes.data_as(C.POINTER(C.c_uint32)), None))
        results[rank] = {"frames": [c.cpu().numpy() for c in copies], "acc": r.accumulator(), "counters": r.counters(),
                         "tiles": mine,
                         "deal": {"balanced": b.value, "tiles": t.value, "deals_built": int(stats[0]),
                                  "exchanges": int(stats[1]), "moves": int(stats[2]), "moves_skipped": int(stats[3]),
                                  "hash": f"{dh.value:016x}"},
                         "deal_per_frame": deals, "exchanges_per_frame": exch, "failed_at": failed_at}
        rt._check(L.rt_comm_destroy(h))
        r.close()
        scene.close()
    except Exception as e:   # reported by the main thread
        errors.append(f"rank {rank}: {type(e).__name__}: {e}")


def main():
    world, mode, recipe, W, H = int(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    plan = plan_for(mode)
    if mode.startswith("fault:"):
        os.environ["RT_MULTI_FAULT"] = mode[len("fault:"):]
    L = rt.lib()
    uid = (C.c_uint8 * rt.RT_COMM_ID_BYTES)()
    rt._check(L.rt_comm_unique_id(uid))
    uid2 = (C.c_uint8 * rt.RT_COMM_ID_BYTES)()
    rt._check(L.rt_comm_unique_id(uid2))
    results, errors = [None] * world, []
    threads = [threading.Thread(target=rank_main, args=(k, world, uid, recipe, W, H, mode, plan, results, errors, uid2))
               for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=400)
    if errors or any(t.is_alive() for t in threads):
        print(json.dumps({"ok": False, "errors": errors, "alive": [t.is_alive() for t in threads]}), flush=True)
        os._exit(1)   # a rank left waiting in a collective: do not join it
    skip = None
    if mode.startswith("fault:"):
        fails = [results[k]["failed_at"] for k in range(world)]
        fail_ok = all(x is not None for x in fails) and len({x[0] for x in fails}) == 1
        if not fail_ok:
            print(json.dumps({"ok": False, "world": world, "mode": mode, "failed_at": fails}), flush=True)
            sys.exit(1)
        skip = fails[0][0]   # no rank rendered the failed frame: Tick skips it too
    ref = rt.Renderer(make_scene(recipe), W, H)
    want = []
    for f, (spp, depth, shift, reset) in enumerate(plan):
        if f == skip:
            continue
        ref.camera = camera_for(W, H, shift)
        want.append(ref.tick_host(spp=spp, depth=depth, frame=f, reset=reset).view(np.int32))
    got = results[0]["frames"]
    bad_frames = [f for f in range(len(want)) if f >= len(got) or not np.array_equal(got[f], want[f])]
    acc = ref.accumulator()
    bad_acc = []
    for k in range(world):   # each rank holds the running averages of the tiles of its final deal
        px = tile_pixels(W, H, results[k]["tiles"])
        if not np.array_equal(results[k]["acc"][px].view(np.uint32), acc[px].view(np.uint32)):
            bad_acc.append(k)
    c = dict(ref.counters())
    if mode == "after_tick":   # every rank also traced the whole-frame Ticks: world - 1 more copies of them
        pre = rt.Renderer(make_scene(recipe), W, H)
        for f in range(TICK_FRAMES):
            spp, depth, shift, reset = plan[f]
            pre.camera = camera_for(W, H, shift)
            pre.tick_host(spp=spp, depth=depth, frame=f, reset=reset)
        cp = pre.counters()
        for key in ("primary", "shadow", "bounce"):
            c[key] += (world - 1) * cp[key]
    sums = {key: sum(results[k]["counters"][key] for k in range(world)) for key in ("primary", "shadow", "bounce")}
    deal = results[0]["deal"]
    deal_ok = True
    if mode in BALANCED_MODES and world > 1:
        # every rank ends on the same balanced deal, having built at least one
        deal_ok = all(results[k]["deal"]["balanced"] == 1 and results[k]["deal"]["deals_built"] >= 1 for k in range(world))
        deal_ok = deal_ok and len({results[k]["deal"]["hash"] for k in range(world)}) == 1   # one deal everywhere
        if mode == "balanced":   # the primary+shadow deal, then a rebalance on path-traced costs (which
            # may cut the frame where the first deal did); every new deal moved the accumulators
            deal_ok = deal_ok and deal["exchanges"] >= 2 and deal["moves"] == deal["deals_built"]
        if mode == "moving":     # no deal change while the camera moves; the new static camera runs a
            # balancing attempt (which may rebuild the same cut: a valid rebalance either way)
            per, ex = results[0]["deal_per_frame"], results[0]["exchanges_per_frame"]
            deal_ok = deal_ok and per[30:40] == [per[29]] * 10 and ex[30:40] == [ex[29]] * 10 and ex[-1] > ex[39]
        if mode == "after_tick":   # every rank held every tile: the first frame moved nothing
            deal_ok = deal_ok and deal["moves"] == deal["deals_built"]
        if mode == "recreate":   # the new communicator starts interleaved and balances again
            per = results[0]["deal_per_frame"]
            deal_ok = deal_ok and per[RECREATE_AT - 1] == 1 and per[RECREATE_AT] == 0 and per[-1] == 1
    ok = len(got) == len(want) and not bad_frames and not bad_acc and all(sums[key] == c[key] for key in sums) and deal_ok
    print(json.dumps({"ok": ok, "world": world, "mode": mode, "frames": len(got), "bad_frames": bad_frames,
                      "failed_at": results[0]["failed_at"],
                      "bad_acc_ranks": bad_acc, "counters": sums, "want_counters": {k: c[k] for k in sums},
                      "deal": deal, "deal_ok": deal_ok,
                      "first_balanced_frame": next((f for f, b in enumerate(results[0]["deal_per_frame"]) if b), None)}),
          flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
