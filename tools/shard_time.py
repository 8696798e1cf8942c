#!/usr/bin/env python3
"""Per-rank frame time of bench.py's N > 1 workload, measured on one GPU: every rank's share of
the frame (its 1/N of the tiles) rendered back to back on a renderer of its own, for N = 1, 2,
4, 8; the slowest rank bounds the frame.  Predicts the driver's scaling efficiency up to the
gather.  Deals: "interleaved" (t % N, rt_render_shard), "balanced" (rt_tile_deal over the
dry-run work map of a full frame, rt_renderer_tile_work -- what RT_MULTI_BALANCED cuts since round
5 -- rendered with rt_render_shard_tiles), "balanced_cycles" (the same over the measured wave
cycles of a full frame, round 4's deal input) or "blocksB" (BxB-tile blocks round-robin).
Weak scaling: spp = N x --spp per rank; --strong: one frame of --spp split N ways.

usage: shard_time.py [--scene teapotF] [--depth 1] [--spp S] [--strong] [--deal interleaved,balanced]
                     [--frames 30] [--warm 80] [--ranks all|last] [--out file.jsonl]
(RT_SPLIT_UNITS=U: split threshold; RT_PS_PIPELINE / RT_PS_DEPTH: frames in flight)"""
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


def time_share(scene, a, spp, frames, render):
    """warm-up frames (walk timing, tile order, frames-in-flight timing), then `frames` timed."""
    r = rt.Renderer(scene, a.w, a.h)
    st = torch.cuda.Stream()
    f, t0 = 0, time.perf_counter()
    while f < a.warm or time.perf_counter() - t0 < a.warm_seconds:   # past the renderer's tuning gate
        render(r, spp, f, st.cuda_stream)
        f += 1
        if f % 200 == 0:   # rare syncs: the renderer's timed groups (up to 32 frames) run back to back
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    c0 = r.counters()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(st):
        ev[0].record()
        h0 = time.perf_counter()
        for f in range(frames):
            render(r, spp, 100000 + f, st.cuda_stream)
        h1 = time.perf_counter()
        ev[1].record()
    torch.cuda.synchronize()
    c1 = r.counters()
    ms = ev[0].elapsed_time(ev[1]) / frames
    rays = sum(c1[k] - c0[k] for k in ("primary", "shadow", "bounce")) / frames
    od = r.overlap_depth()
    out = {"ms": round(ms, 4), "host_ms": round((h1 - h0) * 1e3 / frames, 4), "mrays": round(rays / 1e6, 3), "in_flight": od[0], "choices": r.choices(),
           "in_flight_groups_ms": [round(float(x), 4) for x in od[1]]}
    cost = r.tile_costs().astype(np.float64)
    if cost.size:
        out["tile_cycles_max"] = int(cost.max())
        out["tile_cycles_sum"] = int(cost.sum())
    r.close()
    return out, cost


def spread_deal(w, h, n, cost, nheavy):
    """tile lists per rank: the nheavy costliest tiles snake-dealt, the rest cut in Morton order so
    that every rank's summed cost is the frame's / n (as far as whole tiles allow)"""
    tx, ty = (w + 7) // 8, (h + 7) // 8
    nt = tx * ty
    cost = np.asarray(cost, dtype=np.float64)
    order = np.argsort(-cost, kind="stable")
    heavy = order[:nheavy]
    owner = -np.ones(nt, dtype=np.int64)
    hsum = np.zeros(n)
    for i, t in enumerate(heavy):
        k = i % n if (i // n) % 2 == 0 else n - 1 - i % n
        owner[t] = k
        hsum[k] += cost[t]

    def morton(x, y):
        m = 0
        for b in range(16):
            m |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
        return m
    rest = [t for t in range(nt) if owner[t] < 0]
    rest.sort(key=lambda t: morton(t % tx, t // tx))
    rc = cost[rest]
    pre = np.concatenate([[0.0], np.cumsum(rc)])
    target = cost.sum() / n
    cum, start = 0.0, 0
    for k in range(n):
        cum += max(0.0, target - hsum[k])
        end = len(rest) if k == n - 1 else int(np.clip(np.searchsorted(pre, cum), start, len(rest)))
        for t in rest[start:end]:
            owner[t] = k
        start = end
    tiles = np.concatenate([np.nonzero(owner == k)[0] for k in range(n)]).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum([(owner == k).sum() for k in range(n)])]).astype(np.int64)
    return tiles, off


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="teapotF")
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--warm", type=int, default=80, help="untimed frames per renderer (walk, tile order and "
                    "frames-in-flight timing: ~60 frames after the tuning gate)")
    ap.add_argument("--warm-seconds", type=float, default=0.4, help="... and at least this much wall time (the "
                    "renderer's timed choices start after 100 ms of GPU time, RT_TUNE_DELAY_MS)")
    ap.add_argument("--strong", action="store_true", help="the config's spp per shard (one frame split N ways)")
    ap.add_argument("--spp", type=int, default=1, help="samples per pixel of the whole frame (strong) / per GPU (weak)")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--deal", default="interleaved", help="comma list: interleaved, balanced, balanced_cycles, blocksB")
    ap.add_argument("--ranks", default="all", choices=("all", "last"), help="time every rank's share or the last only")
    ap.add_argument("--out", default=None, help="append the summary line to this jsonl file")
    a = ap.parse_args()
    scene = rt.Scene.recipe(a.scene)
    r0 = rt.Renderer(scene, a.w, a.h)                  # GPU clock ramp (untimed), as bench.py
    o0 = torch.zeros(a.w * a.h, dtype=torch.int32, device="cuda")
    t0, f = time.perf_counter(), 0
    while time.perf_counter() - t0 < 0.5:
        r0.Tick(o0, spp=1, depth=a.depth, frame=f)
        f += 1
        if f % 200 == 0:   # rare syncs: the renderer's timed groups (up to 32 frames) run back to back
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    r0.close()
    ns = [int(x) for x in a.ns.split(",")]
    full_cost = None
    deals = a.deal.split(",")
    work_map = None
    if "balanced" in deals or any(d.startswith("spread") for d in deals):   # the product's deal input
        rw = rt.Renderer(scene, a.w, a.h)
        work_map = rw.tile_work(spp=a.spp if a.strong else a.spp * ns[0], depth=a.depth, frame=100000)
        rw.close()
        q = max(1.0, work_map.mean() / 64.0)          # rt_multi.cpp's 1/64-of-the-mean rounding
        work_map = np.floor(work_map / q + 0.5).astype(np.uint32)
    if "balanced_cycles" in deals and "interleaved" not in deals:
        # the balanced deal cuts the measured cost map of a whole frame: measure it first
        spp = a.spp if a.strong else a.spp * ns[0]
        buf = torch.zeros(((a.w + 7) // 8) * ((a.h + 7) // 8) * 64, dtype=torch.int32, device="cuda")
        _, cost = time_share(scene, a, spp, 4, lambda r, spp_, fr, s: r.render_shard(buf, 0, 1, spp=spp_, depth=a.depth,
                                                                                      frame=fr, stream=s))
        full_cost = cost.astype(np.uint32)
    res = {}
    for deal in a.deal.split(","):
        out = {}
        for n in ns:
            spp = a.spp if a.strong else a.spp * n
            cap = ((a.w + 7) // 8) * ((a.h + 7) // 8) * 64
            buf = torch.zeros(cap, dtype=torch.int32, device="cuda")
            if deal == "balanced":
                tiles, off = rt.tile_deal(a.w, a.h, n, work_map)
            elif deal == "balanced_cycles":
                tiles, off = rt.tile_deal(a.w, a.h, n, full_cost if (full_cost is not None and full_cost.size) else None)
            elif deal.startswith("spread"):   # spreadK: the K*n costliest tiles (work map) dealt snake-wise, the
                # rest in Morton runs that even out each rank's total work (heavy chains shared out)
                K = int(deal[6:] or 4)
                tiles, off = spread_deal(a.w, a.h, n, work_map, K * n)
            elif deal.startswith("blocks"):   # blocksB: BxB-tile blocks dealt round-robin (block b -> rank b % n)
                B = int(deal[6:] or 8)
                tx, ty = (a.w + 7) // 8, (a.h + 7) // 8
                t = np.arange(tx * ty)
                bx, by = (t % tx) // B, (t // tx) // B
                blk = by * ((tx + B - 1) // B) + bx
                owner = blk % n
                order = np.lexsort((t, blk))
                tiles = np.concatenate([order[owner[order] == k] for k in range(n)]).astype(np.uint32)
                off = np.concatenate([[0], np.cumsum([(owner == k).sum() for k in range(n)])]).astype(np.int64)
            ranks = range(n) if a.ranks == "all" else [n - 1]
            per = []
            for k in ranks:
                if deal.startswith("balanced") or deal.startswith("blocks") or deal.startswith("spread"):
                    mine = tiles[off[k]:off[k + 1]]
                    render = lambda r, spp_, fr, s, mine=mine: r.render_shard_tiles(buf, mine, spp=spp_, depth=a.depth, frame=fr, stream=s)
                else:
                    render = lambda r, spp_, fr, s, k=k, n=n: r.render_shard(buf, k, n, spp=spp_, depth=a.depth, frame=fr, stream=s)
                t, cost = time_share(scene, a, spp, a.frames, render)
                if n == 1 and deal == "interleaved" and full_cost is None:
                    full_cost = cost.astype(np.uint32)
                per.append(t)
            worst = max(per, key=lambda x: x["ms"])
            out[n] = {"ms_per_frame_max_rank": worst["ms"], "ms_per_frame_mean_rank": round(float(np.mean([p["ms"] for p in per])), 4),
                      "in_flight_max_rank": worst["in_flight"], "per_rank": per}
            print(deal, n, json.dumps({k: v for k, v in out[n].items() if k != "per_rank"}), flush=True)
        base = out[ns[0]]["ms_per_frame_max_rank"] * ns[0] if a.strong else out[ns[0]]["ms_per_frame_max_rank"]
        eff = {n: round((base / (v["ms_per_frame_max_rank"] * n)) if a.strong else (base / v["ms_per_frame_max_rank"]), 3)
               for n, v in out.items()}
        res[deal] = {"per_n": out, "predicted_efficiency_without_gather": eff}
    line = json.dumps({"scene": a.scene, "depth": a.depth, "spp": a.spp, "strong": a.strong, "size": [a.w, a.h],
                       "ps": os.environ.get("RT_PS_PIPELINE", "-1"), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "deals": res})
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as fo:
            fo.write(line + "\n")


if __name__ == "__main__":
    main()
