#!/usr/bin/env python3
"""The costliest tiles of a primary+shadow frame, explained by their rays' traversal work.

Renders a parameter set until the renderer has recorded its per-tile wave cycles (the cost map
behind the longest-tile-first order, rt_renderer_tile_costs), then takes the dry-run work map of
the same frame with per-pixel counters (rt_renderer_tile_work: closest-hit node visits / prim
tests for the camera rays, any-hit node visits / prim tests for the shadow rays -- camera rays in
the reference's IntersectBVH order, shadow rays in the library's farther-box-first order).  For
the --top costliest tiles by cycles it prints the lane with the longest chain (node visits of its
camera + shadow ray), the tile's mean lane, how many lanes are within half of the longest, and the
camera / shadow split; then how well the work map predicts the cycles over all tiles (the balanced
multi-GPU deals are cut on the work map).

usage: tail_tiles.py [--scene mig16] [--w 1920 --h 1080] [--top 32] [--json out.json]
"""
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
    ap.add_argument("--scene", default="mig16")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--top", type=int, default=32)
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--depth", type=int, default=1, help="> 1: path-traced frames (cycles = level-0 cost map)")
    ap.add_argument("--walk", choices=("lane", "auto"), default="lane",
                    help="camera walk of the rendered frames (lane: the order the work map counts)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    g = rt.Scene.recipe(a.scene)
    if a.walk == "lane":
        g.set_camera_walk(rt.WALK_LANE)
    W, H = a.w, a.h
    r = rt.Renderer(g, W, H)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    f, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 1.0 or r.tile_costs().size == 0:   # past the tuning gate: costs recorded
        for _ in range(20):
            r.Tick(out, spp=a.spp, depth=a.depth, frame=0, stream=st.cuda_stream)
            f += 1
        torch.cuda.synchronize()
        if time.perf_counter() - t0 > 20:
            break
    cyc = r.tile_costs().astype(np.float64)
    work, px = r.tile_work(spp=a.spp, depth=a.depth, frame=0, pixels=True)
    tx, ty = (W + 7) // 8, (H + 7) // 8

    def tiles(v):
        p = np.zeros((ty * 8, tx * 8), np.int64)
        p[:H, :W] = v.reshape(H, W)
        return p.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)

    cam_n, cam_p, sh_n, sh_p = (tiles(px[:, k].astype(np.int64)) for k in range(4))
    chain = cam_n + sh_n
    res = {"scene": a.scene, "size": [W, H], "spp": a.spp, "depth": a.depth, "frames_rendered": f, "walk": a.walk,
           "cycles_mean": round(float(cyc.mean()), 1), "cycles_max": int(cyc.max()),
           "chain_mean_lane": round(float(chain.mean()), 2), "chain_max_lane": int(chain.max())}
    top = np.argsort(-cyc)[:a.top]
    rows = []
    for t in top:
        lmax = int(chain[t].argmax())
        rows.append({"tile": int(t), "xy": [int(t % tx) * 8, int(t // tx) * 8], "cycles": int(cyc[t]),
                     "cycles_over_mean": round(float(cyc[t] / cyc.mean()), 2),
                     "chain_max_lane": int(chain[t, lmax]), "chain_mean_lane": round(float(chain[t].mean()), 1),
                     "lanes_within_half_of_max": int((chain[t] >= 0.5 * chain[t, lmax]).sum()),
                     "max_lane_camera_nodes_prims": [int(cam_n[t, lmax]), int(cam_p[t, lmax])],
                     "max_lane_shadow_nodes_prims": [int(sh_n[t, lmax]), int(sh_p[t, lmax])],
                     "tile_camera_nodes_prims": [int(cam_n[t].sum()), int(cam_p[t].sum())],
                     "tile_shadow_nodes_prims": [int(sh_n[t].sum()), int(sh_p[t].sum())],
                     "work_over_mean": round(float(work[t] / work.mean()), 2)})
    res["top"] = rows
    # how well per-tile work predicts per-tile cycles (the deal's input vs what it stands for)
    preds = {"work_sum": work.astype(np.float64), "chain_max_lane": chain.max(axis=1).astype(np.float64),
             "chain_sum": chain.sum(axis=1).astype(np.float64)}
    res["corr_with_cycles"] = {k: round(float(np.corrcoef(v, cyc)[0, 1]), 4) for k, v in preds.items()}
    # the exact pop-time cull's ceiling: closest-hit pops of entries already beyond the ray's t
    ch = float(px[:, 0].sum())
    res["pop_cull_ceiling"] = {"interior_pops_beyond_t_over_ch_visits": round(float(px[:, 4].sum()) / ch, 4),
                               "leaf_pops_beyond_t_over_ch_visits": round(float(px[:, 5].sum()) / ch, 4),
                               "ch_visits_over_all_visits": round(ch / float(px[:, 0].sum() + px[:, 2].sum()), 4)}
    top_share = {}
    for k, v in preds.items():   # overlap of the top-N by cycles and by the predictor
        tp = set(np.argsort(-v)[:a.top].tolist())
        top_share[k] = len(tp & set(top.tolist())) / a.top
    res["top_overlap_with_cycles"] = top_share
    print(json.dumps({k: v for k, v in res.items() if k != "top"}))
    for row in rows[:10]:
        print(json.dumps(row))
    if a.json:
        with open(a.json, "w") as fo:
            json.dump(res, fo, indent=1)
    r.close()


if __name__ == "__main__":
    main()
