#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary + shadow) of the MI355X ray-tracing hot path.

Workload (BASELINE.json configs[1]): teapot.obj scene TEAPOT-F at
1920x1080, 1 spp, primary + shadow = Renderer::Trace at depth 1 (one closest-hit ray
per pixel, one NEE shadow ray per diffuse hit facing the light), accumulate + RGB8 pack,
all in one kernel launch per frame (a "step").  Inputs are resident in HBM before
timing; synthetic data = the bundled teapot mesh + the synthetic constant sky.

N > 1 (python -m torch.distributed.run ... bench.py --gpus N): weak scaling -- the
frame's 8x8 tiles are interleaved over the ranks and the frame is rendered at spp = N,
so every GPU traces one 1080p frame's worth of samples per step; one RCCL gather of
the packed RGB8 tiles to rank 0 per frame assembles the image there.  The
gather of frame i runs while frame i+1 renders (double-buffered tiles); the timed region
ends after the last frame's gather and assembly.
value = all rays traced by all ranks / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import advancedgraphicsraytracer_amd as rt  # noqa: E402

# Algorithmic bytes per ray, SURVEY.md 8(d): B = 32*A + 40*P (+36 B pixel IO per camera
# sample), A = BVH node reads (one 32-B node per child test), P = primitive tests (4-B index
# + 36-B triangle).  A, P measured with the oracle on this exact workload (per-pixel seeds,
# Trace depth 1); see DESIGN.md section 4.
BYTES_PER_RAY = {
    # recipe: (primary incl. 36 B IO, shadow)
    "teapotF": (32 * 14.235 + 40 * 1.635 + 36, 32 * 16.719 + 40 * 2.133),
    "mig16": (32 * 23.241 + 40 * 1.835 + 36, 32 * 79.366 + 40 * 8.545),
    "cfg5": (32 * 9.371 + 40 * 1.126 + 36, 32 * 10.611 + 40 * 1.567),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scene", default="teapotF", choices=rt.RECIPES)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--ramp-seconds", type=float, default=0.5,
                    help="untimed frames before the warm-up steps until this much wall time has passed: the "
                         "GPU clocks ramp up over ~0.1 s, and 5 warm-up frames are only ~0.5 ms of work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--per-step-events", action="store_true", help="HIP event pair around every launch at N = 1 too")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the CPU baseline sample")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="HBM traffic per launch from rocprofv3 PMC passes (tools/pmc_summary.py)")
    return ap.parse_args()


def cpu_baseline(args, threads):
    """The oracle (CPU restatement, kind "port") on the same workload, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    s = pyoracle.Scene(args.scene, rt.DATA_DIR)
    W, H = args.width, args.height
    acc = np.zeros((W * H, 4), np.float32)
    s.tick(W, H, acc, spp=args.spp, depth=args.depth, frame=0, threads=threads)   # warm
    frames, rays, t0 = 0, 0, time.perf_counter()
    while True:
        _, st = s.tick(W, H, acc, spp=args.spp, depth=args.depth, frame=frames + 1, threads=threads)
        rays += st["isect"] + st["occl"]
        frames += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{frames} full {W}x{H} {args.scene} frames (spp {args.spp}, Trace depth {args.depth}), "
                      f"{dt:.2f} s wall on {threads} OpenMP threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        args.gpus = world if world > 1 else args.gpus
    dist = None
    # one rank per GPU; RT_DIST_BACKEND=gloo + fewer GPUs than ranks rehearses the N > 1 path
    # on a single card (ranks share it; the exchange goes through gloo instead of RCCL)
    device = local % max(1, torch.cuda.device_count()) if world > 1 else 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(device)
        backend = os.environ.get("RT_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(device)

    W, H = args.width, args.height
    spp = args.spp * world                 # weak scaling: spp grows with the tile share shrinking
    scene = rt.Scene.recipe(args.scene, device=device)
    rend = rt.Renderer(scene, W, H)
    stream = torch.cuda.Stream(device=device)
    sptr = stream.cuda_stream
    frame_out = torch.zeros(W * H, dtype=torch.int32, device=f"cuda:{device}")
    sharded = None
    if world > 1:
        from advancedgraphicsraytracer_amd.distributed import ShardedFrame
        sharded = ShardedFrame(rend, device=torch.device("cuda", device))

    def step(i, events=None):
        with torch.cuda.stream(stream):
            if sharded is not None:
                # the one collective per frame: frame i's packed tiles are gathered while
                # frame i+1 renders; rank 0 assembles frame i once its gather is done
                sharded.submit(spp=spp, depth=args.depth, frame=i, stream=sptr, events=events)
                return
            if events is not None:
                events[0].record(stream)
            rend.Tick(frame_out, spp=spp, depth=args.depth, frame=i, stream=sptr)
            if events is not None:
                events[1].record(stream)

    def drain():
        if sharded is not None:
            with torch.cuda.stream(stream):
                sharded.flush(stream=sptr)

    # clock ramp (untimed, before the W warm-up steps): blocks of 20 frames until
    # --ramp-seconds have passed; at N > 1 the ranks agree on every block (the per-frame
    # gather is a collective, so every rank must submit the same frames)
    nf = 0
    t_ramp = time.perf_counter()
    while args.ramp_seconds > 0:
        for _ in range(20):
            step(nf)
            nf += 1
        drain()
        torch.cuda.synchronize(device)
        more = torch.tensor([1 if time.perf_counter() - t_ramp < args.ramp_seconds else 0], device=f"cuda:{device}")
        if dist:
            dist.all_reduce(more, op=dist.ReduceOp.MIN)
        if not more.item():
            break
    ramp_frames = nf
    for i in range(args.warmup):
        step(nf)
        nf += 1
    drain()
    torch.cuda.synchronize(device)
    c0 = rend.counters()
    # HIP events on the launch stream: at N = 1 one pair brackets the timed region (per-launch
    # average = region / steps; no event packets between the frames), at N > 1 a pair around
    # each shard render (the exchange runs between them)
    per_step_events = world > 1 or args.per_step_events
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps if per_step_events else 1)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    if not per_step_events:
        evs[0][0].record(stream)
    for k in range(args.steps):
        step(nf + k, evs[k] if per_step_events else None)
    if not per_step_events:
        evs[0][1].record(stream)
    drain()                                 # the last frame's gather + assembly are inside the timed region
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    c1 = rend.counters()
    elapsed = t1 - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs])) / (1 if per_step_events else args.steps)
    primary = c1["primary"] - c0["primary"]
    shadow = c1["shadow"] - c0["shadow"]
    bounce = c1["bounce"] - c0["bounce"]
    local_rays = torch.tensor([primary + shadow + bounce, primary, shadow], dtype=torch.float64, device=f"cuda:{device}")
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
    if dist:
        dist.all_reduce(local_rays, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    tot_rays, tot_primary, tot_shadow = local_rays.tolist()
    wall = t_max.item()

    if rank == 0:
        bp, bs = BYTES_PER_RAY.get(args.scene, (None, None))
        roofline = None
        if bp is not None and args.depth == 1:
            per_launch = (primary * bp + shadow * bs) / args.steps     # this rank's launch
            achieved = per_launch / (kern_ms * 1e-3) / 1e9
            traffic = valu = None
            try:
                with open(args.pmc_json) as f:
                    pmc = json.load(f)
                key = f"{args.scene}_{W}x{H}_spp{spp}_d{args.depth}"
                if key in pmc:
                    traffic = pmc[key]["hbm_bytes_per_launch"]
                    valu = pmc[key].get("valu_insts_per_launch")
            except (OSError, ValueError, KeyError):
                traffic = None
            roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                        "kernel": rend.kernel_name(spp=spp, depth=args.depth), "kernel_ms": round(kern_ms, 4),
                        "bytes_per_ray": {"primary": round(bp, 1), "shadow": round(bs, 1)},
                        # the algorithmic node / triangle bytes are served by L1/L2 (the scene is
                        # ~0.1 MB): frac > 1 means "beyond the HBM roofline"; the HBM bytes the
                        # PMC counters see per launch, and their rate, are these
                        "hbm_measured_gbs": round(traffic / (kern_ms * 1e-3) / 1e9, 2) if traffic else None,
                        "hbm_measured_frac": round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if traffic else None,
                        # the binding resource: vector issue.  SQ_INSTS_VALU per launch (PMC pass) x 2
                        # cycles per wave64 instruction over 1,024 SIMDs x the launch's cycles at 2.4 GHz
                        "valu_issue_frac": round(valu * 2 / (1024 * kern_ms * 1e-3 * 2.4e9), 4) if valu else None}
        line = {
            "metric": "Mrays/s (primary+shadow) at 1080p",
            "value": round(tot_rays / wall / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_ramp_frames": ramp_frames,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: bundled teapot.obj mesh (SURVEY 8(d) TEAPOT-F recipe) + constant 1024x512 sky, "
                    "per-pixel seeds InitSeed(pixel + W*H*(sample + spp*frame))",
            "config": {"workload": f"{args.scene} {W}x{H}, spp {spp} ({args.spp} per GPU-frame share), "
                                   f"Trace depth {args.depth} (primary + NEE shadow), accumulate + RGB8",
                       "scene": args.scene, "width": W, "height": H, "spp": spp, "depth": args.depth,
                       "parallelism": f"screen-tile x{world}" if world > 1 else "single GPU"},
            "fps": round(args.steps / wall, 3),
            "msamples_per_s": round(W * H * spp / (wall / args.steps) / 1e6, 3),
            "rays": {"primary": int(tot_primary), "shadow": int(tot_shadow), "total": int(tot_rays)},
            "roofline": roofline,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                threads = max(1, min(16, len(os.sched_getaffinity(0))))
                line["cpu_baseline"] = cpu_baseline(args, threads)
            except Exception as e:   # the baseline is reported, never the product
                line["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
