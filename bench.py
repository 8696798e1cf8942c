#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary + shadow) of the MI355X ray-tracing hot path.

Default workload (BASELINE.json configs[1], "config 2"): teapot.obj scene TEAPOT-F
 at 1920x1080, 1 spp, primary + shadow = Renderer::Trace at depth 1 (one
closest-hit ray per pixel, one NEE shadow ray per diffuse hit facing the light),
accumulate + RGB8 pack, all in one kernel launch per frame (a "step").  Inputs are
resident in HBM before timing; synthetic data = the bundled teapot mesh + the synthetic
constant sky.  --config 3 / 4 / 5 select the other BASELINE.json GPU workloads:
CFG3-sub 4 spp depth 4, mig29 x16 primary + shadow, CFG5-sub 16 spp depth 10.

N > 1 (python -m torch.distributed.run ... bench.py --gpus N): the frame's 8x8 tiles are
interleaved over the ranks, each rank renders its shard, ONE RCCL gather per frame brings
the packed tiles to rank 0, which assembles the image.  The exchange is
the library's C-ABI (rt_render_frame_multi: RCCL issued from C++, pipelined so frame i's
gather runs beside frame i+1's render).  Scaling: config 2 and 3 are weak (spp = N x the
config's spp: every GPU traces one frame's worth of samples per step), config 4 and 5 are
strong (one frame split over the N GPUs); --scaling overrides.
value = all rays traced by all ranks / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time


def _gpus_arg(argv):
    """--gpus N from the command line (any prefix argparse would accept: --gpu, --gp), else 1."""
    n = 1
    for i, a in enumerate(argv):
        key, eq, val = a.partition("=")
        if len(key) >= 4 and "--gpus".startswith(key):
            n = int(val if eq else (argv[i + 1] if i + 1 < len(argv) else "1"))
    return n


def launch_plan(argv, env):
    """How many rank processes bench.py must start itself, decided before anything loads HIP.

    A launcher (python -m torch.distributed.run, or any that exports WORLD_SIZE) owns the ranks: 0.
    `python bench.py --gpus N` with N > 1 and no WORLD_SIZE: N -- the parent then only spawns N
    child processes of this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set and never
    touches the GPU itself; silently rendering on one GPU under `--gpus N` would report N = 1 as N."""
    if env.get("WORLD_SIZE"):
        return 0
    n = _gpus_arg(argv)
    if n < 1:
        raise SystemExit(f"bench: --gpus {n}: need at least one GPU")
    return n if n > 1 else 0


def _die_with_parent():   # child side of fork, before exec: SIGKILL when the launcher dies
    try:
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, 9)   # PR_SET_PDEATHSIG, SIGKILL
    except OSError:
        pass


def spawn_ranks(n, argv, script=None, poll_s=0.2):
    """Run N rank processes of `script` (this file) on 127.0.0.1 and wait for all of them.  Their
    stdout / stderr are this process's (rank 0 prints the one JSON line).  The first rank to fail
    ends the others (its own PID only) and its status becomes the launcher's exit status; SIGTERM /
    SIGINT to the launcher are passed on."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = script or os.path.abspath(__file__)
    procs = []

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
        t_end = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def on_signal(sig, _frame):
        stop_all(sig)
        sys.exit(128 + sig)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RT_BENCH_LAUNCHER="bench.py")
            procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                                          preexec_fn=_die_with_parent))
        status = 0
        while [p.poll() for p in procs].count(None):   # poll every rank (any() would stop at the first live one)
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                status = bad[0]
                print(f"bench: a rank exited with status {status}; stopping the other ranks", file=sys.stderr, flush=True)
                stop_all()
                break
            time.sleep(poll_s)
        if status == 0:
            status = next((p.returncode for p in procs if p.returncode), 0)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return 128 - status if status < 0 else status   # killed by signal k: 128 + k, as a shell reports it


if __name__ == "__main__":
    _n_spawn = launch_plan(sys.argv[1:], os.environ)
    if _n_spawn:
        sys.exit(spawn_ranks(_n_spawn, sys.argv[1:]))
    if os.environ.get("RT_BENCH_LAUNCH_CHECK"):   # tests/test_bench_launch.py: the rank's view, no GPU
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT", "RT_BENCH_LAUNCHER")}), flush=True)
        _mode = os.environ["RT_BENCH_LAUNCH_CHECK"].partition(":")
        if _mode[0] == "fail":   # "fail:R": rank R exits 3, the others wait as if in a collective
            if os.environ.get("RANK") == _mode[2]:
                sys.exit(3)
            time.sleep(600)
        sys.exit(0)


def _queues_wanted(argv, world):
    """Hardware queues this command line (--config / --depth) wants, before anything loads HIP:
    16 for config 5 split over N > 1 ranks, 8 for path tracing (trace depth > 1), config 4 and any
    N > 1 run, else None (the environment's / HIP's default)."""
    cfg, depth = 2, None
    for i, a in enumerate(argv):
        key, _, val = a.partition("=")
        if not val and i + 1 < len(argv):
            val = argv[i + 1]
        if key == "--config":
            cfg = int(val)
        elif key == "--depth":
            depth = int(val)
    pt = (depth if depth is not None else {3: 4, 5: 10}.get(cfg, 1)) > 1
    if world > 1 and (cfg == 5 and pt or cfg == 2 and depth in (None, 1)):
        return 16   # config 5 split over the ranks: the default config-2 run times it too (config5)
    return 8 if (pt or cfg == 4 or world > 1) else None


# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues per process (4 by default).  Path
# tracing: the renderer's two path streams then share a queue with the launch stream, whose
# finishing-pass barrier holds back the next frame's levels -- 8 queues, CFG3-sub 2.05 -> 1.92
# ms (profiles/r02/bench_pipe_bhq*.json).  Multi-GPU frames (N > 1) too, since overlapped
# primary+shadow frames: their two renderer streams and the communicator's stream then no longer
# share a queue with the caller's (world-1 multi frame, mig29 x16: 0.471 -> 0.327 ms; TEAPOT-F
# 0.128 either way; profiles/r02/multi_overhead_hwq8.log).  Config 4 at N = 1 too: its frames in
# flight (up to 6 renderer streams) no longer share queues -- 0.3045 / 0.3005 -> 0.280 / 0.270 ms
# (profiles/r03/hwq_ab/).  Config 2 keeps HIP's default: with 8 queues its timed choice drifted to
# 2 frames in flight and the frame to 0.108-0.120 ms.  Config 5 at N > 1 (each rank a 1/N shard of
# 4 M paths, 8 path-state slots = 8 renderer streams beside the caller's and the communicator's):
# 16 queues, 1/8 shard 1.219 / 1.205 -> 1.152 / 1.162 ms interleaved A/B (profiles/r05/c5/
# hwqab.jsonl; config 4 / 2 shards neutral; config 3 at N = 1 slower with 16).  Set before HIP
# initialises.
# The box may export its own value (HIP's default is 4): the bench sets 8 explicitly where its
# design needs it and records the value in effect (config.hip_hw_queues).  --hw-queues N
# overrides; never above 32 (the pool refuses more).
_HWQ_BEFORE = os.environ.get("GPU_MAX_HW_QUEUES")
_HWQ_ARG = next((a.partition("=")[2] or (sys.argv[i + 2] if i + 2 < len(sys.argv) else "")
                 for i, a in enumerate(sys.argv[1:]) if a.startswith("--hw-queues")), None)
_HWQ_WANT = _queues_wanted(sys.argv[1:], int(os.environ.get("WORLD_SIZE", "1")))
if _HWQ_ARG:
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, int(_HWQ_ARG))))
elif _HWQ_WANT:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_HWQ_WANT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import advancedgraphicsraytracer_amd as rt  # noqa: E402
import roofline as rl  # noqa: E402

# BASELINE.json configs[1..4]: scene recipe, spp, Trace depth, N > 1 scaling,
# dominant kernel (the roofline's subject; profiles/pmc_summary.json key cfgN)
CONFIGS = {
    2: dict(scene="teapotF", spp=1, depth=1, scaling="weak", kernel="k_render"),
    3: dict(scene="cfg3", spp=4, depth=4, scaling="weak", kernel="k_pt_lanes"),
    4: dict(scene="mig16", spp=1, depth=1, scaling="strong", kernel="k_render"),
    5: dict(scene="cfg5", spp=16, depth=10, scaling="strong", kernel="k_pt_lanes"),
}
# Algorithmic bytes per ray, SURVEY.md 8(d): B = 32*A + 40*P (+36 B pixel IO per camera
# sample), A = BVH node reads (one 32-B node per child test), P = primitive tests (4-B index
# + 36-B triangle).  A, P measured with the oracle on these workloads (per-pixel seeds, Trace
# depth 1); DESIGN.md section 5.  Not a roofline: those bytes are L1/L2 hits.
BYTES_PER_RAY = {
    "teapotF": (32 * 14.235 + 40 * 1.635 + 36, 32 * 16.719 + 40 * 2.133),
    "mig16": (32 * 23.241 + 40 * 1.835 + 36, 32 * 79.366 + 40 * 8.545),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--scene", default=None, choices=rt.RECIPES)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None)
    ap.add_argument("--ramp-seconds", type=float, default=0.5,
                    help="untimed frames before the warm-up steps until this much wall time has passed: the "
                         "GPU clocks ramp up over ~0.1 s, and 5 warm-up frames are only ~0.5 ms of work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-companion", action="store_true", help="skip the 1280x720 companion run (profiling runs: "
                    "its frames would share the frame kernel's name in the kernel trace)")
    ap.add_argument("--per-step-events", action="store_true", help="HIP event pair around every launch at N = 1 too")
    ap.add_argument("--extra-configs", default="4,3,5", help="BASELINE configs timed after a default config-2 "
                    "headline in the same process (EXTRA_CONFIGS: strong_config4, config3, config5)")
    ap.add_argument("--no-strong", action="store_true", help="skip every extra config line (strong_config4, config3, config5) "
                    "that default config-2 runs add after the headline")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the all-cores CPU baseline sample")
    ap.add_argument("--summary", default=rl.SUMMARY, help="rocprofv3 PMC / kernel-trace summary (tools/roofline.py)")
    ap.add_argument("--hw-queues", type=int, default=None, help="GPU_MAX_HW_QUEUES for this run (applied before HIP "
                    "starts; default: 8 for path-traced and N > 1 runs, else the environment's / HIP's default)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    args.scene = args.scene or cfg["scene"]
    args.spp = args.spp or cfg["spp"]
    args.depth = args.depth if args.depth is not None else cfg["depth"]
    args.scaling = args.scaling or cfg["scaling"]
    return args


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args, spp):
    """The oracle (CPU restatement, kind "port") on the same workload: a bounded sample on
    all the host threads this job may use (OMP_NUM_THREADS, which the GPU box sets to its
    CPU share, else the affinity mask), and one frame on 1 core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    s = pyoracle.Scene(args.scene, rt.DATA_DIR)
    W, H = args.width, args.height
    acc = np.zeros((W * H, 4), np.float32)
    s.tick(W, H, acc, spp=spp, depth=args.depth, frame=0, threads=threads)   # warm
    frames, rays, t0 = 0, 0, time.perf_counter()
    while True:
        _, st = s.tick(W, H, acc, spp=spp, depth=args.depth, frame=frames + 1, threads=threads)
        rays += st["isect"] + st["occl"]
        frames += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    # one core: rows of one frame until ~1/3 of the all-cores budget has passed
    t1, rays1, y = time.perf_counter(), 0, 0
    while y < H and time.perf_counter() - t1 < args.cpu_seconds / 3:
        y1 = min(H, y + 60)
        _, st = s.tick(W, H, acc, spp=spp, depth=args.depth, frame=frames + 1, y0=y, y1=y1, threads=1)
        rays1 += st["isect"] + st["occl"]
        y = y1
    dt1 = time.perf_counter() - t1
    value, single = rays / dt / 1e6, rays1 / dt1 / 1e6
    out = {"value": round(value, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": f"{frames} full {W}x{H} {args.scene} frames (spp {spp}, Trace depth {args.depth}) in "
                     f"{dt:.2f} s on {threads} OpenMP threads; 1 core: rows 0-{y} of one frame in {dt1:.2f} s",
           "single_core": round(single, 3), "cpu_model": cpu_model(), "host_cpus": os.cpu_count()}
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    try:   # the restatement against the reference, both timed in the build container
        with open(cal) as f:
            c = json.load(f).get(f"config{args.config}")
        if c:
            out["calibration"] = {"restatement_over_reference": c["ratio_threads"],
                                  "restatement_over_reference_1core": c["ratio_1core"], "source": "profiles/cpu_calibration.json",
                                  "reference_equivalent_mrays": round(value / c["ratio_threads"], 3)}
    except (OSError, ValueError, KeyError):
        pass
    return out


def companion_rate(scene, W, H, spp, depth, stream, device, warm_s=0.4, frames=300):
    """The same workload at another frame size on a renderer of its own (BASELINE.json's
    metric is quoted at 1280x720 and 1920x1080): warm-up frames for warm_s seconds (the
    renderer's timed choices -- camera walk, split order, frames in flight -- start after 100 ms
    of GPU time and take ~100 frames), then `frames` timed frames between two stream events and a
    wall clock."""
    r = rt.Renderer(scene, W, H)
    out = torch.zeros(W * H, dtype=torch.int32, device=f"cuda:{device}")
    sptr = stream.cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        warm, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < warm_s:
            for _ in range(20):
                r.Tick(out, spp=spp, depth=depth, frame=warm, stream=sptr)
                warm += 1
            torch.cuda.synchronize(device)
        c0 = r.counters()
        t0 = time.perf_counter()
        e0.record(stream)
        for i in range(frames):
            r.Tick(out, spp=spp, depth=depth, frame=warm + i, stream=sptr)
        e1.record(stream)
        torch.cuda.synchronize(device)
        wall = time.perf_counter() - t0
    c1 = r.counters()
    rays = sum(c1[k] - c0[k] for k in ("primary", "shadow", "bounce"))
    return {"width": W, "height": H, "spp": spp, "depth": depth, "frames": frames, "overlapped": r.overlap()[0], "in_flight": r.overlap_depth()[0],
            "ms_per_frame": round(wall / frames * 1e3, 4), "frame_ms_events": round(e0.elapsed_time(e1) / frames, 4),
            "mrays_s": round(rays / wall / 1e6, 3), "fps": round(frames / wall, 3)}


# The other BASELINE.json GPU configs, timed after the headline in the same process (default
# config-2 runs): name, scene, spp per GPU, Trace depth, N > 1 scaling, balanced deal, timed frames
EXTRA_CONFIGS = {
    4: dict(key="strong_config4", scene="mig16", spp=1, depth=1, scaling="strong", balanced=True, frames=200),
    3: dict(key="config3", scene="cfg3", spp=4, depth=4, scaling="weak", balanced=False, frames=100),
    5: dict(key="config5", scene="cfg5", spp=16, depth=10, scaling="strong", balanced=False, frames=30),
}


def extra_config(cfg_no, world, rank, device, dist, stream, summary, backend="nccl", warm_s=1.5, max_warm_s=12.0):
    """One more BASELINE.json config (EXTRA_CONFIGS) beside the default headline, in the same process
    after it, so the driver's own runs time every GPU config: config 4 (mig29 x16, 1080p, 1 spp,
    primary + shadow) is north_star's strong-scaling case -- ONE frame split over the N ranks with the
    cost-balanced deal (RT_MULTI_BALANCED); config 3 (CFG3-sub, 4 spp, depth 4) is weak (each rank a
    1/N shard at spp 4N, interleaved deal); config 5 (CFG5-sub, 16 spp, depth 10) is strong (one
    frame split, interleaved deal: the bounce levels' cost is not the camera rays').  All go
    through rt_render_frame_multi (pipelined) at N > 1 and through Tick at N = 1 (with
    RT_DIST_BACKEND=gloo, the rehearsal on one card, through ShardedFrame's torch.distributed gather).
    Warm-up: blocks of frames until warm_s seconds have passed (and, for config 4 at N > 1, every
    rank renders under the balanced deal; the renderer's timed choices re-run on the new deal's
    tiles), agreed over the ranks.  Then `frames` frames timed between a barrier + synchronize on
    both sides, max over ranks; then an untimed instrumented pass for every rank's render /
    exposed-gather split.  The roofline row is the config's dominant kernel from the tracked PMC
    summary (serial frames)."""
    from advancedgraphicsraytracer_amd.distributed import NativeCommUnavailable, NativeShardedFrame, ShardedFrame
    ec = EXTRA_CONFIGS[cfg_no]
    W, H, depth = 1920, 1080, ec["depth"]
    spp = ec["spp"] * world if ec["scaling"] == "weak" else ec["spp"]
    frames = ec["frames"]
    dev = f"cuda:{device}"
    sc = rt.Scene.recipe(ec["scene"], device=device)
    rx = rt.Renderer(sc, W, H)
    out = torch.zeros(W * H, dtype=torch.int32, device=dev)
    sptr = stream.cuda_stream
    sf, native = None, False
    if world > 1:
        if backend == "nccl":
            try:
                sf = NativeShardedFrame(rx, device=torch.device("cuda", device), balanced=ec["balanced"])
                native = True
            except NativeCommUnavailable:   # raised on every rank together: torch's gather instead
                sf = None
        if sf is None:
            sf = ShardedFrame(rx, device=torch.device("cuda", device))

    def step(i):
        with torch.cuda.stream(stream):
            if sf is not None:
                sf.submit(spp=spp, depth=depth, frame=i, stream=sptr)
            else:
                rx.Tick(out, spp=spp, depth=depth, frame=i, stream=sptr)

    def drain():
        if sf is not None:
            with torch.cuda.stream(stream):
                sf.flush(stream=sptr)

    block = 100 if depth == 1 else 8   # long blocks: the renderer's timed groups (up to 32 frames) fit between syncs
    nf, t0 = 0, time.perf_counter()
    while True:
        for _ in range(block):
            step(nf)
            nf += 1
        drain()
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
        ready = el >= warm_s and (not native or not ec["balanced"] or sf.deal_info()["balanced"] == 1)
        go = torch.tensor([1 if (ready or el > max_warm_s) else 0], device=dev)
        if dist:
            dist.all_reduce(go, op=dist.ReduceOp.MIN)
        if go.item():
            break
    c0 = rx.counters()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    for k in range(frames):
        step(nf + k)
    drain()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    wall = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
    c1 = rx.counters()
    per = [c1[k] - c0[k] for k in ("primary", "shadow", "bounce")]
    rays = torch.tensor([sum(per)] + per, dtype=torch.float64, device=dev)
    kind = "primary + NEE shadow" if depth == 1 else "path tracing"
    split = ("one frame split over the ranks (strong)" if ec["scaling"] == "strong"
             else "each rank a 1/N shard at spp N x %d (weak)" % ec["spp"])
    res = {"workload": f"config {cfg_no}: {ec['scene']} {W}x{H}, spp {spp}, Trace depth {depth} ({kind}), {split}",
           "scene": ec["scene"], "spp": spp, "depth": depth, "scaling": ec["scaling"], "frames": frames,
           "warm_frames": nf}
    if sf is not None:
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        if native:
            sf.set_timing(True)
            for k in range(min(frames, 20)):
                step(nf + frames + k)
            drain()
            torch.cuda.synchronize(device)
            rms, gms, n = sf.timing()
            mine = torch.tensor([rms / max(n, 1), gms / max(n, 1)], dtype=torch.float64, device=dev)
            every = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(every, mine)
            di = sf.deal_info()
            res.update(path="rt_render_frame_multi (pipelined, %s)" % ("RT_MULTI_BALANCED" if ec["balanced"] else "interleaved deal"),
                       deal_rank0={"in_use": "balanced" if di["balanced"] else "interleaved", **di},
                       render_ms_per_frame_by_rank=[round(e[0].item(), 4) for e in every],
                       # per rank max(0, gather end - render end); rank 0 receives without waiting for its own
                       # render, so its figure is how much later than its own tiles the peers' arrived
                       gather_ms_per_frame_by_rank=[round(e[1].item(), 4) for e in every])
        else:
            res.update(path=f"ShardedFrame (torch.distributed gather, {backend}; interleaved deal)")
        sf.close()
    else:
        res.update(path="Renderer.Tick", in_flight=rx.overlap_depth()[0])
        if depth == 1:
            res["timed_choices"] = rx.choices()
    w = wall.item()
    tot, prim, shad, bnc = rays.tolist()
    res.update(ms_per_frame=round(w / frames * 1e3, 4), fps=round(frames / w, 3),
               rays_per_frame=round(tot / frames), rays={"primary": int(prim), "shadow": int(shad), "bounce": int(bnc)},
               mrays_s=round(tot / w / 1e6, 3),
               msamples_per_s=round(W * H * spp / (w / frames) / 1e6, 3),
               hip_hw_queues=os.environ.get("GPU_MAX_HW_QUEUES", "4 (HIP default)"))
    key = f"cfg{cfg_no}"
    if key in summary:   # serial frames' dominant kernel, from the tracked PMC passes
        roof = rl.roofline(summary[key])
        roof["source"] = f"profiles/pmc_summary.json[{key}] (tools/roofline.py, serial frames)"
        res["roofline"] = roof
    rx.close()
    sc.close()
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:   # never report one GPU's frames as N GPUs' (or the reverse)
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE); "
                         "run `python bench.py --gpus N` alone or under torch.distributed.run --nproc-per-node N")
    dist = None
    backend = os.environ.get("RT_DIST_BACKEND", "nccl")
    # one rank per GPU; RT_DIST_BACKEND=gloo + fewer GPUs than ranks rehearses the N > 1 path
    # on a single card (ranks share it; the exchange goes through gloo instead of RCCL)
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and ndev < world:
        raise SystemExit(f"bench: {world} ranks over RCCL need {world} GPUs, {ndev} visible "
                         "(RT_DIST_BACKEND=gloo rehearses N ranks sharing fewer GPUs)")
    device = local % max(1, ndev) if world > 1 else 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(device)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(device)

    W, H = args.width, args.height
    # weak: every GPU traces one frame's worth of samples per step; strong: one frame, split
    spp = args.spp * world if args.scaling == "weak" else args.spp
    scene = rt.Scene.recipe(args.scene, device=device)
    rend = rt.Renderer(scene, W, H)
    stream = torch.cuda.Stream(device=device)
    sptr = stream.cuda_stream
    frame_out = torch.zeros(W * H, dtype=torch.int32, device=f"cuda:{device}")
    sharded = None
    native_fallback = None
    balanced_deal = args.scaling == "strong" and args.depth == 1
    if world > 1:
        from advancedgraphicsraytracer_amd.distributed import NativeCommUnavailable, NativeShardedFrame, ShardedFrame
        if backend == "nccl":   # the product path: RCCL gather from C++ (rt_render_frame_multi)
            # strong-scaling primary+shadow frames (config 4) render compact cost-balanced screen
            # regions per rank once the costs are measured (RT_MULTI_BALANCED: each GPU's caches
            # hold its region's part of the scene); weak scaling keeps the interleaved deal, whose
            # 1/N shards at spp N are statistically identical, and so do path-traced frames: the
            # level-0 cost deal measured slower than interleaving on config 5 (1/8 shard 1.56 vs
            # 1.31 ms, the bounce levels' cost is not the camera rays')
            try:
                sharded = NativeShardedFrame(rend, device=torch.device("cuda", device), balanced=balanced_deal)
            except NativeCommUnavailable as e:   # raised on every rank together: same gather via torch's RCCL
                if rank == 0:
                    print(f"bench: native RCCL communicator unavailable ({e}); torch.distributed gather instead",
                          file=sys.stderr, flush=True)
                native_fallback = str(e)
        if sharded is None:
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

    # clock ramp (untimed, before the W warm-up steps): blocks of frames until
    # --ramp-seconds have passed; at N > 1 the ranks agree on every block (the per-frame
    # gather is a collective, so every rank must submit the same frames).  The renderer times
    # its choices (camera walk, split order, frames in flight) during the ramp, on groups of up
    # to 32 frames submitted back to back, and times a group again when the GPU ran dry inside
    # it: at N = 1 the host waits only for the block before the previous one (the GPU keeps a
    # block queued), at N > 1 every block ends in a drain and a host sync, so blocks are long.
    nf = 0
    t_ramp = time.perf_counter()
    block = 100 if args.depth <= 1 else 4
    pending = []
    while args.ramp_seconds > 0:
        for _ in range(block):
            step(nf)
            nf += 1
        if dist:
            drain()
            torch.cuda.synchronize(device)
        else:
            ev = torch.cuda.Event()
            ev.record(stream)
            pending.append(ev)
            if len(pending) > 2:
                pending.pop(0).synchronize()
        more = 1 if time.perf_counter() - t_ramp < args.ramp_seconds else 0
        if dist:
            t_more = torch.tensor([more], device=f"cuda:{device}")
            dist.all_reduce(t_more, op=dist.ReduceOp.MIN)
            more = int(t_more.item())
        if not more:
            break
    drain()
    torch.cuda.synchronize(device)
    ramp_frames = nf
    for i in range(args.warmup):
        step(nf)
        nf += 1
    drain()
    torch.cuda.synchronize(device)
    c0 = rend.counters()
    # HIP events on the launch stream: one pair brackets the timed region (per-launch average =
    # region / steps; no event packets between the frames).  At N > 1 the per-frame render /
    # gather split comes from a separate instrumented pass after the timed region: timing
    # events around every frame cost ~20 us per frame on the render stream (0.116 -> 0.138 ms
    # per TEAPOT-F frame at world 1, profiles/r02/multi_overhead.json)
    per_step_events = args.per_step_events
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
    if sharded is not None:   # untimed instrumented pass: per-frame render / exposed-gather times
        sharded.set_timing(True)
        for k in range(min(args.steps, 20)):
            step(nf + args.steps + k)
        drain()
        torch.cuda.synchronize(device)
    frame_ms = float(np.mean([a.elapsed_time(b) for a, b in evs])) / (1 if per_step_events else args.steps)
    primary = c1["primary"] - c0["primary"]
    shadow = c1["shadow"] - c0["shadow"]
    bounce = c1["bounce"] - c0["bounce"]
    dev = f"cuda:{device}"
    local_rays = torch.tensor([primary + shadow + bounce, primary, shadow, bounce], dtype=torch.float64, device=dev)
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    multi = None
    if sharded is not None:
        tm = sharded.timing()
        if tm is not None:   # this rank's render and exposed gather time per frame (max over ranks)
            rms, gms, n = tm
            per = torch.tensor([rms / max(n, 1), gms / max(n, 1)], dtype=torch.float64, device=dev)
            dist.all_reduce(per, op=dist.ReduceOp.MAX)
            di = sharded.deal_info()   # the deal this rank's frames actually ran under
            multi = {"exchange": "rt_render_frame_multi (RCCL send/recv to rank 0 from C++, pipelined)",
                     "deal_requested": "balanced (RT_MULTI_BALANCED)" if balanced_deal else "interleaved t % N",
                     "deal_rank0": {"in_use": "balanced" if di["balanced"] else "interleaved", **di},
                     "render_ms_per_frame_max_rank": round(per[0].item(), 4),
                     "gather_ms_per_frame_max_rank": round(per[1].item(), 4)}
        else:
            multi = {"exchange": f"torch.distributed gather ({backend})"}
            if native_fallback:
                multi["native_comm_unavailable"] = native_fallback
    if dist:
        dist.all_reduce(local_rays, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    tot_rays, tot_primary, tot_shadow, tot_bounce = local_rays.tolist()
    wall = t_max.item()
    overlap = rend.overlap()
    in_flight = rend.overlap_depth()
    choices = rend.choices() if args.depth == 1 else None   # the renderer's timed camera-walk / split choices
    walk_check = None
    if choices is not None and choices["walk"] == 1 and sharded is None:
        # untimed: the wave camera walk's counters (lanes re-traced in the reference order, boxes
        # entered through its cull margin) over 10 frames, then 10 frames re-tracing EVERY walked
        # lane in the reference order and counting results that differ (rt_renderer_walk_stats)
        rend.set_walk_check(rt.WALK_CHECK_COUNT)
        for k in range(10):
            step(nf + args.steps + 100 + k)
        w1 = rend.walk_stats()
        rend.set_walk_check(rt.WALK_CHECK_VERIFY)
        for k in range(10):
            step(nf + args.steps + 110 + k)
        w2 = rend.walk_stats()
        rend.set_walk_check(rt.WALK_CHECK_OFF)
        walk_check = {"frames": 10, "rays_walked": w1["walked"], "lanes_retraced": w1["retraced"],
                      "margin_boxes": w1["margin_boxes"], "verify_frames": 10,
                      "verify_rays": w2["walked"] - w1["walked"], "verify_mismatch": w2["verify_mismatch"]}
    extras = {}
    default_cfg2 = (args.config, args.scene, W, H, args.spp, args.depth) == (2, "teapotF", 1920, 1080, 1, 1)
    extra_list = [int(c) for c in args.extra_configs.split(",") if c.strip()] if not args.no_strong else []
    if default_cfg2 and extra_list:
        if sharded is not None:   # the headline communicator is done (its frames are flushed)
            sharded.close()
            sharded = None
        # the headline renderer is done too: its streams would share hardware queues with the
        # next renderer's frames in flight (see the companion below)
        rend.close()
        summary_x = rl.load(args.summary)
        for c in extra_list:
            try:   # deterministic code and collectives that fail on every rank together: all ranks agree
                ec = extra_config(c, world, rank, device, dist, stream, summary_x, backend=backend)
            except Exception as e:   # the headline line still prints; the failure is reported in it
                ec = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
            extras[EXTRA_CONFIGS[c]["key"]] = ec
            if rank == 0:
                print(f"bench: config {c}: " + (f"{ec['ms_per_frame']} ms per frame, {ec['mrays_s']} Mrays/s"
                                                 if "error" not in ec else ec["error"]), file=sys.stderr, flush=True)
    companion = None
    if world == 1 and args.depth == 1 and (W, H) == (1920, 1080) and not args.no_companion:   # the metric's other frame size
        # the measured renderer is done: free its streams first, so that the companion's
        # frames-in-flight streams get hardware queues of their own (with 8 queues a second
        # renderer beside the first ran config 4's 720p frames at 0.234 instead of 0.168 ms)
        rend.close()
        companion = companion_rate(scene, 1280, 720, spp, args.depth, stream, device)

    if rank == 0:
        cfg = CONFIGS[args.config]
        summary = rl.load(args.summary)
        key = f"cfg{args.config}"
        roof = None
        default_workload = (args.scene, W, H, args.spp, args.depth) == (cfg["scene"], 1920, 1080, cfg["spp"], cfg["depth"])
        if key in summary and default_workload:
            # one kernel per frame (depth 1, N = 1, serial frames): its live duration is the
            # frame's event time; overlapped frames share the CUs, so the kernel trace's duration
            # of a serial run is used instead
            live = frame_ms if (args.depth == 1 and world == 1 and overlap[0] != 1) else None
            bp, bs = BYTES_PER_RAY.get(args.scene, (None, None))
            alg = (primary * bp + shadow * bs) / args.steps if (bp and live) else None
            roof = rl.roofline(summary[key], kernel_ms=live, algorithmic_bytes=alg)
            roof["source"] = f"profiles/pmc_summary.json[{key}] (tools/roofline.py)"
        line = {
            "metric": "Mrays/s (primary+shadow) at 1080p" if args.depth == 1 else
                      f"Mrays/s (all traced rays) at {H}p, config {args.config}",
            "value": round(tot_rays / wall / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_ramp_frames": ramp_frames,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: bundled meshes (SURVEY 8(d) {args.scene} recipe) + constant 1024x512 sky, "
                    "per-pixel seeds InitSeed(pixel + W*H*(sample + spp*frame))",
            "config": {"workload": f"config {args.config}: {args.scene} {W}x{H}, spp {spp}"
                                   + (f" ({args.spp} per GPU, weak)" if args.scaling == "weak" and world > 1 else "")
                                   + f", Trace depth {args.depth}"
                                   + (" (primary + NEE shadow)" if args.depth == 1 else " (path tracing)")
                                   + ", accumulate + RGB8",
                       "scene": args.scene, "width": W, "height": H, "spp": spp, "depth": args.depth,
                       "parallelism": f"screen-tile x{world}" if world > 1 else "single GPU",
                       "launcher": ("bench.py (spawned the ranks itself)" if os.environ.get("RT_BENCH_LAUNCHER")
                                    else "external (WORLD_SIZE from the launcher)" if world > 1 else "single process"),
                       "hip_hw_queues": {"effective": os.environ.get("GPU_MAX_HW_QUEUES", "4 (HIP default)"),
                                         "set_by_bench": os.environ.get("GPU_MAX_HW_QUEUES") != _HWQ_BEFORE
                                         or _HWQ_ARG is not None, "environment_before": _HWQ_BEFORE}},
            "fps": round(args.steps / wall, 3),
            "msamples_per_s": round(W * H * spp / (wall / args.steps) / 1e6, 3),
            "rays": {"primary": int(tot_primary), "shadow": int(tot_shadow), "bounce": int(tot_bounce),
                     "total": int(tot_rays)},
            "frame_ms_events": round(frame_ms, 4),
            "roofline": roof,
        }
        if args.depth == 1:   # RT_PS_PIPELINE: serial or overlapped primary+shadow frames (rank 0)
            groups = [g for g in in_flight[1] if g > 0]
            line["overlapped_frames"] = {"state": overlap[0], "in_flight": in_flight[0], "timed_groups_ms": groups,
                                         "groups": ("frames in flight serial, 2, 4, 6, 6, 4, 2, serial (32 frames each, "
                                                    "timed over their last 23 periods)" if len(groups) == 8
                                                    else "frames in flight serial, 2, 2, serial (16 frames each, timed over "
                                                    "their last 13 periods)")}
            if choices is not None:   # walk 0 lane / 1 wave, split 0 plain / 1 half tiles; groups A, B, B, A
                line["timed_choices"] = choices
            if walk_check is not None:
                line["camera_walk_check"] = walk_check
        if multi:
            line["multi_gpu"] = multi
        if companion:
            line["at_720p"] = companion
        line.update(extras)   # strong_config4, config3, config5 (EXTRA_CONFIGS)
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(args, spp)
            except Exception as e:   # the baseline is reported, never the product
                line["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
        print(json.dumps(line), flush=True)
    if sharded is not None:
        sharded.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
