#!/usr/bin/env python3
"""Per-frame cost of the C-ABI multi-GPU frame at world 1 (one GPU): Renderer.Tick frames vs
NativeShardedFrame.submit frames (rt_render_frame_multi, pipelined, as bench.py --gpus N drives
it), both back to back on one stream.  The difference is the multi path's own cost on rank 0
(shard packing, the zero-peer RCCL group, the rank-0 unshuffle, host submission); at world 1
there is no transfer.

usage: multi_overhead.py [--scene teapotF] [--frames 300] [--spp 1] [--depth 1]
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402
from advancedgraphicsraytracer_amd.distributed import NativeShardedFrame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="teapotF")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--warm", type=int, default=400, help="untimed frames first, per mode: past the renderer's "
                    "timed choices (walk, split order, frames in flight: ~170 frames after the tuning gate) ...")
    ap.add_argument("--warm-seconds", type=float, default=1.0, help="... and at least this much wall time (the "
                    "tuning gate opens after 100 ms of GPU time, RT_TUNE_DELAY_MS)")
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--events", choices=("none", "plain", "bench"), default="plain",
                    help="per-frame torch events around the submit: none, two non-timing ones, or as "
                         "bench.py's timed loop did (two timing events + RT_MULTI_TIMING)")
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    g = rt.Scene.recipe(a.scene)
    W, H = 1920, 1080
    r = rt.Renderer(g, W, H)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    res = {}
    with torch.cuda.stream(st):
        sptr = st.cuda_stream
        w0, f = time.perf_counter(), 0
        while f < a.warm or time.perf_counter() - w0 < a.warm_seconds:
            r.Tick(out, spp=a.spp, depth=a.depth, frame=0, stream=sptr)
            f += 1
            if f % 200 == 0:   # rare syncs: the renderer's timed groups (up to 32 frames) run back to back
                st.synchronize()
        st.synchronize()
        t0 = time.perf_counter()
        for f in range(a.frames):
            r.Tick(out, spp=a.spp, depth=a.depth, frame=f, stream=sptr)
        st.synchronize()
        res["tick_ms"] = (time.perf_counter() - t0) * 1e3 / a.frames
        res["tick_in_flight"] = r.overlap_depth()[0]
        sf = NativeShardedFrame(r, timing=False)
        ev = None if a.events == "none" else (torch.cuda.Event(enable_timing=a.events == "bench"),
                                               torch.cuda.Event(enable_timing=a.events == "bench"))
        w0, f = time.perf_counter(), 0
        while f < a.warm or time.perf_counter() - w0 < a.warm_seconds:
            sf.submit(spp=a.spp, depth=a.depth, frame=f, stream=sptr, events=ev)
            f += 1
            if f % 200 == 0:   # rare syncs: the renderer's timed groups (up to 32 frames) run back to back
                st.synchronize()
        sf.flush(stream=sptr)
        st.synchronize()
        if a.events == "bench":
            sf.set_timing(True)
        t0 = time.perf_counter()
        host = 0.0
        for f in range(a.frames):
            h0 = time.perf_counter()
            sf.submit(spp=a.spp, depth=a.depth, frame=f, stream=sptr, events=ev)
            host += time.perf_counter() - h0
        sf.flush(stream=sptr)
        st.synchronize()
        res["multi_submit_ms"] = (time.perf_counter() - t0) * 1e3 / a.frames
        res["multi_submit_host_ms"] = host * 1e3 / a.frames
        res["multi_in_flight"] = r.overlap_depth()[0]
        res["multi_choices"] = r.choices()
        sf.close()
    dist.destroy_process_group()
    res.update(scene=a.scene, spp=a.spp, depth=a.depth, frames=a.frames, events=a.events)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
