#!/usr/bin/env python3
"""Host-side cost of the N > 1 frame loop, measured on ONE GPU: ShardedFrame.submit (render_shard
+ async RCCL gather + flush) over a world-size-1 NCCL group, against plain Tick frames.  If the
sharded loop's wall time per frame exceeds the render time, the multi-GPU bench is host-bound.
usage: python tools/host_overhead.py [--frames 500]"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import advancedgraphicsraytracer_amd as rt  # noqa: E402
from advancedgraphicsraytracer_amd.distributed import ShardedFrame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--modes", default="tick,shard,shard+gather,shard+assemble,sharded,tick,sharded")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    opts = None
    if os.environ.get("RT_NCCL_HIGH_PRIORITY", "0") == "1":
        opts = dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0), pg_options=opts)
    scene = rt.Scene.recipe("teapotF", device=0)
    r = rt.Renderer(scene, 1920, 1080)
    st = torch.cuda.Stream()
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    sf = ShardedFrame(r, device=torch.device("cuda", 0))
    res = {}
    tiles = torch.zeros(r.shard_capacity(1), dtype=torch.int32, device="cuda")
    gathered = torch.zeros(r.shard_capacity(1), dtype=torch.int32, device="cuda")
    from advancedgraphicsraytracer_amd.distributed import gather_into

    def one(name, f):
        if name == "tick":
            r.Tick(out, spp=1, depth=1, frame=f, stream=st.cuda_stream)
        elif name == "shard":
            r.render_shard(tiles, 0, 1, spp=1, depth=1, frame=f, stream=st.cuda_stream)
        elif name == "shard+gather":
            r.render_shard(tiles, 0, 1, spp=1, depth=1, frame=f, stream=st.cuda_stream)
            gather_into(gathered, tiles, None, async_op=True).wait()
        elif name == "shard+assemble":
            r.render_shard(tiles, 0, 1, spp=1, depth=1, frame=f, stream=st.cuda_stream)
            r.assemble(tiles, 1, out, stream=st.cuda_stream)
        else:
            sf.submit(spp=1, depth=1, frame=f, stream=st.cuda_stream)

    for name in a.modes.split(","):
        f0 = 0
        with torch.cuda.stream(st):
            for f in range(200):                      # warm-up / clock ramp
                one(name, f)
            sf.flush(stream=st.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = 0.0
        with torch.cuda.stream(st):
            for f in range(a.frames):
                h0 = time.perf_counter()
                one(name, 200 + f)
                host += time.perf_counter() - h0
            sf.flush(stream=st.cuda_stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        res[name] = (round(wall / a.frames * 1e3, 4), round(host / a.frames * 1e3, 4))
        print(name, "wall ms/frame", res[name][0], "host ms/frame", res[name][1], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
