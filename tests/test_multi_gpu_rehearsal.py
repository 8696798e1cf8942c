"""The N > 1 frame path on real GPU memory with the product kernels: 2 and 3 ranks share
the one card of a 1-GPU box (gloo carries the per-frame gather; on an 8-GPU node it is
RCCL, bench.py --gpus N), each renders its tile shard with librtamd.so, rank 0
assembles -- the frame must equal the single-renderer frame bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H = 200, 112   # 25 x 14 tiles: uneven over 2 and 3 ranks


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import advancedgraphicsraytracer_amd as rt
        from advancedgraphicsraytracer_amd.distributed import ShardedFrame
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        scene = rt.Scene.recipe("teapotF")
        rend = rt.Renderer(scene, W, H)
        sf = ShardedFrame(rend, device=dev)
        frames = []
        for f in range(2):   # two frames: the accumulators must stay per rank
            out = sf.render(spp=2, depth=3, frame=f)
            torch.cuda.synchronize()
            if rank == 0:
                frames.append(out.cpu().numpy().copy())
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):   # pipelined: frame f's gather overlaps frame f+1's render
            for f in range(2, 4):
                out = sf.submit(spp=2, depth=3, frame=f, stream=st.cuda_stream)
                if out is not None:
                    torch.cuda.synchronize()
                    frames.append(out.cpu().numpy().copy())
            out = sf.flush(stream=st.cuda_stream)
        torch.cuda.synchronize()
        if rank == 0:
            frames.append(out.cpu().numpy().copy())
            ref = rt.Renderer(scene, W, H)
            want = [ref.tick_host(spp=2, depth=3, frame=f).view(np.int32) for f in range(4)]
            q.put(len(frames) == 4 and all(np.array_equal(a, b) for a, b in zip(frames, want)))
    except Exception as e:   # report, never hang the parent
        q.put(repr(e))
        raise
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frames_on_gpu_equal_single_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert q.get(timeout=5) is True
