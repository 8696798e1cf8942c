"""The C-ABI multi-GPU frame (rt_comm_* + rt_render_frame_multi, RCCL gather issued from
C++) at world 1 on the one GPU of the box: synchronous and pipelined frames must equal the
single-renderer frames bit for bit.  (RCCL refuses two ranks on one device, so world > 1
runs on the driver's 8-GPU node: bench.py --gpus N.)"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_comm_world1_direct(rt, torch):
    """rt_comm_unique_id / rt_comm_create / rt_render_frame_multi straight through ctypes."""
    L = rt.lib()
    uid = (C.c_uint8 * rt.RT_COMM_ID_BYTES)()
    rt._check(L.rt_comm_unique_id(uid))
    h = C.c_void_p()
    rt._check(L.rt_comm_create(uid, 0, 1, 0, C.byref(h)))
    rank, world = C.c_int(-1), C.c_int(-1)
    rt._check(L.rt_comm_info(h, C.byref(rank), C.byref(world)))
    assert (rank.value, world.value) == (0, 1)
    g = rt.Scene.recipe("teapotF")
    W, H = 160, 96
    r, ref = rt.Renderer(g, W, H), rt.Renderer(g, W, H)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    for f in range(2):
        p = r.params(1, 3, f)
        rt._check(L.rt_render_frame_multi(r.h, h, C.byref(r.camera), C.byref(p), C.c_void_p(out.data_ptr()),
                                          rt.MULTI_TIMING, None))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref.tick_host(spp=1, depth=3, frame=f).view(np.int32))
    a, b, n = C.c_double(), C.c_double(), C.c_uint64()
    rt._check(L.rt_comm_timing(h, C.byref(a), C.byref(b), C.byref(n)))
    assert n.value == 2 and a.value > 0 and b.value >= 0
    assert L.rt_render_frame_multi(r.h, h, C.byref(r.camera), C.byref(r.params(1, 1, 0)), None, 0, None) \
        == rt.RT_ERR_INVALID                              # rank 0 needs an output frame
    rt._check(L.rt_comm_destroy(h))


def test_native_sharded_frame_world1(rt, torch):
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from advancedgraphicsraytracer_amd.distributed import NativeShardedFrame
        g = rt.Scene.recipe("cfg3")
        W, H = 136, 80
        r, ref = rt.Renderer(g, W, H), rt.Renderer(g, W, H)
        sf = NativeShardedFrame(r, timing=True)
        got = []
        for f in range(2):
            got.append(sf.render(spp=2, depth=4, frame=f).cpu().numpy().copy())
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            for f in range(2, 5):
                out = sf.submit(spp=2, depth=4, frame=f, stream=st.cuda_stream)
                if out is not None:
                    st.synchronize()
                    got.append(out.cpu().numpy().copy())
            out = sf.flush(stream=st.cuda_stream)
            st.synchronize()
            got.append(out.cpu().numpy().copy())
        want = [ref.tick_host(spp=2, depth=4, frame=f).view(np.int32) for f in range(5)]
        assert len(got) == 5 and all(np.array_equal(a, b) for a, b in zip(got, want))
        assert np.array_equal(r.accumulator(), ref.accumulator())
        render_ms, gather_ms, n = sf.timing()
        assert n == 5 and render_ms > 0
        sf.close()
    finally:
        dist.destroy_process_group()
