"""rt_render_frame_multi with world 2 and 3 on the box's one GPU: the ranks run as threads of a
child process (tests/multi_inproc.py) whose exchange is the in-process RCCL stand-in
(tests/cpp/libinproc_rccl.so via RT_RCCL_LIB).  Exercises every rank != 0 branch of
csrc/rt_multi.cpp -- the send, rank 0's receive loop over its peers, the double-buffered tile and
gather buffers, the pipelined waits on both sides -- synchronous and RT_MULTI_PIPELINED, with
ragged edge tiles and a rank that owns no tile; rank 0's frames equal Tick bit for bit."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

STANDIN = os.path.join(ROOT, "tests", "cpp", "libinproc_rccl.so")
DRIVER = os.path.join(ROOT, "tests", "multi_inproc.py")


def test_standin_library_exports_the_rccl_subset():
    """The stand-in is built (build() / tests/cpp/Makefile) and exports what rt_multi.cpp binds."""
    import ctypes
    if not os.path.exists(STANDIN):
        pytest.skip("tests/cpp/libinproc_rccl.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(STANDIN)
    for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclCommCount", "ncclCommUserRank",
                 "ncclGroupStart", "ncclGroupEnd", "ncclSend", "ncclRecv", "ncclGetErrorString"):
        assert getattr(lib, name)


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode,recipe,W,H", [(2, "sync", "teapotF", 200, 120), (2, "pipelined", "teapotF", 200, 120),
                                                   (3, "sync", "cfg3", 136, 80), (3, "pipelined", "mig16", 200, 120),
                                                   (3, "pipelined", "teapotF", 16, 8), (2, "balanced", "teapotF", 200, 120),
                                                   (3, "balanced", "mig16", 256, 144), (1, "balanced", "cfg3", 136, 80)])
def test_multi_frame_world_n_on_one_gpu(world, mode, recipe, W, H):
    assert os.path.exists(STANDIN), "tests/cpp/libinproc_rccl.so must be built beforehand (__graft_entry__.build())"
    env = dict(os.environ, RT_RCCL_LIB=STANDIN)
    p = subprocess.run([sys.executable, "-u", DRIVER, str(world), mode, recipe, str(W), str(H)], env=env,
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    res = json.loads(lines[-1])
    assert res["ok"], res
