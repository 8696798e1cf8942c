"""rt_render_frame_multi with world 1, 2, 3 and 8 on the box's one GPU: the ranks run as threads of a
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
@pytest.mark.parametrize("world,mode,recipe,W,H", [
    (2, "sync", "teapotF", 200, 120), (2, "pipelined", "teapotF", 200, 120),
    (3, "sync", "cfg3", 136, 80), (3, "pipelined", "mig16", 200, 120),
    (3, "pipelined", "teapotF", 16, 8),                # ragged: a rank without a tile
    (2, "balanced", "teapotF", 200, 120), (3, "balanced", "mig16", 256, 144), (1, "balanced", "cfg3", 136, 80),
    (3, "moving", "teapotF", 200, 120),                # camera moves every frame: the deal is kept
    (2, "recreate", "teapotF", 200, 120),              # a new communicator around the same renderer
    (3, "after_tick", "mig16", 200, 120),              # renderers that accumulated whole frames first
    (8, "pipelined", "teapotF", 1920, 1080),           # the driver's default N = 8 run (weak config 2 deal)
    (8, "balanced", "mig16", 1920, 1080),              # config 4 at N = 8: balanced + pipelined, two switches
    (8, "ptbal", "cfg5", 480, 270),                    # config 5's scene at N = 8: path-traced balanced deal
    (8, "pt", "cfg5", 1920, 1080),                     # config 5 as the bench splits it: 1080p, 16 spp, depth 10
    (2, "balanced", "chain64", 160, 96),               # a 64-level tree: no work map, cycle costs
])
def test_multi_frame_world_n_on_one_gpu(world, mode, recipe, W, H):
    assert os.path.exists(STANDIN), "tests/cpp/libinproc_rccl.so must be built beforehand (__graft_entry__.build())"
    env = dict(os.environ, RT_RCCL_LIB=STANDIN)
    p = subprocess.run([sys.executable, "-u", DRIVER, str(world), mode, recipe, str(W), str(H)], env=env,
                       capture_output=True, text=True, timeout=500)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    res = json.loads(lines[-1])
    print(json.dumps(res))
    assert res["ok"], res


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode,recipe,W,H", [(3, "balanced", "mig16", 256, 144), (8, "ptbal", "cfg5", 480, 270)])
def test_balanced_deal_is_reproducible(world, mode, recipe, W, H):
    """Balanced deals are cut on the dry-run work map (node visits + primitive tests, not wave
    cycles): two runs of the same frames build the same deal -- equal rt_comm_deal_hash."""
    assert os.path.exists(STANDIN)
    env = dict(os.environ, RT_RCCL_LIB=STANDIN)
    hashes = []
    for _ in range(2):
        p = subprocess.run([sys.executable, "-u", DRIVER, str(world), mode, recipe, str(W), str(H)], env=env,
                           capture_output=True, text=True, timeout=500)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert p.returncode == 0 and lines, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
        res = json.loads(lines[-1])
        assert res["ok"], res
        hashes.append(res["deal"]["hash"])
    print(hashes)
    assert hashes[0] == hashes[1], hashes


@pytest.mark.gpu
@pytest.mark.parametrize("site", ["cost_upload:1", "mig_pack:2", "mig_pack:0"])
def test_collective_failure_reaches_every_rank(site):
    """A local failure inside a per-frame collective (the cost exchange's block upload, the
    accumulator move's pack; RT_MULTI_FAULT injects it on one rank) makes rt_render_frame_multi
    return an error on EVERY rank from the same call -- no rank is left waiting in the group -- and
    the failed attempt is not retried: every later frame renders, and rank 0's frames equal Tick's
    with the failed frame left out (the injected fault stays armed throughout)."""
    assert os.path.exists(STANDIN)
    env = dict(os.environ, RT_RCCL_LIB=STANDIN)
    p = subprocess.run([sys.executable, "-u", DRIVER, "3", "fault:" + site, "teapotF", "200", "120"], env=env,
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    res = json.loads(lines[-1])
    print(json.dumps(res))
    assert res["ok"], res


@pytest.mark.gpu
def test_balanced_deal_with_default_tune_delay():
    """The bench's setting (RT_TUNE_DELAY_MS unset = 100 ms of GPU time before a renderer times its
    camera walk, so its tile costs come late): the cost exchange is retried (frames 6, 12, 24, ...)
    until every rank has costs and the balanced deal then takes over -- here with a short delay so
    the run stays small (mig16, whose walk is timed)."""
    assert os.path.exists(STANDIN)
    env = dict(os.environ, RT_RCCL_LIB=STANDIN, RT_TUNE_DELAY_MS="3", INPROC_PS_FRAMES="400")
    p = subprocess.run([sys.executable, "-u", DRIVER, "2", "balanced", "mig16", "256", "144"], env=env,
                       capture_output=True, text=True, timeout=500)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    res = json.loads(lines[-1])
    print(json.dumps(res))
    assert res["ok"], res
