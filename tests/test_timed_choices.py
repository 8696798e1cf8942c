"""The renderer's timed choices (camera walk, half-tile split order, frames in flight) time groups
of frames submitted back to back.  A group in which the GPU ran dry between two frames (the caller
synchronised) is timed again, at most kTuneRestarts times per choice (csrc/rt_device.hip), so a
caller that synchronises after EVERY frame still gets a decision; frames are the same whatever is
decided."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_choices_decided_when_the_caller_syncs_every_frame(rt, torch):
    g = rt.Scene.recipe("mig16")            # walk timed, tail-bound: split order and deep frames in flight
    W, H = 480, 270
    r = rt.Renderer(g, W, H)
    g_ref = rt.Scene.recipe("mig16")
    g_ref.set_camera_walk(rt.WALK_LANE)
    ref = rt.Renderer(g_ref, W, H)
    for f in range(700):                     # tick_host: a host synchronisation after every frame
        a = r.tick_host(spp=1, depth=1, frame=f)
        if f % 50 == 0 or f > 680:
            b = ref.tick_host(spp=1, depth=1, frame=f)
            assert np.array_equal(a, b), f"frame {f}"
        else:
            ref.tick_host(spp=1, depth=1, frame=f)
    ch = r.choices()
    assert ch["walk"] in (0, 1) and ch["split"] in (0, 1), ch
    assert r.overlap_depth()[0] in (1, 2, 4, 6)
    assert np.array_equal(r.accumulator().view(np.uint32), ref.accumulator().view(np.uint32))
    r.close()
    ref.close()


def test_choices_decided_back_to_back(rt, torch):
    """The usual caller: frames queued on a stream, an occasional synchronisation (every 100
    frames, as bench.py's multi-GPU clock ramp does)."""
    g = rt.Scene.recipe("teapotF")
    W, H = 640, 360
    r = rt.Renderer(g, W, H)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    for f in range(600):
        r.Tick(out, spp=1, depth=1, frame=f, stream=st.cuda_stream)
        if f % 100 == 99:
            st.synchronize()
    torch.cuda.synchronize()
    ch = r.choices()
    assert ch["walk"] in (0, 1) and ch["split"] in (0, 1), ch
    assert r.overlap_depth()[0] in (1, 2, 4, 6)
    r.close()
