"""The reference-shaped C++ hosts (tests/cpp, prebuilt by __graft_entry__.build()) on the GPU:
compat_host (Scene / Ray / RayPacket / Trace / the C-ABI multi frame at world 1) and
reference_main (the reference's main loop on include/rt_compat.hpp: Surface, new Renderer(),
Init, Tick(float), the K key, Shutdown, on the reference's default scene)."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
CPP = os.path.join(ROOT, "tests", "cpp")


@pytest.mark.parametrize("exe", ["compat_host", "reference_main"])
def test_reference_shaped_hosts_on_gpu(rt, exe):
    path = os.path.join(CPP, exe)
    assert os.path.exists(path), f"tests/cpp/{exe} must be built beforehand (__graft_entry__.build())"
    env = dict(os.environ, RT_MESH_DIR=rt.DATA_DIR)
    r = subprocess.run([path, rt.DATA_DIR] if exe == "compat_host" else [path], capture_output=True, text=True,
                       env=env, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
