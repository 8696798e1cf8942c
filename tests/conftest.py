import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))   # tests are allowed to use the oracle (checker)

REFERENCE = "/root/reference"

# the renderers' timed choices (camera walk, split order, frames in flight) start after 100 ms
# of GPU time by default (clock ramp); tests exercise them on their first frames
os.environ.setdefault("RT_TUNE_DELAY_MS", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: CPU test taking more than ~5 s")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def rt():
    import advancedgraphicsraytracer_amd as pkg
    from advancedgraphicsraytracer_amd import build
    build.build()
    return pkg


@pytest.fixture(scope="session")
def reference_assets():
    path = os.path.join(REFERENCE, "assets")
    if not os.path.isdir(path):
        pytest.skip("reference assets not present (GPU box)")
    return path


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
