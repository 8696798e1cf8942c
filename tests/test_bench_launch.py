"""bench.py --gpus N measures N ranks however it is started (CPU only).

Under a launcher (torch.distributed.run exports WORLD_SIZE) the launcher owns the ranks; run
alone, `python bench.py --gpus N` starts N rank processes itself before anything loads HIP, so
the driver's scaling run never reports one GPU's frames as N GPUs'.  The rank processes here
stop at RT_BENCH_LAUNCH_CHECK (they print their rank environment and exit; no GPU)."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_launch_only", BENCH)
    src = open(BENCH).read()
    # only the launch helpers: everything above the first `import numpy` (no torch, no HIP)
    head = src.split("\nimport numpy as np", 1)[0]
    mod = importlib.util.module_from_spec(spec)
    exec(compile(head.replace('if __name__ == "__main__":', "if False:"), BENCH, "exec"), mod.__dict__)
    return mod


@pytest.mark.parametrize("argv,env,want", [
    ([], {}, 0),
    (["--gpus", "1"], {}, 0),
    (["--gpus", "8", "--steps", "5"], {}, 8),
    (["--gpus=4"], {}, 4),
    (["--gpu", "2"], {}, 2),                     # argparse accepts the prefix, so does the plan
    (["--gpus", "8"], {"WORLD_SIZE": "8"}, 0),   # torch.distributed.run owns the ranks
    (["--gpus", "8"], {"WORLD_SIZE": "1"}, 0),   # main() then refuses the mismatch
    (["--config", "4", "--gpus", "2"], {}, 2),
])
def test_launch_plan(argv, env, want):
    assert _bench_module().launch_plan(argv, env) == want


def test_launch_plan_rejects_zero():
    with pytest.raises(SystemExit):
        _bench_module().launch_plan(["--gpus", "0"], {})


def _run(argv, mode, timeout=60):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["RT_BENCH_LAUNCH_CHECK"] = mode
    t0 = time.time()
    p = subprocess.run([sys.executable, BENCH] + argv, env=env, capture_output=True, text=True, timeout=timeout)
    return p, time.time() - t0


def test_spawns_n_ranks_with_their_environment():
    p, _ = _run(["--gpus", "3", "--steps", "5"], "ok")
    assert p.returncode == 0, p.stderr
    ranks = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert sorted(int(r["RANK"]) for r in ranks) == [0, 1, 2]
    assert all(r["WORLD_SIZE"] == "3" and r["LOCAL_RANK"] == r["RANK"] for r in ranks)
    assert all(r["MASTER_ADDR"] == "127.0.0.1" and r["RT_BENCH_LAUNCHER"] == "bench.py" for r in ranks)
    assert len({r["MASTER_PORT"] for r in ranks}) == 1


def test_single_gpu_runs_in_process():
    p, _ = _run(["--gpus", "1"], "ok")
    assert p.returncode == 0, p.stderr
    (r,) = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert r["WORLD_SIZE"] is None and r["RT_BENCH_LAUNCHER"] is None


def test_failed_rank_fails_the_run_and_stops_the_others():
    # rank 1 exits 3 while ranks 0 and 2 wait (as in a collective): the launcher must end them
    # and exit 3 long before their 600 s sleep
    p, dt = _run(["--gpus", "3"], "fail:1", timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert dt < 60
    assert "stopping the other ranks" in p.stderr
