"""bench.py's multi-rank launcher: `python bench.py --gpus N` (no torchrun) starts the N ranks itself and
rank 0 prints exactly one JSON line with n_gpus = N.

CPU: --dry-run (gloo rendezvous, barrier-bracketed timing, max over ranks, no envs).
GPU: the LIDAR workload with two ranks sharing the box's one GPU over gloo (RCCL needs a GPU per rank),
without and with the packed all-gather of the step outputs.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                           "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_self_launch_dry_run_two_ranks():
    out = _run(["--gpus", "2", "--dry-run", "--steps", "5", "--warmup", "1"], 120)
    assert out["n_gpus"] == 2 and out["config"]["ranks"] == 2 and out["steps"] == 5


@pytest.mark.gpu
@pytest.mark.parametrize("gather", [False, True], ids=["shard", "gather"])
def test_self_launch_lidar_two_ranks_one_gpu(gather):
    args = ["--gpus", "2", "--workload", "lidar", "--num-envs", "512", "--steps", "8", "--warmup", "2",
            "--dist-backend", "gloo", "--no-cpu-baseline", "--no-episode"] + (["--gather"] if gather else [])
    out = _run(args, 300)
    assert out["n_gpus"] == 2
    assert out["config"]["num_envs_total"] == 1024
    assert out["value"] > 0
    if gather:
        assert out["config"]["gather_ms"] is not None
