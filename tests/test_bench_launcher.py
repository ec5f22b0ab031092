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
    assert out["config"]["num_envs_per_gpu"] == 65536 and out["scaling"] == "weak"  # config 2: per-GPU envs


def test_dry_run_eight_ranks_tinyimagenet_gather():
    """BASELINE config 5 at 8 ranks: 32768 envs split 8 ways, each rank all-gathers the full-size packed rows
    (reward, glimpse + target glimpse, glimpse_pos, time_step, base_reward, target, loss, stats) of the others."""
    from ap_gym_amd import _native as N
    from ap_gym_amd.image_env import image_output_row_layout

    out = _run(["--gpus", "8", "--dry-run", "--workload", "tinyimagenet-loc", "--gather", "--steps", "2",
                "--warmup", "0"], 300)
    cfg = out["config"]
    row = image_output_row_layout(N.APG_IMAGE_LOCALIZE, (12, 12), 3, True)[1]
    assert out["n_gpus"] == 8 and cfg["ranks"] == 8 and out["scaling"] == "strong"
    assert cfg["num_envs_per_gpu"] == 4096 and cfg["num_envs_total"] == 32768
    assert cfg["row_bytes"] == row and cfg["gather_bytes_per_rank_step"] == 7 * 4096 * row
    assert cfg["parallelism"] == "env-shard x8 + all-gather"


def test_dry_run_eight_ranks_maze127():
    """BASELINE config 3 at 8 ranks: 262144 envs split 8 ways, no data-path collective."""
    out = _run(["--gpus", "8", "--dry-run", "--workload", "maze127", "--steps", "2", "--warmup", "0"], 300)
    cfg = out["config"]
    assert out["n_gpus"] == 8 and out["scaling"] == "strong"
    assert cfg["workload"] == "LIDARLocMaze-v0" and cfg["num_envs_per_gpu"] == 32768
    assert cfg["num_envs_total"] == 262144 and cfg["gather_bytes_per_rank_step"] == 0
    assert cfg["parallelism"] == "env-shard x8"


@pytest.mark.parametrize("workload,per_rank", [("lidar", 65536), ("maze127", 32768), ("tinyimagenet-loc", 4096)])
def test_dry_run_eight_ranks_gather_in_sub_batches(workload, per_rank):
    """BASELINE configs 2 / 3 / 5 at 8 ranks with the all-gather split into two sub-batches (ShardedVectorEnv's
    overlapped layout: sub-batch h of rank r holds global envs [(h*W + r)*m, +m)): every rank receives every row,
    in global env order (run_dry checks the env index carried in each row)."""
    out = _run(["--gpus", "8", "--dry-run", "--workload", workload, "--gather", "--sub-batches", "2", "--steps", "2",
                "--warmup", "0"], 300)
    cfg = out["config"]
    assert out["n_gpus"] == 8 and cfg["num_envs_per_gpu"] == per_rank and cfg["sub_batches"] == 2
    assert cfg["gather_bytes_per_rank_step"] == 7 * per_rank * cfg["row_bytes"]
    assert cfg["parallelism"] == "env-shard x8 + all-gather in 2 overlapped sub-batches"


def test_dry_run_eight_ranks_pipelined_gather():
    """BASELINE config 2 at 8 ranks with the pipelined all-gather (--gather-lag 1: step t's batch returned with step
    t+1's call): the same per-rank rows and traffic as the plain gather; the flag is refused without --gather."""
    out = _run(["--gpus", "8", "--dry-run", "--workload", "lidar", "--gather", "--gather-lag", "1", "--steps", "2",
                "--warmup", "0"], 300)
    cfg = out["config"]
    assert out["n_gpus"] == 8 and cfg["gather_lag"] == 1 and cfg["num_envs_per_gpu"] == 65536
    assert cfg["gather_bytes_per_rank_step"] == 7 * 65536 * cfg["row_bytes"]
    assert cfg["parallelism"] == "env-shard x8 + all-gather (pipelined: step t's batch returned with step t+1)"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gather-lag", "1"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "needs --gather" in p.stderr


def test_dry_run_rejects_an_uneven_split():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--workload", "maze127",
                        "--gpus", "1"], capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env=dict(os.environ, WORLD_SIZE="3", RANK="0"))
    assert p.returncode != 0 and "do not split over 3 ranks" in p.stderr


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
