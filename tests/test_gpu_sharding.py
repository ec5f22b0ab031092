"""GPU sharding: the device envs split into shards (env_offset / num_envs_total) reproduce the unsharded
env bit for bit, and ShardedVectorEnv's packed all-gather reassembles that batch on every rank.

* single process: two shard envs on cuda:0 stepped side by side, concatenated, vs one unsharded env;
* two processes (torch.multiprocessing, gloo — RCCL refuses two ranks on one device) sharing cuda:0,
  ShardedVectorEnv(gather=True) on each: the gathered batch of every rank vs the unsharded env;
* one process in a one-rank RCCL ("nccl") group: the device-side all_gather_into_tensor branch.
Both for the LIDAR path (LIDARLocRooms) and the image path (ImageLocalizationVectorEnv with the
unique-sampler reset), across autoresets.
"""

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_TOTAL = 256


def _make(kind, num_envs, env_offset=0, num_envs_total=None, **kw):
    import ap_gym_amd as ap

    if kind == "lidar":
        return ap.make_vec("LIDARLocRooms-v0", num_envs=num_envs, lidar_beam_count=16,
                           dataset=ap.FloorMapDatasetRooms(32, 32), device="cuda:0", array_backend="torch",
                           env_offset=env_offset, **kw)
    ds = ap.SyntheticImageClassificationDataset(64, (32, 32, 3), 10, 3, seed=3)
    if kind == "image_cls_inv":  # classification with randomly_invert_labels (registration.py:391)
        cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(5, 5), step_limit=8, randomly_invert_labels=True)
        return ap.ImageClassificationVectorEnv(num_envs, cfg, device="cuda:0", array_backend="torch",
                                               num_envs_total=num_envs_total or num_envs, env_offset=env_offset, **kw)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(8, 8), step_limit=8)
    return ap.ImageLocalizationVectorEnv(num_envs, cfg, device="cuda:0", array_backend="torch",
                                         num_envs_total=num_envs_total or num_envs, env_offset=env_offset, **kw)


def _steps(kind):
    return 110 if kind == "lidar" else 30  # both cross autoresets (TimeLimit 100 / step_limit 8)


def _actions(kind, t, n):
    import torch

    g = torch.Generator(device="cuda:0").manual_seed(1000 + t)
    return (torch.rand((n, 2), device="cuda:0", generator=g) * 2 - 1,
            torch.rand((n, 10 if kind == "image_cls_inv" else 2), device="cuda:0", generator=g) * 2 - 1)


def _flat(kind, obs, rew, term, info):
    """The gathered fields of one step as numpy arrays (the same set ShardedVectorEnv packs)."""
    if kind == "lidar":
        d = {"lidar": obs["lidar"], "odometry": obs["odometry"], "time_step": obs["time_step"], "reward": rew,
             "base_reward": info["base_reward"], "target": info["prediction"]["target"],
             "loss": info["prediction"]["loss"], "terminated": term}
    else:
        d = {"glimpse_pos": obs["glimpse_pos"], "time_step": obs["time_step"], "reward": rew,
             "base_reward": info["base_reward"], "target": info["prediction"]["target"],
             "loss": info["prediction"]["loss"], "index": info["index"], "terminated": term}
        if "glimpse" in obs:
            d["glimpse"] = obs["glimpse"]
            if "target_glimpse" in obs:
                d["target_glimpse"] = obs["target_glimpse"]
        if "inverted_label" in obs:  # [num_envs_total]: drawn flags on reset steps, 2s after
            d["inverted_label"] = obs["inverted_label"]
    return {k: v.detach().cpu().numpy().copy() for k, v in d.items()}


def _reference(kind, with_reset=False):
    env = _make(kind, N_TOTAL)
    obs0, info0 = env.reset(seed=5)
    out = []
    if with_reset:
        out.append({k: obs0[k].detach().cpu().numpy().copy() for k in ("lidar", "odometry", "time_step")})
        out[-1]["map_idx"] = info0["map_idx"].cpu().numpy().copy()
    for t in range(_steps(kind)):
        a, p = _actions(kind, t, N_TOTAL)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        out.append(_flat(kind, obs, rew, term, info))
    env.check_errors()
    env.close()
    return out


@pytest.mark.parametrize("kind", ["lidar", "image", "image_cls_inv"])
def test_shards_union_equals_unsharded(gpu, kind):
    import torch

    half = N_TOTAL // 2
    shards = [_make(kind, half, r * half, N_TOTAL) for r in range(2)]
    for s in shards:
        s.reset(seed=5)
    ref = _reference(kind)
    for t in range(_steps(kind)):
        a, p = _actions(kind, t, N_TOTAL)
        parts = []
        for r, s in enumerate(shards):
            obs, rew, term, trunc, info = s.step({"action": a[r * half:(r + 1) * half],
                                                  "prediction": p[r * half:(r + 1) * half]})
            parts.append(_flat(kind, obs, rew, term, info))
        for k, want in ref[t].items():
            got = np.concatenate([parts[0][k], parts[1][k]])
            assert np.array_equal(got, want), f"step {t}: {k}"
    torch.cuda.synchronize()


def _worker(rank, world, port, kind, outdir, backend="gloo", sub=1, lag=0):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    assert dist.get_backend() == backend
    import ap_gym_amd  # noqa: F401
    from ap_gym_amd.sharding import ShardedVectorEnv

    senv = ShardedVectorEnv(lambda num_envs, env_offset, **kw: _make(kind, num_envs, env_offset, N_TOTAL, **kw),
                            N_TOTAL, rank, world, beams=16 if kind == "lidar" else None, gather=True,
                            gather_glimpse=True, sub_batches=sub, gather_lag=lag)
    assert senv._packed  # the step kernels write the all-gather's send rows (LIDAR and image envs)
    ids = torch.as_tensor(senv.local_env_ids, device="cuda:0")
    obs0, info0 = senv.reset(seed=5)
    rows = []
    if kind == "lidar":  # reset returns the gathered batch too
        rows.append({k: obs0[k].detach().cpu().numpy().copy() for k in ("lidar", "odometry", "time_step")})
        rows[-1]["map_idx"] = info0["map_idx"].cpu().numpy().copy()
    for t in range(_steps(kind)):
        a, p = _actions(kind, t, N_TOTAL)
        out = senv.step({"action": a[ids], "prediction": p[ids]})
        if lag:  # the pipelined gather: step t's call returns step t - 1's batch (None first)
            assert (out is None) == (t == 0)
            if out is None:
                continue
        obs, rew, term, trunc, info = out
        rows.append(_flat(kind, obs, rew, term, info))
    if lag:
        obs, rew, term, trunc, info = senv.flush()
        rows.append(_flat(kind, obs, rew, term, info))
    torch.cuda.synchronize()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"),
             **{f"{t}_{k}": v for t, r in enumerate(rows) for k, v in r.items()})
    senv.close()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind", ["lidar", "image", "image_cls_inv"])
def test_two_rank_gather_on_gpu_equals_unsharded(gpu, kind, tmp_path):
    import torch.multiprocessing as mp

    mp.start_processes(_worker, args=(2, _free_port(), kind, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    ref = _reference(kind, with_reset=kind == "lidar")
    got = [np.load(tmp_path / f"rank{r}.npz") for r in range(2)]
    for t, want in enumerate(ref):
        for k, v in want.items():
            for r in range(2):
                assert np.array_equal(got[r][f"{t}_{k}"], v), f"rank {r} step {t}: {k}"


@pytest.mark.parametrize("kind,sub,lag", [("lidar", 1, 0), ("image", 1, 0), ("image_cls_inv", 1, 0), ("lidar", 2, 0),
                                          ("image", 2, 0), ("lidar", 1, 1)])
def test_rccl_gather_branch_single_rank(gpu, kind, sub, lag, tmp_path):
    """The RCCL branch of ShardedVectorEnv._all_gather_rows (dist.all_gather_into_tensor on the device rows;
    sharding.py) on a one-rank "nccl" group: RCCL refuses two ranks on one device, so this is the only way
    one GPU runs that branch.  The gathered batch must equal the unsharded env.  sub = 2: two sub-batches whose
    all-gathers are issued asynchronously right after their steps (RCCL's stream overlaps the next step kernel).
    lag = 1: the pipelined gather (gather_lag=1), the same batches one call late."""
    import torch.multiprocessing as mp

    mp.start_processes(_worker, args=(1, _free_port(), kind, str(tmp_path), "nccl", sub, lag), nprocs=1, join=True,
                       start_method="spawn")
    ref = _reference(kind, with_reset=kind == "lidar")
    got = np.load(tmp_path / "rank0.npz")
    for t, want in enumerate(ref):
        for k, v in want.items():
            assert np.array_equal(got[f"{t}_{k}"], v), f"step {t}: {k}"


@pytest.mark.parametrize("log_stats,sparse", [(False, False), (True, False), (False, True)])
def test_packed_output_rows_equal_dense(gpu, log_stats, sparse):
    """packed_outputs=True (the kernel writes [N, row] rows for the all-gather) vs the dense outputs."""
    import torch

    import ap_gym_amd as ap

    def make(packed):
        e = ap.LIDARLocalization2DVectorEnv(N_TOTAL, ap.FloorMapDatasetRooms(32, 32), lidar_beam_count=16,
                                            device="cuda:0", array_backend="torch", log_stats=log_stats,
                                            sparse=sparse, sparse_reset_info=True, packed_outputs=packed)
        return e

    envs = [make(False), make(True)]
    assert envs[1].output_rows is not None and envs[0].output_rows is None
    for e in envs:
        e.reset(seed=11)
    names = ["lidar", "odometry", "time_step", "reward", "terminated", "truncated", "base_reward", "target", "loss",
             "info_mask", "map_idx_out", "reset_mask"] + (["stats", "stats_len"] if log_stats else []) + (
        ["weight"] if sparse else [])
    for t in range(_steps("lidar")):
        a, p = _actions("lidar", t, N_TOTAL)
        for e in envs:
            e.step({"action": a, "prediction": p})
        for k in names:
            x, y = envs[0]._t[k], envs[1]._t[k]
            if k == "map_idx_out":  # written only for envs that reset: compare where they did
                m = envs[0]._t["reset_mask"]
                x, y = x[m], y[m]
            assert torch.equal(x.cpu(), y.cpu()), f"step {t}: {k}"
    for e in envs:
        e.check_errors()
        e.close()


@pytest.mark.parametrize("kind,log_stats,sparse", [("cls", True, False), ("cls", False, True), ("loc", True, False),
                                                   ("loc", False, False)])
def test_image_packed_output_rows_equal_dense(gpu, kind, log_stats, sparse):
    """Image envs with packed_outputs=True (the fused step kernel, the reset path and the autoreset glimpses write
    [N, row] rows for the all-gather) vs the dense outputs, across two batch autoresets."""
    import torch

    import ap_gym_amd as ap

    ch = 3 if kind == "loc" else 1
    ds = ap.SyntheticImageClassificationDataset(64, (32, 32, ch) if ch == 3 else (28, 28), 10, ch, seed=3)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(8, 8) if kind == "loc" else (5, 5), step_limit=6)
    cls = ap.ImageLocalizationVectorEnv if kind == "loc" else ap.ImageClassificationVectorEnv
    envs = [cls(N_TOTAL, cfg, device="cuda:0", array_backend="torch", log_stats=log_stats, sparse=sparse,
                packed_outputs=p) for p in (False, True)]
    assert envs[1].output_rows is not None and envs[0].output_rows is None
    names = ["glimpse", "glimpse_pos", "time_step", "reward", "base_reward"] + (
        ["target_glimpse", "target_out", "loss_f32"] if kind == "loc" else ["label_target", "loss_f64"]) + (
        ["stats"] + (["stats_idx"] if kind == "cls" else []) if log_stats else [])

    def check(t):
        for k in names:
            assert torch.equal(envs[0]._t[k].cpu(), envs[1]._t[k].cpu()), f"step {t}: {k}"

    for e in envs:
        e.reset(seed=21)
    check(-1)
    g = torch.Generator(device="cuda:0").manual_seed(4)
    for t in range(15):
        a = torch.rand((N_TOTAL, 2), device="cuda:0", generator=g) * 2 - 1
        p = (torch.randn((N_TOTAL, 10), device="cuda:0", generator=g) if kind == "cls"
             else torch.rand((N_TOTAL, 2), device="cuda:0", generator=g) * 2 - 1)
        outs = [e.step({"action": a, "prediction": p}) for e in envs]
        check(t)
        if log_stats and "stats" in outs[0][4]:
            s0, s1 = outs[0][4]["stats"]["scalar"], outs[1][4]["stats"]["scalar"]
            for key in s0:
                assert torch.equal(s0[key].cpu(), s1[key].cpu()), (t, key)
    for e in envs:
        e.check_errors()
        e.close()
