"""Env sharding over torch.distributed (gloo, world_size 2, CPU): the union of the shards, reassembled
by ShardedVectorEnv's packed all-gather, equals one unsharded env bit for bit.

The per-rank env is the C oracle wrapped to the torch output contract of
LIDARLocalization2DVectorEnv(array_backend="torch"), seeded with the shard's env offset exactly as
the device env is (sub-env i of rank r uses seed + r*N + i) — the GPU path itself is covered by
tests/test_gpu_lidar.py; this test covers the sharding/gather host logic on CPU.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_TOTAL, BEAMS, SIZE, STEPS = 16, 8, 32, 110


class _OracleShard:
    def __init__(self, num_envs, env_offset):
        from oracle import oracle

        self.offset = env_offset
        self.e = oracle.OracleLidarVectorEnv(num_envs, "rooms", SIZE, False, 0, BEAMS)

    def reset(self, *, seed=None, options=None):
        self.e.reset(seed + self.offset)
        return {"lidar": torch.from_numpy(self.e.lidar.copy())}, {}

    def step(self, action):
        e = self.e
        e.step(action["action"].numpy(), action["prediction"].numpy())
        obs = {"lidar": torch.from_numpy(e.lidar.copy()), "odometry": torch.from_numpy(e.odometry.copy()),
               "time_step": torch.from_numpy(e.time_step.copy())}
        info = {"base_reward": torch.from_numpy(e.base_reward.copy()),
                "_base_reward": torch.from_numpy(e.info_mask.astype(bool)),
                "prediction": {"target": torch.from_numpy(e.target.copy()), "loss": torch.from_numpy(e.loss.copy())}}
        return (obs, torch.from_numpy(e.reward.copy()), torch.from_numpy(e.terminated.astype(bool)),
                torch.from_numpy(e.truncated.astype(bool)), info)

    def close(self):
        self.e.close()


def _actions():
    rng = np.random.default_rng(1)
    return (rng.uniform(-1, 1, (STEPS, N_TOTAL, 2)).astype(np.float32),
            rng.uniform(-1, 1, (STEPS, N_TOTAL, 2)).astype(np.float32))


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ap_gym_amd.sharding import ShardedVectorEnv

    senv = ShardedVectorEnv(lambda num_envs, env_offset: _OracleShard(num_envs, env_offset), N_TOTAL, rank, world,
                            BEAMS, gather=True)
    acts, preds = _actions()
    lo, n = senv.offset, senv.local_num_envs
    senv.reset(seed=7)
    rows = []
    for t in range(STEPS):
        obs, rew, term, trunc, info = senv.step({"action": torch.from_numpy(acts[t, lo:lo + n]),
                                                 "prediction": torch.from_numpy(preds[t, lo:lo + n])})
        rows.append(np.concatenate([obs["lidar"].numpy().view(np.uint8).ravel(),
                                    obs["odometry"].numpy().view(np.uint8).ravel(),
                                    obs["time_step"].numpy().view(np.uint8).ravel(),
                                    rew.numpy().view(np.uint8).ravel(),
                                    info["base_reward"].numpy().view(np.uint8).ravel(),
                                    info["prediction"]["target"].numpy().view(np.uint8).ravel(),
                                    info["prediction"]["loss"].numpy().view(np.uint8).ravel(),
                                    term.numpy().view(np.uint8).ravel(), trunc.numpy().view(np.uint8).ravel(),
                                    info["_base_reward"].numpy().view(np.uint8).ravel()]))
    np.save(os.path.join(outdir, f"rank{rank}.npy"), np.stack(rows))
    senv.close()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_bounds():
    from ap_gym_amd.sharding import shard_bounds

    assert [shard_bounds(64, r, 4) for r in range(4)] == [(0, 16), (16, 16), (32, 16), (48, 16)]
    with pytest.raises(ValueError):
        shard_bounds(10, 0, 4)


def test_two_rank_gather_equals_unsharded(tmp_path, oracle_mod):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0, r1 = np.load(tmp_path / "rank0.npy"), np.load(tmp_path / "rank1.npy")
    assert np.array_equal(r0, r1)  # every rank holds the full batch

    full = oracle_mod.OracleLidarVectorEnv(N_TOTAL, "rooms", SIZE, False, 0, BEAMS)
    acts, preds = _actions()
    full.reset(7)
    saw_reset = False
    for t in range(STEPS):
        full.step(acts[t], preds[t])
        want = np.concatenate([full.lidar.view(np.uint8).ravel(), full.odometry.view(np.uint8).ravel(),
                               full.time_step.view(np.uint8).ravel(), full.reward.view(np.uint8).ravel(),
                               full.base_reward.view(np.uint8).ravel(), full.target.view(np.uint8).ravel(),
                               full.loss.view(np.uint8).ravel(), full.terminated.ravel(), full.truncated.ravel(),
                               full.info_mask.ravel()])
        assert np.array_equal(r0[t], want), t
        saw_reset |= bool(full.truncated.any() or full.terminated.any())
    assert saw_reset  # the trace crosses the TimeLimit autoreset
    full.close()
