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


class _PackedOracleShard(_OracleShard):
    """The oracle shard with the device env's packed output rows (packed_outputs=True): every step's
    outputs land in one [n, row] buffer, laid out like the kernel writes it (lidar_output_row_layout)."""

    def __init__(self, num_envs, env_offset, packed_outputs=False):
        from ap_gym_amd.lidar_env import lidar_output_row_layout, row_views

        super().__init__(num_envs, env_offset)
        assert packed_outputs
        self.output_layout, row = lidar_output_row_layout(BEAMS)
        self.output_rows = torch.zeros((num_envs, row), dtype=torch.uint8)
        self.v = row_views(self.output_rows, self.output_layout)

    def _fill(self):
        e, v = self.e, self.v
        for k in ("lidar", "odometry", "time_step", "reward", "base_reward", "target", "loss"):
            v[k].copy_(torch.from_numpy(getattr(e, k).copy()))
        for k in ("terminated", "truncated", "info_mask"):
            v[k].copy_(torch.from_numpy(getattr(e, k).astype(bool)))

    def reset(self, *, seed=None, options=None):
        out = super().reset(seed=seed, options=options)
        self._fill()
        return out

    def step(self, action):
        out = super().step(action)
        self._fill()
        return out


def _actions():
    rng = np.random.default_rng(1)
    return (rng.uniform(-1, 1, (STEPS, N_TOTAL, 2)).astype(np.float32),
            rng.uniform(-1, 1, (STEPS, N_TOTAL, 2)).astype(np.float32))


def _worker(rank, world, port, outdir, packed=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ap_gym_amd.sharding import ShardedVectorEnv

    make = _PackedOracleShard if packed else (lambda num_envs, env_offset: _OracleShard(num_envs, env_offset))
    senv = ShardedVectorEnv(make, N_TOTAL, rank, world, BEAMS, gather=True)
    assert senv._packed == packed
    acts, preds = _actions()
    lo, n = senv.offset, senv.local_num_envs
    senv.reset(seed=7)
    rows = []
    for t in range(STEPS):
        obs, rew, term, trunc, info = senv.step({"action": torch.from_numpy(acts[t, lo:lo + n]),
                                                 "prediction": torch.from_numpy(preds[t, lo:lo + n])})
        rows.append(np.concatenate([np.ascontiguousarray(obs["lidar"].numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(obs["odometry"].numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(obs["time_step"].numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(rew.numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(info["base_reward"].numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(info["prediction"]["target"].numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(info["prediction"]["loss"].numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(term.numpy()).view(np.uint8).ravel(), np.ascontiguousarray(trunc.numpy()).view(np.uint8).ravel(),
                                    np.ascontiguousarray(info["_base_reward"].numpy()).view(np.uint8).ravel()]))
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


@pytest.mark.parametrize("packed", [False, True], ids=["copying", "packed_rows"])
def test_two_rank_gather_equals_unsharded(tmp_path, oracle_mod, packed):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), packed), nprocs=2, join=True,
                       start_method="spawn")
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
