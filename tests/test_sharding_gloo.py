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


def _worker(rank, world, port, outdir, packed=False, sub=1, lag=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ap_gym_amd.sharding import ShardedVectorEnv

    make = _PackedOracleShard if packed else (lambda num_envs, env_offset: _OracleShard(num_envs, env_offset))
    senv = ShardedVectorEnv(make, N_TOTAL, rank, world, BEAMS, gather=True, sub_batches=sub, gather_lag=lag)
    assert senv._packed == packed and len(senv.envs) == sub
    acts, preds = _actions()
    ids = senv.local_env_ids  # sub-batches: rank r owns [(h*W + r)*m, +m) for each h
    assert len(ids) == senv.local_num_envs and (sub > 1 or ids[0] == senv.offset)
    senv.reset(seed=7)
    rows = []

    def row(out):  # the gathered batch as bytes (the packed path's views are rewritten by the next call)
        obs, rew, term, trunc, info = out
        parts = [obs["lidar"], obs["odometry"], obs["time_step"], rew, info["base_reward"],
                 info["prediction"]["target"], info["prediction"]["loss"], term, trunc, info["_base_reward"]]
        return np.concatenate([np.ascontiguousarray(x.numpy()).view(np.uint8).ravel() for x in parts])

    for t in range(STEPS):
        out = senv.step({"action": torch.from_numpy(acts[t, ids]), "prediction": torch.from_numpy(preds[t, ids])})
        if lag:  # step t's call returns step t - 1's gathered batch (None first); flush() the last one
            assert (out is None) == (t == 0)
            if out is None:
                continue
        rows.append(row(out))
    if lag:
        rows.append(row(senv.flush()))
        assert senv.flush() is None
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


def test_sub_batch_layout_and_checks():
    """Sub-batch h of rank r holds global envs [(h*W + r)*m, +m); every global env is in exactly one sub-batch."""
    from ap_gym_amd.sharding import ShardedVectorEnv

    made = []

    def make(num_envs, env_offset, packed_outputs=False):
        made.append((num_envs, env_offset))
        env = type("E", (), {})()  # a stand-in: only the constructor's layout is checked here
        env.output_rows = torch.zeros((num_envs, 8), dtype=torch.uint8) if packed_outputs else None
        env.lidar_beam_count = BEAMS
        return env

    ids = []
    for r in range(2):
        made.clear()
        s = ShardedVectorEnv(make, 16, r, 2, BEAMS, gather=True, sub_batches=4)
        assert made == [(2, (h * 2 + r) * 2) for h in range(4)] and s.sub_num_envs == 2
        ids.append(s.local_env_ids)
    assert sorted(np.concatenate(ids).tolist()) == list(range(16))
    with pytest.raises(ValueError, match="gather=True"):
        ShardedVectorEnv(make, 16, 0, 2, BEAMS, gather=False, sub_batches=2)
    with pytest.raises(ValueError, match="divisible"):
        ShardedVectorEnv(make, 16, 0, 2, BEAMS, gather=True, sub_batches=3)
    with pytest.raises(ValueError, match="packed"):
        ShardedVectorEnv(lambda num_envs, env_offset: make(num_envs, env_offset), 16, 0, 2, BEAMS, gather=True,
                         sub_batches=2)
    with pytest.raises(ValueError, match="gather=True"):
        ShardedVectorEnv(make, 16, 0, 2, BEAMS, gather=False, gather_lag=1)
    with pytest.raises(ValueError, match="sub_batches=1"):
        ShardedVectorEnv(make, 16, 0, 2, BEAMS, gather=True, sub_batches=2, gather_lag=1)
    with pytest.raises(ValueError, match="0 or 1"):
        ShardedVectorEnv(make, 16, 0, 2, BEAMS, gather=True, gather_lag=2)


@pytest.mark.parametrize("packed,sub,lag", [(False, 1, 0), (True, 1, 0), (True, 2, 0), (True, 4, 0), (True, 1, 1)],
                         ids=["copying", "packed_rows", "packed_rows_2sub", "packed_rows_4sub", "packed_rows_lag1"])
def test_two_rank_gather_equals_unsharded(tmp_path, oracle_mod, packed, sub, lag):
    """sub > 1: each rank's envs in sub-batches whose all-gathers are issued right after their steps (overlapping
    the next sub-batch's step on RCCL); the gathered batch is still in global env order.  lag = 1: the pipelined
    gather (step t's call returns step t - 1's batch, flush() the last): the same batches shifted by one call."""
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), packed, sub, lag), nprocs=2, join=True,
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


# ---------------------------------------------------------------------------------------- image envs
# Each rank runs the numpy restatement of the whole batch (the image envs draw every batch from one stream, so a
# shard draws the whole batch and keeps its slice, as the device env does with num_envs_total / env_offset) and
# hands over its slice in the torch output contract of the image envs — densely (the copying path) or in the
# packed output rows of image_env.image_output_row_layout (the zero-copy path).
IMG_N, IMG_STEPS, IMG_LIMIT, IMG_SENSOR = 8, 21, 8, (5, 5)


def _img_pool():
    rng = np.random.default_rng(3)
    return rng.integers(0, 256, (32, 16, 16, 1)).astype(np.uint8), rng.integers(0, 10, 32).astype(np.int32)


def _img_actions(kind):
    rng = np.random.default_rng(2)
    a = rng.uniform(-1, 1, (IMG_STEPS, IMG_N, 2)).astype(np.float32)
    p = (rng.standard_normal((IMG_STEPS, IMG_N, 10)) if kind in ("cls", "cls_inv")
         else rng.uniform(-1, 1, (IMG_STEPS, IMG_N, 2))).astype(np.float32)
    return a, p


class _ImageOracleShard:
    def __init__(self, kind, num_envs, env_offset, packed_outputs=False):
        invert = kind == "cls_inv"  # randomly_invert_labels (the registered MNIST-style ids)
        kind = "cls" if invert else kind
        from ap_gym_amd import _native as N
        from ap_gym_amd.image_env import image_output_row_layout, image_row_views
        from oracle import image_oracle as io

        pool, labels = _img_pool()
        self.kname, self.lo, self.n = kind, env_offset, num_envs
        self.kind = N.APG_IMAGE_CLASSIFY if kind == "cls" else N.APG_IMAGE_LOCALIZE
        self.single_observation_space = {"glimpse": np.zeros(IMG_SENSOR + (1,), np.float32)}  # .shape only
        self.e = io.ImageVectorEnvOracle(kind, pool, labels, 10, 1, IMG_N, IMG_SENSOR, step_limit=IMG_LIMIT,
                                         invert=invert)
        self.copy = False
        self._prev_done = False
        self.output_rows = self.output_layout = None
        if packed_outputs:
            self.output_layout, row = image_output_row_layout(self.kind, IMG_SENSOR, 1, log_stats=True)
            self.output_rows = torch.zeros((num_envs, row), dtype=torch.uint8)
            self.v = image_row_views(self.output_rows, self.output_layout)

    def _metric_names(self):
        return ("correct_label_prob", "accuracy") if self.kname == "cls" else ("euclidean_distance", "mse")

    def _sl(self, x):
        return torch.from_numpy(np.ascontiguousarray(np.asarray(x)[self.lo:self.lo + self.n]))

    def _obs(self, o):
        out = {k: self._sl(o[k]) for k in ("glimpse", "glimpse_pos", "time_step")}
        if "target_glimpse" in o:
            out["target_glimpse"] = self._sl(o["target_glimpse"])
        if "inverted_label" in o:  # int32 flags on reset steps, int64 2s after (image_env.py's torch outputs)
            out["inverted_label"] = self._sl(o["inverted_label"])
        return out

    def reset(self, *, seed=None, options=None):
        o, info = self.e.reset(seed)
        self._prev_done = False
        obs = self._obs(o)
        if self.output_rows is not None:
            for k in obs:
                if k in self.v:  # (the target glimpse is not in the row)
                    self.v[k].copy_(obs[k])
        return obs, {"index": self._sl(info["index"])}

    def step(self, action):
        # the other shards' envs step with zeros: an env's outputs depend only on its own action / prediction
        a = np.zeros((IMG_N, 2), np.float32)
        p = np.zeros((IMG_N,) + tuple(action["prediction"].shape[1:]), np.float32)
        a[self.lo:self.lo + self.n] = action["action"].numpy()
        p[self.lo:self.lo + self.n] = action["prediction"].numpy()
        o, r, te, tr, info = self.e.step(a, p)
        self._prev_done = bool(te.any())
        obs = self._obs(o)
        tgt = info["prediction"]["target"]
        loss = info["prediction"]["loss"]
        ti = {"index": self._sl(info["index"]), "base_reward": self._sl(np.asarray(info["base_reward"], np.float32)),
              "prediction": {"target": self._sl(tgt if self.kname == "cls" else np.asarray(tgt, np.float32)),
                             "loss": self._sl(np.asarray(loss, np.float64 if self.kname == "cls" else np.float32))}}
        if "stats" in info:
            ti["stats"] = {"vector": {}, "_vector": self._sl(info["stats"]["_vector"]), "np": info["stats"]}
        if self.output_rows is not None:
            v = self.v
            for k in obs:
                if k in v:  # (the target glimpse is not in the row)
                    v[k].copy_(obs[k])
            v["reward"].copy_(self._sl(np.asarray(r, np.float64)))
            v["base_reward"].copy_(ti["base_reward"])
            if self.kname == "cls":
                v["label_target"].copy_(ti["prediction"]["target"])
                v["loss_f64"].copy_(ti["prediction"]["loss"])
            else:
                v["target_out"].copy_(ti["prediction"]["target"])
                v["loss_f32"].copy_(ti["prediction"]["loss"])
            if "stats" in info:
                sc = info["stats"]["scalar"]
                nm = self._metric_names()
                for j, key in enumerate((f"final_{nm[0]}", f"final_{nm[1]}", f"avg_{nm[0]}", f"avg_{nm[1]}")):
                    v["stats"][j].copy_(self._sl(sc[key]))
                if self.kname == "cls":
                    v["stats_idx"][0].copy_(self._sl(sc["first_correct"]))
                    v["stats_idx"][1].copy_(self._sl(sc["last_incorrect"]))
        return obs, self._sl(np.asarray(r, np.float64)), self._sl(te), self._sl(tr), ti

    def close(self):
        pass


def _img_worker(rank, world, port, outdir, kind, packed, sub=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ap_gym_amd.sharding import ShardedVectorEnv

    def make(num_envs, env_offset, packed_outputs=False):
        return _ImageOracleShard(kind, num_envs, env_offset, packed_outputs)

    senv = ShardedVectorEnv(make, IMG_N, rank, world, gather=True, gather_glimpse=True, sub_batches=sub)
    assert senv._packed == packed or not packed
    if not packed:  # the copying path: a factory without packed_outputs
        senv = ShardedVectorEnv(lambda num_envs, env_offset: _ImageOracleShard(kind, num_envs, env_offset), IMG_N, rank,
                                world, gather=True, gather_glimpse=True)
        assert not senv._packed
    acts, preds = _img_actions(kind)
    ids = senv.local_env_ids
    obs, info = senv.reset(seed=7)
    out = {}
    if packed:  # (the copying path gathers step outputs only)
        out["reset_glimpse"] = obs["glimpse"].numpy().copy()
        out["reset_index"] = info["index"].numpy().copy()
        if "inverted_label" in obs:
            out["reset_inverted_label"] = obs["inverted_label"].numpy().copy()
    for t in range(IMG_STEPS):
        obs, rew, term, trunc, info = senv.step({"action": torch.from_numpy(acts[t, ids]),
                                                 "prediction": torch.from_numpy(preds[t, ids])})
        for k in ("glimpse", "glimpse_pos", "time_step", "target_glimpse", "inverted_label"):
            if k in obs:
                out[f"{k}_{t}"] = obs[k].numpy().copy()
        out[f"reward_{t}"] = rew.numpy().copy()
        out[f"term_{t}"] = term.numpy().copy()
        out[f"base_{t}"] = info["base_reward"].numpy().copy()
        out[f"target_{t}"] = info["prediction"]["target"].numpy().copy()
        out[f"loss_{t}"] = info["prediction"]["loss"].numpy().copy()
        out[f"index_{t}"] = info["index"].numpy().copy()
        if packed and "stats" in info:
            for key, val in info["stats"]["scalar"].items():
                out[f"stats_{t}_{key}"] = val.numpy().copy()
    np.savez(os.path.join(outdir, f"img_rank{rank}.npz"), **out)
    senv.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("packed,sub", [(False, 1), (True, 1), (True, 2)],
                         ids=["copying", "packed_rows", "packed_rows_2sub"])
@pytest.mark.parametrize("kind", ["cls", "loc", "cls_inv"])
def test_two_rank_image_gather_equals_unsharded(tmp_path, kind, packed, sub):
    from oracle import image_oracle as io

    mp.start_processes(_img_worker, args=(2, _free_port(), str(tmp_path), kind, packed, sub), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = np.load(tmp_path / "img_rank0.npz"), np.load(tmp_path / "img_rank1.npz")
    assert sorted(r0.files) == sorted(r1.files)
    for k in r0.files:
        assert np.array_equal(r0[k], r1[k], equal_nan=True), k  # every rank holds the full batch
    pool, labels = _img_pool()
    full = io.ImageVectorEnvOracle("cls" if kind == "cls_inv" else kind, pool, labels, 10, 1, IMG_N, IMG_SENSOR,
                                   step_limit=IMG_LIMIT, invert=kind == "cls_inv")
    o, info = full.reset(7)
    if packed:
        assert np.array_equal(r0["reset_glimpse"], o["glimpse"])
        assert np.array_equal(r0["reset_index"], info["index"])
        if kind == "cls_inv":  # the whole batch's flags, not one shard's
            got = r0["reset_inverted_label"]
            assert got.shape == (IMG_N,) and got.dtype == np.int32 and np.array_equal(got, o["inverted_label"])
    acts, preds = _img_actions(kind)
    ends = 0
    for t in range(IMG_STEPS):
        o, r, te, tr, info = full.step(acts[t], preds[t])
        for k in ("glimpse", "glimpse_pos", "time_step", "target_glimpse", "inverted_label"):
            if k in o:
                assert np.array_equal(r0[f"{k}_{t}"], o[k]), (k, t)
                assert r0[f"{k}_{t}"].dtype == np.asarray(o[k]).dtype, (k, t)
        assert np.array_equal(r0[f"reward_{t}"], np.asarray(r, np.float64)), t
        assert np.array_equal(r0[f"term_{t}"], te), t
        assert np.array_equal(r0[f"base_{t}"], np.asarray(info["base_reward"], np.float32)), t
        assert np.array_equal(r0[f"target_{t}"], np.asarray(info["prediction"]["target"]).astype(r0[f"target_{t}"].dtype))
        assert np.array_equal(r0[f"index_{t}"], info["index"]), t
        if packed and "stats" in info:
            ends += 1
            for key, val in info["stats"]["scalar"].items():
                if not key.startswith("_"):
                    assert np.array_equal(r0[f"stats_{t}_{key}"], val), (t, key)
    assert not packed or ends == 2
