"""numpy restatement of LightDark-v0 as registered — TEST INFRASTRUCTURE ONLY.

Imported only by tests/ as the checker for the HIP LightDark path (ap_gym_amd never imports it).
Restates, per sub-env and in the reference's operation order and dtypes (numpy 2 / NEP 50):
  * LightDarkEnv.reset / _step / __get_obs / __compute_brightness   ap_gym/envs/light_dark.py:93-155
  * TimeLimit(50, issue_termination=True)                          ap_gym/time_limit.py:113-139
  * ActivePerceptionEnv.step + normalized MSE                       active_perception_env.py:101-121,
                                                                    active_regression_env.py:29-76
  * ActiveRegressionLogWrapper per-episode statistics              active_regression_env.py:131-159
  * gymnasium SyncVectorEnv: sub-env i seeded with seed + i, NEXT_STEP autoreset, float64 rewards
  * SparsifyWrapper (sparse=True)                                   sparsify_wrapper.py:93-161
The random streams are numpy's own Generator(PCG64(SeedSequence(seed + i))) objects (uniform and
normal draws exactly as the reference makes them).  Pinned against tests/golden/light_dark_*.npz
(the reference run as-is, tests/test_oracle_golden.py).
"""

from __future__ import annotations

import numpy as np

LIGHT_POS = np.array([0, -0.7], dtype=np.float32)
LIGHT_HEIGHT = 0.2
LOSS_SCALE = np.float32(1 / (2**2 / 12))  # MSE normalized for prediction bounds [-1, 1] (as float32)


def brightness(pos):
    dist_squared = np.sum((pos - LIGHT_POS) ** 2, axis=-1) + LIGHT_HEIGHT**2
    return LIGHT_HEIGHT**2 / dist_squared


class LightDarkVectorOracle:
    def __init__(self, num_envs: int, step_limit: int = 50, sparse: bool = False):
        self.n, self.limit, self.sparse = num_envs, step_limit, sparse

    def _obs(self, i):
        p = self.pos[i]
        obs = p + self.rngs[i].normal(size=2).astype(np.float32) * ((1 - brightness(p)) * 0.3)
        return np.clip(obs, -2, 2)

    def _reset_env(self, i):
        self.pos[i] = self.rngs[i].uniform(-np.ones(2), np.ones(2), size=2).astype(np.float32)
        self.elapsed[i] = 0
        self.hist[i] = ([], [])
        return self._obs(i)

    def reset(self, seed: int, env_ids=None):
        """env_ids: the sub-env indices this oracle follows (default range(num_envs)); sub-env i's
        stream is default_rng(seed + i) whatever the batch size, so any subset can be checked."""
        ids = range(self.n) if env_ids is None else [int(i) for i in env_ids]
        assert len(ids) == self.n
        self.rngs = [np.random.default_rng(seed + i) for i in ids]
        self.pos = [None] * self.n
        self.elapsed = [0] * self.n
        self.hist = [None] * self.n
        self.done = np.zeros(self.n, bool)
        obs = np.stack([self._reset_env(i) for i in range(self.n)])
        return {"noisy_position": obs, "time_step": np.full(self.n, -1.0, np.float32)}

    def step(self, actions, predictions):
        n = self.n
        out = {k: np.zeros(n, dt) for k, dt in (("reward", np.float64), ("terminated", bool), ("truncated", bool),
                                                ("base_reward", np.float32), ("loss", np.float32),
                                                ("info_mask", bool), ("weight", np.float64),
                                                ("stats_len", np.int32), ("time_step", np.float32))}
        out["noisy_position"] = np.zeros((n, 2), np.float32)
        out["target"] = np.zeros((n, 2), np.float32)
        out["stats"] = np.zeros((4, n), np.float64)
        out["stats_vectors"] = {}
        for i in range(n):
            if self.done[i]:  # NEXT_STEP autoreset
                out["noisy_position"][i] = self._reset_env(i)
                out["time_step"][i] = -1.0
                self.done[i] = False
                continue
            action, prediction = actions[i], predictions[i]
            last_pos = self.pos[i].copy()
            base_reward = 1.0 - 1e-3 * np.sum(action**2, axis=-1)
            magnitude = np.linalg.norm(action)
            if magnitude > 1:
                action = action / magnitude
            self.pos[i] = self.pos[i] + action * 0.15
            terminated = bool(np.any(np.abs(self.pos[i]) >= 1))
            self.pos[i] = np.clip(self.pos[i], -1, 1)
            obs = self._obs(i)
            self.elapsed[i] += 1
            if self.elapsed[i] >= self.limit:
                terminated = True
            err = prediction - last_pos
            mse = np.mean(err**2, axis=-1)
            loss = mse * LOSS_SCALE + np.float32(-0.0)
            self.hist[i][0].append(np.linalg.norm(last_pos - prediction))
            self.hist[i][1].append(mse)
            if self.sparse:
                weight = float(terminated)
                reward = base_reward - loss * np.float32(weight)
                out["weight"][i] = weight
            else:
                reward = base_reward - loss
            out["reward"][i] = reward
            out["terminated"][i] = terminated
            out["base_reward"][i] = base_reward
            out["target"][i] = last_pos
            out["loss"][i] = loss
            out["info_mask"][i] = True
            out["noisy_position"][i] = obs
            out["time_step"][i] = np.float32(2.0 * self.elapsed[i] / self.limit - 1.0)
            if terminated:
                ed, ms = self.hist[i]
                out["stats"][:, i] = [float(np.mean(ed)), float(np.mean(ms)), float(ed[-1]), float(ms[-1])]
                out["stats_len"][i] = len(ms)
                out["stats_vectors"][i] = (list(ed), list(ms))
                self.done[i] = True
        return out
