from __future__ import annotations

import copy
import enum
from typing import Any, Generic, TypeVar

_O = TypeVar("_O")
_A = TypeVar("_A")
_R = TypeVar("_R")

import numpy as np

from . import utils  # noqa: F401
from ..core import Env


class AutoresetMode(enum.Enum):
    NEXT_STEP = "NextStep"
    SAME_STEP = "SameStep"
    DISABLED = "Disabled"


class VectorEnv(Generic[_O, _A, _R]):
    metadata: dict[str, Any] = {}
    num_envs: int
    _np_random = None

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            from ..core import np_random

            self._np_random, self._np_random_seed = np_random(seed)
        return None

    def close(self, **kwargs):
        pass

    @property
    def np_random(self):
        if self._np_random is None:
            from ..core import np_random

            self._np_random, self._np_random_seed = np_random()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    @property
    def unwrapped(self):
        return self


class VectorWrapper(VectorEnv):
    def __init__(self, env):
        self.env = env

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, actions):
        return self.env.step(actions)

    def __getattr__(self, name):
        if name.startswith("_") or name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def num_envs(self):
        return self.env.num_envs

    @property
    def unwrapped(self):
        return self.env.unwrapped


class AsyncVectorEnv(VectorEnv):
    pass


class SyncVectorEnv(VectorEnv):
    """gymnasium 1.1 SyncVectorEnv restated (NEXT_STEP autoreset only)."""

    def __init__(self, env_fns, copy: bool = True):
        self.envs = [fn() for fn in env_fns]
        self.num_envs = len(self.envs)
        self.copy = copy
        self.autoreset_mode = AutoresetMode.NEXT_STEP
        self._rewards = np.zeros((self.num_envs,), dtype=np.float64)
        self._terminations = np.zeros((self.num_envs,), dtype=np.bool_)
        self._truncations = np.zeros((self.num_envs,), dtype=np.bool_)
        self._autoreset_envs = np.zeros((self.num_envs,), dtype=np.bool_)
        self._env_obs = [None] * self.num_envs

    def _concat(self):
        first = self._env_obs[0]
        if isinstance(first, dict):
            return {k: np.stack([np.asarray(o[k]) for o in self._env_obs]) for k in first}
        return np.stack(self._env_obs)

    def reset(self, *, seed=None, options=None):
        if seed is None:
            seed = [None] * self.num_envs
        elif isinstance(seed, int):
            seed = [seed + i for i in range(self.num_envs)]
        self._terminations = np.zeros((self.num_envs,), dtype=np.bool_)
        self._truncations = np.zeros((self.num_envs,), dtype=np.bool_)
        self._autoreset_envs = np.zeros((self.num_envs,), dtype=np.bool_)
        infos = {}
        for i, (env, s) in enumerate(zip(self.envs, seed)):
            self._env_obs[i], env_info = env.reset(seed=s, options=options)
            infos = self._add_info(infos, env_info, i)
        obs = self._concat()
        return (copy.deepcopy(obs) if self.copy else obs), infos

    def step(self, actions):
        infos = {}
        for i in range(self.num_envs):
            action = {k: v[i] for k, v in actions.items()} if isinstance(actions, dict) else actions[i]
            if self._autoreset_envs[i]:
                self._env_obs[i], env_info = self.envs[i].reset()
                self._rewards[i] = 0.0
                self._terminations[i] = False
                self._truncations[i] = False
            else:
                (
                    self._env_obs[i],
                    self._rewards[i],
                    self._terminations[i],
                    self._truncations[i],
                    env_info,
                ) = self.envs[i].step(action)
            infos = self._add_info(infos, env_info, i)
        obs = self._concat()
        self._autoreset_envs = np.logical_or(self._terminations, self._truncations)
        return (
            copy.deepcopy(obs) if self.copy else obs,
            np.copy(self._rewards),
            np.copy(self._terminations),
            np.copy(self._truncations),
            infos,
        )

    def _add_info(self, vector_infos, env_info, env_num):
        for key, value in env_info.items():
            if isinstance(value, dict):
                array = self._add_info(vector_infos.get(key, {}), value, env_num)
            else:
                if key not in vector_infos:
                    if type(value) in [int, float, bool] or issubclass(type(value), np.number):
                        array = np.zeros(self.num_envs, dtype=type(value))
                    elif isinstance(value, np.ndarray):
                        array = np.zeros((self.num_envs, *value.shape), dtype=value.dtype)
                    else:
                        array = np.full(self.num_envs, fill_value=None, dtype=object)
                else:
                    array = vector_infos[key]
                array[env_num] = value
            array_mask = vector_infos.get(f"_{key}", np.zeros(self.num_envs, dtype=np.bool_))
            array_mask[env_num] = True
            vector_infos[key], vector_infos[f"_{key}"] = array, array_mask
        return vector_infos

    def close(self, **kwargs):
        for e in self.envs:
            e.close()
