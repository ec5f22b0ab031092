from __future__ import annotations

from typing import Any, Generic, TypeVar

import numpy as np

ObsType = TypeVar("ObsType")
ActType = TypeVar("ActType")
WObs = TypeVar("WObs")
WAct = TypeVar("WAct")


def np_random(seed=None):
    if seed is not None and not (isinstance(seed, (int, np.integer)) and 0 <= seed):
        raise ValueError("seed must be a non-negative int")
    seed_seq = np.random.SeedSequence(seed)
    return np.random.Generator(np.random.PCG64(seed_seq)), seed_seq.entropy


class Env(Generic[ObsType, ActType]):
    metadata: dict[str, Any] = {"render_modes": []}
    render_mode = None
    spec = None
    action_space = None
    observation_space = None
    _np_random = None
    _np_random_seed = None

    def step(self, action):
        raise NotImplementedError

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, self._np_random_seed = np_random(seed)
        return None

    def render(self):
        return None

    def close(self):
        pass

    @property
    def unwrapped(self):
        return self

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, self._np_random_seed = np_random()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value


class Wrapper(Env, Generic[WObs, WAct, ObsType, ActType]):
    def __init__(self, env):
        self.env = env
        self._action_space = None
        self._observation_space = None
        self._metadata = None
        self._cached_spec = None

    def step(self, action):
        return self.env.step(action)

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def render(self):
        return self.env.render()

    def close(self):
        return self.env.close()

    @property
    def unwrapped(self):
        return self.env.unwrapped

    @property
    def action_space(self):
        if self._action_space is None:
            return self.env.action_space
        return self._action_space

    @action_space.setter
    def action_space(self, space):
        self._action_space = space

    @property
    def observation_space(self):
        if self._observation_space is None:
            return self.env.observation_space
        return self._observation_space

    @observation_space.setter
    def observation_space(self, space):
        self._observation_space = space

    @property
    def metadata(self):
        if self._metadata is None:
            return self.env.metadata
        return self._metadata

    @property
    def np_random(self):
        return self.env.np_random

    @property
    def spec(self):
        return self.env.spec
