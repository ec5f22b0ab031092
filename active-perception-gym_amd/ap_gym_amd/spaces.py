"""Space types for the vector envs.

When gymnasium is importable its spaces are used directly (so the envs plug into gymnasium
tooling); otherwise a minimal stand-in with the same attributes (low, high, shape, dtype, spaces)
keeps the package usable on machines without gymnasium, such as the GPU box.  Layout conventions
follow the reference: images are (H, W, C) (ap_gym/image_space.py:9-57).
"""

from __future__ import annotations

import numpy as np

try:  # pragma: no cover - gymnasium is absent in the build image
    import gymnasium as _gym

    Space = _gym.spaces.Space
    Box = _gym.spaces.Box
    Dict = _gym.spaces.Dict
    Discrete = _gym.spaces.Discrete
    MultiDiscrete = _gym.spaces.MultiDiscrete
    Tuple = _gym.spaces.Tuple
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class Space:  # type: ignore[no-redef]
        def __init__(self, shape=None, dtype=None):
            self._shape = None if shape is None else tuple(int(s) for s in shape)
            self.dtype = None if dtype is None else np.dtype(dtype)

        @property
        def shape(self):
            return self._shape

    class Box(Space):  # type: ignore[no-redef]
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            if shape is None:
                shape = np.shape(low) if np.shape(low) != () else np.shape(high)
            super().__init__(shape, dtype)
            self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Discrete(Space):  # type: ignore[no-redef]
        def __init__(self, n, start=0):
            super().__init__((), np.int64)
            self.n = int(n)
            self.start = int(start)

    class MultiDiscrete(Space):  # type: ignore[no-redef]
        def __init__(self, nvec, dtype=np.int64):
            nvec = np.asarray(nvec, dtype=np.int64)
            super().__init__(nvec.shape, dtype)
            self.nvec = nvec

    class Dict(Space):  # type: ignore[no-redef]
        def __init__(self, spaces=None, **kw):
            super().__init__(None, None)
            self.spaces = dict(spaces or {}, **kw)

        def __getitem__(self, k):
            return self.spaces[k]

        def keys(self):
            return self.spaces.keys()

        def items(self):
            return self.spaces.items()

        def __repr__(self):
            return "Dict(" + ", ".join(f"{k!r}: {v}" for k, v in self.spaces.items()) + ")"

    class Tuple(Space):  # type: ignore[no-redef]
        def __init__(self, spaces=()):
            super().__init__(None, None)
            self.spaces = tuple(spaces)

        def __getitem__(self, i):
            return self.spaces[i]

        def __len__(self):
            return len(self.spaces)

        def __repr__(self):
            return "Tuple(" + ", ".join(str(v) for v in self.spaces) + ")"


class LogitSpace(Box):
    """Unbounded logits of a classifier (ap_gym/logit_space.py)."""

    def __repr__(self):
        return f"LogitSpace({self.shape}, {self.dtype})"


class ImageSpace(Box):
    """(…, H, W, C) float image in [low, high] (ap_gym/image_space.py:9-57)."""

    def __init__(self, width, height, channels, batch_shape=(), dtype=np.float32, low=0.0, high=1.0):
        super().__init__(low, high, (*batch_shape, height, width, channels), dtype)

    @property
    def height(self):
        return self.shape[-3]

    @property
    def width(self):
        return self.shape[-2]

    @property
    def channels(self):
        return self.shape[-1]

    @property
    def batch_shape(self):
        return self.shape[:-3]


class ActivePerceptionActionSpace(Dict):
    """{"action": inner, "prediction": prediction} (ap_gym/active_perception_env.py:27-68)."""

    def __init__(self, inner_action_space, prediction_space):
        super().__init__({"action": inner_action_space, "prediction": prediction_space})

    @property
    def inner_action_space(self):
        return self["action"]

    @property
    def prediction_space(self):
        return self["prediction"]


def batch_box(space: Box, n: int) -> Box:
    reps = (n,) + (1,) * len(space.shape)
    return Box(np.tile(space.low, reps), np.tile(space.high, reps), dtype=space.dtype)


def batch_space(space, n: int):
    if isinstance(space, ImageSpace):
        return ImageSpace(space.width, space.height, space.channels, (n, *space.batch_shape), space.dtype)
    if isinstance(space, ActivePerceptionActionSpace):
        return ActivePerceptionActionSpace(batch_space(space["action"], n), batch_space(space["prediction"], n))
    if isinstance(space, Dict):
        return Dict({k: batch_space(v, n) for k, v in space.spaces.items()})
    if isinstance(space, LogitSpace):
        b = batch_box(space, n)
        return LogitSpace(b.low, b.high, b.shape, b.dtype)
    if isinstance(space, Box):
        return batch_box(space, n)
    if isinstance(space, Discrete):
        return MultiDiscrete(np.full(n, space.n))
    if isinstance(space, Tuple):  # gymnasium batches a Tuple element-wise (Tuple(()) stays empty)
        return Tuple(tuple(batch_space(v, n) for v in space.spaces))
    raise TypeError(f"cannot batch {type(space).__name__}")
