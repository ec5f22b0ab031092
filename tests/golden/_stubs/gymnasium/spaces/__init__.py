from __future__ import annotations

import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None, seed=None):
        self._shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self._np_random = None

    @property
    def shape(self):
        return self._shape

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.shape(low) != () else np.shape(high)
        shape = tuple(int(s) for s in shape)
        self.low = np.full(shape, low, dtype=dtype) if np.isscalar(low) else np.asarray(low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype) if np.isscalar(high) else np.asarray(high, dtype=dtype)
        super().__init__(shape, dtype, seed)
        self.low_repr = str(low)
        self.high_repr = str(high)


class Discrete(Space):
    def __init__(self, n, seed=None, start=0):
        self.n = np.int64(n)
        self.start = np.int64(start)
        super().__init__((), np.int64, seed)


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64, seed=None, start=None):
        self.nvec = np.asarray(nvec, dtype=dtype)
        super().__init__(self.nvec.shape, dtype, seed)


class MultiBinary(Space):
    def __init__(self, n, seed=None):
        super().__init__((n,) if np.isscalar(n) else tuple(n), np.int8, seed)


class Tuple(Space):
    def __init__(self, spaces, seed=None):
        self.spaces = tuple(spaces)
        super().__init__(None, None, seed)

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)


class Dict(Space):
    def __init__(self, spaces=None, seed=None, **kw):
        self.spaces = dict(spaces or {}, **kw)
        super().__init__(None, None, seed)

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()
