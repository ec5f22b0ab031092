from __future__ import annotations

from functools import singledispatch

import numpy as np

from ...spaces import Box, Dict, Discrete, Space, Tuple
from . import space_utils


@singledispatch
def batch_space(space: Space, n: int = 1):
    raise TypeError(f"cannot batch {type(space)}")


@batch_space.register(Box)
def _(space, n=1):
    return space_utils._batch_space_box(space, n)


@batch_space.register(Dict)
def _(space, n=1):
    return Dict({k: batch_space(v, n) for k, v in space.spaces.items()})


@batch_space.register(Tuple)
def _(space, n=1):
    return Tuple([batch_space(s, n) for s in space.spaces])


@batch_space.register(Discrete)
def _(space, n=1):
    from ...spaces import MultiDiscrete

    return MultiDiscrete(np.full((n,), space.n, dtype=space.dtype))
