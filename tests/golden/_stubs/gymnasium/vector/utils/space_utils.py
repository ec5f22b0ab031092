import numpy as np


def _batch_space_box(space, n=1):
    from ...spaces import Box

    repeats = tuple([n] + [1] * space.low.ndim)
    low, high = np.tile(space.low, repeats), np.tile(space.high, repeats)
    return Box(low=low, high=high, dtype=space.dtype)
