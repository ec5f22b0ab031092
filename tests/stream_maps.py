"""A floor-map dataset of 2**32 maps that no pool can hold: map idx is drawn from default_rng(idx) (a pure function of
idx, so the reference's per-draw get_data_point and any later fetch of the same index agree).

Shared by tests/golden/make_golden.py (the reference env over it: lidar_env_stream40_b16.npz) and the GPU parity
tests (the backend's streamed maps over it).  Not a rooms or maze generator: walls are a border, a few straight wall
segments and scattered cells.
"""

from __future__ import annotations

import numpy as np

STREAM_LEN = 2**32


def rng_floor_map(idx: int, h: int = 40, w: int = 40) -> np.ndarray:
    r = np.random.default_rng(int(idx))
    m = r.random((h, w)) < 0.04
    m[0, :] = m[-1, :] = m[:, 0] = m[:, -1] = True
    for _ in range(int(r.integers(1, 6))):
        y, x = int(r.integers(1, h - 1)), int(r.integers(1, w - 1))
        length = int(r.integers(3, max(4, min(h, w) // 2)))
        if r.random() < 0.5:
            m[y, x:x + length] = True
        else:
            m[y:y + length, x] = True
    m[h // 2, w // 2] = False  # (every map keeps free cells)
    return m


class StreamFloorMaps:
    """The interface the reference env uses of a FloorMapDataset (floor_map_dataset.py:10-22): map_width /
    map_height, load, __len__ = 2**32, get_data_point(idx).  Counts its fetches."""

    def __init__(self, h: int = 40, w: int = 40, length: int = STREAM_LEN):
        self.h, self.w, self.length = h, w, length
        self.fetches = 0

    @property
    def map_width(self):
        return self.w

    @property
    def map_height(self):
        return self.h

    def load(self):
        pass

    def __len__(self):
        return self.length

    def get_data_point(self, idx):
        self.fetches += 1
        return rng_floor_map(idx, self.h, self.w)
