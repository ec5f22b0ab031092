"""Procedural floor-map datasets (ap_gym/envs/floor_map/*).

Same constructors, sizes and indexing as the reference; maps are generated on the GPU by
apg_map_generate (bit-exact with FloorMapDatasetRooms/Maze.get_data_point) and, for direct
indexing, unpacked to the reference's bool[H, W] arrays.
"""

from __future__ import annotations

import numpy as np

from . import _native as N


class FloorMapDataset:
    map_kind: int

    def __init__(self, map_width: int, map_height: int):
        self._w, self._h = int(map_width), int(map_height)

    @property
    def map_width(self) -> int:
        return self._w

    @property
    def map_height(self) -> int:
        return self._h

    def load(self):
        pass

    def __len__(self):
        return 2**32

    def native_params(self) -> dict:
        raise NotImplementedError

    def get_data_point_batch(self, idx, device="cuda") -> np.ndarray:
        return generate_maps(self, np.asarray(idx, dtype=np.uint64), device=device)

    def get_data_point(self, idx, device="cuda") -> np.ndarray:
        return self.get_data_point_batch([int(idx)], device=device)[0]

    def __getitem__(self, item):
        if isinstance(item, (list, tuple, np.ndarray)):
            return self.get_data_point_batch(item)
        return self.get_data_point(item)


class FloorMapDatasetRooms(FloorMapDataset):
    """floor_map_dataset_rooms.py:10-89 (recursive room split with doors, random transpose)."""

    map_kind = N.APG_MAP_ROOMS

    def __init__(self, width: int = 32, height: int = 32, max_rooms: int = 10, door_width: int = 3):
        self.max_rooms = int(max_rooms)
        self.door_width = int(door_width)
        super().__init__(width, height)

    def native_params(self):
        return dict(max_rooms=self.max_rooms, door_width=self.door_width, branching_prob=1.0)


class FloorMapDatasetMaze(FloorMapDataset):
    """floor_map_dataset_maze.py:10-55 (recursive-backtracker maze on odd-sized grids)."""

    map_kind = N.APG_MAP_MAZE

    def __init__(self, width: int = 21, height: int = 21, branching_prob: float = 1.0):
        if width % 2 == 0 or height % 2 == 0:
            raise ValueError("Width and height must be odd.")
        self.branching_prob = float(branching_prob)
        super().__init__(width, height)

    def native_params(self):
        return dict(max_rooms=10, door_width=3, branching_prob=self.branching_prob)


def unpack_occupancy(occ_words: np.ndarray, h: int, w: int) -> np.ndarray:
    """uint64 bit rows [..., h, wpr] -> bool [..., h, w]."""
    b = occ_words.astype("<u8").view(np.uint8)
    bits = np.unpackbits(b.reshape(*occ_words.shape[:-1], -1), axis=-1, bitorder="little")
    return bits[..., :w].astype(bool)


def generate_maps(ds: FloorMapDataset, idx: np.ndarray, device="cuda") -> np.ndarray:
    import torch

    p = ds.native_params()
    n = int(idx.size)
    h, w = ds.map_height, ds.map_width
    wpr = (w + 63) // 64
    dev = torch.device(device)
    idx_t = torch.as_tensor(idx.astype(np.int64), device=dev)
    occ = torch.zeros((n, h, wpr), dtype=torch.int64, device=dev)
    scratch = None  # reserved ABI slot, unused
    frames = int(N.lib().apg_maze_frames(h, w))
    stack = torch.zeros((n, frames), dtype=torch.int16, device=dev) if ds.map_kind == N.APG_MAP_MAZE else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = N.lib().apg_map_generate(ds.map_kind, N.ptr(idx_t), n, h, w, p["max_rooms"], p["door_width"],
                                  p["branching_prob"], N.ptr(occ), N.ptr(scratch), N.ptr(stack), N.ptr(err),
                                  N.stream_handle(dev))
    N.check(rc, "apg_map_generate")
    if int(err.item()) != 0:
        raise N.ApgError("map generation exceeded an internal bound")
    return unpack_occupancy(occ.cpu().numpy().view(np.uint64), h, w)
