"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / CPU baseline.  The product package never imports this module.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None
MAP_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p)


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("apg_oracle_rng_maps.c", "apg_oracle_lidar.c", "apg_oracle.h")]
    if force or not os.path.exists(LIB_PATH) or any(os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in srcs):
        subprocess.run(["make", "-s", "-C", HERE, "-B" if force else "liboracle.so"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, u64, f32, f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_float, ctypes.c_double
        L.orc_test_draws.argtypes = [u64, i32, ctypes.c_int64, ctypes.c_int64, f64, i32, vp]
        L.orc_rooms_map.argtypes = [u64, i32, i32, i32, i32, vp]
        L.orc_maze_map.argtypes = [u64, i32, i32, f64, vp]
        L.orc_lidar_scan.restype = f32
        L.orc_lidar_scan.argtypes = [vp, i32, i32, f32, f32, f32, f32, ctypes.POINTER(i32)]
        L.orc_lidar_create.restype = vp
        L.orc_lidar_create.argtypes = [i32, i32, i32, i32, i32, i32, i32, f32, i32, vp]
        L.orc_lidar_destroy.argtypes = [vp]
        L.orc_lidar_set_rooms.argtypes = [vp, i32, i32]
        L.orc_lidar_reset.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.orc_lidar_step.restype = i32
        L.orc_lidar_step.argtypes = [vp] + [vp] * 14
        L.orc_lidar_step_mt.restype = i32
        L.orc_lidar_step_mt.argtypes = [vp, i32] + [vp] * 14
        L.orc_lidar_get_state.argtypes = [vp, vp, vp, vp, vp]
        L.orc_lidar_set_pool.restype = i32
        L.orc_lidar_set_pool.argtypes = [vp, vp, ctypes.c_int64, i32]
        L.orc_lidar_set_map_source.restype = i32
        L.orc_lidar_set_map_source.argtypes = [vp, MAP_FN, vp, ctypes.c_int64]
        L.orc_lidar_no_free.restype = i32
        L.orc_lidar_no_free.argtypes = [vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def rooms_map(idx: int, size: int, max_rooms: int = 10, door_width: int = 3) -> np.ndarray:
    out = np.zeros((size, size), np.uint8)
    if lib().orc_rooms_map(idx, size, size, max_rooms, door_width, _p(out)) != 0:
        raise ValueError("rooms map must be square")
    return out


def maze_map(idx: int, h: int, w: int | None = None, branching_prob: float = 1.0) -> np.ndarray:
    w = h if w is None else w
    out = np.zeros((h, w), np.uint8)
    if lib().orc_maze_map(idx, h, w, branching_prob, _p(out)) != 0:
        raise ValueError("Width and height must be odd.")
    return out


def lidar_scan(occ: np.ndarray, p, q):
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    k = ctypes.c_int()
    d = lib().orc_lidar_scan(_p(occ), occ.shape[0], occ.shape[1], float(p[0]), float(p[1]), float(q[0]),
                             float(q[1]), ctypes.byref(k))
    return np.float32(d), k.value


def beam_directions(beams: int, lidar_range: float = 5) -> np.ndarray:
    """lidar_localization2d.py:181-187, evaluated by numpy exactly like the reference."""
    ang = np.linspace(-np.pi, np.pi, beams, dtype=np.float32, endpoint=False)
    return np.ascontiguousarray(np.stack([np.cos(ang), np.sin(ang)], axis=-1) * lidar_range, dtype=np.float32)


class OracleLidarVectorEnv:
    """SyncVectorEnv(TimeLimit(LIDARLocalization2DEnv)) restated in C; numpy in/out."""

    def __init__(self, num_envs, map_kind="rooms", size=32, static_map=False, static_map_index=0, beams=8,
                 lidar_range=5, step_limit=100, sparse=False, max_rooms=10, door_width=3, pool=None,
                 map_fn=None, map_len=None, map_hw=None):
        """map_kind "pool": `pool` holds the maps of a finite FloorMapDataset, bool [len, H, W] (any H x W).
        map_kind "stream": `map_fn(idx) -> bool [H, W]` is the dataset's get_data_point, called at every draw
        (dataset_iterator.py:26-32), `map_len` its len (any size), `map_hw` = (H, W)."""
        self._map_cb = None
        if map_kind == "stream":
            size_hw = tuple(map_hw)
            h_, w_ = size_hw

            def cb(_ctx, idx, out):
                try:
                    m = np.asarray(map_fn(int(idx)), dtype=bool)
                    if m.shape != (h_, w_):
                        return 1
                    ctypes.memmove(out, np.ascontiguousarray(m.view(np.uint8)).ctypes.data, h_ * w_)
                    return 0
                except Exception:  # noqa: BLE001 (reported as a failed draw)
                    return 1

            self._map_cb = MAP_FN(cb)
        elif map_kind == "pool":
            self._pool = np.ascontiguousarray(np.asarray(pool, dtype=bool).view(np.uint8))
            size_hw = self._pool.shape[1:]
        else:
            size_hw = (size, size)
        self.n, self.beams = num_envs, beams
        self.h, self.w = size_hw
        size = self.h
        self.static = static_map
        self.dirs = beam_directions(beams, lidar_range)
        kind = {"rooms": 0, "maze": 1, "pool": 2, "stream": 2}[map_kind]
        self._e = lib().orc_lidar_create(num_envs, kind, self.h, self.w, int(static_map),
                                         static_map_index, beams, float(lidar_range), step_limit, _p(self.dirs))
        if not self._e:
            raise ValueError("invalid map configuration")
        if map_kind == "stream":
            if static_map or lib().orc_lidar_set_map_source(self._e, self._map_cb, None, int(map_len)) != 0:
                raise ValueError("streamed maps: dynamic maps and map_len >= 1")
        elif kind == 2 and lib().orc_lidar_set_pool(self._e, _p(self._pool), len(self._pool), static_map_index) != 0:
            raise ValueError("invalid map pool / static_map_index")
        if (max_rooms, door_width) != (10, 3):
            lib().orc_lidar_set_rooms(self._e, max_rooms, door_width)
        n = num_envs
        self.lidar = np.zeros((n, beams), np.float32)
        self.odometry = np.zeros((n, 2), np.float32)
        self.time_step = np.zeros(n, np.float32)
        self.map = None if static_map else np.zeros((n, self.h, self.w), np.float32)
        self.map_idx = np.zeros(n, np.uint64)
        self.reward = np.zeros(n, np.float64)
        self.terminated = np.zeros(n, np.uint8)
        self.truncated = np.zeros(n, np.uint8)
        self.base_reward = np.zeros(n, np.float32)
        self.target = np.zeros((n, 2), np.float32)
        self.loss = np.zeros(n, np.float32)
        self.info_mask = np.zeros(n, np.uint8)
        self.sparse = sparse
        self.weight = np.zeros(n, np.float64)

    def close(self):
        if self._e:
            lib().orc_lidar_destroy(self._e)
            self._e = None

    __del__ = close

    def reset(self, seed: int):
        lib().orc_lidar_reset(self._e, seed, _p(self.lidar), _p(self.odometry), _p(self.time_step), _p(self.map),
                              _p(self.map_idx))

    def step(self, action, prediction, threads: int = 1) -> int:
        """threads > 1: the OpenMP variant (same outputs; bench.py's multi-core CPU baseline)."""
        a = np.ascontiguousarray(action, np.float32)
        p = np.ascontiguousarray(prediction, np.float32)
        outs = (_p(self.lidar), _p(self.odometry), _p(self.time_step), _p(self.map), _p(self.reward),
                _p(self.terminated), _p(self.truncated), _p(self.base_reward), _p(self.target), _p(self.loss),
                _p(self.info_mask), _p(self.map_idx))
        if threads > 1:
            rc = lib().orc_lidar_step_mt(self._e, threads, _p(a), _p(p), *outs)
        else:
            rc = lib().orc_lidar_step(self._e, _p(a), _p(p), *outs)
        if self.sparse:
            # SparsifyWrapper.step per sub-env (sparsify_wrapper.py:137-151): weight = 1.0 if terminated
            # else 0.0 (SyncVectorEnv merges the floats into float64); reward = base_reward - loss * weight
            # in float32 (np.float32 loss times a Python float), stored as float64
            m = self.info_mask.astype(bool)
            w = np.where(self.terminated.astype(bool), np.float32(1.0), np.float32(0.0))
            with np.errstate(invalid="ignore"):
                r = (self.base_reward - self.loss * w).astype(np.float64)
            self.weight = np.where(m, w.astype(np.float64), 0.0)
            self.reward = np.where(m, r, 0.0)
        return rc

    def no_free_cell(self) -> bool:
        """A map without free cells was drawn (the reference raised ValueError("high <= 0") there)."""
        return bool(lib().orc_lidar_no_free(self._e))

    def state(self):
        n = self.n
        pos, ipos = np.zeros((n, 2), np.float32), np.zeros((n, 2), np.float32)
        el, ar = np.zeros(n, np.int32), np.zeros(n, np.uint8)
        lib().orc_lidar_get_state(self._e, _p(pos), _p(ipos), _p(el), _p(ar))
        return dict(pos=pos, init_pos=ipos, elapsed=el, autoreset=ar)
