"""Streamed floor maps: the host side of APG_MAP_POOL with stream_len > 0 (include/apgym_capi.h).

The reference fetches every episode's map from the dataset when the episode starts: each sub-env's
`DataLoader(DatasetIterator(dataset, seed), prefetch=True)` (lidar_localization2d.py:547-557) draws
`idx = rng.integers(0, len(dataset))` and calls `dataset.get_data_point(idx)` on a background thread
(dataset_iterator.py:26-32, buffered_iterator.py:11-61), and reset() takes the next item (:296-298).  A
dataset too large to read at construction (len 2**32, or a budget's worth of maps), or one the user wants
fetched per draw (`frozen_maps=False`), runs that way here too:

* every env owns one map slot on the device (`pool_occ[e]`, `pool_free[e]`); the kernels draw the
  episode's index from the env's DatasetIterator stream as usual and install slot e;
* which index an env's NEXT reset will draw is known one episode ahead (the stream is advanced by nothing
  else), so `apg_lidar_peek_map_index` reads it from a copy of the stream right after the env's reset;
* a worker thread (the BufferedIterator's) calls `get_data_point(idx)` for those envs, packs the maps
  into bit rows and uploads them into the slots on a side stream;
* an env reset at step t can reset again at step t + 2 at the earliest (its next episode holds at least
  one step), so before launching step t + 2 the env's stream waits for step t's upload (the host blocks
  only if the thread has not even submitted it yet, like `next()` on an empty BufferedIterator).

reset(seed) fetches the first maps synchronously (their indices peeked from the seeded streams).
"""

from __future__ import annotations

import ctypes
from collections import deque
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native as N
from .floor_map import pack_maps


class MapStreamer:
    RING = 3  # peek result buffers (a step's buffers are read by its job before step + 2 is launched)

    def __init__(self, dataset, num_envs: int, device):
        import torch

        self.ds = dataset
        self.n = int(num_envs)
        self.h, self.w = dataset.map_height, dataset.map_width
        self.wpr = (self.w + 63) // 64
        self.device = torch.device(device)
        dev, n = self.device, self.n
        self.slots_occ = torch.zeros((n, self.h, self.wpr), dtype=torch.int64, device=dev)
        self.slots_free = torch.zeros(n, dtype=torch.int32, device=dev)
        self._idx = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(self.RING)]
        self._env = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(self.RING)]
        self._cnt = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(self.RING)]
        self._cnt_host = [torch.zeros(1, dtype=torch.int32).pin_memory() for _ in range(self.RING)]
        self._side = torch.cuda.Stream(dev)
        self._pool = ThreadPoolExecutor(1, thread_name_prefix="apg-map-stream")
        self._jobs: deque = deque()  # (step, future -> upload event or None)
        self.step_no = 0
        self.fetched = 0  # get_data_point calls so far (diagnostics)

    # ------------------------------------------------------------------ device side
    def _peek(self, env, seed: int, use_seed: bool, mask_ptr, slot: int | None):
        """apg_lidar_peek_map_index on the env's current stream: dense into _idx[0] (slot None) or compacted into
        ring slot `slot`."""
        out_env = out_cnt = None
        k = 0 if slot is None else slot
        if slot is not None:
            out_env, out_cnt = self._env[k], self._cnt[k]
        rc = N.lib().apg_lidar_peek_map_index(ctypes.byref(env._cfg), ctypes.byref(env._state),
                                              ctypes.c_uint64(seed & (2**64 - 1)), int(use_seed), mask_ptr,
                                              N.ptr(self._idx[k]), N.ptr(out_env), N.ptr(out_cnt), env._stream())
        N.check(rc, "apg_lidar_peek_map_index")

    def _fetch(self, idx: np.ndarray):
        """DatasetIterator.__next__'s get_data_point(idx) (dataset_iterator.py:31) for each index, packed."""
        k = len(idx)
        bits = np.zeros((k, self.h, self.wpr * 8), np.uint8)
        free = np.zeros(k, np.int32)
        maps = []
        for i in idx.tolist():
            maps.append(self.ds.map_array(int(i)))
        pack_maps(maps, self.h, self.w, bits, free, first=0)
        self.fetched += k
        return bits.view(np.int64).reshape(k, self.h, self.wpr), free

    def _upload(self, envs_np: np.ndarray, bits: np.ndarray, free: np.ndarray, stream):
        import torch

        with torch.cuda.stream(stream):
            e = torch.as_tensor(envs_np.astype(np.int64)).to(self.device, non_blocking=False)
            self.slots_occ.index_copy_(0, e, torch.as_tensor(bits).to(self.device, non_blocking=False))
            self.slots_free.index_copy_(0, e, torch.as_tensor(free).to(self.device, non_blocking=False))

    # ------------------------------------------------------------------ protocol
    def drain(self):
        """Finish every pending fetch and order the env's stream after its uploads."""
        import torch

        while self._jobs:
            _, fut = self._jobs.popleft()
            ev = fut.result()
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)

    def before_reset(self, env, seed: int, use_seed: bool):
        """reset(seed): the maps of every env's first draw, fetched synchronously into the slots."""
        import torch

        self.drain()
        self._peek(env, seed, use_seed, None, None)
        idx = self._idx[0].cpu().numpy()  # (synchronizes the env's stream)
        bits, free = self._fetch(idx)
        self._upload(np.arange(self.n), bits, free, torch.cuda.current_stream(self.device))

    def after_reset(self, env):
        """Every env consumed its slot: the next indices of all of them, fetched by the worker thread."""
        self.step_no = 0
        self._launch_job(env, None, 0)

    def before_step(self):
        """Step t = step_no + 1: the uploads of the resets at steps <= t - 2 must be in the slots first."""
        import torch

        self.step_no += 1
        t = self.step_no
        while self._jobs and self._jobs[0][0] <= t - 2:
            _, fut = self._jobs.popleft()
            ev = fut.result()  # (re-raises a dataset error, like next() on the reference's BufferedIterator)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)

    def after_step(self, env, reset_mask_ptr):
        """The envs this step reset (reset_mask) consumed their slots: peek their next indices, fetch ahead."""
        self._launch_job(env, reset_mask_ptr, self.step_no)

    def _launch_job(self, env, mask_ptr, step: int):
        import torch

        slot = step % self.RING
        self._peek(env, 0, False, mask_ptr, slot)
        main = torch.cuda.current_stream(self.device)
        self._cnt_host[slot].copy_(self._cnt[slot], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(main)
        self._jobs.append((step, self._pool.submit(self._job, slot, ev)))

    def _job(self, slot: int, ready):
        """Worker thread: the envs listed by the peek, their maps fetched, packed and uploaded on the side stream;
        returns the upload's event (None when no env reset)."""
        import torch

        with torch.cuda.device(self.device):
            ready.synchronize()
            k = int(self._cnt_host[slot].item())
            if k == 0:
                return None
            side = self._side
            side.wait_event(ready)
            with torch.cuda.stream(side):
                envs = self._env[slot][:k].cpu().numpy()
                idx = self._idx[slot][:k].cpu().numpy()
            order = np.argsort(envs, kind="stable")  # the envs' own order (the peek's compaction has none)
            envs, idx = envs[order], idx[order]
            bits, free = self._fetch(idx)
            self._upload(envs, bits, free, side)
            done = torch.cuda.Event()
            done.record(side)
            return done

    def close(self):
        try:
            self.drain()
        finally:
            self._pool.shutdown(wait=True)
