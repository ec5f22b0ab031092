"""LIDARLocalization2DVectorEnv — the LIDARLoc* env ids as one batched GPU environment.

Reference behaviour reproduced (ap_gym 0.5.0): `make_vec("LIDARLoc*-v0", N)` builds gymnasium's
SyncVectorEnv over N copies of TimeLimit(100, issue_termination=True) ∘ LIDARLocalization2DEnv
(ap_gym/envs/registration.py:319-356, :753-767).  This class is that whole composition as state in
HBM plus one fused kernel launch per step (include/apgym_capi.h):

  reset(seed=s)   sub-env i seeded with s+i (SyncVectorEnv.reset), map + start cell drawn on device
  step(action)    NEXT_STEP autoreset: envs done at the previous step return their reset obs with
                  reward 0 / terminated False / truncated False and no base_reward/prediction info
  obs             {"lidar": f32[N,B], "odometry": f32[N,2], "map": f32[N,H,W,1] (dynamic maps),
                   "time_step": f32[N]}
  reward          float64 (SyncVectorEnv's reward array), base_reward - normalized MSE loss
  info            {"base_reward", "prediction": {"target", "loss"}, "map_idx"} with `_key` masks, and
                  with log_stats=True (the registered ids, registration.py:348-355) the per-episode
                  "stats" of ActiveRegressionLogWrapper (active_regression_env.py:131-159) for the
                  envs whose episode ended: scalar avg_/final_ euclidean_distance and mse, vector
                  lists of the per-step values
  sparse=True     the "-sparse" ids (registration.py:115-142, SparsifyWrapper sparsify_wrapper.py:93-161
                  on every sub-env): prediction target {"target", "weight" = 1.0 where terminated},
                  reward = base_reward - loss * weight.  The reference's own LIDAR "-sparse" ids raise
                  KeyError('prediction') in reset (SparsifyWrapper.reset needs info["prediction"], which
                  LIDARLocalization2DEnv.reset does not return), and so does this env by default (after
                  resetting its state, as the reference's first sub-env does).  sparse_reset_info=True
                  opts into a working reset (reset info as the dense ids) with the wrapper's step
                  semantics

Two I/O modes (constructor `array_backend`), inputs of either type are accepted:
  "numpy" (default) -> numpy out, host copies and host-side NaN checks, like the reference.  By default
                       (copy=None -> True, SyncVectorEnv's default, which deep-copies the observations) every
                       returned array is the caller's own: writable, never written again by the env, obs["map"]
                       included (a full copy of the map obs per step, 4*H*W bytes per env).
                       obs_snapshot="shared" (opt-in) hands out obs["map"] as one read-only array shared by
                       the steps between two steps with resets instead (no per-step copy: the map obs changes
                       only at resets).  copy=False returns the pinned host mirror of the map obs itself
                       (writable, refreshed in place at resets)
  "torch"           -> torch out on the env's device, no host synchronisation.  Returned tensors
                       are persistent buffers overwritten by the next step (gymnasium's copy=False
                       contract, the default here: copy=None -> False); pass copy=True to get fresh
                       tensors.  NaN errors are raised lazily (at a later step) unless strict_errors=True.
"""

from __future__ import annotations

import ctypes
from typing import Any

import numpy as np

from . import _native as N
from .floor_map import FloorMapDataset, FloorMapDatasetMaze, FloorMapDatasetRooms, as_floor_map_dataset
from .loss_fn import WeightedLossFn, affine_f32, regression_loss
from .spaces import ActivePerceptionActionSpace, Box, Dict, ImageSpace, batch_space
from .vector_env import VectorEnv

NAN_ACTION_MSG = "NaN values detected in action."
NAN_PREDICTION_MSG = "NaN values detected in prediction."


def lidar_beam_directions(beams: int, lidar_range: float) -> np.ndarray:
    """lidar_localization2d.py:181-187 evaluated with numpy exactly as the reference does."""
    ang = np.linspace(-np.pi, np.pi, beams, dtype=np.float32, endpoint=False)
    unscaled = np.stack([np.cos(ang), np.sin(ang)], axis=-1)
    return np.ascontiguousarray(unscaled * lidar_range, dtype=np.float32)


# Packed output rows (apg_lidar_config.out_row_bytes): every per-env output of a step in one row per env,
# 8-byte fields first, so ShardedVectorEnv all-gathers the [N, row] buffer as is (no packing copies) and
# the gathered fields are strided views of the receive buffer.
def lidar_output_row_layout(beams: int, log_stats: bool = False, sparse: bool = False):
    """[(name, torch dtype, per-env shape, byte offset)] of the packed output row, and the row size."""
    import torch

    f64, i64, f32, i32, b8 = torch.float64, torch.int64, torch.float32, torch.int32, torch.bool
    fields = [("reward", f64, ()), ("map_idx_out", i64, ())] + ([("weight", f64, ())] if sparse else []) + [
        ("lidar", f32, (beams,)), ("odometry", f32, (2,)), ("target", f32, (2,)), ("time_step", f32, ()),
        ("base_reward", f32, ()), ("loss", f32, ())] + (
        [("stats", f32, (4,)), ("stats_len", i32, ())] if log_stats else []) + [
        ("terminated", b8, ()), ("truncated", b8, ()), ("info_mask", b8, ()), ("reset_mask", b8, ())]
    out, off = [], 0
    for name, dt, sh in fields:
        out.append((name, dt, sh, off))
        off += torch.empty((), dtype=dt).element_size() * int(np.prod(sh, dtype=np.int64))
    return out, off + (-off) % 8


def row_views(buf, layout) -> dict:
    """Field views of a packed [rows, row_bytes] uint8 buffer (stats as [4, rows] like the dense layout)."""
    import torch

    v = {}
    for name, dt, sh, off in layout:
        nb = torch.empty((), dtype=dt).element_size() * int(np.prod(sh, dtype=np.int64))
        t = buf[:, off:off + nb].view(dt)
        if not sh:
            t = t[:, 0]
        v[name] = t.T if name == "stats" else t
    return v


_NP_DTYPES: dict = {}


def np_dtype(dt) -> np.dtype:
    """numpy dtype of a torch dtype (cached: the numpy backend builds its field views every step)."""
    r = _NP_DTYPES.get(dt)
    if r is None:
        import torch

        r = _NP_DTYPES[dt] = torch.empty((), dtype=dt).numpy().dtype
    return r


def row_views_np(buf: np.ndarray, layout) -> dict:
    """numpy field views of a packed [rows, row_bytes] uint8 host buffer (stats as [4, rows])."""
    v = {}
    for name, dt, sh, off in layout:
        npdt = np_dtype(dt)
        nb = npdt.itemsize * int(np.prod(sh, dtype=np.int64))
        a = buf[:, off:off + nb].view(npdt)
        a = a[:, 0] if not sh else a.reshape(buf.shape[0], *sh)
        v[name] = a.T if name == "stats" else a
    return v


# The numpy backend's output block: the same fields in the dense layout (field-major, each contiguous and
# 256-byte aligned) inside one buffer, so a step's outputs come to the host in ONE D2H copy and every host
# field is a contiguous array (its copy a plain memcpy; packed rows would need strided gathers).
def lidar_output_block_layout(num_envs: int, beams: int, log_stats: bool = False, sparse: bool = False):
    """[(name, torch dtype, shape, byte offset)] of the field-major output block, and its size."""
    import torch

    n = num_envs
    f64, i64, f32, i32, b8 = torch.float64, torch.int64, torch.float32, torch.int32, torch.bool
    fields = [("reward", f64, (n,)), ("map_idx_out", i64, (n,))] + ([("weight", f64, (n,))] if sparse else []) + [
        ("lidar", f32, (n, beams)), ("odometry", f32, (n, 2)), ("target", f32, (n, 2)), ("time_step", f32, (n,)),
        ("base_reward", f32, (n,)), ("loss", f32, (n,))] + (
        [("stats", f32, (4, n)), ("stats_len", i32, (n,))] if log_stats else []) + [
        ("terminated", b8, (n,)), ("truncated", b8, (n,)), ("info_mask", b8, (n,)), ("reset_mask", b8, (n,))]
    out, off = [], 0
    for name, dt, sh in fields:
        out.append((name, dt, sh, off))
        off += torch.empty((), dtype=dt).element_size() * int(np.prod(sh, dtype=np.int64))
        off += (-off) % 256
    return out, off


def block_views(buf, layout) -> dict:
    """Field views of a flat uint8 output block (torch or numpy)."""
    v = {}
    for name, dt, sh, off in layout:
        if isinstance(buf, np.ndarray):
            npdt = np_dtype(dt)
            v[name] = buf[off:off + npdt.itemsize * int(np.prod(sh, dtype=np.int64))].view(npdt).reshape(sh)
        else:
            nb = torch_elem(dt) * int(np.prod(sh, dtype=np.int64))
            v[name] = buf[off:off + nb].view(dt).view(sh)
    return v


def torch_elem(dt) -> int:
    import torch

    return torch.empty((), dtype=dt).element_size()


def torch_index(idx: np.ndarray, device):
    import torch

    return torch.as_tensor(idx, dtype=torch.int64, device=device)


def lidar_spaces(num_envs: int, height: int, width: int, beams: int, static_map: bool, sparse: bool) -> dict:
    """Spaces and loss of the LIDAR ids (lidar_localization2d.py:144-227, time_limit.py:64-70,
    active_regression_env.py:55-76; sparse: sparsify_wrapper.py:93-127)."""
    obs = {"lidar": Box(0, 1, (beams,), np.float32), "odometry": Box(-1, 1, (2,), np.float32)}
    if not static_map:
        obs["map"] = ImageSpace(width=width, height=height, channels=1)
    obs["time_step"] = Box(-1.0, 1.0, (), np.float32)
    single_obs = Dict(obs)
    single_act = ActivePerceptionActionSpace(Box(-1, 1, (2,), np.float32), Box(-1, 1, (2,), np.float32))
    single_target = Box(-1, 1, (2,), np.float32)
    loss_fn = inner_loss = regression_loss(2, -1, 1)
    if sparse:
        single_target = Dict({"target": single_target, "weight": Box(0, 1, (), np.float32)})
        loss_fn = WeightedLossFn(inner_loss)
    return dict(single_observation_space=single_obs, observation_space=batch_space(single_obs, num_envs),
                single_action_space=single_act, action_space=batch_space(single_act, num_envs),
                single_prediction_target_space=single_target,
                prediction_target_space=batch_space(single_target, num_envs), loss_fn=loss_fn, inner_loss=inner_loss)


class LIDARLocalization2DVectorEnv(VectorEnv):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 4, "autoreset_mode": "NextStep"}
    ERROR_POLL_INTERVAL = 128  # steps between the lazy error-word copies (each costs the stream a blit + marker)

    def __init__(self, num_envs: int = 1, dataset: FloorMapDataset | None = None, render_mode: str = "rgb_array",
                 static_map: bool = False, lidar_beam_count: int = 8, lidar_range: float = 5,
                 static_map_index: int = 0, prefetch: bool = True, prefetch_buffer_size: int = 128,
                 max_episode_steps: int = 100, device=None, env_offset: int = 0, copy: bool | None = None,
                 strict_errors: bool = False, array_backend: str = "numpy", log_stats: bool = False,
                 sparse: bool = False, render_envs=None, sparse_reset_info: bool = False, packed_outputs: bool = False,
                 vector_stats: str = "list", frozen_maps: bool | None = None, obs_snapshot: str = "copy"):
        import torch

        if render_mode not in self.metadata["render_modes"]:
            raise ValueError(f"Invalid render mode: {render_mode}")
        if dataset is None:
            dataset = FloorMapDatasetRooms()
        # any other FloorMapDataset (a reference subclass included) runs from a resident map pool (APG_MAP_POOL)
        dataset = as_floor_map_dataset(dataset)
        dataset.load()  # lidar_localization2d.py:176
        self.num_envs = int(num_envs)
        self.dataset = dataset
        self.render_mode = render_mode
        self.static_map = bool(static_map)
        self.lidar_beam_count = int(lidar_beam_count)
        self.lidar_range = lidar_range
        self.max_episode_steps = int(max_episode_steps)
        self.env_offset = int(env_offset)
        if array_backend not in ("numpy", "torch"):
            raise ValueError("array_backend must be 'numpy' or 'torch'")
        self.copy = (array_backend == "numpy") if copy is None else bool(copy)
        self.strict_errors = strict_errors
        self.log_stats = bool(log_stats)
        if vector_stats not in ("list", "array"):
            raise ValueError("vector_stats must be 'list' (the reference's lists of np.float32) or 'array'")
        self.vector_stats = vector_stats  # numpy backend: form of info["stats"]["vector"] entries
        if obs_snapshot not in ("copy", "shared"):
            raise ValueError("obs_snapshot must be 'copy' (writable arrays, SyncVectorEnv(copy=True)) or 'shared'")
        self.obs_snapshot = obs_snapshot  # numpy backend, copy=True: obs["map"] per step or a shared snapshot
        self.sparse = bool(sparse)
        self.sparse_reset_info = bool(sparse_reset_info)
        self.array_backend = array_backend
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("LIDARLocalization2DVectorEnv runs on a GPU device (no CPU fallback)")
        h, w = dataset.map_height, dataset.map_width

        sp = lidar_spaces(self.num_envs, h, w, self.lidar_beam_count, self.static_map, self.sparse)
        inner_loss = sp.pop("inner_loss")
        for k, v in sp.items():
            setattr(self, k, v)

        # ---- native configuration
        p = dataset.native_params()
        pool_occ = pool_free = None
        self._streamer = None
        cfg_static_index, pool_len, stream_len = int(static_map_index), 0, 0
        if dataset.map_kind == N.APG_MAP_POOL:
            if self.static_map:  # dataset[static_map_index] alone (lidar_localization2d.py:177-178), any dataset size
                pool_occ, pool_free = dataset.static_pool(int(static_map_index), self.device)
                cfg_static_index, pool_len = 0, 1
            elif frozen_maps is True or (frozen_maps is None and not dataset.prefers_streaming()):
                pool_occ, pool_free = dataset.device_pool(self.device)  # every map of the dataset, once per device
                pool_len = len(dataset)
            else:  # get_data_point(idx) at every draw, fetched one episode ahead (map_stream.py)
                from .map_stream import MapStreamer

                self._streamer = MapStreamer(dataset, self.num_envs, self.device)
                pool_occ, pool_free = self._streamer.slots_occ, self._streamer.slots_free
                pool_len, stream_len = self.num_envs, len(dataset)
        self.frozen_maps = None if dataset.map_kind != N.APG_MAP_POOL or self.static_map else self._streamer is None
        scale, offset = affine_f32(inner_loss)
        self.output_layout, row_bytes = lidar_output_row_layout(self.lidar_beam_count, self.log_stats, self.sparse)
        if not packed_outputs:
            self.output_layout, row_bytes = None, 0
        self._cfg = N.LidarConfig(num_envs=self.num_envs, height=h, width=w, map_kind=dataset.map_kind,
                                  is_static=int(self.static_map), static_map_index=cfg_static_index,
                                  beams=self.lidar_beam_count, step_limit=self.max_episode_steps,
                                  max_rooms=p["max_rooms"], door_width=p["door_width"],
                                  lidar_range=float(np.float32(lidar_range)), loss_scale=scale, loss_offset=offset,
                                  branching_prob=p["branching_prob"], log_stats=int(self.log_stats),
                                  sparse=int(self.sparse), out_row_bytes=row_bytes,
                                  pool_len=pool_len, stream_len=stream_len)
        L = N.lib()
        sizes = N.LidarSizes()
        N.check(L.apg_lidar_query_sizes(ctypes.byref(self._cfg), ctypes.byref(sizes)), "apg_lidar_query_sizes")

        dev, n, B = self.device, self.num_envs, self.lidar_beam_count
        t = torch
        self._t = dict(
            pos=t.zeros((n, 2), dtype=t.float32, device=dev),
            init_pos=t.zeros((n, 2), dtype=t.float32, device=dev),
            elapsed=t.zeros(n, dtype=t.int32, device=dev),
            flags=t.zeros(n, dtype=t.uint8, device=dev),
            rng=t.zeros((n, 5), dtype=t.int64, device=dev),
            it_rng=t.zeros((n, 5), dtype=t.int64, device=dev),
            occ=t.zeros(max(1, sizes.occ_bytes // 8), dtype=t.int64, device=dev),
            scratch=t.zeros(sizes.scratch_bytes // 8, dtype=t.int64, device=dev) if sizes.scratch_bytes else None,
            stack=t.zeros(sizes.stack_bytes // 2, dtype=t.int16, device=dev) if sizes.stack_bytes else None,
            map_idx=t.full((n,), int(static_map_index) if self.static_map else 0, dtype=t.int64, device=dev),
            beam_dirs=t.as_tensor(lidar_beam_directions(B, lidar_range), device=dev),
            lidar=t.zeros((n, B), dtype=t.float32, device=dev),
            odometry=t.zeros((n, 2), dtype=t.float32, device=dev),
            time_step=t.zeros(n, dtype=t.float32, device=dev),
            map_obs=None if self.static_map else t.zeros((n, h, w, 1), dtype=t.float32, device=dev),
            reward=t.zeros(n, dtype=t.float64, device=dev),
            terminated=t.zeros(n, dtype=t.bool, device=dev),
            truncated=t.zeros(n, dtype=t.bool, device=dev),
            base_reward=t.zeros(n, dtype=t.float32, device=dev),
            target=t.zeros((n, 2), dtype=t.float32, device=dev),
            loss=t.zeros(n, dtype=t.float32, device=dev),
            info_mask=t.zeros(n, dtype=t.bool, device=dev),
            map_idx_out=t.zeros(n, dtype=t.int64, device=dev),
            reset_mask=t.zeros(n, dtype=t.bool, device=dev),
            err=t.zeros(1, dtype=t.int32, device=dev),
            stats_hist=(t.zeros((2, self.max_episode_steps, n), dtype=t.float32, device=dev) if self.log_stats
                        else None),  # step-major: the per-step stores of the kernel are coalesced
            stats=t.zeros((4, n), dtype=t.float32, device=dev) if self.log_stats else None,
            stats_len=t.zeros(n, dtype=t.int32, device=dev) if self.log_stats else None,
            weight=t.zeros(n, dtype=t.float64, device=dev) if self.sparse else None,
            # the next map of every env, generated ahead of its autoreset on a side stream (dynamic mazes): the
            # reference's DataLoader(prefetch=True) thread (lidar_localization2d.py:130-131, 296-298)
            prefetch=(t.zeros(sizes.prefetch_bytes, dtype=t.uint8, device=dev)
                      if prefetch and sizes.prefetch_bytes else None),
            pool_occ=pool_occ, pool_free=pool_free,
        )
        # packed_outputs: the per-env outputs are field views of one [n, row] buffer (ShardedVectorEnv's send)
        self.output_rows = None
        self._out_block = self._block_layout = None
        if row_bytes:
            self.output_rows = t.zeros((n, row_bytes), dtype=t.uint8, device=dev)
            self._t.update(row_views(self.output_rows, self.output_layout))
        elif array_backend == "numpy":  # dense fields inside one block: one D2H copy per step (_host_rows)
            self._block_layout, nbytes = lidar_output_block_layout(n, B, self.log_stats, self.sparse)
            self._out_block = t.zeros(nbytes, dtype=t.uint8, device=dev)
            self._t.update(block_views(self._out_block, self._block_layout))
        T = self._t
        # the prefetcher (C++ in the library): side stream, pinned per-step reset counts, batch events
        self._prefetcher = None
        if T["prefetch"] is not None:
            h_pf = ctypes.c_void_p()
            with torch.cuda.device(dev):
                N.check(L.apg_lidar_prefetcher_create(ctypes.byref(self._cfg), ctypes.byref(h_pf)),
                        "apg_lidar_prefetcher_create")
            self._prefetcher = h_pf.value
        self._state = N.LidarState(*[N.ptr(T[k]) for k in ("pos", "init_pos", "elapsed", "flags", "rng", "it_rng",
                                                            "occ", "scratch", "stack", "map_idx", "beam_dirs",
                                                            "stats_hist", "prefetch")], self._prefetcher,
                                    N.ptr(T["pool_occ"]), N.ptr(T["pool_free"]))
        self._out = N.LidarOutputs(N.ptr(T["lidar"]), N.ptr(T["odometry"]), N.ptr(T["time_step"]),
                                   N.ptr(T["map_obs"]), N.ptr(T["reward"]), N.ptr(T["terminated"]),
                                   N.ptr(T["truncated"]), N.ptr(T["base_reward"]), N.ptr(T["target"]),
                                   N.ptr(T["loss"]), N.ptr(T["info_mask"]), N.ptr(T["map_idx_out"]),
                                   N.ptr(T["reset_mask"]), N.ptr(T["err"]), N.ptr(T["stats"]),
                                   N.ptr(T["stats_len"]), N.ptr(T["weight"]))
        c = self._cfg
        self._ops = N.torch_ops()  # torch.ops.apgym: the reset/step hot path
        self._step_op = self._ops.lidar_step.default  # the overload itself: no per-call overload resolution
        self._dev = N.exact_device(self.device)
        # Eager steps call the C ABI directly (3.8 us of host time per call, against 15 us through the torch
        # dispatcher: tools/host_overhead_image.py); use_torch_op = True routes them through
        # torch.ops.apgym.lidar_step instead, which capture_step_graph always uses.
        self.use_torch_op = False
        self._c_args = None
        self._h = t.classes.apgym.LidarEnv(
            [c.num_envs, c.height, c.width, c.map_kind, c.is_static, c.static_map_index, c.beams, c.step_limit,
             c.max_rooms, c.door_width, c.log_stats, c.sparse, c.out_row_bytes, self._prefetcher or 0, c.pool_len,
             c.stream_len],
            [c.lidar_range, c.loss_scale, c.loss_offset, c.branching_prob],
            N.op_buffers([T[k] for k in ("pos", "init_pos", "elapsed", "flags", "rng", "it_rng", "occ", "scratch",
                                         "stack", "map_idx", "beam_dirs", "stats_hist", "prefetch")] + [None] +
                         [T["pool_occ"], T["pool_free"]], dev),
            N.op_buffers([T[k] for k in ("lidar", "odometry", "time_step", "map_obs", "reward", "terminated",
                                         "truncated", "base_reward", "target", "loss", "info_mask", "map_idx_out",
                                         "reset_mask", "err", "stats", "stats_len", "weight")], dev))
        self._err_host = t.zeros(1, dtype=t.int32).pin_memory()
        self._err_event = t.cuda.Event()
        self._err_pending = False
        self._autoreset_host = np.zeros(n, dtype=bool)
        self._rows_host = self._rows_np = self._map_host = None  # numpy backend: pinned host mirrors
        self._ring, self._ring_copy = [], False  # numpy backend: pinned output blocks (_host_block)
        self._map_snapshot = None  # numpy backend, copy=True, obs_snapshot="shared": read-only map obs until a reset
        self._map_copies = []  # numpy backend, copy=True, obs_snapshot="copy": host blocks handed out as obs["map"]
        self._in_host = self._in_dev = None  # numpy backend: pinned input staging and its device copy
        self._seeded = False
        self._closed = False
        self._kernel_events = None
        self._stats_view = None
        self._steps_since_poll = 0
        N.check(L.apg_lidar_init(ctypes.byref(self._cfg), ctypes.byref(self._state), self._stream()), "apg_lidar_init")
        self._setup_render(render_envs)

    # ------------------------------------------------------------------ render state
    def _setup_render(self, render_envs):
        """Device buffers of the render-only state of the tracked sub-envs (apg_lidar_render_track).
        render_envs=None tracks every sub-env up to render.DEFAULT_TRACKED of them, else none."""
        import torch

        from .render import tracked_envs

        self.render_envs = tracked_envs(render_envs, self.num_envs)
        self._r = self._rstate = None
        k = len(self.render_envs)
        if not k:
            return
        ang = np.linspace(-np.pi, np.pi, self.lidar_beam_count, dtype=np.float32, endpoint=False)
        unscaled = np.stack([np.cos(ang), np.sin(ang)], axis=-1)
        scan = np.arange(0, self.lidar_range, 0.05)[None, :, None] * unscaled[:, None]  # lidar_localization2d.py:188-191
        h, w, dev = self.dataset.map_height, self.dataset.map_width, self.device
        f32, i32 = torch.float32, torch.int32
        self._r = R = dict(
            env=torch.as_tensor(self.render_envs.astype(np.int32), device=dev),
            scan_xy=torch.as_tensor(np.ascontiguousarray(scan, dtype=np.float64), device=dev),
            scan_norm=torch.as_tensor(np.ascontiguousarray(np.linalg.norm(scan, axis=-1), dtype=np.float64), device=dev),
            obs_map=torch.zeros((k, h, (w + 31) // 32), dtype=i32, device=dev),
            traj=torch.zeros((k, self.max_episode_steps, 3), dtype=f32, device=dev),
            traj_len=torch.zeros(k, dtype=i32, device=dev),
            pose=torch.zeros((k, 6), dtype=f32, device=dev),
            has_last=torch.zeros(k, dtype=i32, device=dev),
            lidar_dist=torch.zeros((k, self.lidar_beam_count), dtype=f32, device=dev))
        self._rstate = N.LidarRenderState(k, scan.shape[1], *[N.ptr(R[n]) for n in (
            "env", "scan_xy", "scan_norm", "obs_map", "traj", "traj_len", "pose", "has_last", "lidar_dist")])

    def _track_render(self, prediction):
        if self._rstate is not None:
            N.check(N.lib().apg_lidar_render_track(ctypes.byref(self._cfg), ctypes.byref(self._state),
                                                   N.ptr(prediction), ctypes.byref(self._out),
                                                   ctypes.byref(self._rstate), self._stream()),
                    "apg_lidar_render_track")

    def _occupancy(self, envs: np.ndarray) -> np.ndarray:
        """Current maps (bool [len(envs), H, W]) of the given sub-envs, unpacked from the bit rows."""
        h, w = self.dataset.map_height, self.dataset.map_width
        wpr = (w + 63) // 64
        rows = self._t["occ"].view(-1, h * wpr)
        sel = np.zeros(len(envs), np.int64) if self.static_map else envs
        words = rows[torch_index(sel, self.device)].cpu().numpy()
        bits = np.unpackbits(words.view(np.uint8).reshape(len(envs), h, wpr * 8), axis=-1, bitorder="little")
        return bits[..., :w].astype(bool)

    def render(self):
        """SyncVectorEnv.render(): a tuple with one rgb_array frame per tracked sub-env, drawn from the
        device render state like LIDARLocalization2DEnv.render (lidar_localization2d.py:391-494)."""
        from .render import lidar_frame, no_tracked_error

        if self._rstate is None:
            raise no_tracked_error()
        if not self._seeded:
            raise RuntimeError("render() needs reset() first")
        R = {k: self._r[k].cpu().numpy() for k in ("obs_map", "traj", "traj_len", "pose", "has_last", "lidar_dist")}
        w = self.dataset.map_width
        seen = np.unpackbits(R["obs_map"].view(np.uint8), axis=-1, bitorder="little")[..., :w].astype(bool)
        occ = self._occupancy(self.render_envs)
        dirs = self._t["beam_dirs"].cpu().numpy()
        frames = []
        for j in range(len(self.render_envs)):
            p = R["pose"][j]
            last = bool(R["has_last"][j])
            frames.append(lidar_frame(occ[j], seen[j], R["traj"][j, :R["traj_len"][j]], R["lidar_dist"][j], dirs,
                                      p[4:6], p[0:2] if last else None, p[2:4] if last else None))
        return tuple(frames)

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        return N.stream_handle(self.device)

    @property
    def unwrapped(self):
        return self

    @property
    def prediction_space(self):
        return self.action_space["prediction"]

    @property
    def single_prediction_space(self):
        return self.single_action_space["prediction"]

    @property
    def inner_action_space(self):
        return self.action_space["action"]

    @property
    def single_inner_action_space(self):
        return self.single_action_space["action"]

    def capture_step_graph(self, action, prediction):
        """Capture one device step (torch.ops.apgym.lidar_step on the static `action` / `prediction`
        tensors, float32 [N, 2] on the env's device) into a torch.cuda.CUDAGraph (a hipGraph).  Each
        `graph.replay()` is one env step reading the tensors' current contents; its results land in the
        persistent output buffers (`device_outputs()`).  NaN checks run on the device as usual
        (`check_errors()`); the host-side bookkeeping of `step()` (render tracking, lazy error polling)
        is not part of the graph."""
        import torch

        if not self._seeded:
            raise RuntimeError("capture_step_graph() needs reset() first")
        if self._streamer is not None:
            raise RuntimeError("capture_step_graph(): streamed maps (frozen_maps=False) are fetched by the host "
                               "between steps; a captured step cannot do that")
        for name, x in (("action", action), ("prediction", prediction)):
            if not (isinstance(x, torch.Tensor) and x.dtype == torch.float32 and x.is_contiguous()
                    and x.device == self.device and x.numel() == 2 * self.num_envs):
                raise ValueError(f"{name} must be a contiguous float32 [num_envs, 2] tensor on {self.device}")
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side), torch.cuda.graph(graph, stream=side):
            self._ops.lidar_step(self._h, action, prediction)
        torch.cuda.current_stream(self.device).wait_stream(side)
        return graph

    def device_outputs(self) -> dict:
        """The persistent device buffers every step writes (obs, reward, flags, info fields)."""
        T = self._t
        out = {k: T[k] for k in ("lidar", "odometry", "time_step", "reward", "terminated", "truncated", "base_reward",
                                 "target", "loss", "info_mask", "reset_mask")}
        if not self.static_map:
            out["map"] = T["map_obs"]
        return out

    def _launch_step(self, a_t, p_t):
        if self.use_torch_op:
            self._step_op(self._h, a_t, p_t)
            return
        if N.wrong_current_device(self._dev):  # the op's DeviceGuard, for the direct call
            import torch

            with torch.cuda.device(self._dev):
                return self._launch_step(a_t, p_t)
        if self._c_args is None:  # (the structures' addresses: rebuilt whenever a structure is replaced)
            self._c_args = (N.fast().lidar_step, N.addr(self._cfg), N.addr(self._state), N.addr(self._out))
        fn, cfg, st, out = self._c_args
        rc = fn(cfg, st, a_t.data_ptr(), p_t.data_ptr(), out, N.current_stream_ptr(self._dev))
        if rc:
            N.check(rc, "apg_lidar_step")

    def set_kernel_timing_events(self, begin=None, end=None):
        """Record hipEvent_t handles `begin`/`end` around the step op (torch.ops.apgym.lidar_step: the
        fused step kernel, one launch) of the next step, on its stream (bench.py's live per-launch
        timing).  None disables."""
        self._kernel_events = None if begin is None else (begin, end)

    def _raise_error_bits(self, bits: int):
        if bits & N.APG_ERR_NAN_ACTION:
            raise ValueError(NAN_ACTION_MSG)
        if bits & N.APG_ERR_NAN_PREDICTION:
            raise ValueError(NAN_PREDICTION_MSG)
        if bits & N.APG_ERR_MAPGEN:
            raise N.ApgError("map generation exceeded an internal bound")
        if bits & N.APG_ERR_NO_FREE_CELL:  # numpy's integers(0, 0) in reset (lidar_localization2d.py:302-303)
            raise ValueError("high <= 0")
        if bits & N.APG_ERR_PREFETCH:
            raise N.ApgError("an autoreset found no prefetched map (prefetch protocol violated)")

    def check_errors(self, block: bool = True):
        """Raise the reference's exception for any error flagged by the kernels so far."""
        if block:
            import torch

            torch.cuda.synchronize(self.device)
            bits = int(self._t["err"].item())
        elif self._err_pending and self._err_event.query():
            bits = int(self._err_host.item())
            self._err_pending = False
        else:
            return
        if bits:
            self._t["err"].zero_()
            self._raise_error_bits(bits)

    def _post_launch_error_copy(self):
        """Lazy error reporting: every ERROR_POLL_INTERVAL steps copy the device error word to pinned
        host memory (async) and raise once that copy has landed; strict mode checks every step."""
        if self.strict_errors:
            self.check_errors(block=True)
            return
        self._steps_since_poll += 1
        if self._err_pending or self._steps_since_poll < self.ERROR_POLL_INTERVAL:
            return
        self._steps_since_poll = 0
        self._err_host.copy_(self._t["err"], non_blocking=True)
        self._err_event.record()
        self._err_pending = True

    # ------------------------------------------------------------------ API
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        if self._closed:
            raise RuntimeError("environment is closed")
        if seed is None and not self._seeded:
            seed = int(np.random.SeedSequence().entropy) & ((1 << 62) - 1)
        use_seed = seed is not None
        if use_seed and not isinstance(seed, (int, np.integer)):
            raise TypeError("seed must be an int (sub-env i is seeded with seed + i) or None")
        s = (int(seed) + self.env_offset) if use_seed else 0
        if s < 0 or s + self.num_envs > 2**64:
            raise ValueError("seed must be a non-negative int")
        if self._streamer is not None:
            self._streamer.before_reset(self, s, use_seed)
        self._ops.lidar_reset(self._h, s if s < 2**63 else s - 2**64, bool(use_seed))
        if self._streamer is not None:
            self._streamer.after_reset(self)
        self._track_render(None)
        self._seeded = True
        self._autoreset_host[:] = False
        if self.sparse and not self.sparse_reset_info:
            # SparsifyWrapper.reset (sparsify_wrapper.py:128-135) reads info["prediction"], which
            # LIDARLocalization2DEnv.reset never returns (lidar_localization2d.py:315)
            raise KeyError("prediction")
        T = self._t
        if self.array_backend == "numpy":
            self.check_errors(block=True)
            R = self._host_rows()
            return self._to_numpy_obs(R, None), {"map_idx": R["map_idx_out"].astype(np.int64),
                                                 "_map_idx": np.ones(self.num_envs, dtype=bool)}
        self._post_launch_error_copy()
        return self._obs_out(), {"map_idx": T["map_idx_out"], "_map_idx": T["reset_mask"]}

    def step(self, action):
        import torch

        if self._closed:
            raise RuntimeError("environment is closed")
        a, p = action["action"], action["prediction"]
        numpy_mode = self.array_backend == "numpy"
        if numpy_mode:
            if isinstance(a, torch.Tensor):
                a = a.detach().cpu().numpy()
            if isinstance(p, torch.Tensor):
                p = p.detach().cpu().numpy()
            a_np = np.ascontiguousarray(a, dtype=np.float32).reshape(self.num_envs, 2)
            p_np = np.ascontiguousarray(p, dtype=np.float32).reshape(self.num_envs, 2)
            # one summing pass per input finds that no NaN is present (a NaN or an inf makes the sum non-finite);
            # only then the per-env check, which raises for the first offending active sub-env, action first
            if not (np.isfinite(a_np.sum(dtype=np.float64)) and np.isfinite(p_np.sum(dtype=np.float64))):
                active = ~self._autoreset_host
                bad_a = np.isnan(a_np).view(np.uint16).reshape(-1) != 0
                bad_p = np.isnan(p_np).view(np.uint16).reshape(-1) != 0
                bad_a &= active
                bad_p &= active
                if bad_a.any() or bad_p.any():
                    i = int(np.argmax(bad_a | bad_p))
                    raise ValueError(NAN_ACTION_MSG if bad_a[i] else NAN_PREDICTION_MSG)
            # one H2D copy of both inputs from a pinned staging buffer (the previous step synchronized, so neither
            # the staging buffer nor the device copy is still in use)
            if self._in_host is None:
                self._in_host = torch.empty((2, self.num_envs, 2), dtype=torch.float32).pin_memory()
                self._in_dev = torch.empty((2, self.num_envs, 2), dtype=torch.float32, device=self.device)
            staged = self._in_host.numpy()
            staged[0] = a_np
            staged[1] = p_np
            self._in_dev.copy_(self._in_host, non_blocking=True)
            a_t, p_t = self._in_dev[0], self._in_dev[1]
        else:
            self.check_errors(block=False)
            a_t = N.as_device_f32(a, self._dev, 2 * self.num_envs, name="action")
            p_t = N.as_device_f32(p, self._dev, 2 * self.num_envs, name="prediction")
        if self._streamer is not None:
            self._streamer.before_step()
        if self._kernel_events is None:
            self._launch_step(a_t, p_t)
        else:  # bench timing: hipEvents on the op's stream around the step launch(es)
            ev_b, ev_e = self._kernel_events
            s = self._stream()
            N.event_record(ev_b, s)
            self._launch_step(a_t, p_t)
            N.event_record(ev_e, s)
        if self._streamer is not None:
            self._streamer.after_step(self, N.ptr(self._t["reset_mask"]))
        self._track_render(p_t)
        if numpy_mode:
            return self._numpy_step_result()
        self._post_launch_error_copy()
        T = self._t
        mask = T["info_mask"]
        c = (lambda x: x.clone()) if self.copy else (lambda x: x)
        target = c(T["target"])
        if self.sparse:  # SyncVectorEnv merge of the sub-envs' {"target", "weight": float}
            target = {"target": target, "_target": c(mask), "weight": c(T["weight"]), "_weight": c(mask)}
        info = {"base_reward": c(T["base_reward"]), "_base_reward": c(mask),
                "prediction": {"target": target, "_target": c(mask), "loss": c(T["loss"]),
                               "_loss": c(mask)},
                "_prediction": c(mask),
                "map_idx": c(T["map_idx_out"]), "_map_idx": c(T["reset_mask"])}
        if self.log_stats:
            info.update(self._torch_stats(c))
        return self._obs_out(), c(T["reward"]), c(T["terminated"]), c(T["truncated"]), info

    # ------------------------------------------------------------------ episode statistics
    STAT_NAMES = ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse")

    def _torch_stats(self, c):
        """Device form of info["stats"]: scalars valid where `_stats` (= terminated: every episode of
        these envs ends by termination, TimeLimit(issue_termination=True)); "vector" holds the
        per-step history [N, max_episode_steps] of each metric with its valid length.  Built once
        from persistent buffers (no per-step device work)."""
        if self._stats_view is None:
            T = self._t
            done = T["terminated"]
            scalar = {}
            for j, name in enumerate(self.STAT_NAMES):
                scalar[name] = T["stats"][j]
                scalar["_" + name] = done
            vector = {"euclidean_distance": T["stats_hist"][0].T, "_euclidean_distance": done,
                      "mse": T["stats_hist"][1].T, "_mse": done, "length": T["stats_len"]}  # [N, steps] views
            self._stats_view = {"stats": {"scalar": scalar, "_scalar": done, "vector": vector, "_vector": done},
                                "_stats": done}
        if not self.copy:
            return self._stats_view

        def clone(d):
            return {k: clone(v) if isinstance(v, dict) else v.clone() for k, v in d.items()}

        return clone(self._stats_view)

    def _numpy_stats(self, info: dict, R: dict):
        """SyncVectorEnv's merge of the sub-envs' ActiveRegressionLogWrapper stats (util.py:18-37):
        python-float scalars -> float64 arrays, lists -> object arrays, `_key` masks."""
        T = self._t
        lens = R["stats_len"].copy()
        done = lens > 0
        if not done.any():
            return
        st = R["stats"]
        idx = np.nonzero(done)[0]
        hist = T["stats_hist"][:, :, torch_index(idx, self.device)].permute(2, 0, 1).cpu().numpy()  # [k, 2, steps]
        scalar: dict[str, Any] = {}
        for j, name in enumerate(self.STAT_NAMES):
            scalar[name] = np.where(done, st[j].astype(np.float64), 0.0)
            scalar["_" + name] = done.copy()
        vector: dict[str, Any] = {}
        ln = lens[idx].tolist()
        for m, name in enumerate(("euclidean_distance", "mse")):
            arr = np.full(self.num_envs, None, dtype=object)
            hm = hist[:, m, :]
            if self.vector_stats == "array":  # float32 views of one host block (opt-in: ndarray, not list)
                rows = [r[:n] for r, n in zip(hm, ln)]
            else:  # the reference's list of np.float32 (ActiveRegressionLogWrapper's deque -> list(v)):
                # one np.float32 object per logged value, ~50 ns each, is what an episode end costs
                rows = [list(r[:n]) for r, n in zip(hm, ln)]
            for i, r in zip(idx.tolist(), rows):
                arr[i] = r
            vector[name] = arr
            vector["_" + name] = done.copy()
        info["stats"] = {"scalar": scalar, "_scalar": done.copy(), "vector": vector, "_vector": done.copy()}
        info["_stats"] = done.copy()

    # ------------------------------------------------------------------ output assembly
    def _obs_out(self):
        T = self._t
        c = (lambda x: x.clone()) if self.copy else (lambda x: x)
        obs = {"lidar": c(T["lidar"]), "odometry": c(T["odometry"])}
        if not self.static_map:
            obs["map"] = c(T["map_obs"])
        obs["time_step"] = c(T["time_step"])
        return obs

    HOST_RING = 4  # numpy backend, copy=True: pinned output blocks handed out as the returned arrays

    def _host_block(self):
        """A pinned host block for this step's outputs.  copy=True: a small ring of blocks whose field views ARE the
        returned arrays (no per-field host copies); a block is reused only once no array of an earlier step still
        refers to it (its numpy base has no outside references), else another block is pinned, up to HOST_RING;
        past that (or with copy=False) the outputs land in a private block that is never handed out and the step
        copies its fields from it (self._ring_copy)."""
        import sys

        import torch

        src = self.output_rows if self._out_block is None else self._out_block
        if self.copy:
            for blk in self._ring:
                if sys.getrefcount(blk[1]) <= 2:  # the ring tuple and the call argument: no returned view is alive
                    self._ring_copy = False
                    return blk
            if len(self._ring) < self.HOST_RING:
                t = torch.empty(tuple(src.shape), dtype=torch.uint8).pin_memory()
                self._ring.append((t, t.numpy()))
                self._ring_copy = False
                return self._ring[-1]
        self._ring_copy = True
        if self._rows_host is None:  # the private block
            self._rows_host = torch.empty(tuple(src.shape), dtype=torch.uint8).pin_memory()
            self._rows_np = self._rows_host.numpy()
        return self._rows_host, self._rows_np

    def _host_rows(self) -> dict:
        """numpy backend: the output block (or the packed output rows) and the error word copied D2H into a pinned
        host block in one go, then one synchronize; returns fresh numpy field views of that block (copy=True: the
        block is not written again while any of them is alive, see _host_block)."""
        import torch

        src = self.output_rows if self._out_block is None else self._out_block
        blk_t, blk_np = self._host_block()
        blk_t.copy_(src, non_blocking=True)
        self._err_host.copy_(self._t["err"], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        self._err_pending = False
        return (row_views_np(blk_np, self.output_layout) if self._out_block is None
                else block_views(blk_np, self._block_layout))

    def _own(self, a: np.ndarray) -> np.ndarray:
        """A returned output field: the block view itself, or a copy where the block is shared (copy=False keeps
        the aliasing mirror semantics; a full ring falls back to copies)."""
        return a.copy() if self._ring_copy else a

    MAP_COPIES = 3  # obs_snapshot="copy": host blocks kept for reuse once no returned obs["map"] refers to them

    def _map_refresh(self, reset_mask: np.ndarray | None):
        """The host mirror of the map observation, refreshed only for the sub-envs that reset (the map obs
        changes only then); None refreshes every sub-env.  copy=False: the mirror itself.  copy=True: the caller's
        own copy of it, like SyncVectorEnv(copy=True)'s deepcopy -- a block no earlier returned array refers to any
        more (sys.getrefcount), rewritten whole from the mirror on torch's intra-op threads, or
        (obs_snapshot="shared") one read-only snapshot of the mirror taken again only when the mirror changed."""
        import sys

        import torch

        if self.static_map:
            return None
        T = self._t
        if self._map_host is None:
            self._map_host = torch.empty(tuple(T["map_obs"].shape), dtype=torch.float32).pin_memory()
            reset_mask = None
        changed = reset_mask is None or bool(reset_mask.any())
        if reset_mask is None or reset_mask.all():
            self._map_host.copy_(T["map_obs"])
        elif changed:
            idx = np.nonzero(reset_mask)[0]
            self._map_host.numpy()[idx] = T["map_obs"][torch_index(idx, self.device)].cpu().numpy()
        m = self._map_host.numpy()
        if not self.copy:
            return m
        if self.obs_snapshot == "copy":
            blk = None
            for b in self._map_copies:
                if sys.getrefcount(b[1]) <= 2:  # the list's tuple and the call argument: no returned array is alive
                    blk = b
                    break
            if blk is None:
                t = torch.empty(tuple(self._map_host.shape), dtype=torch.float32)
                blk = (t, t.numpy())
                if len(self._map_copies) < self.MAP_COPIES:
                    self._map_copies.append(blk)
            blk[0].copy_(self._map_host)  # whole: the caller may have written into an earlier hand-out of it
            return blk[1]
        if changed or self._map_snapshot is None:
            # torch's CPU copy runs on the intra-op thread pool (numpy's m.copy() is one thread: 3-4x slower at
            # the 1 GB of a cfg-2 episode end)
            self._map_snapshot = self._map_host.clone().numpy()
            self._map_snapshot.flags.writeable = False
        return self._map_snapshot

    def _to_numpy_obs(self, R: dict | None = None, reset_mask: np.ndarray | None = None):
        if R is None:
            R = self._host_rows()
        obs = {"lidar": self._own(R["lidar"]), "odometry": self._own(R["odometry"])}
        if not self.static_map:
            obs["map"] = self._map_refresh(reset_mask)
        obs["time_step"] = self._own(R["time_step"])
        return obs

    def _numpy_step_result(self):
        R = self._host_rows()  # every per-env output in one D2H copy + one synchronize
        bits = int(self._err_host[0])
        if bits:
            self._t["err"].zero_()
            self._raise_error_bits(bits)
        reset_mask = R["reset_mask"].copy()
        obs = self._to_numpy_obs(R, reset_mask)
        reward = self._own(R["reward"])
        term = self._own(R["terminated"])
        trunc = self._own(R["truncated"])
        mask = R["info_mask"].copy()
        info: dict[str, Any] = {}
        if mask.any():
            full = bool(mask.all())

            def masked(a):  # np.where(mask, a, 0) along the env axis: the field itself when every env reports
                if full:
                    return self._own(a)
                out = a.copy()  # (a copy plus a masked store: np.where broadcasting the [N, 2] target costs ~10x)
                out[~mask] = 0
                return out

            info["base_reward"] = masked(R["base_reward"])
            info["_base_reward"] = mask.copy()
            tgt = masked(R["target"])
            loss = masked(R["loss"])
            if self.sparse:
                tgt = {"target": tgt, "_target": mask.copy(), "weight": masked(R["weight"]), "_weight": mask.copy()}
            info["prediction"] = {"target": tgt, "_target": mask.copy(), "loss": loss, "_loss": mask.copy()}
            info["_prediction"] = mask.copy()
        if self.log_stats:
            self._numpy_stats(info, R)
        if reset_mask.any():
            info["map_idx"] = np.where(reset_mask, R["map_idx_out"], 0).astype(np.int64)
            info["_map_idx"] = reset_mask
        self._autoreset_host = term | trunc
        return obs, reward, term, trunc, info

    def prefetch_stats(self) -> dict | None:
        """Counters of the map prefetcher (None without one): batches launched, steps whose stream waited for a
        batch still running, resets observed, step calls since the last reset."""
        if not self._prefetcher:
            return None
        v = (ctypes.c_int64 * 4)()
        N.check(N.lib().apg_lidar_prefetcher_stats(self._prefetcher, v), "apg_lidar_prefetcher_stats")
        return dict(zip(("batches", "waits", "resets", "steps"), list(v)))

    def close(self, **kwargs):
        if not getattr(self, "_closed", True):
            self._closed = True
            self.closed = True
            if getattr(self, "_prefetcher", None):
                N.lib().apg_lidar_prefetcher_destroy(self._prefetcher)  # synchronizes its side stream
                self._prefetcher = None
            if getattr(self, "_streamer", None) is not None:
                self._streamer.close()
                self._streamer = None
            self._t = {}
            self._h = None  # the op handle keeps every state/output buffer alive
            self._c_args = None
            self.output_rows = self._out_block = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def __repr__(self):
        kind = ("maze" if isinstance(self.dataset, FloorMapDatasetMaze) else
                "rooms" if isinstance(self.dataset, FloorMapDatasetRooms) else f"pool[{len(self.dataset)}]")
        return (f"LIDARLocalization2DVectorEnv(num_envs={self.num_envs}, {kind} "
                f"{self.dataset.map_width}x{self.dataset.map_height}, static={self.static_map}, "
                f"beams={self.lidar_beam_count}, device={self.device})")
