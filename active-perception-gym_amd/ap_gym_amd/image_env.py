"""Image glimpse envs on the GPU: ImageClassificationVectorEnv and ImageLocalizationVectorEnv.

Reference (ap_gym 0.5.0): ap_gym/envs/image_classification.py:22-167,
ap_gym/envs/image_localization.py:24-256 over ImagePerceptionModule
(ap_gym/envs/image/image_perception_module.py:20-477), built by `make_vec("MNIST-v0", N)` and the
other image ids (registration.py:145-192, 516-627).  Same constructor
(num_envs, image_perception_config, render_mode), spaces, reset/step semantics and dtypes; the
dataset is held in HBM as one pool and every per-step array op (glimpse gather, losses, move,
rewards) and every vector-level numpy draw (DatasetBatchIterator, the module's and the env's
generators) runs on the device through the C ABI (include/apgym_capi.h: apg_image_*).

  obs     {"glimpse": f32[N,G0,G1,C], "glimpse_pos": f32[N,2], "time_step": f32[N],
           ("inverted_label": i32/i64[N]), ("target_glimpse": f32[N,G0,G1,C] localization)}
  reward  base_reward - normalized loss (CE: float64; MSE: float32, float64 on autoreset steps)
  info    {"index": i64[N], "base_reward", "prediction": {"target", "loss"}}
  episode all envs terminate together after step_limit steps; the next step resets the batch
          (NEXT_STEP autoreset inside the module, base_reward = zeros(N) float64)

array_backend="numpy" (default) returns numpy exactly like the reference: every step's arrays are the caller's own
(writable, never written again by the env), obs["target_glimpse"] included (the reference computes it anew every step,
image_localization.py:142-146, 170-174); obs_snapshot="shared" (opt-in) hands out the target glimpse as one read-only
array shared by the steps of a batch instead (it changes only with the batch).  "torch" returns persistent device
tensors without host synchronisation (errors raised lazily, like the LIDAR env).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Any, Sequence

import numpy as np

from . import _native as N
from .image_dataset import ImageClassificationDataset, as_pool_dataset
from .loss_fn import CrossEntropyLossFn, WeightedLossFn, affine_f32, regression_loss
from .spaces import ActivePerceptionActionSpace, Box, Dict, Discrete, ImageSpace, LogitSpace, MultiDiscrete, batch_space
from .vector_env import VectorEnv

NAN_ACTION_MSG = "NaN values detected in action."
NAN_PREDICTION_MSG = "NaN values detected in prediction."
OOB_MSG = "One of the requested xi is out of bounds in dimension %d"


@dataclass(frozen=True)
class ImagePerceptionConfig:
    """image_perception_module.py:20-34 (same fields and defaults)."""

    dataset: ImageClassificationDataset
    sensor_size: tuple[int, int] = (5, 5)
    sensor_scale: float = 1.0
    max_step_length: float | Sequence[float] = 0.2
    step_limit: int = 16
    display_visitation: bool = True
    render_unvisited_opacity: float = 0.0
    render_visited_opacity: float = 0.3
    prefetch_buffer_size: int = 128
    prefetch: bool = True
    unique_sampling_max_grid_cell_size_rel = 0.2  # class attribute in the reference too
    unique_sampling_top_k: int = 10
    randomly_invert_labels: bool = False


def sensor_pos_lim_pixels(image_hw, sensor_size, sensor_scale) -> np.ndarray:
    """image_perception_module.py:419-423, evaluated with numpy like the reference."""
    eff = np.array(sensor_size) * sensor_scale
    return (np.flip(np.array(image_hw)) - 1) / 2 - (eff - 1) / 2


def unique_sampling_grid(image_hw, sensor_size, sensor_scale, rel=0.2):
    """Sampling positions and cell size of sample_unique_glimpse_positions (:254-267)."""
    eff = np.array(sensor_size) * sensor_scale
    cell = (eff / sensor_pos_lim_pixels(image_hw, sensor_size, sensor_scale)) * rel
    cnt = np.ceil(2 / cell)
    grid = np.stack(np.meshgrid(np.linspace(-1, 1, int(cnt[0])), np.linspace(-1, 1, int(cnt[1])), indexing="ij"),
                    axis=-1).reshape(-1, 2)
    return np.ascontiguousarray(grid), cell


def device_pool_u8(pool: np.ndarray, dev):
    """A uint8 image pool on `dev` with N.APG_U8_POOL_PAD readable bytes after the last image (the glimpse kernels
    read taps with whole-dword loads, apgym_capi.h); the returned tensor is the [M, H, W, C] view."""
    import torch

    nb = pool.nbytes
    buf = torch.zeros(nb + N.APG_U8_POOL_PAD, dtype=torch.uint8, device=dev)
    buf[:nb].copy_(torch.from_numpy(np.ascontiguousarray(pool).reshape(-1)))
    return buf[:nb].view(pool.shape)


def tiled_pool_bytes(h: int, w: int) -> int:
    """Bytes of one image of an APG_POOL_U8_TILED pool (apgym_capi.h): ceil(H/4) x ceil(W/8) tiles of 128 bytes."""
    return ((h + 3) // 4) * ((w + 7) // 8) * 128


def use_tiled_pools() -> bool:
    """RGB u8 pools go to the device as RGBX 8 x 4-pixel tiles (APG_POOL_U8_TILED) unless APG_IMAGE_TILED=0 (A/B)."""
    import os

    return os.environ.get("APG_IMAGE_TILED", "1") != "0"


def device_pool_u8_tiled(pool: np.ndarray, dev, chunk: int = 4096):
    """An RGB uint8 pool [M, H, W, 3] laid out on `dev` as APG_POOL_U8_TILED: pixel (y, x) of image m at byte
    m * img + (y // 4) * ceil(W/8) * 128 + (x // 8) * 128 + (y % 4) * 32 + (x % 8) * 4 + channel (the 4th byte 0),
    re-tiled on the device in chunks of images; N.APG_U8_POOL_PAD spare bytes after the last image.  Returned as the
    flat byte tensor of the M images (the kernels address it through apg_image_config.pool_dtype)."""
    import torch

    m, h, w, c = pool.shape
    assert c == 3 and pool.dtype == np.uint8
    th, tw = (h + 3) // 4, (w + 7) // 8
    img = th * tw * 128
    buf = torch.zeros(m * img + N.APG_U8_POOL_PAD, dtype=torch.uint8, device=dev)
    for lo in range(0, m, chunk):
        hi = min(m, lo + chunk)
        src = torch.from_numpy(np.ascontiguousarray(pool[lo:hi])).to(dev)
        padded = torch.zeros((hi - lo, th * 4, tw * 8, 4), dtype=torch.uint8, device=dev)
        padded[:, :h, :w, :3] = src
        tiles = padded.view(hi - lo, th, 4, tw, 8, 4).permute(0, 1, 3, 2, 4, 5).reshape(-1)
        buf[lo * img:hi * img].copy_(tiles)
    return buf[:m * img]


def padded_device_pool_u8(pool_t):
    """A device uint8 pool (e.g. from a dataset's device_pool_tensors) as the glimpse kernels need it: contiguous with
    N.APG_U8_POOL_PAD readable bytes after the last image in its own allocation (apgym_capi.h).  The tensor itself
    when its storage already extends that far, else a padded copy."""
    import torch

    nb = pool_t.numel()
    if (pool_t.is_contiguous() and
            pool_t.untyped_storage().nbytes() - pool_t.storage_offset() >= nb + N.APG_U8_POOL_PAD):
        return pool_t
    buf = torch.zeros(nb + N.APG_U8_POOL_PAD, dtype=torch.uint8, device=pool_t.device)
    buf[:nb].copy_(pool_t.reshape(-1))
    return buf[:nb].view(tuple(pool_t.shape))


def softmax_nan_rows(logits: np.ndarray) -> np.ndarray:
    """Rows where scipy.special.softmax(row)[label] is NaN: a NaN or +inf logit, or all -inf."""
    return np.isnan(logits).any(-1) | np.isposinf(logits).any(-1) | np.isneginf(logits).all(-1)


# Packed output rows (apg_image_config.out_row_bytes): every per-env output of a step in one row per env, 8-byte
# fields first, so ShardedVectorEnv all-gathers the [N, row] buffer as is (no packing copies) and the gathered fields
# are strided views of the receive buffer.  Names are the env's output buffer names.
def image_output_row_layout(kind: int, sensor: tuple, channels: int, log_stats: bool = False):
    """[(name, torch dtype, per-env shape, byte offset)] of the packed output row, and the row size."""
    import torch

    f64, f32, i32 = torch.float64, torch.float32, torch.int32
    g = (int(sensor[0]), int(sensor[1]), int(channels))
    cls = kind == N.APG_IMAGE_CLASSIFY
    # (the localization target glimpse is not in the row: it changes only with the batch, so a sharded run
    # gathers it on reset / autoreset steps only)
    fields = [("reward", f64, ())] + ([("loss_f64", f64, ())] if cls else []) + [("glimpse", f32, g)] + [
        ("glimpse_pos", f32, (2,)), ("time_step", f32, ()), ("base_reward", f32, ())] + (
        [("label_target", i32, ())] if cls else [("target_out", f32, (2,)), ("loss_f32", f32, ())]) + (
        [("stats", f32, (4,))] if log_stats else []) + ([("stats_idx", i32, (2,))] if log_stats and cls else [])
    out, off = [], 0
    for name, dt, sh in fields:
        out.append((name, dt, sh, off))
        off += torch.empty((), dtype=dt).element_size() * int(np.prod(sh, dtype=np.int64))
    return out, off + (-off) % 8


def image_row_views(buf, layout) -> dict:
    """Field views of a packed [rows, row_bytes] uint8 buffer (stats / stats_idx as [M, rows] like the dense
    layout)."""
    import torch

    v = {}
    for name, dt, sh, off in layout:
        nb = torch.empty((), dtype=dt).element_size() * int(np.prod(sh, dtype=np.int64))
        t = buf[:, off:off + nb].view(dt)
        t = t[:, 0] if not sh else t.view(buf.shape[0], *sh)
        v[name] = t.T if name in ("stats", "stats_idx") else t
    return v


class _ImageVectorEnv(VectorEnv):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 2, "autoreset_mode": "NextStep"}
    ERROR_POLL_INTERVAL = 128  # steps between the lazy error-word copies (each costs the stream a blit + marker)
    kind: int

    def __init__(self, num_envs: int, image_perception_config: ImagePerceptionConfig,
                 render_mode: str = "rgb_array", device=None, copy: bool = False, strict_errors: bool = False,
                 array_backend: str = "numpy", num_envs_total: int | None = None, env_offset: int = 0,
                 log_stats: bool = False, sparse: bool = False, render_envs=None, packed_outputs: bool = False,
                 draw_ahead: bool = True, vector_stats: str = "list", obs_snapshot: str = "copy"):
        import torch

        if render_mode not in self.metadata["render_modes"]:
            raise ValueError(f"Unsupported render mode: {render_mode}")
        if array_backend not in ("numpy", "torch"):
            raise ValueError("array_backend must be 'numpy' or 'torch'")
        if vector_stats not in ("list", "array"):
            raise ValueError("vector_stats must be 'list' (the reference's lists of np.float32) or 'array'")
        self.vector_stats = vector_stats  # numpy backend: form of info["stats"]["vector"] entries (as the LIDAR env)
        if obs_snapshot not in ("copy", "shared"):
            raise ValueError("obs_snapshot must be 'copy' (a writable target glimpse per step) or 'shared'")
        self.obs_snapshot = obs_snapshot  # numpy backend: obs["target_glimpse"] per step or a shared snapshot
        cfg = image_perception_config
        self.config = cfg
        self.num_envs = n = int(num_envs)
        # sharding (ap_gym_amd.sharding): this env is envs [env_offset, env_offset + num_envs) of a batch
        # of num_envs_total; every rank draws the whole batch from the same streams and keeps its slice
        self.num_envs_total = nt = int(num_envs_total) if num_envs_total is not None else n
        self.env_offset = int(env_offset)
        if self.env_offset < 0 or self.env_offset + n > nt:
            raise ValueError("the shard [env_offset, env_offset + num_envs) must lie inside num_envs_total")
        self.render_mode = render_mode
        self.copy, self.strict_errors, self.array_backend = copy, strict_errors, array_backend
        if packed_outputs and array_backend != "torch":
            raise ValueError("packed_outputs (the all-gather row layout) needs array_backend='torch'")
        # the registered ids wrap the env in ActiveClassificationVectorLogWrapper /
        # ActiveRegressionVectorLogWrapper (registration.py:185-192, 263-269): info["stats"]
        self.log_stats = bool(log_stats)
        # the "-sparse" ids wrap that in SparsifyVectorWrapper (sparsify_wrapper.py:23-92): target
        # {"target", "weight" = terminated as float32}, reward = base_reward - loss * weight
        self.sparse = bool(sparse)
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("the image envs run on a GPU device (no CPU fallback)")
        ds = as_pool_dataset(cfg.dataset)
        ds.load()
        if hasattr(ds, "device_pool_tensors"):  # procedural datasets render their pool on the device
            pool_t, labels_t = ds.device_pool_tensors(self.device)
            pool, pool_tiled = None, False
            pool_is_u8 = pool_t.dtype == torch.uint8
            if pool_is_u8:  # the kernels' dword tap loads read up to APG_U8_POOL_PAD - 1 bytes past the last image
                pool_t = padded_device_pool_u8(pool_t)
        else:
            # one upload per dataset and device, shared by every env built on it (ShardedVectorEnv's sub-batches, a
            # train and an eval env): the pool is read-only on the device
            cache = ds.__dict__.setdefault("_apg_device_pools", {}) if hasattr(ds, "__dict__") else {}
            key = (str(self.device), use_tiled_pools())
            if key not in cache:
                pool, labels = ds.device_pool()
                tiled = key[1] and pool.dtype == np.uint8 and pool.shape[-1] == 3
                cache[key] = (device_pool_u8_tiled(pool, self.device) if tiled else
                              device_pool_u8(pool, self.device) if pool.dtype == np.uint8
                              else torch.from_numpy(np.ascontiguousarray(pool)).to(self.device),
                              torch.from_numpy(np.ascontiguousarray(labels)).to(self.device), pool, tiled)
            pool_t, labels_t, pool, pool_tiled = cache[key]
            pool_is_u8 = pool_t.dtype == torch.uint8
        m, h, w, pc = pool.shape if pool_tiled else pool_t.shape
        c = int(ds.num_channels)
        if c not in (1, 3):
            raise ValueError(f"Target channels must be either 1 or 3 but is {c}.")
        if pc != c and not (pc == 1 and c == 3):
            raise ValueError(f"Invalid image format. Expected {c} channels but got {pc}")
        s0, s1 = (int(v) for v in cfg.sensor_size)
        eff = np.array(cfg.sensor_size) * cfg.sensor_scale
        if np.any(np.array([h, w]) < eff):
            raise ValueError(f"Image size {(h, w)} cannot be smaller than effective sensor size {tuple(eff)}.")
        self.image_size = (h, w)
        k = int(ds.num_classes)
        self._k = k

        # ---- spaces (image_perception_module.py:51-91, image_classification.py:86-103,
        #      image_localization.py:86-118, active_{classification,regression}_env.py)
        obs = {"glimpse": ImageSpace(s1, s0, c), "glimpse_pos": Box(-1, 1, (2,), np.float32),
               "time_step": Box(-1, 1, (), np.float32)}
        if cfg.randomly_invert_labels:
            obs["inverted_label"] = Discrete(3)
        if self.kind == N.APG_IMAGE_LOCALIZE:
            obs["target_glimpse"] = ImageSpace(s1, s0, c)
            pred_space = Box(-1, 1, (2,), np.float32)
            self.single_prediction_target_space = Box(-1, 1, (2,), np.float32)
            self.prediction_target_space = batch_space(self.single_prediction_target_space, n)
            self.loss_fn = regression_loss(2, -1, 1)
        else:
            pred_space = LogitSpace(-np.inf, np.inf, (k,), np.float32)
            self.single_prediction_target_space = Discrete(k)
            self.prediction_target_space = MultiDiscrete([k] * n)
            self.loss_fn = CrossEntropyLossFn(num_classes=k).normalized
        inner_loss = self.loss_fn
        if self.sparse:
            self.single_prediction_target_space = Dict({"target": self.single_prediction_target_space,
                                                        "weight": Box(0, 1, (), np.float32)})
            self.prediction_target_space = batch_space(self.single_prediction_target_space, n)
            self.loss_fn = WeightedLossFn(inner_loss)
        self.single_observation_space = Dict(obs)
        self.observation_space = batch_space(self.single_observation_space, n)
        self.single_action_space = ActivePerceptionActionSpace(Box(-1, 1, (2,), np.float32), pred_space)
        self.action_space = batch_space(self.single_action_space, n)

        # ---- native configuration
        grid, cell = unique_sampling_grid((h, w), cfg.sensor_size, cfg.sensor_scale,
                                          cfg.unique_sampling_max_grid_cell_size_rel)
        msl = np.ones(2) * np.array(cfg.max_step_length)
        if self.kind == N.APG_IMAGE_CLASSIFY:
            ce = inner_loss
            ce_scale, ce_offset = float(ce.scale), float(ce.offset)
            mse_scale, mse_offset = 1.0, 0.0
        else:
            ce_scale, ce_offset = 1.0, 0.0
            mse_scale, mse_offset = affine_f32(inner_loss)
        self._cfg = N.ImageConfig(
            num_envs=n, kind=self.kind, height=h, width=w, pool_channels=pc, channels=c,
            pool_dtype=(N.APG_POOL_U8_TILED if pool_tiled else N.APG_POOL_U8 if pool_is_u8 else N.APG_POOL_F32),
            sensor_h=s0, sensor_w=s1,
            step_limit=int(cfg.step_limit), num_classes=k, invert_labels=int(bool(cfg.randomly_invert_labels)),
            top_k=int(cfg.unique_sampling_top_k), unique_points=int(grid.shape[0]), num_envs_total=nt,
            env_offset=self.env_offset, pool_len=m,
            sensor_scale=float(cfg.sensor_scale), max_step=(ctypes.c_double * 2)(*msl.tolist()),
            cell=(ctypes.c_double * 2)(*cell.tolist()), ce_scale=ce_scale, ce_offset=ce_offset,
            mse_scale=mse_scale, mse_offset=mse_offset, log_stats=int(self.log_stats), sparse=int(self.sparse))
        self.output_layout, row_bytes = image_output_row_layout(self.kind, cfg.sensor_size, c, self.log_stats)
        if not packed_outputs:
            self.output_layout, row_bytes = None, 0
        self._cfg.out_row_bytes = row_bytes

        t, dev = torch, self.device
        gshape = (n, s0, s1, c)
        work = max(N.lib().apg_rng_fill_work_elems(nt, b) for b in (m, int(cfg.unique_sampling_top_k), 2))
        self._t = T = dict(
            pool=pool_t, pool_labels=labels_t,
            unique_grid=t.from_numpy(grid).to(dev),
            index=t.zeros(n, dtype=t.int64, device=dev), label=t.zeros(n, dtype=t.int32, device=dev),
            inverted=t.zeros(n, dtype=t.int32, device=dev), pos=t.zeros((n, 2), dtype=t.float64, device=dev),
            target=t.zeros((n, 2), dtype=t.float32, device=dev), rng=t.zeros((3, 5), dtype=t.int64, device=dev),
            scratch_i64=t.zeros(2 * nt, dtype=t.int64, device=dev),
            scratch_f64=t.zeros(2 * nt, dtype=t.float64, device=dev),
            top_k=t.zeros((n, int(cfg.unique_sampling_top_k)), dtype=t.int32, device=dev),
            rng_work=t.zeros(work, dtype=t.int64, device=dev),
            glimpse=t.zeros(gshape, dtype=t.float32, device=dev),
            glimpse_pos=t.zeros((n, 2), dtype=t.float32, device=dev),
            time_step=t.zeros(n, dtype=t.float32, device=dev),
            target_glimpse=t.zeros(gshape, dtype=t.float32, device=dev) if self.kind == N.APG_IMAGE_LOCALIZE else None,
            reward=t.zeros(n, dtype=t.float64, device=dev), base_reward=t.zeros(n, dtype=t.float32, device=dev),
            target_out=t.zeros((n, 2), dtype=t.float32, device=dev),
            label_target=t.zeros(n, dtype=t.int32, device=dev),
            loss_f64=t.zeros(n, dtype=t.float64, device=dev), loss_f32=t.zeros(n, dtype=t.float32, device=dev),
            err=t.zeros(1, dtype=t.int32, device=dev),
            stats_hist=(t.zeros((n, 2, int(cfg.step_limit)), dtype=t.float32, device=dev) if self.log_stats
                        else None),
            stats=t.zeros((4, n), dtype=t.float32, device=dev) if self.log_stats else None,
            stats_idx=t.zeros((2, n), dtype=t.int32, device=dev) if self.log_stats else None,
            # the next batch autoreset's draws, made ahead on a side stream (apg_image_draw_ahead)
            ahead_i64=t.zeros(2 * nt, dtype=t.int64, device=dev),
            ahead_f64=t.zeros(4 * nt, dtype=t.float64, device=dev),
            rng_saved=t.zeros((3, 5), dtype=t.int64, device=dev))
        # packed_outputs: the per-env outputs are field views of one [n, row] buffer (ShardedVectorEnv's send)
        self.output_rows = None
        if row_bytes:
            self.output_rows = t.zeros((n, row_bytes), dtype=t.uint8, device=dev)
            T.update(image_row_views(self.output_rows, self.output_layout))
        self._state = N.ImageState(*[N.ptr(T[k_]) for k_ in ("pool", "pool_labels", "unique_grid", "index", "label",
                                                              "inverted", "pos", "target", "rng", "scratch_i64",
                                                              "scratch_f64", "top_k", "rng_work", "stats_hist",
                                                              "ahead_i64", "ahead_f64", "rng_saved")])
        self._out = N.ImageOutputs(*[N.ptr(T[k_]) for k_ in ("glimpse", "glimpse_pos", "time_step", "target_glimpse",
                                                              "reward", "base_reward", "target_out", "label_target",
                                                              "loss_f64", "loss_f32", "err", "stats", "stats_idx")])
        c = self._cfg
        self._ops = N.torch_ops()  # torch.ops.apgym: the reset/step hot path
        self._step_op = self._ops.image_step.default  # the overload itself: no per-call overload resolution
        self._dev = N.exact_device(self.device)
        # Eager steps call the C ABI directly (3.8 us of host time per call, against 15 us through the torch
        # dispatcher, which made MNIST host-bound: tools/host_overhead_image.py); use_torch_op = True routes
        # them through torch.ops.apgym.image_step instead.
        self.use_torch_op = False
        self._c_args = None
        self._kernel_events = None
        self._h = t.classes.apgym.ImageEnv(
            [c.num_envs, c.kind, c.height, c.width, c.pool_channels, c.channels, c.pool_dtype, c.sensor_h,
             c.sensor_w, c.step_limit, c.num_classes, c.invert_labels, c.top_k, c.unique_points, c.num_envs_total,
             c.env_offset, c.pool_len, c.log_stats, c.sparse, c.out_row_bytes],
            [c.sensor_scale, c.max_step[0], c.max_step[1], c.cell[0], c.cell[1], c.ce_scale, c.ce_offset,
             c.mse_scale, c.mse_offset],
            N.op_buffers([T[k_] for k_ in ("pool", "pool_labels", "unique_grid", "index", "label", "inverted", "pos",
                                           "target", "rng", "scratch_i64", "scratch_f64", "top_k", "rng_work",
                                           "stats_hist", "ahead_i64", "ahead_f64", "rng_saved")], dev),
            N.op_buffers([T[k_] for k_ in ("glimpse", "glimpse_pos", "time_step", "target_glimpse", "reward",
                                           "base_reward", "target_out", "label_target", "loss_f64", "loss_f32", "err",
                                           "stats", "stats_idx")], dev))
        # The next batch's draws depend only on the module / iterator / env streams, never on actions, so they are
        # made right after each batch reset on a low-priority side stream (the reference draws them inside the
        # autoreset step): that step then installs them in the fused step kernel, one launch instead of five.
        self.draw_ahead = bool(draw_ahead)
        self._ahead_stream = t.cuda.Stream(dev, priority=0) if self.draw_ahead else None
        # stream-ordering events (device-scope release: N.DeviceEvent): the draws made ahead -> the step installing
        # them; the batch autoreset step -> the draws of the next batch
        self._ahead_event = self._main_event = None
        if self.draw_ahead:
            with t.cuda.device(dev):
                self._ahead_event, self._main_event = N.DeviceEvent(), N.DeviceEvent()
        self._ahead_side = self._ahead_stream.cuda_stream if self.draw_ahead else None
        self._ahead = False  # draws made ahead and not yet installed
        self._err_host = t.zeros(1, dtype=t.int32).pin_memory()
        self._err_event = t.cuda.Event()
        self._err_pending = False
        self._steps_since_poll = 0
        self._seeded = False
        self._closed = False
        self._t_step = 0
        self._prev_done = False
        self._done_consts = None
        self._stats_view = None
        # numpy backend: pinned input staging, the device byte block the step outputs are packed into and a ring of
        # pinned host blocks handed out as the returned arrays (_np_block), the target glimpse's host snapshot
        self._in_host = self._in_dev = self._np_dev = None
        self._np_ring, self._np_layout, self._tg_host = [], None, None
        from .render import tracked_envs

        self.render_envs = tracked_envs(render_envs, n)
        self._pool_host = pool  # render: images of the tracked envs (host pools)
        self._visits = [[] for _ in self.render_envs]  # (pre-step position f64 [2], quality) since the reset
        self._last_prediction = None

    # ------------------------------------------------------------------ properties
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

    @property
    def current_labels(self):
        return self._t["label"]

    def _stream(self):
        return N.stream_handle(self.device)

    # ------------------------------------------------------------------ errors
    @staticmethod
    def _raise_error_bits(bits: int):
        if bits & N.APG_ERR_NAN_PREDICTION:
            raise ValueError(NAN_PREDICTION_MSG)
        if bits & N.APG_ERR_NAN_ACTION:
            raise ValueError(NAN_ACTION_MSG)
        if bits & N.APG_ERR_OOB_Y:
            raise ValueError(OOB_MSG % 0)
        if bits & N.APG_ERR_OOB_X:
            raise ValueError(OOB_MSG % 1)

    def check_errors(self, block: bool = True):
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
        L = N.lib()
        if seed is None and not self._seeded:
            seed = int(np.random.SeedSequence().entropy) & ((1 << 63) - 1)
        if seed is not None and (not isinstance(seed, (int, np.integer)) or int(seed) < 0 or int(seed) >= 2**64):
            raise ValueError("seed must be a non-negative int below 2**64")
        if self._ahead:  # the batch is replaced here: the streams go back to before the draws made ahead
            import torch

            self._ahead_event.wait(N.current_stream_ptr(self._dev))
            N.check(L.apg_image_discard_ahead(ctypes.byref(self._cfg), ctypes.byref(self._state), self._stream()),
                    "apg_image_discard_ahead")
            self._ahead = False
        if seed is not None:
            N.check(L.apg_image_seed(ctypes.byref(self._cfg), ctypes.byref(self._state), int(seed), self._stream()),
                    "apg_image_seed")
            self._seeded = True
        self._ops.image_reset(self._h)
        self._launch_draw_ahead()
        self._t_step = 0
        self._prev_done = False
        self._visits = [[] for _ in self.render_envs]  # module.reset clears the overlay (:184-186)
        self._last_prediction = None
        if self.array_backend == "numpy":
            self.check_errors(block=True)
            self._tg_host = None  # (the next step takes a new target-glimpse snapshot)
            return self._numpy_obs(), {"index": self._t["index"].cpu().numpy()}
        self._post_launch_error_copy()
        return self._torch_obs(), {"index": self._c(self._t["index"])}

    def step(self, action):
        import torch

        if self._closed:
            raise RuntimeError("environment is closed")
        a, p = action["action"], action["prediction"]
        n = self.num_envs
        numpy_mode = self.array_backend == "numpy"
        pdim = self._k if self.kind == N.APG_IMAGE_CLASSIFY else 2
        if numpy_mode:
            if isinstance(a, torch.Tensor):
                a = a.detach().cpu().numpy()
            if isinstance(p, torch.Tensor):
                p = p.detach().cpu().numpy()
            a_np = np.ascontiguousarray(a, dtype=np.float32).reshape(n, 2)
            p_np = np.ascontiguousarray(p, dtype=np.float32).reshape(n, pdim)
            # the module checks the prediction quality first, then (if it does not reset) the action.  A finite f64
            # sum rules out every NaN / inf in one pass (|sum| <= 3.4e38 * N stays far below the f64 range); the
            # exact row tests (softmax_nan_rows: ~12 ms at N = 65536, K = 10) run only when it is not finite
            if not np.isfinite(p_np.sum(dtype=np.float64)):
                bad_p = softmax_nan_rows(p_np) if self.kind == N.APG_IMAGE_CLASSIFY else np.isnan(p_np).any(-1)
                if bad_p.any():
                    raise ValueError(NAN_PREDICTION_MSG)
            if not self._prev_done and not np.isfinite(a_np.sum(dtype=np.float64)) and np.isnan(a_np).any():
                raise ValueError(NAN_ACTION_MSG)
            a_t, p_t = self._stage_inputs(a_np, p_np)
        else:
            self.check_errors(block=False)
            a_t = N.as_device_f32(a, self._dev, 2 * n, (n, 2), name="action")
            p_t = N.as_device_f32(p, self._dev, pdim * n, (n, pdim), name="prediction")
        resetting = self._prev_done
        flags = 0
        if resetting:
            flags = 1
            if self._ahead:  # install the draws made ahead (the step's stream waits for the side stream)
                self._ahead_event.wait(N.current_stream_ptr(self._dev))
                flags |= 2
                self._ahead = False
        self._track_render(p_np if numpy_mode else p_t, resetting)
        ev = self._kernel_events
        if ev is not None:  # bench timing: hipEvents on the launch stream right around the step's launches
            N.event_record(ev[0], N.current_stream_ptr(self._dev))
        if self.use_torch_op:
            self._step_op(self._h, a_t, p_t, int(self._t_step), flags)
        elif N.wrong_current_device(self._dev):  # the op's DeviceGuard, for the direct call
            with torch.cuda.device(self._dev):
                self._c_step(a_t, p_t, flags)
        else:
            self._c_step(a_t, p_t, flags)
        if ev is not None:
            N.event_record(ev[1], N.current_stream_ptr(self._dev))
        if resetting:
            self._launch_draw_ahead()  # the next batch's draws, while this episode steps
            self._t_step = 0
            terminated = False
        else:
            self._t_step += 1
            terminated = self._t_step >= self.config.step_limit
        self._prev_done = terminated
        if numpy_mode:
            return self._numpy_step(resetting, terminated)
        self._post_launch_error_copy()
        return self._torch_step(resetting, terminated)

    def set_kernel_timing_events(self, begin=None, end=None):
        """Record hipEvent_t handles `begin`/`end` around the next steps' kernel launches (not around the
        Python step), on their stream (bench.py's live timing).  None disables."""
        self._kernel_events = None if begin is None else (begin, end)

    def _launch_draw_ahead(self):
        """The next batch autoreset's draws (apg_image_draw_ahead) on the side stream, after the work queued so far
        on the env's stream (the reset that just replaced the batch)."""
        if not self.draw_ahead:
            return
        import torch

        # (cached events and the side stream's raw handle: the C call takes the stream, no stream context needed)
        self._main_event.record(N.current_stream_ptr(self._dev))
        self._main_event.wait(self._ahead_side)
        N.check(N.lib().apg_image_draw_ahead(ctypes.byref(self._cfg), ctypes.byref(self._state), self._ahead_side),
                "apg_image_draw_ahead")
        self._ahead_event.record(self._ahead_side)
        self._ahead = True

    def _c_step(self, a_t, p_t, flags):
        if self._c_args is None:  # the fast-call entry point and the structures' addresses
            self._c_args = (N.fast().image_step, N.addr(self._cfg), N.addr(self._state), N.addr(self._out))
        fn, cfg, st, out = self._c_args
        rc = fn(cfg, st, a_t.data_ptr(), p_t.data_ptr(), self._t_step, flags, out, N.current_stream_ptr(self._dev))
        if rc:
            N.check(rc, "apg_image_step")

    # ------------------------------------------------------------------ outputs
    def _c(self, x):
        return x.clone() if self.copy else x

    def _numpy_obs(self):
        T = self._t
        obs = {"glimpse": T["glimpse"].cpu().numpy(), "glimpse_pos": T["glimpse_pos"].cpu().numpy(),
               "time_step": T["time_step"].cpu().numpy()}
        if self.config.randomly_invert_labels:
            obs["inverted_label"] = (np.full(self.num_envs, 2) if self._t_step > 0
                                     else T["inverted"].cpu().numpy().astype(np.int32))
        if self.kind == N.APG_IMAGE_LOCALIZE:
            obs["target_glimpse"] = T["target_glimpse"].cpu().numpy()
        return obs

    def _torch_obs(self):
        import torch

        T = self._t
        obs = {"glimpse": self._c(T["glimpse"]), "glimpse_pos": self._c(T["glimpse_pos"]),
               "time_step": self._c(T["time_step"])}
        if self.config.randomly_invert_labels:
            obs["inverted_label"] = (torch.full((self.num_envs,), 2, dtype=torch.int64, device=self.device)
                                     if self._t_step > 0 else self._c(T["inverted"]))
        if self.kind == N.APG_IMAGE_LOCALIZE:
            obs["target_glimpse"] = self._c(T["target_glimpse"])
        return obs

    def _stage_inputs(self, a_np, p_np):
        """numpy backend: action and prediction through one pinned staging buffer and one H2D copy (a pageable
        source would make each copy synchronous); the buffer is rewritten only after the previous step synchronized."""
        import torch

        na, npd = a_np.size, p_np.size
        if self._in_host is None:
            self._in_host = torch.empty(na + npd, dtype=torch.float32).pin_memory()
            self._in_dev = torch.empty(na + npd, dtype=torch.float32, device=self.device)
        h = self._in_host.numpy()
        np.copyto(h[:na], a_np.reshape(-1))
        np.copyto(h[na:], p_np.reshape(-1))
        self._in_dev.copy_(self._in_host, non_blocking=True)
        return self._in_dev[:na].view(a_np.shape), self._in_dev[na:].view(p_np.shape)

    HOST_RING = 4  # numpy backend: pinned output blocks handed out as the returned arrays

    def _np_fields(self):
        """(name, device tensor) of the outputs copied every numpy-backend step, 8-byte fields first (so every
        field of the packed byte block stays aligned)."""
        T = self._t
        loc = self.kind == N.APG_IMAGE_LOCALIZE
        f8 = [("reward", T["reward"]), ("index", T["index"])] + ([] if loc else [("loss", T["loss_f64"])])
        f4 = [("glimpse", T["glimpse"]), ("glimpse_pos", T["glimpse_pos"]), ("time_step", T["time_step"]),
              ("base_reward", T["base_reward"]), ("target", T["target_out"] if loc else T["label_target"])] + (
            [("loss", T["loss_f32"])] if loc else []) + [("err", T["err"])] + (
            [("target_glimpse", T["target_glimpse"])] if loc and self.obs_snapshot == "copy" else [])
        return f8 + f4

    def _np_block(self):
        """The step's outputs packed on the device into one byte block (one kernel), copied D2H in one go into a
        pinned host block and one synchronize; returns numpy views of that host block.  The host blocks form a ring
        that is reused only once no returned array refers to a block any more (every step's arrays stay valid, as
        the reference's freshly computed arrays do); past HOST_RING live blocks a private block is allocated."""
        import sys

        import torch

        fields = self._np_fields()
        if self._np_layout is None:
            lay, off = [], 0
            for name, t in fields:
                nb = t.numel() * t.element_size()
                lay.append((name, off, nb, torch.empty((), dtype=t.dtype).numpy().dtype, tuple(t.shape)))
                off += nb
            self._np_layout = (lay, off)
            self._np_dev = torch.empty(off, dtype=torch.uint8, device=self.device)
        lay, total = self._np_layout
        torch.cat([t.reshape(-1).view(torch.uint8) for _, t in fields], out=self._np_dev)
        blk = None
        for b in self._np_ring:
            if sys.getrefcount(b[1]) <= 2:  # the ring tuple and the call argument: no returned view is alive
                blk = b
                break
        if blk is None:
            t = torch.empty(total, dtype=torch.uint8).pin_memory()
            blk = (t, t.numpy())
            if len(self._np_ring) < self.HOST_RING:
                self._np_ring.append(blk)
        blk[0].copy_(self._np_dev, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return {name: blk[1][off:off + nb].view(dt).reshape(shape) for name, off, nb, dt, shape in lay}

    def _numpy_step(self, resetting, terminated):
        import torch

        T = self._t
        v = self._np_block()  # one D2H copy of every per-step output + one synchronize
        bits = int(v["err"][0])
        if bits:
            T["err"].zero_()
            self._raise_error_bits(bits)
        n = self.num_envs
        obs = {"glimpse": v["glimpse"], "glimpse_pos": v["glimpse_pos"], "time_step": v["time_step"]}
        if self.config.randomly_invert_labels:
            obs["inverted_label"] = (np.full(n, 2) if self._t_step > 0
                                     else T["inverted"].cpu().numpy().astype(np.int32))
        if self.kind == N.APG_IMAGE_LOCALIZE and self.obs_snapshot == "copy":
            obs["target_glimpse"] = v["target_glimpse"]  # (a field of this step's host block: the caller's own)
        elif self.kind == N.APG_IMAGE_LOCALIZE:
            # the target glimpse changes only with the batch: a read-only host snapshot refreshed on batch changes
            if resetting or self._tg_host is None:
                self._tg_host = T["target_glimpse"].cpu().numpy()
                self._tg_host.flags.writeable = False
            obs["target_glimpse"] = self._tg_host
        reward = v["reward"]
        if self.kind == N.APG_IMAGE_LOCALIZE and not resetting:
            reward = reward.astype(np.float32)  # every value is a float32 (base - loss in f32)
        target, loss = v["target"], v["loss"]
        base = np.zeros(n) if resetting else v["base_reward"]
        if self.sparse:
            target = {"target": target, "weight": np.full(n, terminated, dtype=np.float32)}
        info = {"index": v["index"], "base_reward": base, "prediction": {"target": target, "loss": loss}}
        if self.log_stats and terminated:
            info["stats"] = self._numpy_stats()
        return obs, reward, np.full(n, terminated), np.zeros(n, dtype=np.bool_), info

    def _metric_names(self):
        if self.kind == N.APG_IMAGE_CLASSIFY:
            return ("correct_label_prob", "accuracy")
        return ("euclidean_distance", "mse")

    def _numpy_stats(self):
        """update_info_metrics_vec (util.py:40-80) as the vector log wrappers call it on the step that
        ends every env's episode (image episodes end together)."""
        T = self._t
        n, lim = self.num_envs, int(self.config.step_limit)
        done = np.ones(n, dtype=np.bool_)
        st = T["stats"].cpu().numpy()
        hist = T["stats_hist"].cpu().numpy()
        names = self._metric_names()
        scalar: dict[str, Any] = {}
        for j, nm in enumerate(names):
            scalar[f"final_{nm}"] = st[j].copy()
        for nm in names:
            scalar[f"_final_{nm}"] = done
        for j, nm in enumerate(names):
            scalar[f"avg_{nm}"] = st[2 + j].copy()
        for nm in names:
            scalar[f"_avg_{nm}"] = done
        vector: dict[str, Any] = {}
        for j, nm in enumerate(names):
            arr = np.empty(n, dtype=object)
            hj = hist[:, j, :lim]
            if self.vector_stats == "array":  # float32 row views of one host block (opt-in: ndarray, not list)
                for i in range(n):
                    arr[i] = hj[i]
            else:  # the reference's list of np.float32 per env (update_info_metrics_vec, util.py:68-77)
                for i in range(n):
                    arr[i] = list(hj[i])
            vector[nm] = arr
        for nm in names:
            vector[f"_{nm}"] = done
        if self.kind == N.APG_IMAGE_CLASSIFY:
            idx = T["stats_idx"].cpu().numpy()
            scalar.update(first_correct=idx[0].copy(), _first_correct=idx[0] >= 0,
                          last_incorrect=idx[1].copy(), _last_incorrect=idx[1] >= 0)
        return {"scalar": scalar, "_scalar": done, "vector": vector, "_vector": done}

    def _torch_stats(self):
        """Device form of info["stats"] (built once from persistent buffers): scalars [N] and the
        per-step history [N, step_limit] of each metric as "vector"."""
        if self._stats_view is None:
            import torch

            T = self._t
            done = torch.ones(self.num_envs, dtype=torch.bool, device=self.device)
            names = self._metric_names()
            scalar, vector = {}, {}
            for j, nm in enumerate(names):
                scalar[f"final_{nm}"] = T["stats"][j]
                scalar[f"_final_{nm}"] = done
                scalar[f"avg_{nm}"] = T["stats"][2 + j]
                scalar[f"_avg_{nm}"] = done
                vector[nm] = T["stats_hist"][:, j]
                vector[f"_{nm}"] = done
            if self.kind == N.APG_IMAGE_CLASSIFY:
                scalar.update(first_correct=T["stats_idx"][0], last_incorrect=T["stats_idx"][1])
            self._stats_view = {"scalar": scalar, "_scalar": done, "vector": vector, "_vector": done}
        if not self.copy:
            return self._stats_view

        def clone(d):
            return {k: clone(v) if isinstance(v, dict) else v.clone() for k, v in d.items()}

        return clone(self._stats_view)

    def _torch_step(self, resetting, terminated):
        import torch

        T = self._t
        n = self.num_envs
        if self.kind == N.APG_IMAGE_LOCALIZE:
            target, loss = T["target_out"], T["loss_f32"]
        else:
            target, loss = T["label_target"], T["loss_f64"]
        # episodes end for the whole batch at once: terminated is all-True or all-False, never truncated
        if self._done_consts is None:
            self._done_consts = (torch.zeros(n, dtype=torch.bool, device=self.device),
                                 torch.ones(n, dtype=torch.bool, device=self.device),
                                 torch.zeros(n, dtype=torch.float32, device=self.device),
                                 torch.ones(n, dtype=torch.float32, device=self.device))
        target = self._c(target)
        if self.sparse:
            target = {"target": target, "weight": self._c(self._done_consts[3 if terminated else 2])}
        info = {"index": self._c(T["index"]), "base_reward": self._c(T["base_reward"]),
                "prediction": {"target": target, "loss": self._c(loss)}}
        term = self._c(self._done_consts[1 if terminated else 0])
        trunc = self._c(self._done_consts[0])
        if self.log_stats and terminated:
            info["stats"] = self._torch_stats()
        return self._torch_obs(), self._c(T["reward"]), term, trunc, info

    # ------------------------------------------------------------------ render
    def _track_render(self, prediction, resetting: bool):
        """Visitation overlay history of the tracked envs (image_perception_module.py:196, 219-234): the
        module records the sensor rectangle at the position *before* the step with the prediction quality,
        then (on the batch autoreset) clears the overlay.  Kept as (position, quality) rows and replayed
        by render()."""
        if not len(self.render_envs):
            return
        import torch

        if isinstance(prediction, torch.Tensor):
            self._last_prediction = prediction[torch.as_tensor(self.render_envs, device=self.device)].cpu().numpy()
        else:
            self._last_prediction = np.asarray(prediction)[self.render_envs].copy()
        if resetting:  # the overlay written by this step is cleared by module.reset() right after
            self._visits = [[] for _ in self.render_envs]
            return
        idx = torch.as_tensor(self.render_envs, device=self.device)
        pos = self._t["pos"][idx].cpu().numpy()
        p = self._last_prediction
        if self.kind == N.APG_IMAGE_CLASSIFY:  # softmax(prediction)[label] (image_classification.py:114-116)
            from scipy.special import softmax

            lab = self._t["label"][idx].cpu().numpy()
            quality = softmax(p, axis=-1)[np.arange(len(p)), lab]
        else:  # 1 - |prediction - target| / sqrt(4) (image_localization.py:157-159)
            quality = 1 - np.linalg.norm(p - self._t["target"][idx].cpu().numpy(), axis=-1) / np.sqrt(4)
        for j, v in enumerate(self._visits):
            v.append((pos[j].copy(), quality[j]))

    def _render_geometry(self):
        """render_size / render_scaling / sensor_pos_lim_pixels as the module derives them
        (image_perception_module.py:167-171, 403-445, 464-465)."""
        h, w = self.image_size
        s0, s1 = (int(v) for v in self.config.sensor_size)
        width = max(128, s1)
        scaling = width / w
        size = (width, int(round(scaling * h)))
        eff = np.array(self.config.sensor_size) * self.config.sensor_scale
        lim = (np.flip(np.array([h, w])) - 1) / 2 - (eff - 1) / 2
        border = max(1, int(round(1 / 128 * size[0])))
        return size, scaling, eff, lim, border

    def render(self):
        """rgb_array frames [len(render_envs), H_r, W_r, 3] like ImagePerceptionModule.render
        (image_perception_module.py:333-401) plus, for localization, ImageLocalizationVectorEnv.render
        (image_localization.py:183-223)."""
        from PIL import Image, ImageDraw

        from .render import COLOR_AGENT, COLOR_PRED, no_tracked_error, quality_color

        if not len(self.render_envs):
            raise no_tracked_error()
        if not self._seeded:
            raise RuntimeError("render() needs reset() first")
        import torch

        size, scaling, eff, lim, border = self._render_geometry()
        cfg = self.config

        def to_render(pn):
            return pn * lim * scaling + np.array(size) / 2

        idx = torch.as_tensor(self.render_envs, device=self.device)
        index = self._t["index"][idx].cpu().numpy()
        pool = self._pool_host if self._pool_host is not None else self._t["pool"][
            torch.as_tensor(index, device=self.device)].cpu().numpy()
        imgs = pool[index] if self._pool_host is not None else pool
        if imgs.dtype == np.uint8:
            imgs = imgs.astype(np.float32) / 255
        if imgs.shape[-1] == 1 and int(self.config.dataset.num_channels) == 3:
            imgs = np.repeat(imgs, 3, axis=-1)
        if imgs.shape[-1] == 1:
            imgs = imgs[..., 0]
        pos_now = self._t["pos"][idx].cpu().numpy()
        targets = self._t["target"][idx].cpu().numpy() if self.kind == N.APG_IMAGE_LOCALIZE else None
        rect = eff * scaling
        frames = []
        for j in range(len(self.render_envs)):
            counts = np.zeros((size[1], size[0]), dtype=np.int32)
            qmap = np.zeros((size[1], size[0]), dtype=np.float32)
            rs = np.round(np.flip(rect)).astype(np.int32)
            for pn, q in self._visits[j]:  # __update_visitation_overlay (:219-234)
                pi = np.round(to_render(pn)).astype(np.int32)
                xs = np.clip(pi[0] + np.arange(rs[0]) - rs[0] // 2, 0, size[0] - 1)
                ys = np.clip(pi[1] + np.arange(rs[1]) - rs[1] // 2, 0, size[1] - 1)
                counts[ys[:, None], xs[None, :]] += 1
                qmap[ys[:, None], xs[None, :]] = np.clip(q, 0, 1)
            visited = counts > 0
            ol = (visited[..., None] * np.concatenate(
                [np.stack(quality_color(qmap[None]))[..., :3].reshape(size[1], size[0], 3),
                 np.full_like(qmap[..., None], int(255 * cfg.render_visited_opacity))], axis=-1)
                  + ~visited[..., None] * (0, 0, 0, int(255 * cfg.render_unvisited_opacity))).round().astype(np.uint8)
            img = Image.fromarray((imgs[j] * 255).astype(np.uint8)).resize(
                size, resample=Image.Resampling.NEAREST).convert("RGB")
            if cfg.display_visitation:
                alpha = ol[..., -1:] / 255
                img = Image.fromarray((np.array(img) * (1 - alpha) + alpha * ol[..., :-1]).astype(np.uint8))
            draw = ImageDraw.Draw(img, "RGBA")
            c = to_render(pos_now[j])
            box = np.concatenate([c - rect / 2, c + rect / 2])
            draw.rectangle(tuple(box + border), outline=(0, 0, 0, 80), width=border)
            draw.rectangle(tuple(box), outline=COLOR_AGENT, width=border)
            if targets is not None:
                t_c = to_render(targets[j])
                draw.rectangle((tuple(t_c - rect / 2), tuple(t_c + rect / 2)), outline=COLOR_PRED + (100,),
                               width=border)
                if self._last_prediction is not None:
                    lp = to_render(self._last_prediction[j])
                    lp_box = np.concatenate([lp - rect / 2, lp + rect / 2])
                    draw.rectangle(tuple(lp_box), outline=COLOR_PRED, width=border)
                    draw.rectangle(tuple(lp_box + border), outline=(0, 0, 0, 80), width=border)
            frames.append(np.asarray(img))
        return np.asarray(frames)

    def close(self, **kwargs):
        if not getattr(self, "_closed", True):
            self._closed = True
            self.closed = True
            if getattr(self, "_ahead_stream", None) is not None:
                # the draw-ahead kernels on the side stream may still write the streams and ahead buffers, which
                # the caching allocator would otherwise hand to a new allocation of the main stream
                self._ahead_stream.synchronize()
                for ev in (self._ahead_event, self._main_event):
                    ev.destroy()
            self._t = {}
            self._h = None  # the op handle keeps every state/output buffer alive
            self._c_args = None
            self.output_rows = None


class ImageClassificationVectorEnv(_ImageVectorEnv):
    """image_classification.py:22-167 (target = current labels after the module step)."""

    kind = N.APG_IMAGE_CLASSIFY


class ImageLocalizationVectorEnv(_ImageVectorEnv):
    """image_localization.py:24-256 (unique-glimpse targets at reset, uniform targets after autoreset)."""

    kind = N.APG_IMAGE_LOCALIZE
