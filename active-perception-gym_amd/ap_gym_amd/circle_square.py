"""CircleSquare datasets and the CircleSquareHideAndSeek wrapper on the GPU.

Reference (ap_gym 0.5.0): ap_gym/envs/image/circle_square_dataset.py:11-178 (BaseCircleSquareDataset,
CircleSquareDataset, DoubleCircleSquareDataset) and ap_gym/envs/circle_square_catch_or_flee.py:20-107
(CircleSquareHideAndSeekVectorWrapper), registered at ap_gym/envs/registration.py:358-512.

The datasets are procedural: data point `idx` is (label, object position) unpacked from `idx`, and
its image is a distance gradient with the object drawn on top.  The image envs keep a dataset as
one device-resident pool, so `device_pool_tensors` renders the whole dataset into HBM with one
HIP kernel (`apg_circle_square_pool`; 2.8 GB float32 for DoubleCircleSquare 28x28) and the glimpse
kernels read it like any other float32 pool.  `get_data_point[_batch]` (the reference's dataset
API) renders the requested points with the same kernel and copies them to the host.

The hide-and-seek reward (sign(label) * distance between the glimpse and the object, folded into
info["base_reward"] and the reward) runs as one HIP kernel per step on the inner env's device
outputs (`apg_hide_and_seek_reward`).
"""

from __future__ import annotations

import ctypes
from copy import copy
from typing import Any, Sequence

import numpy as np

from . import _native as N
from .image_dataset import ImageClassificationDataset
from .loss_fn import WeightedLossFn, ZeroLossFn
from .spaces import ActivePerceptionActionSpace, Box, Dict, Tuple, batch_space
from .vector_env import VectorEnv


class BaseCircleSquareDataset(ImageClassificationDataset):
    """circle_square_dataset.py:11-76: packing of (label, position) into an index, one channel."""

    _kind: int

    def __init__(self, image_shape: tuple[int, int] = (28, 28), object_extents: int = 8):
        self._image_shape = tuple(int(v) for v in image_shape)
        self._object_extents = object_extents

    def _get_num_channels(self) -> int:
        return 1

    def _get_max_vals(self) -> Sequence[int]:
        raise NotImplementedError

    def _pack(self, vals: Sequence[int]) -> int:
        multiplier, value_packed = 1, 0
        for val, max_val in zip(vals, self._get_max_vals()):
            value_packed += val * multiplier
            multiplier *= max_val
        return value_packed

    def _unpack(self, value_packed):
        remainder, vals = value_packed, []
        for max_val in self._get_max_vals():
            val = remainder % max_val
            vals.append(val)
            remainder = (remainder - val) // max_val
        return vals

    def _get_length(self) -> int:
        return int(np.prod(self._get_max_vals()))

    # ------------------------------------------------------------------ device rendering
    def _native_config(self) -> N.CircleSquareConfig:
        raise NotImplementedError

    def _positions_tensor(self, device):
        return None

    def render_device(self, first: int, count: int, device="cuda"):
        """Data points [first, first + count) as device tensors (images f32 [count, H, W, 1], labels i32)."""
        import torch

        dev = torch.device(device)
        h, w = self._image_shape
        images = torch.empty((count, h, w, 1), dtype=torch.float32, device=dev)
        labels = torch.empty(count, dtype=torch.int32, device=dev)
        pos = self._positions_tensor(dev)
        cfg = self._native_config()
        N.check(N.lib().apg_circle_square_pool(ctypes.byref(cfg), N.ptr(pos), int(first), int(count), N.ptr(images),
                                               N.ptr(labels), N.stream_handle(dev)), "apg_circle_square_pool")
        return images, labels

    def device_pool_tensors(self, device):
        """The whole dataset as a resident pool (what the image envs gather glimpses from)."""
        return self.render_device(0, len(self), device)

    def _get_data_point_batch(self, idx):
        import torch

        idx = np.asarray(idx, dtype=np.int64)
        if not torch.cuda.is_available():
            raise N.NativeLibraryError("CircleSquare datasets render on the GPU (no CPU fallback)")
        n = len(self)
        if np.any((idx < 0) | (idx >= n)):
            raise IndexError("data point index out of range")
        images = np.empty((idx.shape[0], *self._image_shape, 1), dtype=np.float32)
        labels = np.empty(idx.shape[0], dtype=np.int32)
        for j, i in enumerate(idx):  # contiguous single-point renders (the dataset API is not a hot path)
            im, lb = self.render_device(int(i), 1)
            images[j] = im[0].cpu().numpy()
            labels[j] = int(lb[0].item())
        return images, labels

    def device_pool(self):
        images, labels = self.render_device(0, len(self))
        return images.cpu().numpy(), labels.cpu().numpy()


class CircleSquareDataset(BaseCircleSquareDataset):
    """circle_square_dataset.py:79-113: a circle (label 1) or square (label 0) of side/diameter
    object_extents at any pixel, over an optional distance gradient towards it."""

    def __init__(self, show_gradient: bool = True, image_shape: tuple[int, int] = (28, 28), object_extents: int = 8):
        super().__init__(image_shape=image_shape, object_extents=object_extents)
        self._show_gradient = show_gradient

    def _get_max_vals(self) -> Sequence[int]:
        return [2, self._image_shape[1], self._image_shape[0]]

    def _get_num_classes(self) -> int:
        return 2

    def get_object_position_and_label(self, idx):
        label, pos_x, pos_y = self._unpack(idx)
        return np.stack([pos_y, pos_x], axis=-1), label

    def _native_config(self):
        h, w = self._image_shape
        return N.CircleSquareConfig(kind=N.APG_DS_CIRCLE_SQUARE, height=h, width=w,
                                    show_gradient_a=int(bool(self._show_gradient)), show_gradient_b=0, num_positions=0,
                                    half_extent=float(self._object_extents / 2),
                                    max_dist=float(np.sqrt(np.sum(np.array(self._image_shape) ** 2))))


class DoubleCircleSquareDataset(BaseCircleSquareDataset):
    """circle_square_dataset.py:116-178: two objects at least object_extents + 1 apart along one
    axis; label = the shared shape, or 2 for one of each."""

    def __init__(self, show_gradient_a: bool = True, show_gradient_b: bool = True,
                 image_shape: tuple[int, int] = (28, 28), object_extents: int = 8):
        super().__init__(image_shape=image_shape, object_extents=object_extents)
        self._show_gradient_a, self._show_gradient_b = show_gradient_a, show_gradient_b
        h, w = self._image_shape
        # the reference's valid coordinate pairs, in its order (:129-146): pair (a, b) of row-major pixel
        # indices, a <= b, far enough apart along at least one axis
        a, b = np.divmod(np.arange(h * w), w)
        coords = np.stack([a, b], axis=-1)
        ia, ib = np.meshgrid(np.arange(h * w), np.arange(h * w), indexing="ij")
        ia, ib = ia.reshape(-1), ib.reshape(-1)
        ca, cb = coords[ia], coords[ib]
        valid = ((np.abs(ca - cb) >= object_extents + 1).any(axis=-1) & (ca[:, 0] <= cb[:, 0])
                 & ((ca[:, 0] < cb[:, 0]) | (ca[:, 1] <= cb[:, 1])))
        self._positions = np.stack([ca[valid], cb[valid]], axis=1)  # [P, 2, 2] (row, col)
        self._positions_dev = {}

    def _get_num_classes(self) -> int:
        return 3

    def _get_max_vals(self) -> Sequence[int]:
        return [2, 2, len(self._positions)]

    @property
    def positions(self) -> np.ndarray:
        return self._positions

    def _positions_tensor(self, device):
        import torch

        key = str(device)
        if key not in self._positions_dev:
            self._positions_dev[key] = torch.from_numpy(self._positions.astype(np.int16).reshape(-1, 4)).to(device)
        return self._positions_dev[key]

    def _native_config(self):
        h, w = self._image_shape
        return N.CircleSquareConfig(kind=N.APG_DS_DOUBLE_CIRCLE_SQUARE, height=h, width=w,
                                    show_gradient_a=int(bool(self._show_gradient_a)),
                                    show_gradient_b=int(bool(self._show_gradient_b)),
                                    num_positions=len(self._positions), half_extent=float(self._object_extents / 2),
                                    max_dist=float(np.sqrt(np.sum(np.array(self._image_shape) ** 2))))


class CircleSquareHideAndSeekVectorWrapper(VectorEnv):
    """circle_square_catch_or_flee.py:20-107 over the GPU ImageClassificationVectorEnv.

    reward += sign * |glimpse_pos - object position (normalized)|, sign = +1 for circles (label 1),
    -1 for squares; info["base_reward"] gets the same term.  mask_prediction=True (the NoPrediction
    id) drops the prediction: ZeroLossFn, empty prediction/target spaces, reward = base_reward.
    sparse=True applies SparsifyVectorWrapper on top (the -sparse ids)."""

    def __init__(self, env, mask_prediction: bool = False, sparse: bool = False):
        import torch

        if not isinstance(env.config.dataset, CircleSquareDataset):
            raise AssertionError("CircleSquareHideAndSeekVectorWrapper needs a CircleSquareDataset")
        if getattr(env, "sparse", False):
            raise ValueError("pass sparse=True to the wrapper, not to the inner env")
        self.env = env
        self.num_envs = n = env.num_envs
        self._dataset = env.config.dataset
        self._mask = bool(mask_prediction)
        self.sparse = bool(sparse)
        self.single_observation_space = env.single_observation_space
        self.observation_space = env.observation_space
        self.metadata = env.metadata
        self.loss_fn = ZeroLossFn() if self._mask else env.loss_fn
        if self._mask:
            self.single_prediction_target_space = Tuple(())
            self.single_action_space = ActivePerceptionActionSpace(env.single_inner_action_space, Tuple(()))
        else:
            self.single_prediction_target_space = env.single_prediction_target_space
            self.single_action_space = env.single_action_space
        if self.sparse:
            self.single_prediction_target_space = Dict({"target": self.single_prediction_target_space,
                                                        "weight": Box(0, 1, (), np.float32)})
            self.loss_fn = WeightedLossFn(self.loss_fn)
        self.prediction_target_space = batch_space(self.single_prediction_target_space, n)
        self.action_space = batch_space(self.single_action_space, n)
        h, w = env.image_size
        from .image_env import sensor_pos_lim_pixels

        lim = sensor_pos_lim_pixels((h, w), env.config.sensor_size, env.config.sensor_scale)
        dev = env.device
        self._buf = {k: torch.zeros(n, dtype=torch.float64, device=dev) for k in ("base", "reward", "additional")}
        self._args = N.HideAndSeekArgs(num_envs=n, height=h, width=w, lim=(ctypes.c_double * 2)(*lim.tolist()),
                                       base_reward_out=N.ptr(self._buf["base"]),
                                       reward_out=N.ptr(self._buf["reward"]),
                                       additional=N.ptr(self._buf["additional"]))
        self._zero_pred = None

    # ------------------------------------------------------------------ passthrough
    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    @property
    def config(self):
        return self.env.config

    @property
    def render_mode(self):
        return self.env.render_mode

    @property
    def closed(self):
        return self.env.closed

    @property
    def prediction_space(self):
        return self.action_space["prediction"]

    @property
    def single_prediction_space(self):
        return self.single_action_space["prediction"]

    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        obs, info = self.env.reset(seed=seed, options=options)
        info = dict(info)
        if self._mask:
            # the reference assigns info["prediction"]["target"] on a reset info that has no
            # "prediction" entry (circle_square_catch_or_flee.py:61-64): the same KeyError
            info["prediction"]["target"] = ()
        return obs, info

    def step(self, actions):
        import torch

        env = self.env
        n = self.num_envs
        if self._mask:
            if self._zero_pred is None:
                self._zero_pred = (np.zeros(env.prediction_space.shape) if env.array_backend == "numpy"
                                   else torch.zeros(env.prediction_space.shape, device=env.device))
            actions = {"action": actions["action"], "prediction": self._zero_pred}
        resetting = env._prev_done
        obs, reward, terminated, truncated, info = env.step(actions)
        done = bool(env._prev_done)  # image episodes end for the whole batch at once (host-tracked)
        T = env._t
        a = self._args
        a.resetting, a.terminated = int(resetting), int(done)
        a.mask_prediction, a.sparse = int(self._mask), int(self.sparse)
        a.index, a.glimpse_pos = N.ptr(T["index"]), N.ptr(T["glimpse_pos"])
        a.base_reward_in, a.reward_in, a.loss = N.ptr(T["base_reward"]), N.ptr(T["reward"]), N.ptr(T["loss_f64"])
        N.check(N.lib().apg_hide_and_seek_reward(ctypes.byref(a), env._stream()), "apg_hide_and_seek_reward")
        info = copy(info)
        info["prediction"] = dict(info["prediction"])
        numpy_mode = env.array_backend == "numpy"
        B = self._buf
        if numpy_mode:
            base = B["base"].cpu().numpy()
            base = base if resetting else base.astype(np.float32)
            rew = B["reward"].cpu().numpy()
            if self._mask and not resetting:
                rew = rew.astype(np.float32)
        else:  # persistent float64 buffers (cloned when the inner env copies), float32 views where numpy's are
            base = (B["base"].clone() if env.copy else B["base"]) if resetting else B["base"].to(torch.float32)
            if self._mask and not resetting:
                rew = B["reward"].to(torch.float32)
            else:
                rew = B["reward"].clone() if env.copy else B["reward"]
        info["base_reward"] = base
        if self._mask:
            info["prediction"]["target"] = ()
        if self.sparse:
            weight = (np.full(n, done, dtype=np.float32) if numpy_mode
                      else torch.full((n,), float(done), dtype=torch.float32, device=env.device))
            info["prediction"]["target"] = {"target": info["prediction"]["target"], "weight": weight}
        return obs, rew, terminated, truncated, info

    def render(self):
        return self.env.render()

    def close(self, **kwargs):
        if "env" in self.__dict__:
            self.env.close(**kwargs)
