"""Prediction losses with the reference's interface (ap_gym/loss_fn.py:25-349).

`env.loss_fn(prediction, target, batch_shape)` is what users call to train their predictors; the
envs evaluate the same losses inside their step kernels.  numpy evaluation reproduces the
reference bit for bit (same ops, same NEP 50 dtype promotion); `torch` gives differentiable
tensors on any device.
"""

from __future__ import annotations

import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _log_softmax_np(x: np.ndarray) -> np.ndarray:
    # scipy.special.log_softmax: x - max - log(sum(exp(x - max)))
    x = np.asarray(x)
    x_max = np.amax(x, axis=-1, keepdims=True)
    x_max = np.where(np.isfinite(x_max), x_max, 0)
    tmp = x - x_max
    s = np.sum(np.exp(tmp), axis=-1, keepdims=True)
    with np.errstate(divide="ignore"):
        return tmp - np.log(s)


class LossFn:
    def numpy(self, prediction, target, batch_shape=()):
        raise NotImplementedError

    def torch(self, prediction, target, batch_shape=()):
        raise NotImplementedError("Loss function is not implemented for torch.")

    def jax(self, prediction, target, batch_shape=()):
        raise NotImplementedError("Loss function is not implemented for jax.")

    def __call__(self, prediction, target, batch_shape=()):
        return self.numpy(prediction, target, batch_shape)

    @property
    def lower_bound(self) -> float:
        return self._lower_bound()

    def _lower_bound(self):
        return -np.inf

    @property
    def blind_guessing_expected_value(self):
        return self._blind_guessing_expected_value()

    def _blind_guessing_expected_value(self):
        return None

    @property
    def normalized(self) -> "LossFnAffineTransformation":
        """Affine map sending [lower_bound, blind-guess expectation] to [0, 1] (loss_fn.py:69-83)."""
        hi = self.blind_guessing_expected_value
        if hi is None:
            raise ValueError("Cannot normalize loss function without blind guessing expected value.")
        lo = self.lower_bound
        if hi <= lo:
            raise ValueError(
                "Cannot normalize loss function when blind guessing expected value is not greater than lower bound.")
        scale = 1 / (hi - lo)
        return LossFnAffineTransformation(self, scale, -lo * scale)


class LossFnAffineTransformation(LossFn):
    def __init__(self, inner: LossFn, scale: float, offset: float):
        self.inner = inner
        self.scale = scale
        self.offset = offset

    def numpy(self, prediction, target, batch_shape=()):
        return self.inner.numpy(prediction, target, batch_shape=batch_shape) * self.scale + self.offset

    def torch(self, prediction, target, batch_shape=()):
        return self.inner.torch(prediction, target, batch_shape=batch_shape) * self.scale + self.offset

    def _lower_bound(self):
        return self.inner.lower_bound * self.scale + self.offset

    def _blind_guessing_expected_value(self):
        v = self.inner.blind_guessing_expected_value
        return None if v is None else v * self.scale + self.offset


class LambdaLossFn(LossFn):
    def __init__(self, np, torch=None, jax=None, lower_bound=-np.inf, blind_guessing_expected_value=None):
        self._np, self._torch, self._jax = np, torch, jax
        self._lb, self._bg = lower_bound, blind_guessing_expected_value

    def numpy(self, prediction, target, batch_shape=()):
        return self._np(prediction, target, batch_shape)

    def torch(self, prediction, target, batch_shape=()):
        if self._torch is None:
            raise NotImplementedError("Loss function is not implemented for torch.")
        return self._torch(prediction, target, batch_shape)

    def _lower_bound(self):
        return self._lb

    def _blind_guessing_expected_value(self):
        return self._bg


class ZeroLossFn(LossFn):
    def numpy(self, prediction, target, batch_shape=()):
        return np.zeros(batch_shape, dtype=np.float32)

    def torch(self, prediction, target, batch_shape=()):
        return torch.zeros(batch_shape)

    def _lower_bound(self):
        return 0.0

    def _blind_guessing_expected_value(self):
        return 0.0


class CrossEntropyLossFn(LossFn):
    """-log_softmax(prediction)[target] (loss_fn.py:207-250); blind guess = log(num_classes)."""

    def __init__(self, num_classes: int | None = None):
        self.num_classes = num_classes

    def numpy(self, prediction, target, batch_shape=()):
        lsm = _log_softmax_np(prediction)
        return -np.take_along_axis(lsm, np.asarray(target)[..., None], axis=-1)[..., 0]

    def torch(self, prediction, target, batch_shape=()):
        lsm = torch.nn.functional.log_softmax(prediction, dim=-1)
        return -torch.take_along_dim(lsm, target[..., None], dim=-1)[..., 0]

    def _lower_bound(self):
        return 0.0

    def _blind_guessing_expected_value(self):
        return None if self.num_classes is None else np.log(self.num_classes)


class MSELossFn(LossFn):
    """mean((prediction - target)**2, -1) (loss_fn.py:253-289); blind guess = mean(target_std**2)."""

    def __init__(self, target_std=None):
        self._bg = None if target_std is None else float(np.mean(np.asarray(target_std) ** 2))

    def numpy(self, prediction, target, batch_shape=()):
        return np.mean((prediction - target) ** 2, axis=-1)

    def torch(self, prediction, target, batch_shape=()):
        return torch.mean((prediction - target) ** 2, dim=-1)

    def _lower_bound(self):
        return 0.0

    def _blind_guessing_expected_value(self):
        return self._bg


class WeightedLossFn(LossFn):
    def __init__(self, inner: LossFn, min_weight: float = 0.0, average_weight: float | None = None):
        self.inner, self.min_weight, self.average_weight = inner, min_weight, average_weight

    def numpy(self, prediction, target, batch_shape=()):
        return self.inner.numpy(prediction, target["target"], batch_shape) * target["weight"]

    def torch(self, prediction, target, batch_shape=()):
        return self.inner.torch(prediction, target["target"], batch_shape) * target["weight"]

    def _lower_bound(self):
        return self.min_weight * self.inner.lower_bound

    def _blind_guessing_expected_value(self):
        v = self.inner.blind_guessing_expected_value
        if v is None or self.average_weight is None:
            return None
        return self.average_weight * v


def regression_loss(target_dim: int, low: float, high: float, target_std: float | None = None) -> LossFn:
    """active_regression_env.py:29-52: MSE normalised by a uniform-target std when bounded."""
    if target_std is None and np.isfinite(low) and np.isfinite(high):
        target_std = (high - low) / np.sqrt(12)
    fn = MSELossFn(target_std=target_std)
    return fn.normalized if target_std is not None else fn


def affine_f32(fn: LossFn) -> tuple[float, float]:
    """(scale, offset) as the float32 values numpy applies to a float32 loss (NEP 50)."""
    if isinstance(fn, LossFnAffineTransformation):
        return float(np.float32(fn.scale)), float(np.float32(fn.offset))
    return 1.0, 0.0
