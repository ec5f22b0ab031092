"""numpy restatement of the reference's image glimpse path — TEST INFRASTRUCTURE ONLY.

Imported only by tests/ (and __graft_entry__.smoke()) as the checker for the HIP image path.  The
product package never imports this module.

What it restates (reference files at /root/reference, ap_gym 0.5.0):
  * glimpse()             ImagePerceptionModule.get_glimpse (image_perception_module.py:294-331) with
                          scipy 1.15 RegularGridInterpolator(method="linear", bounds_error=True) evaluated
                          in the order of scipy/interpolate/_rgi.py:_evaluate_linear (values are 3-D, so
                          the generic path): ((((0 + v00*w00) + v01*w01) + v10*w10) + v11*w11), with
                          w = (1*w_y)*w_x and w_y = y - g_i (unit grid), all f64; then clip(0, 1) -> f32.
  * pairwise_sum_f32()    numpy's pairwise summation (loops_utils.h.src pairwise_sum, PW_BLOCKSIZE 128)
                          that np.mean(..., axis=(-3, -2, -1)) applies to a contiguous f32 block.
  * unique_top_k()        sample_unique_glimpse_positions (image_perception_module.py:253-292) up to the
                          top-k selection; exact ties are ordered by index (numpy's argsort order for exact
                          ties is not restated: parity unpinned for that case only).
  * ImageVectorEnvOracle  ImagePerceptionModule.seed/reset/step (:105-217) composed with
                          ImageClassificationVectorEnv (image_classification.py:107-151) or
                          ImageLocalizationVectorEnv (image_localization.py:131-181) and
                          ActivePerceptionVectorEnv.step (active_perception_vector_env.py:84-111),
                          numpy Generator draws in the reference's order, scipy.special for the losses.
Pinned against tests/golden/image_*.npz (the reference run as-is; tests/test_oracle_golden.py).
"""

from __future__ import annotations

import numpy as np
import scipy.special

PW_BLOCK = 128


def pairwise_sum_f32(x: np.ndarray) -> np.ndarray:
    """Sum over the last axis in numpy's pairwise order, f32 accumulation, vectorised over the rest."""
    x = np.asarray(x, np.float32)
    n = x.shape[-1]
    if n < 8:
        r = np.zeros(x.shape[:-1], np.float32)
        for i in range(n):
            r = r + x[..., i]
        return r
    if n <= PW_BLOCK:
        r = [x[..., j].copy() for j in range(8)]
        i = 8
        while i < n - n % 8:
            for j in range(8):
                r[j] = r[j] + x[..., i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res = res + x[..., i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise_sum_f32(x[..., :n2]) + pairwise_sum_f32(x[..., n2:])


def sensor_pos_lim(image_hw, sensor, scale) -> np.ndarray:
    """sensor_pos_lim_pixels (:419-423): (flip(H, W) - 1)/2 - (sensor*scale - 1)/2 (x first)."""
    eff = np.array(sensor) * scale
    return (np.flip(np.array(image_hw)) - 1) / 2 - (eff - 1) / 2


def sensor_offsets(sensor, scale):
    o0 = (np.arange(sensor[0]) - (sensor[0] - 1) / 2) * scale
    o1 = (np.arange(sensor[1]) - (sensor[1] - 1) / 2) * scale
    return o0, o1


def glimpse(images: np.ndarray, pos: np.ndarray, sensor, scale) -> np.ndarray:
    """images f32 [N, H, W, C]; pos [N, ..., 2] (x, y normalised) -> f32 [N, ..., s0, s1, C]."""
    n, h, w, c = images.shape
    lim = sensor_pos_lim((h, w), sensor, scale)
    o0, o1 = sensor_offsets(sensor, scale)
    pos = np.asarray(pos)
    # flip(denormalize(pos)): (y, x) pixel offsets from the image centre, f64
    py = pos[..., 1] * lim[1]
    px = pos[..., 0] * lim[0]
    y = py[..., None, None] + o0[:, None]
    x = px[..., None, None] + o1[None, :]
    y, x = np.broadcast_arrays(y, x)
    cy, cx = (h - 1) / 2, (w - 1) / 2
    for d, (v, cc) in enumerate(((y, cy), (x, cx))):
        if not (np.all(-cc <= v) and np.all(v <= cc)):
            raise ValueError("One of the requested xi is out of bounds in dimension %d" % d)
    # interval index with g[i] <= v < g[i+1], clipped to [0, n-2] (scipy find_interval_ascending)
    iy = np.clip(np.floor(y + cy).astype(np.int64), 0, h - 2)
    ix = np.clip(np.floor(x + cx).astype(np.int64), 0, w - 2)
    iy = np.where(iy - cy > y, iy - 1, iy)
    ix = np.where(ix - cx > x, ix - 1, ix)
    iy = np.clip(iy, 0, h - 2)
    ix = np.clip(ix, 0, w - 2)
    wy = y - (iy - cy)
    wx = x - (ix - cx)
    ny_, nx_ = 1 - wy, 1 - wx
    b = np.arange(n).reshape((n,) + (1,) * (y.ndim - 1))

    def px_(yy, xx):
        return images[b, yy, xx].astype(np.float64)

    val = 0 + px_(iy, ix) * (ny_ * nx_)[..., None]
    val = val + px_(iy, ix + 1) * (ny_ * wx)[..., None]
    val = val + px_(iy + 1, ix) * (wy * nx_)[..., None]
    val = val + px_(iy + 1, ix + 1) * (wy * wx)[..., None]
    return np.clip(val, 0, 1).astype(np.float32)


def unique_grid(image_hw, sensor, scale, rel=0.2):
    """Sampling grid and cell size of sample_unique_glimpse_positions (:254-267)."""
    eff = np.array(sensor) * scale
    lim = sensor_pos_lim(image_hw, sensor, scale)
    cell = (eff / lim) * rel
    cnt = np.ceil(2 / cell)
    grid = np.stack(np.meshgrid(np.linspace(-1, 1, int(cnt[0])), np.linspace(-1, 1, int(cnt[1])), indexing="ij"),
                    axis=-1).reshape(-1, 2)
    return grid, cell


def uniqueness(g: np.ndarray) -> np.ndarray:
    """g f32 [N, P, L] -> f64 [N, P]: min over b != a of mean_f32((g_b - g_a)^2)."""
    n, p, l = g.shape
    out = np.empty((n, p), np.float64)
    for a in range(p):
        d = (g - g[:, a:a + 1]) ** 2  # f32 [N, P, L], element order as numpy's broadcast difference
        m = (np.float32(0) + pairwise_sum_f32(d)) / np.float32(l)
        m = m.astype(np.float64)
        m[:, a] = np.inf
        out[:, a] = m.min(axis=1)
    return out


def unique_top_k(images, sensor, scale, k=10, rel=0.2):
    grid, cell = unique_grid(images.shape[1:3], sensor, scale, rel)
    g = glimpse(images, np.broadcast_to(grid[None], (images.shape[0],) + grid.shape), sensor, scale)
    u = uniqueness(g.reshape(g.shape[0], g.shape[1], -1))
    top = np.argsort(-u, axis=-1, kind="stable")[:, :k]
    return top, grid, cell, u


def images_f32(pool: np.ndarray, channels: int) -> np.ndarray:
    """_process_imgs_np (image_classification_dataset.py:66-84)."""
    x = pool.astype(np.float32) / 255 if pool.dtype == np.uint8 else pool.astype(np.float32)
    if x.ndim == 3:
        x = x[..., None]
    if x.shape[-1] == 1 and channels == 3:
        x = np.repeat(x, 3, axis=-1)
    return x


def project_sphere(x, radius=1.0):
    mag = np.linalg.norm(x, axis=-1, keepdims=True)
    return np.where(mag > radius, x / np.maximum(mag, radius) * radius, x)


class ImageVectorEnvOracle:
    """Vector image env restated with numpy Generators (kind "cls" or "loc")."""

    def __init__(self, kind, pool, labels, num_classes, channels, num_envs, sensor=(5, 5), scale=1.0,
                 step_limit=16, max_step_length=0.2, invert=False, top_k=10, rel=0.2, log_stats=True,
                 sparse=False):
        self.kind, self.n = kind, num_envs
        self.pool = images_f32(pool, channels)
        self.labels_pool = np.asarray(labels).astype(np.int32)
        self.k = num_classes
        self.sensor, self.scale, self.limit = tuple(sensor), scale, step_limit
        self.msl = np.ones(2) * np.array(max_step_length)
        self.invert, self.top_k, self.rel = invert, top_k, rel
        self.log_stats = log_stats
        self.sparse = sparse

    # --- seeding chain: VectorEnv.reset(seed) -> _np_random setter -> module.seed
    def seed(self, seed):
        self.np_random = np.random.default_rng(seed)
        self.cur = np.random.default_rng(self.np_random.integers(0, 2**32 - 1, endpoint=True))
        self.it = np.random.default_rng(self.cur.integers(0, 2**32 - 1, endpoint=True))

    def _module_reset(self):
        idx = self.it.integers(0, len(self.pool), self.n)
        self.idx = idx
        self.images = self.pool[idx]
        labels = self.labels_pool[idx]
        if self.invert:
            self.inverted = self.cur.integers(0, 2, size=self.n) == 1
            labels = np.where(self.inverted, self.k - labels - 1, labels)
        self.cur_labels = labels
        self.pos = self.cur.uniform(-1, 1, size=(self.n, 2))
        self.t = 0
        self.prev_done = np.zeros(self.n, bool)
        return self._obs()

    def _obs(self):
        o = {"glimpse": glimpse(self.images, self.pos, self.sensor, self.scale),
             "glimpse_pos": self.pos.astype(np.float32),
             "time_step": np.full(self.n, (self.t / self.limit) * 2 - 1, np.float32)}
        if self.invert:
            o["inverted_label"] = np.full(self.n, 2) if self.t > 0 else self.inverted.astype(np.int32)
        return o

    def reset(self, seed):
        self.seed(seed)
        obs = self._module_reset()
        if self.kind == "loc":
            top, grid, cell, _ = unique_top_k(self.images, self.sensor, self.scale, self.top_k, self.rel)
            sel = self.cur.integers(0, self.top_k, size=self.n)
            base = grid[top[np.arange(self.n), sel]]
            self.target = np.clip(base + self.cur.uniform(-cell, cell, (self.n, 2)), -1, 1).astype(np.float32)
            self.env_prev_done = np.zeros(self.n, bool)
            obs["target_glimpse"] = glimpse(self.images, self.target, self.sensor, self.scale)
        self.hist = [[] for _ in range(self.n)]
        self.log_prev_done = np.zeros(self.n, bool)
        return obs, {"index": self.idx}

    def _log(self, prediction, info, done):
        """The registered ids' vector log wrapper (ActiveClassificationVectorLogWrapper,
        active_classification_env.py:116-197 / ActiveRegressionVectorLogWrapper,
        active_regression_env.py:160-227, util.py:40-80), restated."""
        target = info["prediction"]["target"]
        if self.kind == "cls":
            prob = scipy.special.softmax(prediction, axis=-1)[np.arange(self.n), target]
            vals = [(prob[i],) for i in range(self.n)]
            names = ["correct_label_prob"]
        else:
            d = target - prediction
            ed, ms = np.linalg.norm(d, axis=-1), np.mean(d ** 2, axis=-1)
            vals = [(ed[i], ms[i]) for i in range(self.n)]
            names = ["euclidean_distance", "mse"]
        for i in range(self.n):
            if self.log_prev_done[i]:
                self.hist[i] = []
            else:
                self.hist[i].append(vals[i])
        self.log_prev_done = done
        if not done.any():
            return info
        metrics = {nm: [np.array([h[j] for h in self.hist[i]], np.float32) for i in range(self.n)]
                   for j, nm in enumerate(names)}
        if self.kind == "cls":
            is_correct = [m > 1 / self.k for m in metrics["correct_label_prob"]]
            metrics["accuracy"] = [c.astype(np.float32) for c in is_correct]
        scalar, vector = {}, {}
        for nm, per_env in metrics.items():
            scalar[f"final_{nm}"] = np.array([e[-1] if t else np.nan for t, e in zip(done, per_env)], np.float32)
            scalar[f"_final_{nm}"] = done
        for nm, per_env in metrics.items():
            scalar[f"avg_{nm}"] = np.array([np.mean(e) if t else np.nan for t, e in zip(done, per_env)], np.float32)
            scalar[f"_avg_{nm}"] = done
        for nm, per_env in metrics.items():
            vector[nm] = np.array([(list(e) if t else []) for e, t in zip(per_env, done)] + [None], dtype=object)[:-1]
            vector[f"_{nm}"] = done
        if self.kind == "cls":
            fc, fcv = np.full(self.n, -1, np.int32), np.zeros(self.n, bool)
            li, liv = np.full(self.n, -1, np.int32), np.zeros(self.n, bool)
            for i, c in enumerate(is_correct):
                w = np.nonzero(c)[0]
                if len(w):
                    fc[i], fcv[i] = w[0], True
                w = np.nonzero(~c)[0]
                if len(w):
                    li[i], liv[i] = w[-1], True
            scalar.update(first_correct=fc, _first_correct=fcv, last_incorrect=li, _last_incorrect=liv)
        info["stats"] = {"scalar": scalar, "_scalar": done, "vector": vector, "_vector": done}
        return info

    def step(self, action, prediction):
        action = np.asarray(action, np.float32)
        prediction = np.asarray(prediction, np.float32)
        if self.kind == "loc":
            pred_target = self.target.copy()
            if np.any(self.env_prev_done):
                self.target[self.env_prev_done] = self.np_random.uniform(
                    -1, 1, (int(np.sum(self.env_prev_done)), 2)).astype(np.float32)
            quality = 1 - np.linalg.norm(prediction - self.target, axis=-1) / np.sqrt(4)
        else:
            quality = scipy.special.softmax(prediction, axis=-1)[np.arange(self.n), self.cur_labels]
        if np.any(np.isnan(quality)):
            raise ValueError("NaN values detected in prediction.")
        if np.any(self.prev_done):
            obs = self._module_reset()
            terminated = False
            base = np.zeros(self.n)
        else:
            if np.any(np.isnan(action)):
                raise ValueError("NaN values detected in action.")
            self.pos = np.clip(self.pos + self.msl * project_sphere(action), -1, 1)
            base = -np.linalg.norm(action, axis=-1) * 1e-3
            self.t += 1
            terminated = self.t >= self.limit
            obs = self._obs()
        term = np.full(self.n, terminated)
        trunc = np.zeros(self.n, bool)
        self.prev_done = term | trunc
        if self.kind == "loc":
            self.env_prev_done = self.prev_done
            obs["target_glimpse"] = glimpse(self.images, self.target, self.sensor, self.scale)
            target = pred_target
            loss = self._mse_normalized(prediction, target)
        else:
            target = self.cur_labels
            ce = -np.take_along_axis(scipy.special.log_softmax(prediction, axis=-1), target[..., None], -1)[..., 0]
            scale = 1 / (np.log(self.k) - 0.0)
            loss = ce * scale + (-0.0 * scale)
        info = {"index": self.idx, "base_reward": base, "prediction": {"target": target, "loss": loss}}
        if self.log_stats:
            info = self._log(prediction, info, term | trunc)
        if self.sparse:
            # SparsifyVectorWrapper.step (sparsify_wrapper.py:61-87) with WeightedLossFn (loss_fn.py:307-316)
            weight = term.astype(np.float32)
            info["prediction"]["target"] = {"target": target, "weight": weight}
            return obs, base - loss * weight, term, trunc, info
        return obs, base - loss, term, trunc, info

    @staticmethod
    def _mse_normalized(prediction, target):
        # MSELossFn(target_std=(1 - -1)/sqrt(12)).normalized (active_regression_env.py:29-52, loss_fn.py)
        std = (1 - -1) / np.sqrt(12)
        bg = float(np.mean(std ** 2))
        scale = 1 / (bg - 0.0)
        return np.mean((prediction - target) ** 2, axis=-1) * scale + (-0.0 * scale)


# ------------------------------------------------------------------ CircleSquare datasets (test oracle)
def circle_square_positions(image_shape, object_extents=8) -> np.ndarray:
    """DoubleCircleSquareDataset's valid coordinate pairs (circle_square_dataset.py:129-146), [P, 2, 2]."""
    h, w = image_shape
    coords = np.stack(np.meshgrid(np.arange(h), np.arange(w), indexing="ij"), axis=-1).reshape(-1, 2)
    pairs = np.stack(np.broadcast_arrays(coords[:, None], coords[None, :]), axis=-2).reshape(-1, 2, 2)
    valid = ((np.abs(pairs[:, 0] - pairs[:, 1]) >= object_extents + 1).any(axis=-1)
             & (pairs[:, 0, 0] <= pairs[:, 1, 0])
             & ((pairs[:, 0, 0] < pairs[:, 1, 0]) | (pairs[:, 0, 1] <= pairs[:, 1, 1])))
    return pairs[valid]


def _cs_object(coords, pos, label, ext):
    """_draw_object (circle_square_dataset.py:32-55), vectorised over a batch of positions/labels."""
    p = pos[:, None, None, :]
    half = ext / 2
    rect = ((p[..., 0] - half <= coords[..., 0]) & (coords[..., 0] <= p[..., 0] + half)
            & (p[..., 1] - half <= coords[..., 1]) & (coords[..., 1] <= p[..., 1] + half))
    circ = np.linalg.norm(p - coords, axis=-1) <= half
    return np.where((np.asarray(label) == 0)[:, None, None], rect, circ)


def circle_square_images(kind: str, image_shape, idx, show_gradient_a=True, show_gradient_b=True, object_extents=8,
                         positions=None):
    """get_data_point_batch of CircleSquareDataset ("single") / DoubleCircleSquareDataset ("double")
    (circle_square_dataset.py:98-107, 149-172; float64 arithmetic, then float32): images [n, H, W, 1],
    labels int32."""
    idx = np.asarray(idx, np.int64)
    h, w = image_shape
    coords = np.stack(np.meshgrid(np.arange(h), np.arange(w), indexing="ij"), axis=-1)
    max_dist = np.sqrt(np.sum(np.array(image_shape) ** 2))
    if kind == "single":
        label, rest = idx % 2, idx // 2
        pos = np.stack([(rest // w) % h, rest % w], axis=-1)
        if show_gradient_a:
            img = 1 - np.linalg.norm(pos[:, None, None, :] - coords, axis=-1) / max_dist
        else:
            img = np.zeros((idx.shape[0], h, w))
        img[_cs_object(coords, pos, label, object_extents)] = 1.0
        labels = label
    else:
        if positions is None:
            positions = circle_square_positions(image_shape, object_extents)
        l1, l2, pi = idx % 2, (idx // 2) % 2, (idx // 4) % len(positions)
        p1, p2 = positions[pi, 0], positions[pi, 1]
        n1 = np.linalg.norm(p1[:, None, None, :] - coords, axis=-1)
        n2 = np.linalg.norm(p2[:, None, None, :] - coords, axis=-1)
        img = 1 - np.minimum(n1 * show_gradient_a, n2 * show_gradient_b) / max_dist
        img[_cs_object(coords, p1, l1, object_extents) | _cs_object(coords, p2, l2, object_extents)] = 1.0
        labels = np.where(l1 == l2, l1, 2)
    return img.astype(np.float32)[..., None], labels.astype(np.int32)


def hide_and_seek_additional_reward(index, glimpse_pos, image_shape, sensor, scale):
    """CircleSquareHideAndSeekVectorWrapper.step's additional reward (circle_square_catch_or_flee.py:79-92)."""
    h, w = image_shape
    index = np.asarray(index)
    label, rest = index % 2, index // 2
    positions = np.stack([(rest // w) % h, rest % w], axis=-1)
    sign = label * 2 - 1
    positions_norm = np.flip(positions, axis=-1) / sensor_pos_lim((h, w), sensor, scale) - 1
    return sign * np.linalg.norm(glimpse_pos - positions_norm, axis=-1)
