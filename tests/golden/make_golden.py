"""Generate the golden fixtures under tests/golden/ from the reference (build container only).

    python tests/golden/make_golden.py            # all sections
    python tests/golden/make_golden.py maps lidar # some sections

Sources of truth, per fixture:
  rng.npz          numpy 2.2.6 Generator(PCG64(SeedSequence)) itself.
  maps.npz         the reference's FloorMapDatasetRooms / FloorMapDatasetMaze (numpy only, run as-is).
  loss.npz         the reference's MSELossFn / CrossEntropyLossFn (normalized as the envs build them).
  lidar_scan.npz   the reference's LIDARLocalization2DEnv.__lidar_scan (lidar_localization2d.py:496-536)
                   with tests/golden/_stubs/shapely (exact-rational GEOS model) in place of shapely.
  lidar_env_*.npz  the reference's LIDARLocalization2DEnv wrapped exactly as registration.py:319-356
                   composes it (TimeLimit(100, issue_termination=True) + ActiveRegressionLogWrapper),
                   vectorised by the gymnasium SyncVectorEnv restatement in tests/golden/_stubs.
  image_*.npz      the reference's ImageClassificationVectorEnv / ImageLocalizationVectorEnv
                   (ImagePerceptionModule, scipy RegularGridInterpolator, CE/MSE losses) run as-is on
                   small synthetic uint8 pools (HF datasets are not available offline), seeded through
                   the gymnasium VectorEnv.reset restatement in tests/golden/_stubs.
The fixtures hold data only (inputs and expected outputs).  See DESIGN.md §Oracle for what each pins.
"""

from __future__ import annotations

import os
import sys
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path), "bytes")


# --------------------------------------------------------------------------- rng
def make_rng():
    seeds = np.array(list(range(64)) + [2**32 - 1, 2**32, 2**40 + 7, 2**63 + 5, 2**64 - 1], dtype=np.uint64)
    raw = np.stack([np.random.default_rng(int(s)).bit_generator.random_raw(16) for s in seeds])
    u32e = np.stack([[np.random.default_rng(int(s)).integers(0, 2**32, endpoint=True)] for s in seeds])
    his = np.array([2, 3, 7, 10, 61, 1000, 4096, 2**31 + 5, 2**32 - 1, 2**32], dtype=np.int64)
    ints = np.zeros((len(seeds), len(his), 8), np.int64)
    for i, s in enumerate(seeds):
        for j, hi in enumerate(his):
            g = np.random.default_rng(int(s))
            ints[i, j] = [g.integers(0, int(hi)) for _ in range(8)]
    binom = np.zeros((len(seeds), 9, 8), np.int64)
    for i, s in enumerate(seeds):
        for n in range(9):
            g = np.random.default_rng(int(s))
            binom[i, n] = [g.binomial(n, 0.3) for _ in range(8)]
    unif = np.stack([np.random.default_rng(int(s)).uniform(-1, 1, 8) for s in seeds])
    rand = np.stack([np.random.default_rng(int(s)).random(8) for s in seeds])
    perm = np.stack([np.random.default_rng(int(s)).permutation(4) for s in seeds])
    save("rng.npz", seeds=seeds, raw=raw, u32_endpoint=u32e, his=his, ints=ints, binom=binom,
         uniform=unif, random=rand, perm4=perm)


# --------------------------------------------------------------------------- maps
def make_maps():
    fm = refload.load("envs.floor_map")
    out = {}
    for m, n in ((32, 64), (64, 32), (16, 16)):
        ds = fm.FloorMapDatasetRooms(m, m)
        idx = np.array(list(range(n - 3)) + [123456789, 2**32 - 1, 4000000000], dtype=np.uint64)
        out[f"rooms{m}_idx"] = idx
        out[f"rooms{m}_bits"] = np.packbits(np.stack([ds.get_data_point(int(i)) for i in idx]), axis=-1)
    for m, n in ((21, 32), (63, 4), (127, 3)):
        ds = fm.FloorMapDatasetMaze(m, m)
        idx = np.array(list(range(n - 1)) + [2**32 - 1], dtype=np.uint64)
        out[f"maze{m}_idx"] = idx
        out[f"maze{m}_bits"] = np.packbits(np.stack([ds.get_data_point(int(i)) for i in idx]), axis=-1)
    save("maps.npz", **out)


# --------------------------------------------------------------------------- loss
def make_loss():
    refload.load_core()
    lf = refload.load("loss_fn")
    are = refload.load("active_regression_env")
    rng = np.random.default_rng(5)
    mse, _ = are._make_mse_loss_fn_and_target_space(2, -1, 1, None)
    pred = rng.uniform(-1.5, 1.5, (512, 2)).astype(np.float32)
    tgt = rng.uniform(-1, 1, (512, 2)).astype(np.float32)
    mse_out = np.stack([mse(p, t, ()) for p, t in zip(pred, tgt)])
    out = dict(mse_pred=pred, mse_target=tgt, mse_loss=mse_out)
    for k in (10, 200):
        ce = lf.CrossEntropyLossFn(k).normalized
        logits = rng.standard_normal((256, k)).astype(np.float32) * 3
        labels = rng.integers(0, k, 256).astype(np.int32)
        out[f"ce{k}_logits"] = logits
        out[f"ce{k}_labels"] = labels
        out[f"ce{k}_loss"] = np.asarray(ce(logits, labels, (256,)))
    save("loss.npz", **out)


# --------------------------------------------------------------------------- lidar
def _lidar_module():
    refload.load_core()
    return refload.load("envs.lidar_localization2d")


def make_lidar_scan():
    lmod = _lidar_module()
    fm = refload.load("envs.floor_map")
    Env = lmod.LIDARLocalization2DEnv
    rng = np.random.default_rng(11)
    maps, segs, dist = [], [], []
    ds = fm.FloorMapDatasetRooms(32, 32)
    env = Env(dataset=ds, static_map=True, lidar_beam_count=8, prefetch=False)
    scan = env._LIDARLocalization2DEnv__lidar_scan
    set_map = env._LIDARLocalization2DEnv__set_map
    map_sources = [fm.FloorMapDatasetRooms(32, 32).get_data_point(i) for i in (0, 1, 2)]
    # a hand-made map with pinch points (diagonal touches), a 1-cell hole and isolated cells
    hand = np.zeros((32, 32), bool)
    hand[0, :] = hand[-1, :] = hand[:, 0] = hand[:, -1] = True
    hand[10, 10] = hand[11, 11] = hand[12, 10] = True
    hand[20:23, 20:23] = True
    hand[21, 21] = False
    hand[5, 5] = hand[6, 7] = hand[5, 9] = hand[15:17, 3:5] = True
    map_sources.append(hand)
    for mi, m in enumerate(map_sources):
        set_map(m, mi)
        free = np.argwhere(~m)
        for k in range(700):
            cy, cx = free[rng.integers(len(free))]
            mode = k % 7
            if mode == 0:  # cell centre, beam directions like the env (incl. exact diagonals)
                p = np.array([cx, cy], np.float32) + 0.5
                ang = np.linspace(-np.pi, np.pi, 8, dtype=np.float32, endpoint=False)
                d = np.stack([np.cos(ang), np.sin(ang)], -1) * 5
                q = p + d[k % 8]
            elif mode == 1:  # lattice / half-lattice start, axis or diagonal direction
                p = (np.array([cx, cy], np.float32) + rng.integers(0, 3, 2).astype(np.float32) * 0.5)
                d = np.array([[1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [1, -1], [-1, -1],
                              [2, 1], [1, -2]], np.float32)[rng.integers(10)]
                q = p + d * np.float32(rng.integers(1, 6))
            elif mode == 2:  # short moves (<= 1) from generic positions
                p = np.array([cx, cy], np.float32) + rng.uniform(0, 1, 2).astype(np.float32)
                q = p + rng.uniform(-1, 1, 2).astype(np.float32)
            elif mode == 3:  # start exactly on a wall boundary line
                p = np.array([cx + rng.integers(0, 2), cy + rng.uniform(0, 1)], np.float32)
                q = p + rng.uniform(-5, 5, 2).astype(np.float32)
            elif mode == 4:  # integer endpoints (corner-to-corner)
                p = np.array([cx, cy], np.float32) + rng.integers(0, 2, 2).astype(np.float32)
                q = p + rng.integers(-5, 6, 2).astype(np.float32)
            else:  # generic beams of length 5
                p = np.array([cx, cy], np.float32) + rng.uniform(0, 1, 2).astype(np.float32)
                a = rng.uniform(-np.pi, np.pi)
                q = p + (np.array([np.cos(a), np.sin(a)]) * 5).astype(np.float32)
            p = p.astype(np.float32)
            q = q.astype(np.float32)
            if np.array_equal(p, q):
                continue
            dd, _ = scan(p, q[None])
            maps.append(mi)
            segs.append(np.concatenate([p, q]))
            dist.append(dd[0])
    save("lidar_scan.npz", maps=np.packbits(np.stack(map_sources), axis=-1), map_hw=np.array([32, 32]),
         map_index=np.array(maps, np.int32), segments=np.stack(segs).astype(np.float32),
         distance=np.array(dist, np.float32))


def _reset_prediction_info_shim(ap):
    """Generation harness for the LIDAR "-sparse" fixtures only.  The reference's SparsifyWrapper.reset
    reads info["prediction"]["target"] (sparsify_wrapper.py:128-135, 160), which
    LIDARLocalization2DEnv.reset does not return (lidar_localization2d.py:315), so the reference's
    LIDARLoc*-sparse ids raise KeyError in reset.  This wrapper, placed below SparsifyWrapper, adds
    info["prediction"] = {"target": None} to reset infos so that the wrapper's unmodified step can
    be recorded.  Step infos pass through untouched."""

    class ResetPredictionInfo(ap.ActivePerceptionWrapper):
        def reset(self, **kwargs):
            obs, info = self.env.reset(**kwargs)
            info["prediction"] = {"target": None}
            return obs, info

    return ResetPredictionInfo


def run_lidar_env(name, dataset, static, beams, n_envs, steps, seed, action_mode, sparse=False, static_map_index=0,
                  extra=None):
    lmod = _lidar_module()
    gym = sys.modules["gymnasium"]
    ap = sys.modules["ap_gym"]
    sw = refload.load("sparsify_wrapper") if sparse else None

    def mk():
        env = lmod.LIDARLocalization2DEnv(dataset=dataset, static_map=static, lidar_beam_count=beams,
                                          prefetch=False, static_map_index=static_map_index)
        env = ap.TimeLimit(env, max_episode_steps=100, issue_termination=True)
        env = ap.ActiveRegressionLogWrapper(env)
        # the "-sparse" ids (registration.py:115-142): SparsifyWrapper over the registered composition
        return sw.SparsifyWrapper(_reset_prediction_info_shim(ap)(env)) if sparse else env

    venv = gym.vector.SyncVectorEnv([mk for _ in range(n_envs)])
    obs, info = venv.reset(seed=seed)
    arng = np.random.default_rng(1)
    if action_mode == "uniform":
        actions = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    elif action_mode == "wide":
        actions = arng.uniform(-2.5, 2.5, (steps, n_envs, 2)).astype(np.float32)
    else:  # "grid": axis/diagonal half-steps keep positions on lattice and half-lattice lines
        choices = np.array([[0.5, 0], [-0.5, 0], [0, 0.5], [0, -0.5], [0.5, 0.5], [-0.5, 0.5], [0.5, -0.5],
                            [-0.5, -0.5], [1, 0], [0, -1], [0, 0]], np.float32)
        actions = choices[arng.integers(0, len(choices), (steps, n_envs))]
    preds = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    if sparse:  # overflowing squared errors: loss inf, and inf * weight 0 is NaN in the sparse reward
        preds[5::7, 0] = np.float32(1e20)
    rec = {k: [] for k in ("weight",) if sparse}
    rec.update({k: [] for k in ("lidar", "odometry", "time_step", "map", "reward", "terminated", "truncated",
                           "base_reward", "target", "loss", "info_mask", "stats_mask", "stats_avg_euclidean_distance",
                           "stats_avg_mse", "stats_final_euclidean_distance", "stats_final_mse",
                           "stats_len")})
    vec = {"euclidean_distance": [], "mse": []}  # ActiveRegressionLogWrapper "vector" lists, concatenated
    reset_obs = obs
    reset_map_idx = np.asarray(info["map_idx"], dtype=np.int64)
    for t in range(steps):
        obs, rew, term, trunc, info = venv.step({"action": actions[t], "prediction": preds[t]})
        rec["lidar"].append(obs["lidar"])
        rec["odometry"].append(obs["odometry"])
        rec["time_step"].append(obs["time_step"])
        if "map" in obs:
            rec["map"].append(np.packbits(obs["map"][..., 0] > 0, axis=-1))
        rec["reward"].append(rew)
        rec["terminated"].append(term)
        rec["truncated"].append(trunc)
        mask = info.get("_base_reward", np.zeros(n_envs, bool))
        rec["info_mask"].append(mask)
        rec["base_reward"].append(np.where(mask, info.get("base_reward", np.zeros(n_envs, np.float32)), 0))
        tgt = info["prediction"]["target"] if "prediction" in info else None
        if sparse and tgt is not None:
            w = np.asarray(tgt["weight"])
            # (autoreset envs carry the shim's reset info too; only the stepped envs are recorded)
            assert w.dtype == np.float64 and np.all(tgt["_weight"][mask])
            rec["weight"].append(np.where(mask, w, 0.0))
            tgt = np.stack([np.zeros(2, np.float32) if v is None else v for v in tgt["target"]])
        elif sparse:
            rec["weight"].append(np.zeros(n_envs))
        rec["target"].append(np.where(mask[:, None], tgt if tgt is not None
                                      else np.zeros((n_envs, 2), np.float32), 0).astype(np.float32))
        rec["loss"].append(np.where(mask, info["prediction"]["loss"] if "loss" in info.get("prediction", {})
                                    else np.zeros(n_envs, np.float32), 0).astype(np.float32))
        smask = info.get("_stats", np.zeros(n_envs, bool))
        rec["stats_mask"].append(smask)
        lens = np.zeros(n_envs, np.int32)
        for key in ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse"):
            v = info["stats"]["scalar"][key] if smask.any() else np.zeros(n_envs)
            assert not smask.any() or v.dtype == np.float64
            rec["stats_" + key].append(np.where(smask, v, 0.0))
        for i in np.nonzero(smask)[0]:
            for key in vec:
                lst = info["stats"]["vector"][key][i]
                assert all(type(x) is np.float32 for x in lst)
                vec[key].extend(lst)
            lens[i] = len(info["stats"]["vector"]["mse"][i])
        rec["stats_len"].append(lens)
    arrays = {k: np.stack(v) for k, v in rec.items() if v}
    for key, v in vec.items():
        arrays["stats_vector_" + key] = np.array(v, np.float32)
    arrays["reward_dtype"] = np.array(str(rew.dtype))
    arrays["base_reward_dtype"] = np.array(str(np.asarray(info.get("base_reward", np.zeros(1, np.float32))).dtype))
    arrays["lidar_dtype"] = np.array(str(obs["lidar"].dtype))
    save(f"lidar_env_{name}.npz", actions=actions, predictions=preds, seed=np.array(seed),
         reset_lidar=reset_obs["lidar"], reset_odometry=reset_obs["odometry"],
         reset_time_step=reset_obs["time_step"], reset_map_idx=reset_map_idx,
         reset_map=(np.packbits(reset_obs["map"][..., 0] > 0, axis=-1) if "map" in reset_obs
                    else np.zeros(0, np.uint8)), **arrays, **(extra or {}))


def fixed_floor_maps(n=37, h=40, w=48, seed=2024, open_every=0):
    """The maps of the custom-dataset fixtures: walls, blocks and scattered cells; map 7 has 6 free cells.  With
    open_every = k every k-th map has no border (agents walk off it: early terminations).  Only square maps may be
    open: for H != W the reference's __get_obs raises IndexError once a scan point passes the map edge
    (lidar_localization2d.py:254-259 compares (x, y) with map.shape = (h, w))."""
    rng = np.random.default_rng(seed)
    maps = np.zeros((n, h, w), bool)
    for i in range(n):
        m = maps[i]
        if not open_every or i % open_every != open_every - 1:
            m[0, :] = m[-1, :] = m[:, 0] = m[:, -1] = True
        for _ in range(int(rng.integers(2, 9))):
            y, x = int(rng.integers(0, h)), int(rng.integers(0, w))
            if rng.random() < 0.5:  # a wall line
                if rng.random() < 0.5:
                    m[y, x:x + int(rng.integers(3, 30))] = True
                else:
                    m[y:y + int(rng.integers(3, 30)), x] = True
            else:  # a block
                m[y:y + int(rng.integers(1, 8)), x:x + int(rng.integers(1, 8))] = True
        m |= rng.random((h, w)) < 0.02
    maps[7] = True
    maps[7, h // 2:h // 2 + 2, w // 2:w // 2 + 3] = False
    return maps


def make_pool():
    """LIDAR envs over a user FloorMapDataset subclass (floor_map_dataset.py:10-22): the DatasetIterator draws
    integers(0, len(dataset)) (dataset_iterator.py:26-32), any H x W."""
    fm = refload.load("envs.floor_map")
    maps = fixed_floor_maps()

    class FixedFloorMaps(fm.FloorMapDataset):
        def __init__(self, m):
            super().__init__(m.shape[2], m.shape[1])
            self._m = m

        def _get_length(self):
            return len(self._m)

        def get_data_point(self, idx):
            return self._m[int(idx)].copy()

        def get_data_point_batch(self, idx):
            return self._m[np.asarray(idx)].copy()

    def extra(m):
        return dict(pool_bits=np.packbits(m, axis=-1), pool_hw=np.array(m.shape[1:]))

    def first_seed(fn, seeds):
        """fn(seed) for the first seed whose reference run does not raise IndexError: for H != W the reference's
        __get_obs indexes observation_map with scan points it bounds-checks against the swapped shape
        (lidar_localization2d.py:254-259), which raises once a non-occluded scan point passes the bottom edge
        (the "touch plus crossing is no hit" beams pass through the border wall)."""
        for sd in seeds:
            try:
                return fn(sd)
            except IndexError as e:
                print("seed", sd, "raised IndexError in the reference:", e)
        raise RuntimeError("no seed ran through")

    first_seed(lambda sd: run_lidar_env("pool48x40_b16", FixedFloorMaps(maps), False, 16, 8, 110, sd, "wide",
                                        extra=extra(maps)), range(5, 40))
    first_seed(lambda sd: run_lidar_env("pool48x40_static_b8", FixedFloorMaps(maps), True, 8, 6, 60, sd, "uniform",
                                        static_map_index=5, extra=extra(maps)), range(2, 40))
    open_maps = fixed_floor_maps(23, 36, 36, seed=7, open_every=3)
    run_lidar_env("pool36_open_b8", FixedFloorMaps(open_maps), False, 8, 12, 110, 11, "wide", extra=extra(open_maps))


def make_lidar_env():
    fm = refload.load("envs.floor_map")
    run_lidar_env("rooms_static_b16", fm.FloorMapDatasetRooms(), True, 16, 16, 210, 0, "uniform")
    run_lidar_env("rooms_static_b8_grid", fm.FloorMapDatasetRooms(), True, 8, 16, 120, 3, "grid")
    run_lidar_env("rooms64_b32", fm.FloorMapDatasetRooms(64, 64), False, 32, 6, 110, 0, "wide")
    run_lidar_env("maze21_b8", fm.FloorMapDatasetMaze(), False, 8, 8, 110, 7, "uniform")
    run_lidar_env("maze21_b8_grid", fm.FloorMapDatasetMaze(), False, 8, 8, 60, 9, "grid")
    run_lidar_env("maze127_b64", fm.FloorMapDatasetMaze(127, 127), False, 64, 2, 25, 0, "uniform")


# --------------------------------------------------------------------------- image envs
def _image_modules():
    pkg = refload.load_core()
    v2s = refload.load("vector_to_single_wrapper")
    for k, v in vars(v2s).items():
        if not k.startswith("_"):
            setattr(pkg, k, v)
    return (refload.load("envs.image.image_perception_module"), refload.load("envs.image.image_classification_dataset"),
            refload.load("envs.image_classification"), refload.load("envs.image_localization"))


def run_image_env(name, kind, pool_shape, channels, num_classes, sensor, scale, step_limit, invert, n_envs,
                  steps, seed, pool_len, pool_seed, sparse=False):
    ipm, icd, ic, il = _image_modules()
    prng = np.random.default_rng(pool_seed)
    pool = prng.integers(0, 256, (pool_len, *pool_shape), dtype=np.uint8)
    # smooth a little so glimpses differ in structured ways (ties in uniqueness are rare either way)
    labels = prng.integers(0, num_classes, pool_len).astype(np.int64)

    class PoolDataset(icd.ImageClassificationDataset):
        def _get_length(self):
            return pool_len

        def _get_num_classes(self):
            return num_classes

        def _get_num_channels(self):
            return channels

        def _get_data_point_batch(self, idx):
            return pool[np.asarray(idx)], labels[np.asarray(idx)]

    cfg = ipm.ImagePerceptionConfig(dataset=PoolDataset(), sensor_size=sensor, sensor_scale=scale,
                                    step_limit=step_limit, prefetch=False, randomly_invert_labels=invert)
    env = (ic.ImageClassificationVectorEnv if kind == "cls" else il.ImageLocalizationVectorEnv)(n_envs, cfg)
    # the registered ids wrap the vector env in the vector log wrapper (registration.py:185-192, 263-269)
    ap = sys.modules["ap_gym"]
    env = (ap.ActiveClassificationVectorLogWrapper if kind == "cls" else ap.ActiveRegressionVectorLogWrapper)(env)
    if sparse:  # the "-sparse" ids (registration.py:115-142)
        env = refload.load("sparsify_wrapper").SparsifyVectorWrapper(env)
    out = {"pool": pool, "labels": labels,
           "config": np.array([pool_shape[0], pool_shape[1], channels, num_classes, sensor[0], sensor[1],
                               step_limit, int(invert), n_envs, steps], np.int64),
           "sensor_scale": np.array(scale, np.float64), "kind": np.array(kind)}
    _trace_image_env(env, kind, n_envs, num_classes, steps, seed, sparse, out)
    save(f"image_{name}.npz", **out)


def _trace_image_env(env, kind, n_envs, num_classes, steps, seed, sparse, out, mask_prediction=False):
    """Reset with `seed`, step with seeded actions/predictions, record every output into `out`."""
    obs, info = env.reset(seed=seed)
    arng = np.random.default_rng(11)
    actions = arng.uniform(-1.5, 1.5, (steps, n_envs, 2)).astype(np.float32)
    if kind == "cls":
        preds = arng.standard_normal((steps, n_envs, num_classes)).astype(np.float32)
    else:
        preds = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    if sparse:  # infinite losses: inf * weight 0 is NaN in the sparse reward
        if kind == "cls":
            preds[2::5, 0, 1:] = -np.inf
        else:
            preds[2::5, 0] = np.float32(1e20)
    out.update(actions=actions, predictions=preds, seed=np.array(seed))
    for k, v in obs.items():
        out[f"reset_{k}"] = np.asarray(v)
    out["reset_index"] = np.asarray(info["index"], np.int64)
    rec = {}
    for t in range(steps):
        pred_t = () if mask_prediction else preds[t]
        obs, rew, term, trunc, info = env.step({"action": actions[t], "prediction": pred_t})
        fields = dict(obs)
        tgt = info["prediction"]["target"]
        if sparse:
            fields["weight"] = np.asarray(tgt["weight"])
            tgt = tgt["target"]
        if mask_prediction:
            assert tgt == ()
            tgt = np.zeros(0)
        fields.update(reward=rew, terminated=term, truncated=trunc, index=np.asarray(info["index"], np.int64),
                      base_reward=np.asarray(info["base_reward"]), target=np.asarray(tgt),
                      loss=np.asarray(info["prediction"]["loss"]))
        for k, v in fields.items():
            v = np.asarray(v)
            rec.setdefault(k, []).append(v)
            rec.setdefault(k + "_dtype", []).append(str(v.dtype))
        # vector log wrapper statistics (active_{classification,regression}_env.py, util.py:40-80)
        smask = np.asarray(info["stats"]["_scalar"]) if "stats" in info else np.zeros(n_envs, bool)
        rec.setdefault("stats_mask", []).append(smask)
        if smask.any():
            st = info["stats"]
            for key, val in st["scalar"].items():
                out.setdefault(f"stats_t{t}_scalar_{key}", np.asarray(val))
            for key, val in st["vector"].items():
                if key.startswith("_"):
                    out[f"stats_t{t}_vector_{key}"] = np.asarray(val)
                else:
                    assert all(type(x) is np.float32 for lst in val for x in lst)
                    out[f"stats_t{t}_vector_{key}_len"] = np.array([len(lst) for lst in val], np.int32)
                    out[f"stats_t{t}_vector_{key}"] = np.array([x for lst in val for x in lst], np.float32)
    for k, v in rec.items():
        out["step_" + k] = np.array(v) if k.endswith("_dtype") else np.stack(v)
    env.close()


def make_image_env():
    run_image_env("cls_mnist", "cls", (28, 28), 1, 10, (5, 5), 1.0, 16, False, 8, 40, 0, 40, 100)
    run_image_env("cls_tin", "cls", (64, 64, 3), 3, 200, (10, 10), 1.0, 16, False, 4, 20, 3, 12, 101)
    run_image_env("cls_gray3_rect", "cls", (20, 24), 3, 4, (5, 5), 1.5, 8, True, 6, 30, 5, 16, 102)
    run_image_env("loc_mnist", "loc", (28, 28), 1, 10, (5, 5), 1.0, 16, False, 6, 40, 1, 30, 103)
    run_image_env("loc_tin12", "loc", (64, 64, 3), 3, 200, (12, 12), 1.0, 16, False, 2, 20, 4, 6, 104)
    run_image_env("loc_rect", "loc", (24, 20, 3), 3, 5, (4, 4), 1.25, 6, False, 4, 16, 9, 10, 105)


def make_sparse_env():
    """The "-sparse" ids (registration.py:115-142): SparsifyWrapper / SparsifyVectorWrapper."""
    fm = refload.load("envs.floor_map")
    run_lidar_env("maze21_b8_sparse", fm.FloorMapDatasetMaze(), False, 8, 8, 110, 7, "uniform", sparse=True)
    run_image_env("cls_mnist_sparse", "cls", (28, 28), 1, 10, (5, 5), 1.0, 16, False, 8, 40, 0, 40, 100, sparse=True)
    run_image_env("loc_rect_sparse", "loc", (24, 20, 3), 3, 5, (4, 4), 1.25, 6, False, 4, 16, 9, 10, 105,
                  sparse=True)


# --------------------------------------------------------------------------- CircleSquare family
def _circle_square_modules():
    ipm, icd, ic, il = _image_modules()
    csd = refload.load("envs.image.circle_square_dataset")
    return ipm, ic, csd


def make_circle_square():
    """circle_square_dataset.py renders (sampled data points of every registered shape) and traces of
    the CircleSquare ids (registration.py:358-512), incl. CircleSquareHideAndSeekVectorWrapper."""
    ipm, ic, csd = _circle_square_modules()
    out = {}
    rng = np.random.default_rng(21)
    cases = [("cs28g", csd.CircleSquareDataset(image_shape=(28, 28), show_gradient=True)),
             ("cs20n", csd.CircleSquareDataset(image_shape=(20, 20), show_gradient=False)),
             ("cs15g", csd.CircleSquareDataset(image_shape=(15, 15), show_gradient=True)),
             ("csrect", csd.CircleSquareDataset(image_shape=(12, 17), show_gradient=True, object_extents=5)),
             ("dcs15g", csd.DoubleCircleSquareDataset(image_shape=(15, 15))),
             ("dcs15n", csd.DoubleCircleSquareDataset(image_shape=(15, 15), show_gradient_a=False,
                                                      show_gradient_b=False)),
             ("dcs15ab", csd.DoubleCircleSquareDataset(image_shape=(15, 15), show_gradient_a=True,
                                                       show_gradient_b=False)),
             ("dcs20g", csd.DoubleCircleSquareDataset(image_shape=(20, 20))),
             ("dcs28g", csd.DoubleCircleSquareDataset(image_shape=(28, 28)))]
    for name, ds in cases:
        n = len(ds)
        idx = np.unique(np.concatenate([np.arange(min(n, 8)), [n - 1, n // 2],
                                        rng.integers(0, n, 56)])).astype(np.int64)
        imgs, labels = ds.get_data_point_batch(idx)
        out[f"{name}_len"] = np.array(n, np.int64)
        out[f"{name}_idx"] = idx
        out[f"{name}_images"] = np.asarray(imgs, np.float32)
        out[f"{name}_labels"] = np.asarray(labels, np.int32)
        if isinstance(ds, csd.CircleSquareDataset):
            pos, lab = ds.get_object_position_and_label(idx)
            out[f"{name}_obj_pos"] = np.asarray(pos, np.int64)
            out[f"{name}_obj_label"] = np.asarray(lab, np.int64)
    save("circle_square_data.npz", **out)

    ap = sys.modules["ap_gym"]
    hs = refload.load("envs.circle_square_catch_or_flee")
    sp = refload.load("sparsify_wrapper")

    def trace(name, ds, step_limit, invert, n_envs, steps, seed, wrap=None, sparse=False, mask=False,
              log=True):
        cfg = ipm.ImagePerceptionConfig(dataset=ds, step_limit=step_limit, prefetch=False,
                                        randomly_invert_labels=invert)
        env = ic.ImageClassificationVectorEnv(n_envs, cfg)
        if wrap is not None:
            env = wrap(env)
        if log:
            env = ap.ActiveClassificationVectorLogWrapper(env)
        if sparse:
            env = sp.SparsifyVectorWrapper(env)
        k = ds.num_classes
        res = {"config": np.array([step_limit, int(invert), n_envs, steps, k], np.int64)}
        _trace_image_env(env, "cls", n_envs, k, steps, seed, sparse, res, mask_prediction=mask)
        save(f"cs_env_{name}.npz", **res)

    trace("cs28", csd.CircleSquareDataset(image_shape=(28, 28)), 16, False, 6, 36, 0)
    trace("csinv15n", csd.CircleSquareDataset(image_shape=(15, 15), show_gradient=False), 16, True, 5, 36, 3)
    trace("dcs15", csd.DoubleCircleSquareDataset(image_shape=(15, 15)), 16, False, 5, 20, 4)
    trace("hs28", csd.CircleSquareDataset(image_shape=(28, 28)), 32, False, 6, 70, 5,
          wrap=hs.CircleSquareHideAndSeekVectorWrapper)
    trace("hs28_sparse", csd.CircleSquareDataset(image_shape=(28, 28)), 32, False, 4, 40, 6,
          wrap=hs.CircleSquareHideAndSeekVectorWrapper, sparse=True)
    # the NoPrediction variant: the reference's reset raises KeyError('prediction') (its reset info has
    # no "prediction" entry, circle_square_catch_or_flee.py:61-64); record that
    env = hs.CircleSquareHideAndSeekVectorWrapper(
        ic.ImageClassificationVectorEnv(3, ipm.ImagePerceptionConfig(dataset=csd.CircleSquareDataset(), step_limit=32,
                                                                     prefetch=False)), mask_prediction=True)
    try:
        env.reset(seed=0)
        reset_error = ""
    except KeyError as e:
        reset_error = f"KeyError:{e.args[0]}"
    save("cs_env_hs_noprediction_reset.npz", reset_error=np.array(reset_error))


# --------------------------------------------------------------------------- LightDark
def run_light_dark(name, n_envs, steps, seed, action_scale, sparse=False):
    """LightDark-v0 as registered (registration.py:640-647): TimeLimit(50, issue_termination=True) +
    ActiveRegressionLogWrapper over LightDarkEnv, vectorised by the SyncVectorEnv restatement."""
    ap = refload.load_core()
    ld = refload.load("envs.light_dark")
    gym = sys.modules["gymnasium"]
    sw = refload.load("sparsify_wrapper") if sparse else None

    def mk():
        env = ap.TimeLimit(ld.LightDarkEnv(), max_episode_steps=50, issue_termination=True)
        env = ap.ActiveRegressionLogWrapper(env)
        return sw.SparsifyWrapper(_reset_prediction_info_shim(ap)(env)) if sparse else env

    venv = gym.vector.SyncVectorEnv([mk for _ in range(n_envs)])
    obs, info = venv.reset(seed=seed)
    arng = np.random.default_rng(2)
    actions = arng.uniform(-action_scale, action_scale, (steps, n_envs, 2)).astype(np.float32)
    preds = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    if sparse:
        preds[5::7, 0] = np.float32(1e20)
    out = {"actions": actions, "predictions": preds, "seed": np.array(seed),
           "reset_noisy_position": obs["noisy_position"], "reset_time_step": obs["time_step"],
           "reset_info_keys": np.array(sorted(info.keys()), dtype=str)}
    rec = {}
    vec = {"euclidean_distance": [], "mse": []}
    for t in range(steps):
        obs, rew, term, trunc, info = venv.step({"action": actions[t], "prediction": preds[t]})
        mask = info.get("_base_reward", np.zeros(n_envs, bool))
        fields = {"noisy_position": obs["noisy_position"], "time_step": obs["time_step"], "reward": rew,
                  "terminated": term, "truncated": trunc, "info_mask": mask,
                  "base_reward": np.where(mask, info.get("base_reward", np.zeros(n_envs, np.float32)), 0)
                  .astype(np.float32)}
        tgt = info["prediction"]["target"] if "prediction" in info else None
        if sparse:
            w = np.asarray(tgt["weight"]) if tgt is not None else np.zeros(n_envs)
            fields["weight"] = np.where(mask, w, 0.0)
            tgt = (np.stack([np.zeros(2, np.float32) if v is None else v for v in tgt["target"]])
                   if tgt is not None else None)
        fields["target"] = np.where(mask[:, None], tgt if tgt is not None else np.zeros((n_envs, 2), np.float32),
                                    0).astype(np.float32)
        fields["loss"] = np.where(mask, info["prediction"]["loss"] if "loss" in info.get("prediction", {})
                                  else np.zeros(n_envs, np.float32), 0).astype(np.float32)
        smask = info.get("_stats", np.zeros(n_envs, bool))
        fields["stats_mask"] = smask
        lens = np.zeros(n_envs, np.int32)
        for key in ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse"):
            v = info["stats"]["scalar"][key] if smask.any() else np.zeros(n_envs)
            fields["stats_" + key] = np.where(smask, v, 0.0)
        for i in np.nonzero(smask)[0]:
            for key in vec:
                lst = info["stats"]["vector"][key][i]
                assert all(type(x) is np.float32 for x in lst)
                vec[key].extend(lst)
            lens[i] = len(info["stats"]["vector"]["mse"][i])
        fields["stats_len"] = lens
        for k, v in fields.items():
            rec.setdefault(k, []).append(np.asarray(v))
    for k, v in rec.items():
        out["step_" + k] = np.stack(v)
    for key, v in vec.items():
        out["stats_vector_" + key] = np.array(v, np.float32)
    out["reward_dtype"] = np.array(str(rew.dtype))
    save(f"light_dark_{name}.npz", **out)


def make_light_dark():
    run_light_dark("n8", 8, 130, 0, 1.0)
    run_light_dark("n6_wide", 6, 120, 5, 3.0)
    run_light_dark("n5_sparse", 5, 110, 2, 2.0, sparse=True)


# --------------------------------------------------------------------------- render
def run_lidar_render(name, dataset, static, beams, n_envs, steps, seed, render_at):
    """Frames of the reference's LIDARLocalization2DEnv.render() (lidar_localization2d.py:391-494) for every
    sub-env of the registered composition, after reset (step 0) and after the steps in `render_at`."""
    lmod = _lidar_module()
    gym = sys.modules["gymnasium"]
    ap = sys.modules["ap_gym"]

    def mk():
        env = lmod.LIDARLocalization2DEnv(dataset=dataset, static_map=static, lidar_beam_count=beams, prefetch=False)
        return ap.TimeLimit(env, max_episode_steps=100, issue_termination=True)

    venv = gym.vector.SyncVectorEnv([mk for _ in range(n_envs)])
    venv.reset(seed=seed)
    arng = np.random.default_rng(4)
    actions = arng.uniform(-1.5, 1.5, (steps, n_envs, 2)).astype(np.float32)
    preds = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    frames = []
    if 0 in render_at:
        frames.append(np.stack([e.render() for e in venv.envs]))
    for t in range(steps):
        venv.step({"action": actions[t], "prediction": preds[t]})
        if t + 1 in render_at:
            frames.append(np.stack([e.render() for e in venv.envs]))
    save(f"render_lidar_{name}.npz", actions=actions, predictions=preds, seed=np.array(seed),
         render_at=np.array(sorted(render_at)), frames=np.stack(frames))


def run_light_dark_render(name, n_envs, steps, seed, action_scale, render_at):
    """Frames of the reference's LightDarkEnv.render() (light_dark.py:152-243) for every sub-env of
    TimeLimit(50, issue_termination=True) over LightDarkEnv, after reset (step 0) and the steps in render_at."""
    ap = refload.load_core()
    ld = refload.load("envs.light_dark")
    gym = sys.modules["gymnasium"]
    venv = gym.vector.SyncVectorEnv([lambda: ap.TimeLimit(ld.LightDarkEnv(), max_episode_steps=50,
                                                          issue_termination=True) for _ in range(n_envs)])
    venv.reset(seed=seed)
    arng = np.random.default_rng(6)
    actions = arng.uniform(-action_scale, action_scale, (steps, n_envs, 2)).astype(np.float32)
    preds = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    frames = []
    if 0 in render_at:
        frames.append(np.stack([e.render() for e in venv.envs]))
    for t in range(steps):
        venv.step({"action": actions[t], "prediction": preds[t]})
        if t + 1 in render_at:
            frames.append(np.stack([e.render() for e in venv.envs]))
    save(f"render_light_dark_{name}.npz", actions=actions, predictions=preds, seed=np.array(seed),
         render_at=np.array(sorted(render_at)), frames=np.stack(frames))


def run_image_render(name, kind, pool_shape, channels, num_classes, sensor, scale, step_limit, n_envs, steps, seed,
                     pool_len, pool_seed, opacity, render_at):
    """Frames of the reference's ImageClassificationVectorEnv / ImageLocalizationVectorEnv render()
    (image_perception_module.py:333-401, image_localization.py:183-223) on a synthetic uint8 pool, after
    reset (step 0) and the steps in render_at (crossing the batch autoreset)."""
    ipm, icd, ic, il = _image_modules()
    prng = np.random.default_rng(pool_seed)
    pool = prng.integers(0, 256, (pool_len, *pool_shape), dtype=np.uint8)
    labels = prng.integers(0, num_classes, pool_len).astype(np.int64)

    class PoolDataset(icd.ImageClassificationDataset):
        def _get_length(self):
            return pool_len

        def _get_num_classes(self):
            return num_classes

        def _get_num_channels(self):
            return channels

        def _get_data_point_batch(self, idx):
            return pool[np.asarray(idx)], labels[np.asarray(idx)]

    kw = {} if opacity is None else dict(render_unvisited_opacity=opacity[0], render_visited_opacity=opacity[1])
    cfg = ipm.ImagePerceptionConfig(dataset=PoolDataset(), sensor_size=sensor, sensor_scale=scale,
                                    step_limit=step_limit, prefetch=False, **kw)
    env = (ic.ImageClassificationVectorEnv if kind == "cls" else il.ImageLocalizationVectorEnv)(n_envs, cfg)
    env.reset(seed=seed)
    arng = np.random.default_rng(12)
    actions = arng.uniform(-1.5, 1.5, (steps, n_envs, 2)).astype(np.float32)
    if kind == "cls":
        preds = (arng.standard_normal((steps, n_envs, num_classes)) * 2).astype(np.float32)
    else:
        preds = arng.uniform(-1, 1, (steps, n_envs, 2)).astype(np.float32)
    frames = [env.render()] if 0 in render_at else []
    for t in range(steps):
        env.step({"action": actions[t], "prediction": preds[t]})
        if t + 1 in render_at:
            frames.append(env.render())
    save(f"render_image_{name}.npz", pool=pool, labels=labels,
         config=np.array([channels, num_classes, sensor[0], sensor[1], step_limit, n_envs], np.int64),
         sensor_scale=np.array(scale, np.float64), kind=np.array(kind),
         opacity=np.array(opacity if opacity is not None else (0.0, 0.3), np.float64), actions=actions,
         predictions=preds, seed=np.array(seed), render_at=np.array(sorted(render_at)), frames=np.stack(frames))


def run_circle_square_render(name, double, shape, step_limit, n_envs, steps, seed, render_at):
    """render() frames of CircleSquareHideAndSeek over ImageClassificationVectorEnv on the procedural
    CircleSquare / DoubleCircleSquare datasets (float32 images), registered render opacities."""
    ipm, ic, csd = _circle_square_modules()
    hs = refload.load("envs.circle_square_catch_or_flee")
    ds = csd.DoubleCircleSquareDataset(image_shape=shape) if double else csd.CircleSquareDataset(image_shape=shape)
    cfg = ipm.ImagePerceptionConfig(dataset=ds, step_limit=step_limit, prefetch=False, render_unvisited_opacity=0.5,
                                    render_visited_opacity=0.25)
    env = ic.ImageClassificationVectorEnv(n_envs, cfg)
    if not double:
        env = hs.CircleSquareHideAndSeekVectorWrapper(env)
    env.reset(seed=seed)
    arng = np.random.default_rng(13)
    actions = arng.uniform(-1.5, 1.5, (steps, n_envs, 2)).astype(np.float32)
    preds = (arng.standard_normal((steps, n_envs, ds.num_classes)) * 2).astype(np.float32)
    frames = [env.render()] if 0 in render_at else []
    for t in range(steps):
        env.step({"action": actions[t], "prediction": preds[t]})
        if t + 1 in render_at:
            frames.append(env.render())
    save(f"render_cs_{name}.npz", config=np.array([int(double), shape[0], shape[1], step_limit, n_envs], np.int64),
         actions=actions, predictions=preds, seed=np.array(seed), render_at=np.array(sorted(render_at)),
         frames=np.stack(frames))


def make_render():
    run_circle_square_render("hs28", False, (28, 28), 6, 3, 9, 3, {0, 2, 6, 7, 9})
    run_circle_square_render("dcs15", True, (15, 15), 4, 2, 6, 1, {0, 3, 5})
    run_image_render("cls_mnist", "cls", (28, 28), 1, 10, (5, 5), 1.0, 8, 3, 12, 0, 20, 200, (0.5, 0.25),
                     {0, 1, 5, 8, 9, 12})
    run_image_render("cls_gray3_rect", "cls", (20, 24), 3, 4, (5, 5), 1.5, 6, 2, 9, 5, 10, 201, None, {0, 3, 6, 7})
    run_image_render("loc_tin12", "loc", (64, 64, 3), 3, 200, (12, 12), 1.0, 5, 2, 8, 4, 6, 202, (0.5, 0.25),
                     {0, 2, 5, 6, 8})
    run_light_dark_render("n3", 3, 54, 2, 1.5, {0, 1, 2, 20, 50, 51, 54})
    fm = refload.load("envs.floor_map")
    run_lidar_render("rooms32_b8", fm.FloorMapDatasetRooms(32, 32), False, 8, 3, 104, 5, {0, 1, 2, 40, 100, 101, 104})
    run_lidar_render("maze21_b16_static", fm.FloorMapDatasetMaze(), True, 16, 2, 30, 9, {0, 3, 30})


# --------------------------------------------------------------------------- HF data ingestion
def write_hf_parquet(root, images, labels, label_names, splits):
    """A local Hugging Face dataset directory (data/<split>-00000-of-00001.parquet, PNG-encoded images,
    ClassLabel labels) that `datasets.load_dataset(root)` loads offline.  Shared with tests/test_host.py
    (which rebuilds the same directory from the fixture's arrays)."""
    from datasets import ClassLabel, Dataset, Features, Image

    feats = Features({"image": Image(), "label": ClassLabel(names=list(label_names))})
    os.makedirs(os.path.join(root, "data"), exist_ok=True)
    start = 0
    for split, n in splits:
        ims = [images[i] for i in range(start, start + n)]
        Dataset.from_dict({"image": ims, "label": [int(v) for v in labels[start:start + n]]}, features=feats).to_parquet(
            os.path.join(root, "data", f"{split}-00000-of-00001.parquet"))
        start += n


def make_hf():
    """The reference's HuggingfaceImageClassificationDataset (huggingface_image_classification_dataset.py)
    on small local datasets: lengths, class counts, filter_labels remapping and processed batches."""
    import tempfile

    refload.load_core()
    hf = refload.load("envs.image.huggingface_image_classification_dataset")
    out = {}
    rng = np.random.default_rng(21)
    for name, shape, channels in (("rgb", (9, 7, 3), 3), ("grey", (8, 8), 1), ("grey_to_rgb", (8, 8), 3)):
        images = rng.integers(0, 256, (18, *shape), dtype=np.uint8)
        labels = rng.integers(0, 5, 18)
        names = ["zero", "one", "two", "three", "four"]
        out[f"{name}_images"], out[f"{name}_labels"] = images, labels
        out[f"{name}_channels"] = np.array(channels)
        with tempfile.TemporaryDirectory() as root:
            write_hf_parquet(root, images, labels, names, (("train", 12), ("test", 6)))
            for split in ("train", "test"):
                for filt in (None, ["three", "one"]):
                    ds = hf.HuggingfaceImageClassificationDataset(root, channels=channels, split=split,
                                                                  filter_labels=filt)
                    ds.load()
                    key = f"{name}_{split}_{'filt' if filt else 'all'}"
                    idx = np.arange(len(ds))[::-1]
                    imgs, labs = ds.get_data_point_batch(idx)
                    out[key + "_len"] = np.array(len(ds))
                    out[key + "_num_classes"] = np.array(ds.num_classes)
                    out[key + "_idx"] = idx
                    out[key + "_batch_images"] = np.asarray(imgs)
                    out[key + "_batch_labels"] = np.asarray(labs)
    save("hf_dataset.npz", **out)


def make_stream():
    """LIDAR envs over a user FloorMapDataset of len 2**32 whose maps come from default_rng(idx) (tests/stream_maps.py):
    too large for any pool, the backend streams it (get_data_point at every draw, like the reference's DatasetIterator,
    dataset_iterator.py:26-32).  The fixture records the maps of every reset (reset_map / map) and their indices."""
    fm = refload.load("envs.floor_map")
    sys.path.insert(0, os.path.dirname(HERE))
    from stream_maps import STREAM_LEN, rng_floor_map

    class RngFloorMaps(fm.FloorMapDataset):
        def __init__(self):
            super().__init__(40, 40)

        def _get_length(self):
            return STREAM_LEN

        def get_data_point(self, idx):
            return rng_floor_map(int(idx))

        def get_data_point_batch(self, idx):
            return np.stack([rng_floor_map(int(i)) for i in idx])

    run_lidar_env("stream40_b16", RngFloorMaps(), False, 16, 64, 110, 42, "wide")


SECTIONS = {"rng": make_rng, "maps": make_maps, "loss": make_loss, "scan": make_lidar_scan,
            "lidar": make_lidar_env, "image": make_image_env,
            "sparse": make_sparse_env, "circle_square": make_circle_square,
            "light_dark": make_light_dark, "render": make_render, "hf": make_hf, "pool": make_pool,
            "stream": make_stream}


def main(argv):
    sys.setrecursionlimit(200000)
    threading.stack_size(1024 * 1024 * 1024)
    names = argv or list(SECTIONS)
    err = []

    def run():
        try:
            for n in names:
                SECTIONS[n]()
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            raise

    th = threading.Thread(target=run)
    th.start()
    th.join()
    if err:
        raise SystemExit(1)


if __name__ == "__main__":
    main(sys.argv[1:])
