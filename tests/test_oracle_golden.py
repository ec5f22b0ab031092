"""The oracle (oracle/liboracle.so) against the golden fixtures made from the reference.

CPU only.  These pin the restatement before it is trusted as the checker of the HIP kernels:
  rng.npz        numpy 2.2.6 itself
  maps.npz       reference FloorMapDatasetRooms/Maze
  lidar_scan.npz reference __lidar_scan + exact-rational GEOS model
  lidar_env_*    reference LIDARLocalization2DEnv + TimeLimit + SyncVectorEnv composition
"""

import numpy as np
import pytest

from conftest import check_image_stats, golden

ENV_CASES = {
    "rooms_static_b16": ("rooms", 32, True, 16),
    "rooms_static_b8_grid": ("rooms", 32, True, 8),
    "rooms64_b32": ("rooms", 64, False, 32),
    "maze21_b8": ("maze", 21, False, 8),
    "maze21_b8_grid": ("maze", 21, False, 8),
    "maze127_b64": ("maze", 127, False, 64),
    "maze21_b8_sparse": ("maze", 21, False, 8),  # LIDARLocMaze-sparse-v0 (SparsifyWrapper per sub-env)
    # a user FloorMapDataset subclass of fixed maps (48 wide x 40 high; 36 x 36 with open borders)
    "pool48x40_b16": ("pool", 0, False, 16),
    "pool48x40_static_b8": ("pool", 0, True, 8),
    "pool36_open_b8": ("pool", 0, False, 8),
    # a user FloorMapDataset of len 2**32, maps from default_rng(idx) (tests/stream_maps.py): fetched per draw
    "stream40_b16": ("stream", 0, False, 16),
}
POOL_STATIC_INDEX = 5  # make_golden.make_pool's static_map_index


def pool_maps(d) -> np.ndarray:
    """The fixture's dataset maps, bool [len, H, W]."""
    h, w = (int(x) for x in d["pool_hw"])
    return np.unpackbits(d["pool_bits"], axis=-1)[..., :w].astype(bool).reshape(-1, h, w)


def _draws(O, seed, kind, a=0, b=0, p=0.0, n=8):
    out = np.zeros(n)
    O.lib().orc_test_draws(int(seed), kind, a, b, p, n, out.ctypes.data)
    return out


def test_rng_matches_numpy(oracle_mod):
    g = golden("rng.npz")
    for i, s in enumerate(g["seeds"]):
        assert np.array_equal(_draws(oracle_mod, s, 0, n=16), g["raw"][i].astype(np.float64))
        assert _draws(oracle_mod, s, 4, n=1)[0] == g["u32_endpoint"][i][0]
        for j, hi in enumerate(g["his"]):
            assert np.array_equal(_draws(oracle_mod, s, 3, 0, int(hi)), g["ints"][i, j].astype(np.float64))
        for n in range(9):
            assert np.array_equal(_draws(oracle_mod, s, 5, n, 0, 0.3), g["binom"][i, n].astype(np.float64))
        assert np.array_equal(_draws(oracle_mod, s, 6, -1, 1), g["uniform"][i])
        assert np.array_equal(_draws(oracle_mod, s, 2), g["random"][i])


@pytest.mark.parametrize("kind,size", [("rooms", 32), ("rooms", 64), ("rooms", 16), ("maze", 21), ("maze", 63),
                                       ("maze", 127)])
def test_maps_match_reference(oracle_mod, kind, size):
    g = golden("maps.npz")
    idx = g[f"{kind}{size}_idx"]
    ref = np.unpackbits(g[f"{kind}{size}_bits"], axis=-1)[..., :size].astype(bool)
    for i, k in enumerate(idx):
        m = oracle_mod.rooms_map(int(k), size) if kind == "rooms" else oracle_mod.maze_map(int(k), size)
        assert np.array_equal(m.astype(bool), ref[i]), f"{kind}{size} idx={k}"


def test_maze_even_size_raises(oracle_mod):
    with pytest.raises(ValueError):
        oracle_mod.maze_map(0, 128)


def test_scan_matches_reference_model(oracle_mod):
    g = golden("lidar_scan.npz")
    h, w = (int(x) for x in g["map_hw"])
    maps = np.unpackbits(g["maps"], axis=-1)[..., :w].astype(np.uint8)
    kinds = np.zeros(6, int)
    got = np.zeros(len(g["distance"]), np.float32)
    for i, (mi, seg) in enumerate(zip(g["map_index"], g["segments"])):
        got[i], k = oracle_mod.lidar_scan(maps[mi], seg[:2], seg[2:])
        kinds[k] += 1
    assert np.array_equal(got, g["distance"])
    # the fixture exercises every GEOS result type the reference branches on
    assert (kinds > 0).all(), kinds


@pytest.mark.parametrize("name", sorted(ENV_CASES))
def test_vector_env_trace(oracle_mod, name):
    kind, size, static, beams = ENV_CASES[name]
    d = golden(f"lidar_env_{name}.npz")
    n = d["actions"].shape[1]
    sparse = name.endswith("_sparse")
    if kind == "pool":
        env = oracle_mod.OracleLidarVectorEnv(n, "pool", 0, static, POOL_STATIC_INDEX if static else 0, beams,
                                              pool=pool_maps(d))
    elif kind == "stream":
        from stream_maps import STREAM_LEN, rng_floor_map

        env = oracle_mod.OracleLidarVectorEnv(n, "stream", 0, False, 0, beams, map_fn=rng_floor_map,
                                              map_len=STREAM_LEN, map_hw=(40, 40))
    else:
        env = oracle_mod.OracleLidarVectorEnv(n, kind, size, static, 0, beams, sparse=sparse)
    env.reset(int(d["seed"]))
    assert np.array_equal(env.lidar, d["reset_lidar"])
    assert np.array_equal(env.odometry, d["reset_odometry"])
    assert np.array_equal(env.time_step, d["reset_time_step"])
    assert np.array_equal(env.map_idx.astype(np.int64), d["reset_map_idx"])
    for t in range(d["actions"].shape[0]):
        env.step(d["actions"][t], d["predictions"][t])
        for key, got in (("lidar", env.lidar), ("odometry", env.odometry), ("time_step", env.time_step),
                         ("reward", env.reward), ("terminated", env.terminated.astype(bool)),
                         ("truncated", env.truncated.astype(bool)), ("base_reward", env.base_reward),
                         ("target", env.target), ("loss", env.loss), ("info_mask", env.info_mask.astype(bool))):
            assert np.array_equal(got, d[key][t], equal_nan=got.dtype.kind == "f"), f"{name} step {t} {key}"
        if sparse:
            assert np.array_equal(env.weight, d["weight"][t]), f"{name} step {t} weight"
        if not static:
            assert np.array_equal(np.packbits(env.map > 0, axis=-1), d["map"][t]), f"{name} step {t} map"
    assert str(d["reward_dtype"]) == "float64" and str(d["base_reward_dtype"]) == "float32"


IMAGE_CASES = ["cls_mnist", "cls_tin", "cls_gray3_rect", "loc_mnist", "loc_tin12", "loc_rect",
               "cls_mnist_sparse", "loc_rect_sparse"]  # *_sparse: SparsifyVectorWrapper over the log wrapper


@pytest.mark.parametrize("name", IMAGE_CASES)
def test_image_oracle_matches_reference_trace(name):
    """oracle/image_oracle.py against the reference's own image envs (tests/golden/image_*.npz)."""
    from oracle import image_oracle as io

    g = golden(f"image_{name}.npz")
    h, w, c, k, s0, s1, lim, inv, n, steps = (int(v) for v in g["config"])
    env = io.ImageVectorEnvOracle(str(g["kind"]), g["pool"], g["labels"], k, c, n, (s0, s1),
                                  float(g["sensor_scale"]), lim, invert=bool(inv), sparse=name.endswith("_sparse"))
    obs, info = env.reset(int(g["seed"]))
    for key, v in obs.items():
        assert np.array_equal(v, g["reset_" + key]) and v.dtype == g["reset_" + key].dtype, key
    assert np.array_equal(info["index"], g["reset_index"])
    for t in range(steps):
        with np.errstate(invalid="ignore", over="ignore"):
            obs, rew, term, trunc, info = env.step(g["actions"][t], g["predictions"][t])
        tgt = info["prediction"]["target"]
        fields = dict(obs, reward=rew, terminated=term, truncated=trunc, index=info["index"],
                      base_reward=info["base_reward"], loss=info["prediction"]["loss"])
        if isinstance(tgt, dict):
            fields.update(target=tgt["target"], weight=tgt["weight"])
        else:
            fields["target"] = tgt
        assert set(k for k in fields) == set(k[5:] for k in g.files if k.startswith("step_") and
                                             not k.endswith("_dtype") and k != "step_stats_mask")
        for key, v in fields.items():
            v = np.asarray(v)
            assert np.array_equal(v, g["step_" + key][t], equal_nan=v.dtype.kind == "f"), (t, key)
            assert str(v.dtype) == g["step_" + key + "_dtype"][t], (t, key)
        assert ("stats" in info) == bool(g["step_stats_mask"][t].any())
        if "stats" in info:
            check_image_stats(info["stats"], g, t)


def test_pairwise_sum_matches_numpy_mean():
    """The restated pairwise order is the one np.mean uses over a contiguous float32 block."""
    from oracle import image_oracle as io

    rng = np.random.default_rng(0)
    for shape in ((5, 5, 1), (12, 12, 3), (10, 10, 3), (3, 3, 1), (129,), (1000,), (4, 4, 3)):
        x = rng.random((64, *shape)).astype(np.float32) ** 2
        want = np.mean(x, axis=tuple(range(1, x.ndim)))
        n = int(np.prod(shape))
        got = (np.float32(0) + io.pairwise_sum_f32(x.reshape(64, n))) / np.float32(n)
        assert np.array_equal(got, want), shape


# ---------------------------------------------------------------------------- CircleSquare family
CS_DATA_CASES = {  # golden prefix: (kind, shape, show_gradient_a, show_gradient_b, object_extents)
    "cs28g": ("single", (28, 28), True, True, 8), "cs20n": ("single", (20, 20), False, False, 8),
    "cs15g": ("single", (15, 15), True, True, 8), "csrect": ("single", (12, 17), True, True, 5),
    "dcs15g": ("double", (15, 15), True, True, 8), "dcs15n": ("double", (15, 15), False, False, 8),
    "dcs15ab": ("double", (15, 15), True, False, 8), "dcs20g": ("double", (20, 20), True, True, 8),
    "dcs28g": ("double", (28, 28), True, True, 8),
}


@pytest.mark.parametrize("name", sorted(CS_DATA_CASES))
def test_circle_square_oracle_matches_reference_renders(name):
    from oracle import image_oracle as io

    g = golden("circle_square_data.npz")
    kind, shape, ga, gb, ext = CS_DATA_CASES[name]
    if kind == "double":
        assert int(g[f"{name}_len"]) == 4 * len(io.circle_square_positions(shape, ext))
    else:
        assert int(g[f"{name}_len"]) == 2 * shape[0] * shape[1]
    imgs, labels = io.circle_square_images(kind, shape, g[f"{name}_idx"], ga, gb, ext)
    assert np.array_equal(imgs, g[f"{name}_images"])
    assert np.array_equal(labels, g[f"{name}_labels"])


def test_circle_square_host_api_matches_reference():
    """Index packing and get_object_position_and_label of the product's dataset classes (host logic)."""
    import ap_gym_amd as ap

    g = golden("circle_square_data.npz")
    for name, (kind, shape, ga, gb, ext) in CS_DATA_CASES.items():
        if kind == "single":
            ds = ap.CircleSquareDataset(show_gradient=ga, image_shape=shape, object_extents=ext)
            pos, lab = ds.get_object_position_and_label(g[f"{name}_idx"])
            assert np.array_equal(pos, g[f"{name}_obj_pos"]) and np.array_equal(lab, g[f"{name}_obj_label"])
        else:
            ds = ap.DoubleCircleSquareDataset(ga, gb, image_shape=shape, object_extents=ext)
        assert len(ds) == int(g[f"{name}_len"]) and ds.num_classes == (2 if kind == "single" else 3)
        assert ds._unpack(ds._pack([1, 0, 3])) == [1, 0, 3]


def test_hide_and_seek_oracle_matches_reference_autoreset_steps():
    """On the batch autoreset step the inner base_reward is float64 zeros, so the reference's
    info["base_reward"] is exactly the additional reward."""
    from oracle import image_oracle as io

    g = golden("cs_env_hs28.npz")
    lim = int(g["config"][0])
    for t in (lim, 2 * lim + 1):
        assert str(g["step_base_reward_dtype"][t]) == "float64"
        add = io.hide_and_seek_additional_reward(g["step_index"][t], g["step_glimpse_pos"][t], (28, 28), (5, 5), 1.0)
        assert np.array_equal(add, g["step_base_reward"][t])


# ---------------------------------------------------------------------------- LightDark
LIGHT_DARK_CASES = {"n8": False, "n6_wide": False, "n5_sparse": True}


def check_light_dark_step(g, t, got, rtol=0.0):
    """One step of a LightDark vector env (oracle or GPU, numpy-mode dict form) against the fixture."""
    for key in ("noisy_position", "time_step", "reward", "terminated", "truncated", "info_mask"):
        assert np.array_equal(got[key], g["step_" + key][t], equal_nan=got[key].dtype.kind == "f"), (t, key)
    m = g["step_info_mask"][t]
    for key in ("base_reward", "loss"):
        assert np.array_equal(np.where(m, got[key], 0), g["step_" + key][t], equal_nan=True), (t, key)
    assert np.array_equal(np.where(m[:, None], got["target"], 0), g["step_target"][t]), t
    if "step_weight" in g.files:
        assert np.array_equal(np.where(m, got["weight"], 0.0), g["step_weight"][t]), t
    assert np.array_equal(got["stats_len"], g["step_stats_len"][t]), t
    names = ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse")
    for j, key in enumerate(names):
        assert np.array_equal(np.where(got["stats_len"] > 0, got["stats"][j], 0.0), g["step_stats_" + key][t]), (t, key)


@pytest.mark.parametrize("name", sorted(LIGHT_DARK_CASES))
def test_light_dark_oracle_matches_reference_trace(name):
    from oracle.light_dark_oracle import LightDarkVectorOracle

    g = golden(f"light_dark_{name}.npz")
    steps, n = g["actions"].shape[:2]
    ref = LightDarkVectorOracle(n, 50, sparse=LIGHT_DARK_CASES[name])
    obs = ref.reset(int(g["seed"]))
    assert np.array_equal(obs["noisy_position"], g["reset_noisy_position"])
    assert np.array_equal(obs["time_step"], g["reset_time_step"])
    vec = {"euclidean_distance": [], "mse": []}
    for t in range(steps):
        out = ref.step(g["actions"][t], g["predictions"][t])
        check_light_dark_step(g, t, out)
        for i in sorted(out["stats_vectors"]):
            ed, ms = out["stats_vectors"][i]
            vec["euclidean_distance"] += ed
            vec["mse"] += ms
    for key, v in vec.items():
        assert np.array_equal(np.array(v, np.float32), g["stats_vector_" + key]), key
