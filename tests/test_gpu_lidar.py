"""GPU parity: the HIP kernels (through the C ABI) against the golden fixtures and the oracle.

Bar: bit-exact for integer work (RNG, maps, flags, indices) and for every float output (the kernels
restate numpy/GEOS arithmetic operation by operation; the north_star tolerance of 1e-6 is not used
because nothing needs it).
"""

import ctypes

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ENV_CASES = {
    "rooms_static_b16": ("rooms", 32, True, 16),
    "rooms_static_b8_grid": ("rooms", 32, True, 8),
    "rooms64_b32": ("rooms", 64, False, 32),
    "maze21_b8": ("maze", 21, False, 8),
    "maze21_b8_grid": ("maze", 21, False, 8),
    "maze127_b64": ("maze", 127, False, 64),
    "maze21_b8_sparse": ("maze", 21, False, 8),  # LIDARLocMaze-sparse-v0 (SparsifyWrapper per sub-env)
    # a user FloorMapDataset subclass (make_golden.make_pool): the resident map pool (APG_MAP_POOL)
    "pool48x40_b16": ("pool", 0, False, 16),
    "pool48x40_static_b8": ("pool", 0, True, 8),
    "pool36_open_b8": ("pool", 0, False, 8),
}
POOL_STATIC_INDEX = 5  # make_golden.make_pool's static_map_index


class UserFloorMaps:
    """Stand-in for a user subclass of the reference's FloorMapDataset (floor_map_dataset.py:10-22, not importable
    on the GPU box): the interface the reference env uses -- map_width / map_height, load, __len__,
    get_data_point(idx) -> bool [H, W].  The backend sees it through ForeignFloorMapView."""

    def __init__(self, maps):
        self._m = np.asarray(maps, dtype=bool)
        self.loads = 0

    @property
    def map_width(self):
        return self._m.shape[2]

    @property
    def map_height(self):
        return self._m.shape[1]

    def load(self):
        self.loads += 1

    def __len__(self):
        return len(self._m)

    def get_data_point(self, idx):
        return self._m[int(idx)].copy()


def pool_maps(d) -> np.ndarray:
    h, w = (int(x) for x in d["pool_hw"])
    return np.unpackbits(d["pool_bits"], axis=-1)[..., :w].astype(bool).reshape(-1, h, w)


def _ds(ap, kind, size, d=None):
    if kind == "pool":
        return UserFloorMaps(pool_maps(d))
    return ap.FloorMapDatasetRooms(size, size) if kind == "rooms" else ap.FloorMapDatasetMaze(size, size)


def test_device_rng_matches_numpy(gpu):
    import torch

    from ap_gym_amd import _native as N

    g = golden("rng.npz")
    seeds = torch.as_tensor(g["seeds"].view(np.int64), device=gpu)
    m = len(g["seeds"])

    def draws(kind, a=0, b=0, n=8):
        out = torch.zeros((m, n), dtype=torch.float64, device=gpu)
        N.check(N.lib().apg_rng_draws(N.ptr(seeds), m, kind, a, b, n, N.ptr(out), N.stream_handle(gpu)))
        return out.cpu().numpy()

    assert np.array_equal(draws(0, n=16), g["raw"].astype(np.float64))
    assert np.array_equal(draws(4, n=1), g["u32_endpoint"].astype(np.float64))
    assert np.array_equal(draws(2), g["random"])
    for j, hi in enumerate(g["his"]):
        assert np.array_equal(draws(3, 0, int(hi)), g["ints"][:, j].astype(np.float64)), hi
    for n in range(9):
        assert np.array_equal(draws(5, n), g["binom"][:, n].astype(np.float64)), n


@pytest.mark.parametrize("kind,size", [("rooms", 32), ("rooms", 64), ("rooms", 16), ("maze", 21), ("maze", 63),
                                       ("maze", 127)])
def test_device_maps_match_reference(gpu, kind, size):
    import ap_gym_amd as ap

    g = golden("maps.npz")
    ref = np.unpackbits(g[f"{kind}{size}_bits"], axis=-1)[..., :size].astype(bool)
    got = _ds(ap, kind, size).get_data_point_batch(g[f"{kind}{size}_idx"], device=gpu)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("kind,size,count", [("rooms", 64, 4096), ("rooms", 32, 2048), ("maze", 127, 256),
                                             ("maze", 21, 2048)])
def test_device_maps_match_oracle_random_idx(gpu, oracle_mod, kind, size, count):
    import ap_gym_amd as ap

    idx = np.random.default_rng(size).integers(0, 2**32, count).astype(np.uint64)
    got = _ds(ap, kind, size).get_data_point_batch(idx, device=gpu)
    for i in range(0, count, max(1, count // 256)):
        m = oracle_mod.rooms_map(int(idx[i]), size) if kind == "rooms" else oracle_mod.maze_map(int(idx[i]), size)
        assert np.array_equal(got[i], m.astype(bool)), (kind, size, int(idx[i]))


@pytest.mark.parametrize("h,w,bp,count", [(21, 21, 0.5, 512), (21, 35, 0.0, 512), (63, 63, 0.3, 256),
                                           (127, 127, 0.7, 64), (3, 3, 1.0, 16), (127, 9, 1.0, 64),
                                           (255, 255, 1.0, 32), (255, 101, 0.6, 32), (301, 301, 1.0, 16),
                                           (257, 9, 0.5, 32), (11, 511, 1.0, 16), (301, 275, 0.4, 8)])
def test_device_maze_branching_matches_oracle(gpu, oracle_mod, h, w, bp, count):
    """branching_prob < 1 (rng.random() draws decide later branches; mazes need not be perfect, so the
    stream consumption differs from the bp = 1 mazes the stream length is sized for) and odd rectangles."""
    import ap_gym_amd as ap

    idx = np.random.default_rng(h * w).integers(0, 2**32, count).astype(np.uint64)
    got = ap.FloorMapDatasetMaze(w, h, branching_prob=bp).get_data_point_batch(idx, device=gpu)
    for i in range(count):
        assert np.array_equal(got[i], oracle_mod.maze_map(int(idx[i]), h, w, bp).astype(bool)), (h, w, bp, int(idx[i]))


def test_device_maze_stream_overflow_matches_oracle(gpu, oracle_mod, tmp_path):
    """APG_MAZE_STREAM_GROUPS=8 (256 precomputed outputs per maze instead of ~7400 at 127 x 127): every maze
    draws past its precomputed stream and the DFS steps the LCG from the stored state, in a child process
    (the library reads the knob once)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "maps.npy"
    code = (f"import sys, numpy as np; sys.path.insert(0, {os.path.join(root, 'active-perception-gym_amd')!r}); "
            "import ap_gym_amd as ap; "
            "idx = np.random.default_rng(5).integers(0, 2**32, 96).astype(np.uint64); "
            "m = np.concatenate([ap.FloorMapDatasetMaze(s, s, branching_prob=bp).get_data_point_batch(idx[:32], "
            "device='cuda:0').reshape(32, -1) for s, bp in ((127, 1.0), (63, 0.5), (21, 1.0))], axis=1); "
            f"np.save({str(out)!r}, m)")
    env = {k: v for k, v in os.environ.items() if not k.startswith("APG_")}
    env["APG_MAZE_STREAM_GROUPS"] = "8"
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    got = np.load(out)
    idx = np.random.default_rng(5).integers(0, 2**32, 96).astype(np.uint64)
    for i in range(32):
        ref = np.concatenate([oracle_mod.maze_map(int(idx[i]), s, s, bp).astype(bool).reshape(-1)
                              for s, bp in ((127, 1.0), (63, 0.5), (21, 1.0))])
        assert np.array_equal(got[i], ref), int(idx[i])


@pytest.mark.parametrize("size,max_rooms,door_width", [(128, 17, 3), (128, 10, 3), (96, 17, 2), (48, 6, 4),
                                                       (160, 24, 3), (200, 32, 2), (255, 17, 3), (64, 24, 2),
                                                       (320, 48, 3), (511, 64, 2), (300, 40, 6), (257, 33, 1)])
def test_device_rooms_parameters_match_oracle(gpu, oracle_mod, size, max_rooms, door_width):
    import ap_gym_amd as ap

    idx = np.random.default_rng(size + max_rooms).integers(0, 2**32, 1024).astype(np.uint64)
    got = ap.FloorMapDatasetRooms(size, size, max_rooms=max_rooms, door_width=door_width).get_data_point_batch(
        idx, device=gpu)
    for i in range(0, 1024, 8):
        m = oracle_mod.rooms_map(int(idx[i]), size, max_rooms, door_width)
        assert np.array_equal(got[i], m.astype(bool)), (size, max_rooms, int(idx[i]))


def _scan_gpu(gpu, maps_bool, map_index, segs):
    import torch

    from ap_gym_amd import _native as N

    nm, h, w = maps_bool.shape
    wpr = (w + 63) // 64
    padded = np.zeros((nm, h, wpr * 64), np.uint8)
    padded[..., :w] = maps_bool
    words = np.packbits(padded, axis=-1, bitorder="little").view("<u8").astype(np.uint64)
    occ = torch.as_tensor(words.view(np.int64).copy(), device=gpu)
    mi = torch.as_tensor(np.asarray(map_index, np.int32), device=gpu)
    sg = torch.as_tensor(np.ascontiguousarray(segs, np.float32), device=gpu)
    n = len(segs)
    dist = torch.zeros(n, dtype=torch.float32, device=gpu)
    kind = torch.zeros(n, dtype=torch.int32, device=gpu)
    N.check(N.lib().apg_lidar_scan_batch(N.ptr(occ), N.ptr(mi), h, w, N.ptr(sg), n, N.ptr(dist), N.ptr(kind),
                                         N.stream_handle(gpu)))
    return dist.cpu().numpy(), kind.cpu().numpy()


def test_device_scan_matches_reference_model(gpu):
    g = golden("lidar_scan.npz")
    h, w = (int(x) for x in g["map_hw"])
    maps = np.unpackbits(g["maps"], axis=-1)[..., :w].astype(bool)
    dist, kinds = _scan_gpu(gpu, maps, g["map_index"], g["segments"])
    assert np.array_equal(dist, g["distance"])
    assert set(np.unique(kinds)) == set(range(6))


def test_device_scan_matches_oracle_degenerate_sweep(gpu, oracle_mod):
    """Random + lattice-aligned segments (corner touches, collinear runs) on 64x64 rooms and 127 mazes."""
    rng = np.random.default_rng(3)
    for kind, size in (("rooms", 64), ("maze", 127)):
        maps = np.stack([(oracle_mod.rooms_map(i, size) if kind == "rooms" else oracle_mod.maze_map(i, size))
                         for i in range(4)]).astype(bool)
        n = 40000
        mi = rng.integers(0, 4, n).astype(np.int32)
        p = rng.integers(0, size, (n, 2)).astype(np.float32) + rng.choice(
            np.array([0.0, 0.5, 0.25], np.float32), (n, 2))
        gen = rng.uniform(0, size, (n, 2)).astype(np.float32)
        p = np.where((np.arange(n) % 3 == 0)[:, None], gen, p)
        d = rng.choice(np.array([[5, 0], [0, 5], [-5, 0], [0, -5], [5, 5], [-5, 5], [3, -3], [1, 2], [-2, 1],
                                 [0.5, 0.5], [1, 0], [0, -1]], np.float32), n)
        d = np.where((np.arange(n) % 5 == 0)[:, None], rng.uniform(-5, 5, (n, 2)).astype(np.float32), d)
        q = (p + d).astype(np.float32)
        segs = np.concatenate([p, q], axis=1)
        dist, kinds = _scan_gpu(gpu, maps, mi, segs)
        for i in range(n):
            od, ok = oracle_mod.lidar_scan(maps[mi[i]], segs[i, :2], segs[i, 2:])
            assert od == dist[i] and ok == kinds[i], (kind, i, segs[i], od, dist[i], ok, kinds[i])


def test_device_scan_matches_oracle_generic_and_near_grid(gpu, oracle_mod):
    """The walk's fast path (p, q off the grid lines, no lattice crossing: runs of occupied cells decide
    LINE / MULTILINE / EMPTY) and its hand-over to the general walk: uniform segments up to 12 cells
    long on rooms, mazes and 35 %-noise maps (many runs: MULTILINE), endpoints one ulp off a grid line,
    directions one ulp off an axis or a diagonal, and segments through lattice points."""
    rng = np.random.default_rng(11)
    size = 64
    noise = [rng.random((size, size)) < 0.35 for _ in range(2)]
    maps = np.stack([oracle_mod.rooms_map(0, size), oracle_mod.rooms_map(1, size),
                     np.pad(oracle_mod.maze_map(2, size - 1), ((0, 1), (0, 1))), *noise]).astype(bool)
    n = 60000
    mi = rng.integers(0, len(maps), n).astype(np.int32)
    p = rng.uniform(14, size - 14, (n, 2)).astype(np.float32)
    ang = rng.uniform(0, 2 * np.pi, n)
    ln = rng.uniform(0.05, 12, n)
    d = np.stack([np.cos(ang) * ln, np.sin(ang) * ln], 1).astype(np.float32)
    k = np.arange(n) % 8
    # endpoints one ulp beside a grid line (either side), and exactly on one (general walk)
    up = np.nextafter(np.floor(p), np.float32(np.inf)).astype(np.float32)
    dn = np.nextafter(np.floor(p), np.float32(-np.inf)).astype(np.float32)
    p = np.where((k == 1)[:, None], up, p)
    p = np.where((k == 2)[:, None], dn, p)
    p = np.where((k == 3)[:, None], np.floor(p), p)
    # directions one ulp off an axis / the diagonal, and exact diagonals from lattice-aligned p
    tiny = np.float32(1e-7)
    d = np.where((k == 4)[:, None], np.stack([d[:, 0], np.full(n, tiny, np.float32)], 1), d)
    d = np.where((k == 5)[:, None], np.stack([ln.astype(np.float32), np.nextafter(ln.astype(np.float32), 0)], 1), d)
    p = np.where((k == 6)[:, None], (np.floor(p) + np.float32(0.5)), p)
    d = np.where((k == 6)[:, None], np.float32(3.0) * np.sign(d).astype(np.float32), d)
    # axis-parallel segments (the slide scans' shape): vertical / horizontal, from generic points, from
    # points with the travel coordinate on a grid line, and along a grid line (general walk)
    i = np.arange(n)
    sgn = np.where(rng.random(n) < 0.5, -1, 1).astype(np.float32)
    lf = (ln * sgn).astype(np.float32)
    zero = np.zeros(n, np.float32)
    d = np.where((i % 16 == 0)[:, None], np.stack([zero, lf], 1), d)
    d = np.where((i % 16 == 8)[:, None], np.stack([lf, zero], 1), d)
    p = np.where((i % 64 == 24)[:, None], np.stack([np.floor(p[:, 0]), p[:, 1]], 1), p)
    p = np.where((i % 64 == 48)[:, None], np.floor(p), p)
    q = (p + d).astype(np.float32)
    # q on a grid line (x, or both coordinates), and p on a grid line with a generic direction
    q = np.where((k == 7)[:, None], np.stack([np.floor(q[:, 0]), np.where(np.arange(n) % 16 == 7,
                                                                          np.floor(q[:, 1]), q[:, 1])], 1), q)
    segs = np.concatenate([p, q], axis=1).astype(np.float32)
    dist, kinds = _scan_gpu(gpu, maps, mi, segs)
    bad = []
    counts = np.zeros(6, int)
    for i in range(n):
        od, ok = oracle_mod.lidar_scan(maps[mi[i]], segs[i, :2], segs[i, 2:])
        counts[ok] += 1
        if not (od == dist[i] and ok == kinds[i]):
            bad.append((i, segs[i], od, dist[i], ok, kinds[i]))
    assert not bad, (len(bad), bad[:5])
    assert counts[1] > 1000 and counts[2] > 1000 and counts[0] > 1000, counts  # LINE, MULTILINE, EMPTY
    assert counts[3] > 0 and counts[5] > 0, counts  # POINT, COLLECTION (endpoints on the boundary)


@pytest.mark.parametrize("name", sorted(ENV_CASES))
def test_vector_env_matches_reference_trace(gpu, name):
    import ap_gym_amd as ap

    kind, size, static, beams = ENV_CASES[name]
    d = golden(f"lidar_env_{name}.npz")
    n = d["actions"].shape[1]
    sparse = name.endswith("_sparse")
    env = ap.LIDARLocalization2DVectorEnv(num_envs=n, dataset=_ds(ap, kind, size, d), static_map=static,
                                          lidar_beam_count=beams, device=gpu, log_stats=True, sparse=sparse,
                                          sparse_reset_info=sparse,
                                          static_map_index=POOL_STATIC_INDEX if kind == "pool" and static else 0)
    obs, info = env.reset(seed=int(d["seed"]))
    vec_off = 0
    assert np.array_equal(obs["lidar"], d["reset_lidar"])
    assert np.array_equal(obs["odometry"], d["reset_odometry"])
    assert np.array_equal(obs["time_step"], d["reset_time_step"])
    assert np.array_equal(info["map_idx"], d["reset_map_idx"])
    if not static:
        assert np.array_equal(np.packbits(obs["map"][..., 0] > 0, axis=-1), d["reset_map"])
    for t in range(d["actions"].shape[0]):
        obs, rew, term, trunc, info = env.step({"action": d["actions"][t], "prediction": d["predictions"][t]})
        assert rew.dtype == np.float64 and obs["lidar"].dtype == np.float32
        assert np.array_equal(obs["lidar"], d["lidar"][t]), (name, t)
        assert np.array_equal(obs["odometry"], d["odometry"][t]), (name, t)
        assert np.array_equal(obs["time_step"], d["time_step"][t]), (name, t)
        assert np.array_equal(rew, d["reward"][t], equal_nan=True), (name, t)
        assert np.array_equal(term, d["terminated"][t]) and np.array_equal(trunc, d["truncated"][t]), (name, t)
        mask = d["info_mask"][t]
        if mask.any():
            assert np.array_equal(info["_base_reward"], mask)
            assert np.array_equal(info["base_reward"], d["base_reward"][t]), (name, t)
            tgt = info["prediction"]["target"]
            if sparse:  # {"target", "_target", "weight" (float64), "_weight"} as SyncVectorEnv merges them
                assert np.array_equal(tgt["_target"], mask) and np.array_equal(tgt["_weight"], mask)
                assert tgt["weight"].dtype == np.float64 and np.array_equal(tgt["weight"], d["weight"][t]), (name, t)
                tgt = tgt["target"]
            assert np.array_equal(tgt, d["target"][t]), (name, t)
            assert np.array_equal(info["prediction"]["loss"], d["loss"][t]), (name, t)
        else:
            assert "base_reward" not in info
        if not static:
            assert np.array_equal(np.packbits(obs["map"][..., 0] > 0, axis=-1), d["map"][t]), (name, t)
            assert set(np.unique(obs["map"])) <= {np.float32(0), np.float32(1) / np.float32(255)}
        # ActiveRegressionLogWrapper episode statistics, merged by SyncVectorEnv
        smask = d["stats_mask"][t]
        if smask.any():
            assert np.array_equal(info["_stats"], smask)
            st = info["stats"]
            assert np.array_equal(st["_scalar"], smask) and np.array_equal(st["_vector"], smask)
            for key in ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse"):
                assert st["scalar"][key].dtype == np.float64
                assert np.array_equal(st["scalar"][key], d["stats_" + key][t]), (name, t, key)
                assert np.array_equal(st["scalar"]["_" + key], smask)
            for i in np.nonzero(smask)[0]:
                ln = int(d["stats_len"][t][i])
                for key in ("euclidean_distance", "mse"):
                    lst = st["vector"][key][i]
                    assert len(lst) == ln and all(type(x) is np.float32 for x in lst)
                    assert np.array_equal(np.array(lst), d["stats_vector_" + key][vec_off:vec_off + ln]), (name, t, i)
                vec_off += ln
        else:
            assert "stats" not in info
    assert vec_off == len(d["stats_vector_mse"])
    env.close()


@pytest.mark.parametrize("kind,size,beams,n,steps,sparse", [("rooms", 64, 32, 1024, 230, False),
                                                            ("maze", 21, 8, 1024, 120, False),
                                                            ("maze", 127, 64, 64, 40, False),
                                                            ("maze", 255, 32, 32, 110, False),
                                                            ("maze", 301, 32, 16, 110, False),
                                                            ("rooms", 32, 16, 512, 120, False),
                                                            ("rooms", 64, 32, 1024, 120, True)])
def test_vector_env_matches_oracle(gpu, oracle_mod, kind, size, beams, n, steps, sparse):
    import ap_gym_amd as ap

    env = ap.LIDARLocalization2DVectorEnv(num_envs=n, dataset=_ds(ap, kind, size), lidar_beam_count=beams,
                                          device=gpu, log_stats=True, sparse=sparse,
                                          sparse_reset_info=sparse)
    ref = oracle_mod.OracleLidarVectorEnv(n, kind, size, False, 0, beams, sparse=sparse)
    obs, _ = env.reset(seed=123)
    ref.reset(123)
    assert np.array_equal(obs["lidar"], ref.lidar)
    rng = np.random.default_rng(9)
    hist = [[] for _ in range(n)]  # ActiveRegressionLogWrapper metrics, restated per env
    for t in range(steps):
        a = rng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        if sparse:  # a few overflowing losses: inf * weight 0 is NaN in the sparse reward
            p[rng.random(n) < 0.01] = np.float32(3e19)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        ref.step(a, p)
        for i in np.nonzero(ref.info_mask)[0]:
            d = ref.target[i] - p[i]
            with np.errstate(over="ignore"):
                hist[i].append((np.linalg.norm(d), np.mean(d ** 2)))
        done = (ref.terminated | ref.truncated).astype(bool)
        assert np.array_equal(info.get("_stats", np.zeros(n, bool)), done), t
        for i in np.nonzero(done)[0]:
            ed = np.array([h[0] for h in hist[i]], np.float32)
            ms = np.array([h[1] for h in hist[i]], np.float32)
            sc = info["stats"]["scalar"]
            assert sc["avg_euclidean_distance"][i] == float(np.mean(ed)) and sc["final_mse"][i] == float(ms[-1])
            assert sc["avg_mse"][i] == float(np.mean(ms)) and sc["final_euclidean_distance"][i] == float(ed[-1])
            assert np.array_equal(np.array(info["stats"]["vector"]["mse"][i]), ms)
            hist[i] = []
        assert np.array_equal(obs["lidar"], ref.lidar), t
        assert np.array_equal(obs["odometry"], ref.odometry), t
        assert np.array_equal(obs["time_step"], ref.time_step), t
        assert np.array_equal(rew, ref.reward, equal_nan=True), t
        assert np.array_equal(term, ref.terminated.astype(bool)), t
        if sparse and "prediction" in info:
            m = ref.info_mask.astype(bool)
            assert np.array_equal(info["prediction"]["target"]["weight"][m], ref.weight[m]), t
        assert np.array_equal(obs["map"][..., 0], ref.map), t
    env.close()


@pytest.mark.parametrize("kind,size,static,beams,lidar_range,n", [("rooms", 64, False, 32, 8.0, 1024),
                                                                   ("rooms", 64, True, 32, 9.5, 512),
                                                                   ("rooms", 64, False, 16, 9.9, 512),
                                                                   ("rooms", 32, False, 16, 6.5, 512),
                                                                   ("maze", 63, False, 32, 9.0, 512),
                                                                   ("rooms", 64, False, 16, 12.0, 512),
                                                                   ("maze", 63, False, 32, 20.0, 256),
                                                                   ("rooms", 32, True, 8, 10.5, 256),
                                                                   ("rooms", 64, False, 8, 28.0, 128),
                                                                   ("rooms", 64, False, 8, 40.0, 128),
                                                                   ("maze", 63, False, 16, 60.0, 128),
                                                                   ("rooms", 128, False, 16, 45.5, 128)])
def test_long_range_matches_oracle(gpu, oracle_mod, kind, size, static, beams, lidar_range, n):
    """Ranges past the default 5: 6.5-10 (the staged-window instance with bounding boxes 9-12 rows tall, whose
    pre-test ORs the middle rows of the 4-row table) and > 10 (the rows-from-global-memory instance, 64-column row
    windows: ranges up to 60): observations, rewards and terminations of 110 steps (one autoreset) against the
    oracle env."""
    import ap_gym_amd as ap

    env = ap.LIDARLocalization2DVectorEnv(num_envs=n, dataset=_ds(ap, kind, size), lidar_beam_count=beams,
                                          lidar_range=lidar_range, static_map=static, device=gpu)
    ref = oracle_mod.OracleLidarVectorEnv(n, kind, size, static, 0, beams, lidar_range=lidar_range)
    obs, _ = env.reset(seed=11)
    ref.reset(11)
    assert np.array_equal(obs["lidar"], ref.lidar)
    rng = np.random.default_rng(4)
    for t in range(110):
        a = rng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        ref.step(a, p)
        assert np.array_equal(obs["lidar"], ref.lidar), t
        assert np.array_equal(obs["odometry"], ref.odometry), t
        assert np.array_equal(rew, ref.reward, equal_nan=True), t
        assert np.array_equal(term, ref.terminated.astype(bool)), t
        if not static:
            assert np.array_equal(obs["map"][..., 0], ref.map), t
    env.close()


@pytest.mark.parametrize("size,max_rooms,n", [(160, 24, 256), (130, 10, 256), (64, 24, 512), (320, 48, 32)])
def test_large_rooms_env_matches_oracle(gpu, oracle_mod, size, max_rooms, n):
    """Rooms maps past the fused step kernel's generator (maps > 128, max_rooms > 17: the autoresets run
    in k_lidar_reset before the unfused step kernel): 110 steps (one autoreset) against the oracle env."""
    import ap_gym_amd as ap

    env = ap.LIDARLocalization2DVectorEnv(num_envs=n, dataset=ap.FloorMapDatasetRooms(size, size, max_rooms=max_rooms),
                                          lidar_beam_count=16, device=gpu)
    ref = oracle_mod.OracleLidarVectorEnv(n, "rooms", size, False, 0, 16, max_rooms=max_rooms)
    obs, _ = env.reset(seed=21)
    ref.reset(21)
    assert np.array_equal(obs["lidar"], ref.lidar)
    assert np.array_equal(obs["map"][..., 0], ref.map)
    rng = np.random.default_rng(6)
    for t in range(110):
        a = rng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        ref.step(a, p)
        assert np.array_equal(obs["lidar"], ref.lidar), t
        assert np.array_equal(obs["odometry"], ref.odometry), t
        assert np.array_equal(rew, ref.reward, equal_nan=True), t
        assert np.array_equal(term, ref.terminated.astype(bool)), t
        assert np.array_equal(obs["map"][..., 0], ref.map), t
    env.close()


@pytest.mark.parametrize("step_limit,n,steps", [(1200, 64, 1210), (969, 32, 975)])
def test_long_episode_stats_match_oracle(gpu, oracle_mod, step_limit, n, steps):
    """log_stats past 968 steps (the episode-end pairwise sums of k_episode_stats, seven split levels):
    the ActiveRegressionLogWrapper scalars of every episode end against numpy's means of the restated
    per-step metrics, the observations against the oracle env."""
    import ap_gym_amd as ap

    env = ap.LIDARLocalization2DVectorEnv(num_envs=n, dataset=_ds(ap, "rooms", 32), lidar_beam_count=8, device=gpu,
                                          log_stats=True, max_episode_steps=step_limit)
    ref = oracle_mod.OracleLidarVectorEnv(n, "rooms", 32, False, 0, 8, step_limit=step_limit)
    env.reset(seed=7)
    ref.reset(7)
    rng = np.random.default_rng(3)
    hist = [[] for _ in range(n)]
    ends = 0
    for t in range(steps):
        a = rng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        ref.step(a, p)
        for i in np.nonzero(ref.info_mask)[0]:
            d = ref.target[i] - p[i]
            hist[i].append((np.linalg.norm(d), np.mean(d ** 2)))
        done = (ref.terminated | ref.truncated).astype(bool)
        assert np.array_equal(info.get("_stats", np.zeros(n, bool)), done), t
        for i in np.nonzero(done)[0]:
            ed = np.array([h[0] for h in hist[i]], np.float32)
            ms = np.array([h[1] for h in hist[i]], np.float32)
            sc = info["stats"]["scalar"]
            assert sc["avg_euclidean_distance"][i] == float(np.mean(ed)) and sc["final_mse"][i] == float(ms[-1])
            assert sc["avg_mse"][i] == float(np.mean(ms)) and sc["final_euclidean_distance"][i] == float(ed[-1])
            hist[i] = []
            ends += 1
        assert np.array_equal(obs["lidar"], ref.lidar), t
        assert np.array_equal(rew, ref.reward, equal_nan=True), t
    assert ends >= n  # every env ended at least one long episode
    env.close()


@pytest.mark.parametrize("env_id", ["LIDARLocRooms-v0", "LIDARLocRooms-sparse-v0"])
def test_torch_backend_matches_numpy_backend(gpu, env_id):
    import torch

    import ap_gym_amd as ap

    kw = dict(num_envs=256, lidar_beam_count=32, dataset=ap.FloorMapDatasetRooms(64, 64), device=gpu)
    if env_id.endswith("-sparse-v0"):
        with pytest.raises(KeyError, match="prediction"):  # the reference's own -sparse LIDAR reset
            ap.make_vec(env_id, **kw).reset(seed=5)
        kw["sparse_reset_info"] = True
    e_np = ap.make_vec(env_id, **kw)
    e_t = ap.make_vec(env_id, array_backend="torch", **kw)
    assert e_np.sparse == env_id.endswith("-sparse-v0")
    e_np.reset(seed=5)
    e_t.reset(seed=5)
    rng = np.random.default_rng(2)
    for t in range(105):
        a = rng.uniform(-1, 1, (256, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (256, 2)).astype(np.float32)
        o1, r1, te1, tr1, i1 = e_np.step({"action": a, "prediction": p})
        o2, r2, te2, tr2, i2 = e_t.step({"action": torch.from_numpy(a).to(gpu), "prediction": torch.from_numpy(p).to(gpu)})
        assert isinstance(r2, torch.Tensor) and r2.device.type == "cuda"
        assert np.array_equal(o1["lidar"], o2["lidar"].cpu().numpy())
        assert np.array_equal(r1, r2.cpu().numpy())
        assert np.array_equal(te1, te2.cpu().numpy())
        assert np.array_equal(o1["map"], o2["map"].cpu().numpy())
        if e_np.sparse and "prediction" in i1:
            m = i1["_base_reward"]
            w1, w2 = i1["prediction"]["target"]["weight"], i2["prediction"]["target"]["weight"].cpu().numpy()
            assert np.array_equal(w1[m], w2[m]) and np.array_equal(w1[m], te1[m].astype(np.float64))
            assert np.array_equal(i2["prediction"]["target"]["_weight"].cpu().numpy(), m)
    e_t.check_errors()


def _torch_outputs(env):
    out = {k: v.clone() for k, v in env.device_outputs().items()}
    for k in ("pos", "map_idx_out", "stats", "stats_len", "elapsed"):
        out[k] = env._t[k].clone()
    return out


@pytest.mark.parametrize("size,beams,n,limit", [(21, 8, 512, 7), (63, 16, 256, 3), (127, 64, 64, 5)])
def test_maze_prefetch_matches_synchronous_generation(gpu, size, beams, n, limit):
    """The maze prefetch (next maps generated on the side stream, installed by the fused step kernel) gives the
    outputs of synchronous generation bit for bit: many autoresets, a NaN-delayed env whose episode ends at a
    step no other env resets at, reset() and reset(seed) mid-episode, and a captured graph (synchronous steps)
    followed by eager steps."""
    import torch

    import ap_gym_amd as ap

    ds = ap.FloorMapDatasetMaze(size, size)
    kw = dict(num_envs=n, dataset=ds, lidar_beam_count=beams, device=gpu, array_backend="torch",
              max_episode_steps=limit, log_stats=True)
    pf = ap.LIDARLocalization2DVectorEnv(prefetch=True, **kw)
    sy = ap.LIDARLocalization2DVectorEnv(prefetch=False, **kw)
    assert pf._prefetcher and not sy._prefetcher
    g = torch.Generator(device=gpu).manual_seed(5)

    def step_both(a, p):
        pf.step({"action": a, "prediction": p})
        sy.step({"action": a, "prediction": p})
        o1, o2 = _torch_outputs(pf), _torch_outputs(sy)
        for k in o1:
            assert torch.equal(o1[k], o2[k]), k

    def rand():
        return torch.rand((n, 2), generator=g, device=gpu) * 2 - 1, torch.rand((n, 2), generator=g, device=gpu) * 2 - 1

    pf.reset(seed=11)
    sy.reset(seed=11)
    for t in range(4 * (limit + 1) + 3):
        a, p = rand()
        if t == limit + 3:  # env 3's step is refused: its episode (and its resets) shift by one step
            a[3, 0] = float("nan")
        step_both(a, p)
        if t == limit + 3:
            for e in (pf, sy):
                with pytest.raises(ValueError, match="NaN values detected in action."):
                    e.check_errors()
    for e in (pf, sy):
        e.reset()  # streams continue
    for t in range(limit + 4):
        step_both(*rand())
    for e in (pf, sy):
        e.reset(seed=12)
    for t in range(limit // 2):
        step_both(*rand())
    # a captured step (the synchronous path) replayed across an autoreset, then eager steps again
    a_s, p_s = rand()
    graphs = [e.capture_step_graph(a_s, p_s) for e in (pf, sy)]
    for t in range(limit + 2):
        for gr in graphs:
            gr.replay()
        o1, o2 = _torch_outputs(pf), _torch_outputs(sy)
        for k in o1:
            assert torch.equal(o1[k], o2[k]), k
    for t in range(2 * (limit + 1) + 1):
        step_both(*rand())
    for e in (pf, sy):
        e.check_errors()
    st = pf.prefetch_stats()
    assert st["batches"] >= 5 and st["resets"] > 0
    pf.close()
    sy.close()


@pytest.mark.parametrize("kind", ["rooms", "maze"])
def test_numpy_backend_copy_semantics(gpu, kind):
    """copy=None (numpy backend -> True, SyncVectorEnv's default): observations returned at step t keep their
    values after later autoresets; copy=False aliases the host map mirror (refreshed in place at resets)."""
    import ap_gym_amd as ap

    n = 16
    ds = ap.FloorMapDatasetRooms(32, 32) if kind == "rooms" else ap.FloorMapDatasetMaze(21, 21)
    env_id = "LIDARLocRooms-v0" if kind == "rooms" else "LIDARLocMaze-v0"
    env = ap.make_vec(env_id, num_envs=n, lidar_beam_count=8, dataset=ds, device=gpu, max_episode_steps=3)
    alias = ap.make_vec(env_id, num_envs=n, lidar_beam_count=8, dataset=ds, device=gpu, max_episode_steps=3,
                        copy=False)
    assert env.copy and not alias.copy
    obs0, _ = env.reset(seed=3)
    obs0_a, _ = alias.reset(seed=3)
    held = [(obs0, {k: v.copy() for k, v in obs0.items()})]
    rng = np.random.default_rng(0)
    for t in range(9):  # three episodes: autoresets at steps 4 and 8
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        o, r, te, tr, info = env.step({"action": a, "prediction": p})
        oa, *_ = alias.step({"action": a, "prediction": p})
        assert np.array_equal(o["map"], oa["map"]) and np.array_equal(o["lidar"], oa["lidar"])
        held.append((o, {k: v.copy() for k, v in o.items()}))
    for o, snap in held:  # nothing handed out by the copying env changed afterwards
        for k in snap:
            assert np.array_equal(o[k], snap[k]), k
    assert held[-1][0]["map"].flags.writeable  # the caller's own copy (SyncVectorEnv(copy=True) deep-copies)
    assert not np.array_equal(held[0][1]["map"], held[-1][1]["map"])  # the maps did change at the resets
    assert np.shares_memory(oa["map"], obs0_a["map"])  # copy=False: one mirror, rewritten in place
    assert env._ring_copy and len(env._ring) == env.HOST_RING  # 10 steps held: the ring is full, later steps copy
    env.close()
    alias.close()
    # a loop that keeps only the latest step's arrays alternates between two pinned blocks and copies nothing:
    # the returned fields are views of the block the outputs were copied into
    env = ap.make_vec(env_id, num_envs=n, lidar_beam_count=8, dataset=ds, device=gpu, max_episode_steps=3)
    env.reset(seed=3)
    prev = None
    for t in range(7):
        o, r, te, tr, info = env.step({"action": np.zeros((n, 2), np.float32), "prediction": np.zeros((n, 2), np.float32)})
        assert not env._ring_copy and o["lidar"].base is r.base is te.base
        if prev is not None:
            assert o["lidar"].base is not prev.base  # the previous step's arrays were alive during this step
        prev = o["lidar"]
        snap = (o["lidar"].copy(), r.copy())
    assert len(env._ring) == 2
    assert np.array_equal(prev, snap[0]) and np.array_equal(r, snap[1])
    env.close()


def test_numpy_vector_stats_array_mode(gpu):
    """vector_stats="array": float32 arrays with the values of the reference's np.float32 lists."""
    import ap_gym_amd as ap

    kw = dict(num_envs=64, lidar_beam_count=8, dataset=ap.FloorMapDatasetRooms(32, 32), device=gpu,
              max_episode_steps=5)
    e1 = ap.make_vec("LIDARLocRooms-v0", **kw)
    e2 = ap.make_vec("LIDARLocRooms-v0", vector_stats="array", **kw)
    e1.reset(seed=1)
    e2.reset(seed=1)
    rng = np.random.default_rng(4)
    seen = 0
    for t in range(12):
        a = rng.uniform(-1, 1, (64, 2)).astype(np.float32)
        _, _, _, _, i1 = e1.step({"action": a, "prediction": a})
        _, _, _, _, i2 = e2.step({"action": a, "prediction": a})
        assert ("stats" in i1) == ("stats" in i2)
        if "stats" in i1:
            for name in ("euclidean_distance", "mse"):
                v1, v2 = i1["stats"]["vector"][name], i2["stats"]["vector"][name]
                for j in np.nonzero(i1["stats"]["_vector"])[0]:
                    assert isinstance(v1[j], list) and isinstance(v1[j][0], np.float32)
                    assert isinstance(v2[j], np.ndarray) and v2[j].dtype == np.float32
                    assert np.array_equal(np.array(v1[j], np.float32), v2[j])
                    seen += 1
    assert seen > 0
    with pytest.raises(ValueError):
        ap.make_vec("LIDARLocRooms-v0", vector_stats="bad", **kw)


def test_mazes_never_terminate_before_the_time_limit(gpu):
    """The maze prefetch protocol (apg_lidar.hip pf_before_step) relies on an env not resetting again within
    step_limit + 1 steps of its reset; mazes guarantee it because their border rows and columns are walls
    (floor_map_dataset_maze.py:24-55 carves odd cells only), so no move leaves the map and only the TimeLimit
    terminates.  Pushed at the border with oversized actions toward it, every env must run its 100 steps."""
    import ap_gym_amd as ap

    n = 2048
    env = ap.make_vec("LIDARLocMaze-v0", num_envs=n, lidar_beam_count=8, dataset=ap.FloorMapDatasetMaze(21, 21),
                      device=gpu)
    obs, _ = env.reset(seed=4)
    term_steps = []
    rng = np.random.default_rng(0)
    for t in range(205):
        pos = env._t["pos"].cpu().numpy()  # push toward the nearest border, sometimes along it
        a = np.where(pos < 10.5, -3.0, 3.0).astype(np.float32)
        a[rng.random(n) < 0.3, rng.integers(0, 2)] = 0.0
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": np.zeros((n, 2), np.float32)})
        if term.any():
            term_steps.append((t, int(term.sum())))
    # every episode ends exactly at step 100 of it: steps 99 and 200 (the autoreset step 100 in between)
    assert term_steps == [(99, n), (200, n)], term_steps
    assert env.prefetch_stats()["batches"] >= 2
    env.close()


def test_nan_action_raises(gpu):
    import torch

    import ap_gym_amd as ap

    env = ap.make_vec("LIDARLocRoomsStatic-v0", num_envs=4, device=gpu)
    env.reset(seed=0)
    a = np.zeros((4, 2), np.float32)
    p = np.zeros((4, 2), np.float32)
    a[2, 0] = np.nan
    with pytest.raises(ValueError, match="NaN values detected in action."):
        env.step({"action": a, "prediction": p})
    a[2, 0] = 0
    p[1, 1] = np.nan
    with pytest.raises(ValueError, match="NaN values detected in prediction."):
        env.step({"action": a, "prediction": p})
    et = ap.make_vec("LIDARLocRoomsStatic-v0", num_envs=4, device=gpu, array_backend="torch", strict_errors=True)
    et.reset(seed=0)
    with pytest.raises(ValueError, match="prediction"):
        et.step({"action": torch.zeros((4, 2), device=gpu), "prediction": torch.from_numpy(p).to(gpu)})


@pytest.mark.parametrize("kind,size,beams,n", [("rooms", 64, 32, 65536), ("maze", 127, 64, 262144)],
                         ids=["cfg2_rooms64_b32_n65536", "cfg3_maze127_b64_n262144"])
def test_full_size_properties(gpu, oracle_mod, kind, size, beams, n):
    """BASELINE configs 2 and 3 at full size on one GPU (cfg 3 is the whole 262144-env batch the 8-GPU
    run shards): size-independent invariants over 203 steps (two synchronized autoreset bursts), the
    reset maps of sampled envs against the oracle's generator, and the complete step trace (lidar,
    odometry, reward, termination) of sampled envs against a one-env oracle seeded with seed + e."""
    import torch

    import ap_gym_amd as ap

    env_id = "LIDARLocRooms-v0" if kind == "rooms" else "LIDARLocMaze-v0"
    env = ap.make_vec(env_id, num_envs=n, lidar_beam_count=beams, dataset=_ds(ap, kind, size), device=gpu,
                      array_backend="torch")
    obs, info = env.reset(seed=0)
    g = torch.Generator(device=gpu).manual_seed(0)
    sample = np.sort(np.random.default_rng(0).choice(n, 8, replace=False))
    sample[-1] = n - 1  # the last env of the last workgroup
    idx0 = info["map_idx"].cpu().numpy().astype(np.uint64)
    maps = obs["map"][torch.as_tensor(sample, device=gpu), ..., 0].cpu().numpy()
    refs = []
    for j, e in enumerate(sample):
        want = (oracle_mod.rooms_map(int(idx0[e]), size) if kind == "rooms"
                else oracle_mod.maze_map(int(idx0[e]), size)).astype(bool)
        assert np.array_equal(maps[j] > 0, want), f"reset map of env {e}"
        ref = oracle_mod.OracleLidarVectorEnv(1, kind, size, False, 0, beams)
        ref.reset(int(e))  # sub-env 0 seeded with seed + e, like env e of the batch
        assert np.array_equal(obs["lidar"][int(e)].cpu().numpy(), ref.lidar[0]), f"reset lidar of env {e}"
        refs.append(ref)
    sel = torch.as_tensor(sample, device=gpu)
    resets = 0
    for t in range(1, 203):
        a = torch.rand((n, 2), device=gpu, generator=g) * 2 - 1
        p = torch.rand((n, 2), device=gpu, generator=g) * 2 - 1
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        lid = obs["lidar"]
        assert bool(((lid >= 0) & (lid <= 1)).all())
        assert not bool(trunc.any())
        if t % 101 == 100:  # TimeLimit(100) terminates every env still in its first episode
            assert int(term.sum()) >= 0.99 * n
        if t % 101 == 0:
            resets += 1
            reset_now = ~info["_base_reward"]
            assert int(reset_now.sum()) >= 0.99 * n and bool((rew[reset_now] == 0).all())
        a_s, p_s = a[sel].cpu().numpy(), p[sel].cpu().numpy()
        got = {k: v[sel].cpu().numpy() for k, v in (("lidar", lid), ("odometry", obs["odometry"]), ("reward", rew),
                                                      ("terminated", term))}
        for j, ref in enumerate(refs):
            ref.step(a_s[j:j + 1], p_s[j:j + 1])
            e = int(sample[j])
            assert np.array_equal(got["lidar"][j], ref.lidar[0]), f"step {t} env {e}: lidar"
            assert np.array_equal(got["odometry"][j], ref.odometry[0]), f"step {t} env {e}: odometry"
            assert got["reward"][j] == ref.reward[0], f"step {t} env {e}: reward"
            assert bool(got["terminated"][j]) == bool(ref.terminated[0]), f"step {t} env {e}: terminated"
    env.check_errors()
    assert resets == 2
    for ref in refs:
        ref.close()


@pytest.mark.parametrize("use_torch_op", [False, True], ids=["c_abi", "torch_op"])
@pytest.mark.parametrize("kind,size,beams", [("rooms", 64, 32), ("maze", 21, 8)])
def test_step_through_ops_and_graph_replay(gpu, kind, size, beams, use_torch_op):
    """Eager steps call the C ABI directly (use_torch_op=False, the default) or go through
    torch.ops.apgym.lidar_step (use_torch_op=True); one step captured in a torch.cuda.CUDAGraph (hipGraph,
    always through the op) and replayed over 230 steps (two autoreset bursts) is bit-identical to eager
    env.step either way."""
    import torch

    import ap_gym_amd as ap

    n = 512
    kw = dict(num_envs=n, lidar_beam_count=beams, dataset=_ds(ap, kind, size), device=gpu, array_backend="torch")
    eager = ap.make_vec(f"LIDARLoc{'Rooms' if kind == 'rooms' else 'Maze'}-v0", **kw)
    graphed = ap.make_vec(f"LIDARLoc{'Rooms' if kind == 'rooms' else 'Maze'}-v0", **kw)
    assert eager._ops is torch.ops.apgym
    eager.use_torch_op = use_torch_op
    eager.reset(seed=11)
    graphed.reset(seed=11)
    a_buf = torch.zeros((n, 2), dtype=torch.float32, device=gpu)
    p_buf = torch.zeros((n, 2), dtype=torch.float32, device=gpu)
    graph = graphed.capture_step_graph(a_buf, p_buf)
    g = torch.Generator(device=gpu).manual_seed(3)
    out_g = graphed.device_outputs()
    for t in range(230):
        a = torch.rand((n, 2), device=gpu, generator=g) * 2.2 - 1.1
        p = torch.rand((n, 2), device=gpu, generator=g) * 2 - 1
        obs, rew, term, trunc, info = eager.step({"action": a, "prediction": p})
        a_buf.copy_(a)
        p_buf.copy_(p)
        graph.replay()
        for k, v in (("lidar", obs["lidar"]), ("odometry", obs["odometry"]), ("time_step", obs["time_step"]),
                     ("reward", rew), ("terminated", term), ("base_reward", info["base_reward"]),
                     ("target", info["prediction"]["target"]), ("loss", info["prediction"]["loss"])):
            assert torch.equal(out_g[k], v), (t, k)
        assert torch.equal(graphed._t["map_obs"], obs["map"]), t
    eager.check_errors()
    graphed.check_errors()


@pytest.mark.parametrize("snapshot", ["copy", "shared"])
def test_numpy_backend_returned_arrays_are_writable(gpu, oracle_mod, snapshot):
    """SyncVectorEnv(copy=True) deep-copies the observations it returns: a caller may normalise them in place.
    Writes into every returned array (obs["map"] included) on consecutive steps leave the next steps' values
    unaffected (checked against the oracle).  obs_snapshot="shared" (opt-in) returns obs["map"] read-only."""
    import ap_gym_amd as ap

    n = 64
    env = ap.LIDARLocalization2DVectorEnv(num_envs=n, dataset=ap.FloorMapDatasetRooms(32, 32), lidar_beam_count=8,
                                          device=gpu, max_episode_steps=4, obs_snapshot=snapshot)
    ref = oracle_mod.OracleLidarVectorEnv(n, "rooms", 32, False, 0, 8, step_limit=4)
    obs, _ = env.reset(seed=1)
    ref.reset(1)
    rng = np.random.default_rng(3)
    for t in range(12):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        p = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        ref.step(a, p)
        assert np.array_equal(obs["lidar"], ref.lidar) and np.array_equal(obs["map"][..., 0], ref.map), t
        assert np.array_equal(rew, ref.reward), t
        for k, v in obs.items():
            if k == "map" and snapshot == "shared":
                assert not v.flags.writeable
                continue
            v[...] = -7  # in-place "normalisation" by the caller
        rew[...] = 123.0
    env.close()
