"""Host-side logic that needs no GPU: C-ABI symbol export, loss functions, spaces, registry."""

import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden


def _header_functions():
    src = open(os.path.join(ROOT, "include", "apgym_capi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(apg_\w+)\s*\(", src, flags=re.M)))


def test_capi_library_exports_every_declared_symbol():
    import ctypes

    from ap_gym_amd import _native

    names = _header_functions()
    assert len(names) >= 9
    lib = ctypes.CDLL(_native.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert {s[0] for s in _native.SYMBOLS} == set(names)
    assert _native.lib().apg_version().startswith(b"apgym-mi355x")


def test_fast_call_module_reaches_the_c_abi():
    """_apgfast (csrc/apg_pyfast.cpp): the per-step C-ABI calls without ctypes marshalling.  Invalid configurations
    return the C ABI's validation error before any HIP call, so this runs without a GPU."""
    import ctypes

    from ap_gym_amd import _native as N

    F = N.fast()
    assert os.path.dirname(F.__file__) == N.LIB_DIR
    for name, args, cfg, st, out in (("lidar_step", 6, N.LidarConfig(), N.LidarState(), N.LidarOutputs()),
                                     ("image_step", 8, N.ImageConfig(), N.ImageState(), N.ImageOutputs()),
                                     ("light_dark_step", 6, N.LightDarkConfig(), N.LightDarkState(),
                                      N.LightDarkOutputs())):
        fn = getattr(F, name)
        tail = [N.addr(out), 0] if args == 6 else [3, 0, N.addr(out), 0]
        assert fn(N.addr(cfg), N.addr(st), 0, 0, *tail) == N.APG_E_INVALID, name
        assert N.lib().apg_last_error()  # the C ABI's own message
        with pytest.raises(TypeError):
            fn(N.addr(cfg))
        with pytest.raises(TypeError):
            fn(N.addr(cfg), N.addr(st), "x", 0, *tail)
        # the same validation result as the ctypes entry point
        c_fn = getattr(N.lib(), "apg_" + name)
        c_tail = [ctypes.byref(out), None] if args == 6 else [3, 0, ctypes.byref(out), None]
        assert c_fn(ctypes.byref(cfg), ctypes.byref(st), None, None, *c_tail) == N.APG_E_INVALID


def test_capi_validation_without_gpu():
    import ctypes

    from ap_gym_amd import _native as N

    cfg = N.LidarConfig(num_envs=4, height=64, width=64, map_kind=N.APG_MAP_ROOMS, is_static=0, beams=32,
                        step_limit=100, max_rooms=10, door_width=3, lidar_range=5.0, loss_scale=3.0,
                        branching_prob=1.0)
    sz = N.LidarSizes()
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0
    assert sz.wpr == 1 and sz.occ_bytes == 4 * 64 * 8 and sz.scratch_bytes == 0 and sz.stack_bytes == 0
    cfg.map_kind = N.APG_MAP_MAZE
    cfg.height = cfg.width = 127
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0
    assert sz.wpr == 2 and sz.stack_bytes == sz.maze_frames * 4 * 2
    cfg.height = cfg.width = 128  # even maze sizes are rejected like FloorMapDatasetMaze
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    assert b"odd" in N.lib().apg_last_error()
    # the envelope: mazes up to 511 x 511 (past 255: k_maze_big), rooms up to 255,
    # lidar_range up to 60
    cfg.height, cfg.width = 255, 101
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0 and sz.wpr == 2
    cfg.height = cfg.width = 301
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0 and sz.wpr == 5
    # k_maze_big's scratch: visited bits (150 rows x 3 words) + a u32 frame per cell and one more, 64-B rounded
    assert sz.maze_frames * 2 == (150 * 3 * 8 + 4 * (150 * 150 + 1) + 63) // 64 * 64
    cfg.height = cfg.width = 513
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    cfg.map_kind = N.APG_MAP_ROOMS
    cfg.height = cfg.width = 320
    cfg.max_rooms, cfg.door_width = 48, 3
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0 and sz.wpr == 5
    cfg.max_rooms = 65
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    cfg.max_rooms = 48
    cfg.height = cfg.width = 512
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    assert b"rooms" in N.lib().apg_last_error()
    cfg.map_kind = N.APG_MAP_MAZE
    cfg.height = cfg.width = 127
    cfg.lidar_range = 60.0
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0
    cfg.lidar_range = 60.5
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    cfg.lidar_range = 5.0
    # packed output rows must hold every enabled field (the Python row layout's size is the minimum)
    from ap_gym_amd.lidar_env import lidar_output_row_layout

    for log_stats, sparse in ((0, 0), (1, 0), (0, 1), (1, 1)):
        cfg.log_stats, cfg.sparse = log_stats, sparse
        _, row = lidar_output_row_layout(cfg.beams, bool(log_stats), bool(sparse))
        cfg.out_row_bytes = row
        assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0
        cfg.out_row_bytes = row - 8
        assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
        assert b"out_row_bytes" in N.lib().apg_last_error()
    cfg.out_row_bytes = cfg.log_stats = cfg.sparse = 0
    # pool maps (any FloorMapDataset): any H x W from 1 to 511, at least one map, static index inside the pool
    cfg.map_kind, cfg.height, cfg.width, cfg.pool_len = N.APG_MAP_POOL, 40, 48, 37
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0
    assert sz.wpr == 1 and sz.stack_bytes == 0 and sz.prefetch_bytes == 0
    cfg.height, cfg.width = 1, 511
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0 and sz.wpr == 8
    cfg.width = 512
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    cfg.width, cfg.pool_len = 48, 0
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    assert b"pool" in N.lib().apg_last_error()
    cfg.pool_len, cfg.is_static, cfg.static_map_index = 37, 1, 37
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == -1
    cfg.static_map_index = 36
    assert N.lib().apg_lidar_query_sizes(ctypes.byref(cfg), ctypes.byref(sz)) == 0
    # the pool buffers are required before anything reaches the device
    st = N.LidarState()
    assert N.lib().apg_lidar_init(ctypes.byref(cfg), ctypes.byref(st), None) == -1
    assert b"pool_occ" in N.lib().apg_last_error()


def test_pool_floor_map_datasets_pack_the_maps():
    """PoolFloorMapDataset.host_pool: bit x % 64 of word x // 64 of row y is map[y, x] (include/apgym_capi.h,
    apg_lidar_state.pool_occ), free-cell counts per map; ForeignFloorMapView over the reference interface checks
    shapes (lidar_localization2d.py:279) and dtypes like the reference env relies on them."""
    import ap_gym_amd as ap
    from ap_gym_amd.floor_map import as_floor_map_dataset

    rng = np.random.default_rng(0)
    maps = rng.random((7, 13, 130)) < 0.3
    ds = ap.ArrayFloorMapDataset(maps)
    bits, free = ds.host_pool()
    assert bits.shape == (7, 13, 3) and bits.dtype == np.dtype("<u8")
    y, x = np.nonzero(np.ones((13, 130), bool))
    for i in range(7):
        got = (bits[i][y, x // 64] >> (x % 64).astype(np.uint64)) & np.uint64(1)
        assert np.array_equal(got.astype(bool), maps[i][y, x])
        assert free[i] == (~maps[i]).sum()
    assert np.all(bits[:, :, 2] >> np.uint64(2) == 0)  # no bits past W
    assert np.array_equal(ds.get_data_point(3), maps[3]) and ds.get_data_point_batch([1, 2]).shape == (2, 13, 130)

    class Ref:  # the reference FloorMapDataset interface
        map_width, map_height = 130, 13

        def __len__(self):
            return 7

        def get_data_point(self, i):
            return maps[i]

    view = as_floor_map_dataset(Ref())
    assert isinstance(view, ap.ForeignFloorMapView) and len(view) == 7
    assert np.array_equal(view.host_pool()[0], bits)
    assert as_floor_map_dataset(ds) is ds

    class Uint8Maps(Ref):
        def get_data_point(self, i):
            return maps[i].astype(np.uint8)

    with pytest.raises(TypeError, match="boolean"):
        as_floor_map_dataset(Uint8Maps()).host_pool()
    with pytest.raises(TypeError, match="FloorMapDataset"):
        as_floor_map_dataset(object())


def test_mse_loss_matches_reference_golden():
    from ap_gym_amd.loss_fn import affine_f32, regression_loss

    g = golden("loss.npz")
    fn = regression_loss(2, -1, 1)
    got = np.stack([fn(p, t, ()) for p, t in zip(g["mse_pred"], g["mse_target"])])
    assert got.dtype == np.float32
    assert np.array_equal(got, g["mse_loss"])
    assert affine_f32(fn) == (3.0, -0.0)


@pytest.mark.parametrize("k", [10, 200])
def test_ce_loss_matches_reference_golden(k):
    from ap_gym_amd.loss_fn import CrossEntropyLossFn

    g = golden("loss.npz")
    fn = CrossEntropyLossFn(k).normalized
    got = fn(g[f"ce{k}_logits"], g[f"ce{k}_labels"], (256,))
    assert got.dtype == g[f"ce{k}_loss"].dtype == np.float64
    assert np.array_equal(got, g[f"ce{k}_loss"])


def test_ce_loss_numpy_vs_torch():
    """The reference's only unit test (test/test_active_classification_env.py:17-50), restated."""
    import torch

    from ap_gym_amd.loss_fn import CrossEntropyLossFn

    fn = CrossEntropyLossFn()
    rng = np.random.default_rng(0)
    blen = rng.integers(0, 5, size=20)
    plen = blen + rng.integers(1, 5, size=blen.shape)
    shapes = [tuple(rng.integers(1, 10, size=d)) for d in plen]
    for bl, shape in zip(blen, shapes):
        pred = rng.standard_normal(shape)
        tgt = rng.integers(0, shape[-1], size=shape[:-1])
        exp = fn.numpy(pred, tgt, shape[:bl])
        got = fn.torch(torch.from_numpy(pred), torch.from_numpy(tgt), shape[:bl]).numpy()
        np.testing.assert_allclose(got, exp, rtol=1e-4)


def test_registry_and_spaces():
    import ap_gym_amd as ap
    from ap_gym_amd.spaces import ActivePerceptionActionSpace, batch_space

    assert {"LIDARLocRooms-v0", "LIDARLocRoomsStatic-v0", "LIDARLocMaze-v0", "LIDARLocMazeStatic-v0"} <= set(
        ap.registry)
    with pytest.raises(KeyError):
        ap.make_vec("NoSuchEnv-v0", 2)
    sp = ActivePerceptionActionSpace(ap.spaces.Box(-1, 1, (2,)), ap.spaces.Box(-1, 1, (2,)))
    b = batch_space(sp, 7)
    assert b["action"].shape == (7, 2) and b["prediction"].shape == (7, 2)
    im = ap.ImageSpace(64, 48, 1)
    assert im.shape == (48, 64, 1) and batch_space(im, 3).shape == (3, 48, 64, 1)
    with pytest.raises(ValueError):
        ap.FloorMapDatasetMaze(128, 128)


def test_make_vec_vectorization_modes():
    """registration.py:753-767 passes vectorization_mode through to gymnasium: "sync" and "async" give the
    same batches, so both build the batched env; unknown modes and per-sub-env wrappers are refused."""
    from ap_gym_amd.registration import EnvSpec, make_vec

    built = []
    spec = EnvSpec("Probe-v0", lambda num_envs, **kw: built.append((num_envs, kw)) or "env", {"a": 1}, 7)

    class Mode:  # a gymnasium.VectorizeMode-like enum member
        value = "async"

    for mode in (None, "vector_entry_point", "sync", "async", Mode()):
        assert make_vec(spec, 3, vectorization_mode=mode, b=2) == "env"
    assert built == [(3, {"a": 1, "max_episode_steps": 7, "b": 2})] * 5
    with pytest.raises(ValueError):
        make_vec(spec, 3, vectorization_mode="threads")
    with pytest.raises(NotImplementedError):
        make_vec(spec, 3, wrappers=[lambda e: e])


def test_beam_directions_match_reference_formula():
    from ap_gym_amd import lidar_beam_directions

    for b in (8, 16, 32, 64):
        ang = np.linspace(-np.pi, np.pi, b, dtype=np.float32, endpoint=False)
        ref = np.stack([np.cos(ang), np.sin(ang)], axis=-1) * 5
        d = lidar_beam_directions(b, 5)
        assert d.dtype == np.float32 and np.array_equal(d, ref)


def test_image_host_helpers_match_reference_formulas():
    import scipy.special

    from ap_gym_amd.image_env import sensor_pos_lim_pixels, softmax_nan_rows, unique_sampling_grid
    from oracle import image_oracle as io

    for hw, sensor, scale in (((28, 28), (5, 5), 1.0), ((64, 64), (10, 10), 1.0), ((64, 64), (12, 12), 1.0),
                              ((20, 24), (5, 5), 1.5)):
        assert np.array_equal(sensor_pos_lim_pixels(hw, sensor, scale), io.sensor_pos_lim(hw, sensor, scale))
        g1, c1 = unique_sampling_grid(hw, sensor, scale)
        g2, c2 = io.unique_grid(hw, sensor, scale)
        assert np.array_equal(g1, g2) and np.array_equal(c1, c2)
    rows = np.array([[0, 1, 2], [np.nan, 0, 0], [np.inf, 0, 0], [-np.inf, -np.inf, -np.inf], [-np.inf, 0, 1],
                     [1e30, -1e30, 0]], np.float32)
    with np.errstate(invalid="ignore"):
        want = np.isnan(scipy.special.softmax(rows, axis=-1)).any(-1)
    assert np.array_equal(softmax_nan_rows(rows), want)


def test_image_registry_and_spaces():
    import ap_gym_amd as ap

    for i in ("MNIST-v0", "MNIST-test-v0", "CIFAR10-c3-v0", "TinyImageNet-v0", "MNISTLoc-v0", "TinyImageNetLoc-v0"):
        assert i in ap.registry
    ds = ap.SyntheticImageClassificationDataset(20, (28, 28), 10, seed=1)
    imgs, labels = ds.get_data_point_batch([0, 3])
    assert imgs.shape == (2, 28, 28, 1) and imgs.dtype == np.float32 and labels.dtype == np.int32
    pool, lab = ds.device_pool()
    assert pool.dtype == np.uint8 and pool.shape == (20, 28, 28, 1)
    assert np.array_equal(imgs, pool[[0, 3]].astype(np.float32) / 255)


def test_ctypes_layouts_match_the_c_header(tmp_path):
    """Every ctypes mirror in _native.py has the size and field offsets gcc gives include/apgym_capi.h."""
    import ctypes
    import os
    import shutil
    import subprocess

    from ap_gym_amd import _native as N

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"apg_pcg64": N.Pcg64, "apg_lidar_config": N.LidarConfig, "apg_lidar_state": N.LidarState,
               "apg_lidar_outputs": N.LidarOutputs, "apg_lidar_state_sizes": N.LidarSizes,
               "apg_image_config": N.ImageConfig, "apg_image_state": N.ImageState,
               "apg_image_outputs": N.ImageOutputs, "apg_circle_square_config": N.CircleSquareConfig,
               "apg_hide_and_seek_args": N.HideAndSeekArgs, "apg_light_dark_config": N.LightDarkConfig,
               "apg_light_dark_state": N.LightDarkState, "apg_light_dark_outputs": N.LightDarkOutputs,
               "apg_lidar_render_state": N.LidarRenderState}
    lines = ["#include <stdio.h>", "#include \"apgym_capi.h\"", "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'  printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                              text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_sparse_ids_and_weighted_loss():
    """registration.py:115-142: every id has a "-sparse" twin; WeightedLossFn (loss_fn.py:292-349)."""
    import ap_gym_amd as ap
    from ap_gym_amd.registration import sparse_id

    dense = [i for i in ap.registry if "-sparse-" not in i]
    assert dense and all(sparse_id(i) in ap.registry for i in dense)
    assert sparse_id("MNIST-train-v0") == "MNIST-train-sparse-v0"
    assert ap.registry["LIDARLocRooms-sparse-v0"].kwargs["sparse"] is True
    assert "sparse" not in ap.registry["LIDARLocRooms-v0"].kwargs
    assert len(ap.registry) == 2 * len(dense)
    inner = ap.MSELossFn(target_std=2 / np.sqrt(12)).normalized
    fn = ap.WeightedLossFn(inner)
    rng = np.random.default_rng(0)
    p = rng.uniform(-1, 1, (6, 2)).astype(np.float32)
    t = rng.uniform(-1, 1, (6, 2)).astype(np.float32)
    w = np.array([0, 1, 0, 1, 1, 0], np.float32)
    got = fn.numpy(p, {"target": t, "weight": w}, (6,))
    assert np.array_equal(got, inner.numpy(p, t, (6,)) * w) and got.dtype == np.float32


def test_torch_ops_library_registers_the_ops():
    """libapgym_torch.so (csrc/apg_torch_ops.cpp) loads on a CPU-only host and registers
    TORCH_LIBRARY(apgym) ops and env handle classes (no GPU call is made)."""
    import torch

    from ap_gym_amd import _native as N

    ops = N.torch_ops()
    assert ops is torch.ops.apgym
    for name in ("lidar_reset", "lidar_step", "image_reset", "image_step"):
        assert callable(getattr(ops, name)), name
    assert torch.classes.apgym.LidarEnv is not None and torch.classes.apgym.ImageEnv is not None
    with pytest.raises(RuntimeError, match="16 ints"):
        torch.classes.apgym.LidarEnv([1], [0.0], [], [])


def test_foreign_dataset_view_fetches_in_chunks_and_warns():
    """A reference-interface dataset becomes a device pool: fetched once, in chunks, with a warning about the
    frozen (static-pool) semantics."""
    import warnings

    import numpy as np

    from ap_gym_amd.image_dataset import ForeignDatasetView

    class RefLike:
        num_classes, num_channels = 3, 1

        def __init__(self):
            self.calls = 0

        def __len__(self):
            return 10

        def _get_data_point_batch(self, idx):
            self.calls += 1
            idx = np.asarray(idx)
            return (idx[:, None, None] * np.ones((len(idx), 4, 5), np.uint8)).astype(np.uint8), idx % 3

    inner = RefLike()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        view = ForeignDatasetView(inner)
    assert any("frozen" in str(x.message) for x in w)
    view.FETCH_CHUNK = 4
    imgs, labels = view.device_pool()
    assert inner.calls == 3 and imgs.shape == (10, 4, 5, 1) and imgs.dtype == np.uint8
    assert np.array_equal(imgs[:, 0, 0, 0], np.arange(10)) and np.array_equal(labels, np.arange(10) % 3)


def test_u8_tap_value_pair_is_exact():
    """apg_image.hip u8_value_f32: fma(v, c_hi, v * c_lo) in f32 (c_hi + c_lo = 1/255 to ~2^-48) equals the
    correctly rounded v / 255 (the reference's u8 -> float32 / 255 value path) for every byte, checked with
    exact rationals (the kernel's glimpse taps use it instead of an LDS table)."""
    from fractions import Fraction

    def round_f32(fr):
        c = np.float32(float(fr))
        best = None
        for k in range(-2, 3):
            v = c
            for _ in range(abs(k)):
                v = np.nextafter(v, np.float32(np.inf if k > 0 else -np.inf))
            err = abs(Fraction(float(v)) - fr)
            even = (np.array(v, dtype=np.float32).view(np.uint32) & 1) == 0
            if best is None or err < best[0] or (err == best[0] and even):
                best = (err, float(v))
        return best[1]

    c_hi, c_lo = float.fromhex("0x1.010102p-8"), float.fromhex("-0x1.fdfdfep-33")
    assert float(np.float32(c_hi)) == c_hi and float(np.float32(c_lo)) == c_lo
    for v in range(256):
        p = round_f32(Fraction(v) * Fraction(c_lo))
        got = round_f32(Fraction(v) * Fraction(c_hi) + Fraction(p))
        assert got == round_f32(Fraction(v, 255)) == float(np.float32(v / 255.0)), v


def test_lidar_output_block_layout():
    """The numpy backend's field-major output block: every field 256-byte aligned, contiguous, disjoint, and
    views of one buffer (torch and numpy) that alias the same bytes."""
    import torch

    from ap_gym_amd.lidar_env import block_views, lidar_output_block_layout

    for n, beams, stats, sparse in ((1, 8, False, False), (1000, 32, True, True), (65536, 64, True, False)):
        layout, nbytes = lidar_output_block_layout(n, beams, stats, sparse)
        names = [f[0] for f in layout]
        assert ("stats" in names) == stats and ("weight" in names) == sparse and "lidar" in names
        end = 0
        for name, dt, shape, off in layout:
            assert off % 256 == 0 and off >= end
            end = off + torch.empty((), dtype=dt).element_size() * int(np.prod(shape))
        assert end <= nbytes and nbytes % 256 == 0
        if n <= 1000:
            buf = torch.zeros(nbytes, dtype=torch.uint8)
            tv, nv = block_views(buf, layout), block_views(buf.numpy(), layout)
            tv["lidar"][-1, -1] = 2.5
            tv["reward"][0] = -1.25
            assert nv["lidar"][-1, -1] == 2.5 and nv["reward"][0] == -1.25
            assert all(v.is_contiguous() for v in tv.values()) and all(v.flags.c_contiguous for v in nv.values())


def test_binomial_constant_table_matches_host_libm():
    """csrc/apg_binom_table.hpp (the rooms generator's random_binomial_inversion constants in constant memory) is
    what tools/gen_binom_table.py computes with this host's libm, numpy's own evaluation of qn and bound."""
    import os
    import re
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    from gen_binom_table import table

    text = open(os.path.join(root, "active-perception-gym_amd", "csrc", "apg_binom_table.hpp")).read()

    def macro(name):
        m = re.search(r"#define " + name + r" \\\n((?:.*\\\n)*.*)\n", text)
        return [v.strip() for v in m.group(1).replace("\\", "").split(",") if v.strip()]

    p, q, qn, bound = table()
    assert [float.fromhex(v) for v in macro("APG_BINOM_QN")] == qn
    assert [int(v) for v in macro("APG_BINOM_BOUND")] == bound
    assert len(qn) == 64 and qn[1] == 0.7 and bound[:3] == [0, 1, 2]


@pytest.mark.parametrize("family", ["lidar", "image"])
def test_kernel_source_hash_covers_the_include_closure(family):
    """bench.py keys its PMC / duration tables by a hash of the kernel sources; the hash must cover every file
    the translation unit compiles (its quoted #include closure), which the compiler's own dependency list
    (hipcc -MM) names."""
    import os
    import shutil
    import subprocess

    import bench

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not (os.path.exists(hipcc) or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    root = bench.ROOT
    src = os.path.join(root, "active-perception-gym_amd", "csrc", bench.KERNEL_ROOTS[family])
    out = subprocess.run([hipcc, "-MM", "--offload-arch=gfx950", "-I", os.path.join(root, "include"), src],
                         capture_output=True, text=True, check=True).stdout
    deps = {os.path.normpath(os.path.join(root, t)) for t in out.replace("\\\n", " ").split()
            if t.endswith((".hip", ".hpp", ".h")) and not t.startswith("/opt")}
    deps = {d if os.path.isabs(d) else os.path.join(root, d) for d in deps}
    assert deps and deps == set(bench.kernel_sources(family))
    assert any(p.endswith("apgym_capi.h") for p in deps)


def _np_fma(a, b, c):
    # float32 fma: the float32 product is exact in float64, the sum rounded there and then to float32 (no case in
    # the ranges below rounds differently from a single rounding: the sweep matches numpy bit for bit)
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def _np_exp_restated(x):
    """apg_image.hip's np_expf in numpy (normal-range outputs)."""
    f = np.float32
    q = ((x * f(1.4426950216293335)).astype(f) + f(12582912.0)).astype(f) - f(12582912.0)
    r = _np_fma(q, f(-0.693145751953125), x)
    r = _np_fma(q, f(-1.428606765330187e-06), r)
    num = _np_fma(f(5.082762800157070e-04), r, f(6.757896859198809e-03))
    for c in (5.1145121455192566e-02, 2.4736154079437256e-01, 7.2576647996902466e-01, 1.0):
        num = _np_fma(num, r, f(c))
    den = _np_fma(_np_fma(f(2.1595094352960587e-02), r, f(-2.7423354983329773e-01)), r, f(1.0))
    poly = (num.astype(np.float64) / den.astype(np.float64)).astype(f)
    return np.ldexp(poly.astype(np.float64), q.astype(np.int32)).astype(f)


def _np_log_restated(x):
    """apg_image.hip's np_logf in numpy (positive finite inputs)."""
    f = np.float32
    m, e = np.frexp(x)
    m, ex = m.astype(f), e.astype(f)
    low = m <= f(0.70710676908493042)
    m = np.where(low, (m + m).astype(f), m)
    ex = np.where(low, ex - f(1), ex).astype(f)
    r = (m - f(1)).astype(f)
    num = _np_fma(f(2.5899792090058327e-02), r, f(3.8088378310203552e-01))
    for c in (1.4800006151199341, 2.1126775741577148, 1.0, 0.0):
        num = _np_fma(num, r, f(c))
    den = _np_fma(f(5.8750952593982220e-03), r, f(1.5464763343334198e-01))
    for c in (9.8649430274963379e-01, 2.4530060291290283, 2.6126775741577148, 1.0):
        den = _np_fma(den, r, f(c))
    return _np_fma(ex, f(0.69314718246459961), (num.astype(np.float64) / den.astype(np.float64)).astype(f))


def test_numpy_float32_exp_log_restatement():
    """The float32 exp / log algorithms the cross-entropy kernels run (apg_image.hip np_expf / np_logf: numpy's
    AVX-512F loops, its coefficients) against np.exp / np.log on a strided sweep of every float32 a log-softmax feeds
    them: exp on [-87.3, 0] (normal results), log on [1, 65536].  (The full sweeps, 1.1e9 and 1.3e8 inputs, matched
    bit for bit when the restatement was written; the GPU suite checks the kernels against numpy the same way.)"""
    f = np.float32
    lo = np.array([-87.3], f).view(np.uint32)[0]
    bits = np.arange(0x80000000, int(lo) + 1, 101, dtype=np.uint64).astype(np.uint32)
    x = bits.view(f)
    assert np.array_equal(_np_exp_restated(x).view(np.uint32), np.exp(x).view(np.uint32))
    a, b = np.array([1.0, 65536.0], f).view(np.uint32)
    x = np.arange(a, b + 1, 13, dtype=np.uint64).astype(np.uint32).view(f)
    assert np.array_equal(_np_log_restated(x).view(np.uint32), np.log(x).view(np.uint32))


def test_procedural_subclasses_recognised_through_the_mro():
    """A subclass of the reference's FloorMapDatasetRooms / FloorMapDatasetMaze that keeps get_data_point and the
    2**32 length runs on the device generators with its parameters; one that overrides get_data_point (or the
    length) is a foreign dataset read through ForeignFloorMapView.  Stand-ins carry the reference's class names,
    module and private attributes (floor_map_dataset_rooms.py:10-24, floor_map_dataset_maze.py:10-22)."""
    import ap_gym_amd as ap
    from ap_gym_amd.floor_map import as_floor_map_dataset, procedural_equivalent

    class FloorMapDatasetRooms:  # the reference's public surface, under its own module name
        def __init__(self, width=32, height=32, max_rooms=10, door_width=3):
            self.map_width, self.map_height = width, height
            self._FloorMapDatasetRooms__max_rooms = max_rooms
            self._FloorMapDatasetRooms__door_width = door_width

        def __len__(self):
            return 2**32

        def get_data_point(self, idx):
            raise AssertionError("the device generator must be used")

    FloorMapDatasetRooms.__module__ = "ap_gym.envs.floor_map.floor_map_dataset_rooms"

    class FloorMapDatasetMaze(FloorMapDatasetRooms):
        def __init__(self, width=21, height=21, branching_prob=1.0):
            super().__init__(width, height)
            self._FloorMapDatasetMaze__branching_prob = branching_prob

    FloorMapDatasetMaze.__module__ = "ap_gym.envs.floor_map.floor_map_dataset_maze"

    class MyRooms(FloorMapDatasetRooms):  # a user subclass that only changes defaults
        def __init__(self):
            super().__init__(64, 64, max_rooms=7, door_width=2)

    class MyMaps(FloorMapDatasetRooms):  # its own maps
        def get_data_point(self, idx):
            return np.zeros((self.map_height, self.map_width), bool)

    class Finite(FloorMapDatasetRooms):  # a finite length changes the DatasetIterator's draws
        def __len__(self):
            return 1000

    p = procedural_equivalent(MyRooms())
    assert isinstance(p, ap.FloorMapDatasetRooms) and (p.map_width, p.max_rooms, p.door_width) == (64, 7, 2)
    q = procedural_equivalent(FloorMapDatasetMaze(31, 31, 0.5))
    assert isinstance(q, ap.FloorMapDatasetMaze) and q.branching_prob == 0.5 and q.map_height == 31
    assert procedural_equivalent(MyMaps()) is None and procedural_equivalent(Finite()) is None
    assert isinstance(as_floor_map_dataset(MyMaps()), ap.ForeignFloorMapView)
    assert isinstance(as_floor_map_dataset(MyRooms()), ap.FloorMapDatasetRooms)

    class NotReference(FloorMapDatasetRooms):
        pass

    NotReference.__module__ = "user_module"  # (the MRO still holds the reference class: recognised)
    assert isinstance(procedural_equivalent(NotReference()), ap.FloorMapDatasetRooms)

    class OwnGen(ap.FloorMapDatasetRooms):  # ap_gym_amd's own class with user maps
        def get_data_point(self, idx, device=None):
            return np.zeros((self.map_height, self.map_width), bool)

    assert isinstance(as_floor_map_dataset(OwnGen(16, 16)), ap.ForeignFloorMapView)
    assert isinstance(as_floor_map_dataset(ap.FloorMapDatasetRooms(16, 16)), ap.FloorMapDatasetRooms)


def test_map_source_choice_and_static_pool():
    """frozen_maps=None: datasets up to POOL_AUTO_MAPS maps (and POOL_AUTO_BYTES of bit rows) are read once into a
    frozen pool, larger ones are streamed per episode; a static env reads dataset[static_map_index] alone."""
    import ap_gym_amd as ap
    from ap_gym_amd.floor_map import ForeignFloorMapView, pack_maps

    class Big:
        map_width = map_height = 40

        def __init__(self, n):
            self.n, self.fetched = n, []

        def __len__(self):
            return self.n

        def get_data_point(self, idx):
            self.fetched.append(int(idx))
            m = np.zeros((40, 40), bool)
            m[0] = True
            return m

    assert ForeignFloorMapView(Big(2**32)).prefers_streaming()
    assert ForeignFloorMapView(Big(2**16 + 1)).prefers_streaming()
    assert not ForeignFloorMapView(Big(1000)).prefers_streaming()
    inner = Big(2**32)
    occ, free = ForeignFloorMapView(inner).static_pool(2**32 - 3, "cpu")
    assert inner.fetched == [2**32 - 3] and tuple(occ.shape) == (1, 40, 1) and int(free[0]) == 40 * 39
    assert int(occ[0, 0, 0]) == (1 << 40) - 1 and int(occ[0, 1, 0]) == 0
    bits, fr = np.zeros((1, 3, 8), np.uint8), np.zeros(1, np.int32)
    with pytest.raises(ValueError, match="shape"):
        pack_maps([np.zeros((4, 3), bool)], 3, 4, bits, fr)
    with pytest.raises(TypeError, match="boolean"):
        pack_maps([np.zeros((3, 4), np.uint8)], 3, 4, bits, fr)
    with pytest.raises(ValueError, match="streamed"):
        ap.ArrayFloorMapDataset.host_pool(ForeignFloorMapView(Big(2**31)))


def test_device_u8_pools_are_padded_for_the_dword_taps():
    """apgym_capi.h: the glimpse kernels read u8 taps with whole-dword loads up to APG_U8_POOL_PAD - 1 bytes past the
    last image; a pool handed over as a tensor (a dataset's device_pool_tensors) is re-homed into a padded
    allocation unless its storage already extends that far (CPU tensors stand in for device ones here)."""
    import torch

    from ap_gym_amd import _native as N
    from ap_gym_amd.image_env import padded_device_pool_u8

    pool = torch.arange(10 * 4 * 5 * 3, dtype=torch.int64).remainder(251).to(torch.uint8).reshape(10, 4, 5, 3)
    padded = padded_device_pool_u8(pool)
    assert padded is not pool and torch.equal(padded, pool)
    assert padded.untyped_storage().nbytes() >= pool.numel() + N.APG_U8_POOL_PAD
    assert padded_device_pool_u8(padded) is padded  # already padded: used as is
    sliced = padded_device_pool_u8(torch.zeros(64, dtype=torch.uint8)[:48].view(2, 4, 6, 1))
    assert sliced.untyped_storage().nbytes() == 64  # 16 spare bytes behind the view: kept


@pytest.mark.parametrize("h,w", [(64, 64), (33, 29), (5, 6)])
def test_tiled_rgb_pool_layout(h, w):
    """APG_POOL_U8_TILED (apgym_capi.h): pixel (y, x) of image m at m * img + (y // 4) * ceil(W/8) * 128 +
    (y % 4) * 32 + (x // 8) * 128 + (x % 8) * 4 + channel, the 4th byte zero; built here on CPU tensors in chunks."""
    from ap_gym_amd import _native as N
    from ap_gym_amd.image_env import device_pool_u8_tiled, tiled_pool_bytes

    rng = np.random.default_rng(h * w)
    pool = rng.integers(0, 256, (5, h, w, 3), dtype=np.uint8)
    t = device_pool_u8_tiled(pool, "cpu", chunk=2)
    img, trow = tiled_pool_bytes(h, w), ((w + 7) // 8) * 128
    assert t.numel() == 5 * img and t.untyped_storage().nbytes() >= 5 * img + N.APG_U8_POOL_PAD
    b = t.numpy()
    m, y, x = np.meshgrid(np.arange(5), np.arange(h), np.arange(w), indexing="ij")
    off = m * img + (y // 4) * trow + (y % 4) * 32 + (x // 8) * 128 + (x % 8) * 4
    for ch in range(3):
        assert np.array_equal(b[off + ch], pool[..., ch])
    assert not b[off + 3].any()
