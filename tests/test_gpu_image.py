"""GPU parity of the image glimpse path: HIP kernels (through the C ABI) against numpy itself (the
vector-level streams), the reference-generated goldens (tests/golden/image_*.npz) and the numpy
oracle (oracle/image_oracle.py) at larger sizes.

Bar: bit-exact for every integer and float output (glimpses, positions, targets, MSE and cross-entropy losses,
rewards, RNG streams).  The cross-entropy loss runs numpy's own float32 exp / log algorithms on the device
(apg_image.hip: np_expf / np_logf, restated from numpy's AVX-512F loops), so it is compared bit for bit too
(round 4 held it to the north-star tolerance |got - want| <= 1e-6 + 1e-6 |want| with the device libm).
"""

import ctypes

import numpy as np
import pytest

from conftest import check_image_stats, golden

pytestmark = pytest.mark.gpu

CE_RTOL = 0.0  # (bit-exact: numpy's float32 exp / log restated on the device)
CE_ATOL = 0.0
GOLDEN_CASES = ["cls_mnist", "cls_tin", "cls_gray3_rect", "loc_mnist", "loc_tin12", "loc_rect",
                "cls_mnist_sparse", "loc_rect_sparse"]  # *_sparse: the "-sparse" ids (SparsifyVectorWrapper)


def _state_from_numpy(gen: np.random.Generator):
    st = gen.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    words = [s >> 64, s & (2**64 - 1), inc >> 64, inc & (2**64 - 1),
             (st["has_uint32"] & 0xFFFFFFFF) | ((st["uinteger"] & 0xFFFFFFFF) << 32)]
    return np.array(words, dtype=np.uint64).view(np.int64)


def _state_equal(dev_words: np.ndarray, gen: np.random.Generator) -> bool:
    want = _state_from_numpy(gen)
    got = dev_words.copy()
    if (want[4] & 0xFFFFFFFF) == 0:  # buffered word is irrelevant when nothing is buffered
        got[4] &= 0xFFFFFFFF
        want = want.copy()
        want[4] &= 0xFFFFFFFF
    return np.array_equal(got, want)


@pytest.mark.parametrize("bound", [1, 2, 10, 60000, 100000, 2**31 + 5, 3 * 2**30, 2**32 - 1, 2**32])
@pytest.mark.parametrize("n", [1, 7, 1000, 70001])
@pytest.mark.parametrize("pre", [0, 1])
def test_rng_fill_integers_matches_numpy(gpu, bound, n, pre):
    import torch

    from ap_gym_amd import _native as N

    gen = np.random.default_rng(1234 + n + bound % 1000)
    if pre:  # leave a buffered half word in the generator (next_uint32)
        gen.integers(0, 5)
    st = torch.as_tensor(_state_from_numpy(gen), device=gpu)
    out = torch.zeros(n, dtype=torch.int64, device=gpu)
    work = torch.zeros(max(1, N.lib().apg_rng_fill_work_elems(n, bound)), dtype=torch.int64, device=gpu)
    N.check(N.lib().apg_rng_fill(N.ptr(st), N.APG_DRAW_INTEGERS, n, 1, None, None, 3, bound, N.ptr(out),
                                 N.ptr(work), N.stream_handle(gpu)))
    want = gen.integers(3, 3 + bound, n)
    assert np.array_equal(out.cpu().numpy(), want)
    assert _state_equal(st.cpu().numpy(), gen)


@pytest.mark.parametrize("with_work", [False, True])
@pytest.mark.parametrize("n,cols", [(1, 2), (513, 2), (65536, 2), (1000, 1)])
def test_rng_fill_uniform_matches_numpy(gpu, n, cols, with_work):
    """Uniform draws with work=NULL (a second launch advances the state) and with a zeroed work buffer (the last
    workgroup advances it in the same launch, counting finished workgroups in work[0], which it leaves at 0)."""
    import torch

    from ap_gym_amd import _native as N

    gen = np.random.default_rng(77 + n)
    gen.integers(0, 3)  # buffered half word must survive next64 draws untouched
    st = torch.as_tensor(_state_from_numpy(gen), device=gpu)
    low = np.array([-1.0, -0.3][:cols])
    high = np.array([1.0, 0.3][:cols])
    out = torch.zeros((n, cols), dtype=torch.float64, device=gpu)
    lo_c = (ctypes.c_double * cols)(*low.tolist())
    rg_c = (ctypes.c_double * cols)(*(high - low).tolist())
    work = torch.zeros(1, dtype=torch.int64, device=gpu) if with_work else None
    for rep in range(2):  # the work buffer is reused as the env does: it must come back zeroed
        N.check(N.lib().apg_rng_fill(N.ptr(st), N.APG_DRAW_UNIFORM, n, cols, lo_c, rg_c, 0, 0, N.ptr(out),
                                     N.ptr(work) if with_work else None, N.stream_handle(gpu)))
        want = gen.uniform(low, high, (n, cols))
        assert np.array_equal(out.cpu().numpy(), want)
        assert _state_equal(st.cpu().numpy(), gen)
        if with_work:
            assert int(work[0]) == 0


# ---------------------------------------------------------------------------------------- glimpse
GLIMPSE_CASES = [  # (H, W, pool C, obs C, sensor, scale, dtype)
    (28, 28, 1, 1, (5, 5), 1.0, np.uint8),
    (64, 64, 3, 3, (12, 12), 1.0, np.uint8),
    (64, 64, 3, 3, (10, 10), 1.0, np.uint8),
    (20, 24, 1, 3, (5, 5), 1.5, np.uint8),
    (24, 20, 3, 3, (4, 4), 1.25, np.float32),
    (17, 31, 1, 1, (3, 3), 2.0, np.uint8),
]


def _cfg(N, n, kind, h, w, pc, c, sensor, scale, dtype, pool_len, k=10, top_k=10, points=0, cell=(0.0, 0.0)):
    return N.ImageConfig(num_envs=n, kind=kind, height=h, width=w, pool_channels=pc, channels=c,
                         pool_dtype=N.APG_POOL_U8 if dtype == np.uint8 else N.APG_POOL_F32, sensor_h=sensor[0],
                         sensor_w=sensor[1], step_limit=16, num_classes=k, invert_labels=0, top_k=top_k,
                         unique_points=points, num_envs_total=n, env_offset=0, pool_len=pool_len, sensor_scale=scale,
                         max_step=(ctypes.c_double * 2)(0.2, 0.2), cell=(ctypes.c_double * 2)(*cell), ce_scale=1.0,
                         ce_offset=0.0, mse_scale=1.0, mse_offset=0.0)


def _pool(rng, m, h, w, pc, dtype):
    if dtype == np.uint8:
        return rng.integers(0, 256, (m, h, w, pc), dtype=np.uint8)
    return rng.uniform(-0.2, 1.2, (m, h, w, pc)).astype(np.float32)


def _dev_pool(pool, dev):
    """The pool on the device as the envs upload it: u8 pools with APG_U8_POOL_PAD bytes of slack (apgym_capi.h)."""
    import torch

    from ap_gym_amd.image_env import device_pool_u8

    return device_pool_u8(pool, dev) if pool.dtype == np.uint8 else torch.as_tensor(pool, device=dev)


@pytest.mark.parametrize("case", range(len(GLIMPSE_CASES)))
def test_glimpse_matches_oracle(gpu, case):
    import torch

    from ap_gym_amd import _native as N
    from oracle import image_oracle as io

    h, w, pc, c, sensor, scale, dtype = GLIMPSE_CASES[case]
    rng = np.random.default_rng(case)
    n, npos, m = 37, 64, 9
    pool = _pool(rng, m, h, w, pc, dtype)
    index = rng.integers(0, m, n)
    pos = rng.uniform(-1, 1, (n, npos, 2))
    pos[:, :8] = np.array([[-1, -1], [1, 1], [-1, 1], [1, -1], [0, 0], [0.5, -0.5], [1, 0], [0, -1]])
    lim = io.sensor_pos_lim((h, w), sensor, scale)
    pos[:, 8, 0] = 3 / lim[0]  # grid-exact sensing points
    pos[:, 8, 1] = -2 / lim[1]
    cfg = _cfg(N, n, N.APG_IMAGE_CLASSIFY, h, w, pc, c, sensor, scale, dtype, m)
    out = torch.zeros((n, npos, sensor[0], sensor[1], c), dtype=torch.float32, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    idx_t, pos_t = (torch.as_tensor(x, device=gpu) for x in (index, pos))
    pool_t = _dev_pool(pool, gpu)
    N.check(N.lib().apg_image_glimpse(ctypes.byref(cfg), N.ptr(pool_t), N.ptr(idx_t), N.ptr(pos_t), 0, npos,
                                      N.ptr(out), N.ptr(err), N.stream_handle(gpu)))
    imgs = io.images_f32(pool, c)[index]
    want = io.glimpse(imgs, pos, sensor, scale)
    assert int(err.item()) == 0
    assert np.array_equal(out.cpu().numpy(), want)
    # float32 positions (the target glimpse path)
    pos32 = pos.astype(np.float32)
    pos32_t = torch.as_tensor(pos32, device=gpu)
    N.check(N.lib().apg_image_glimpse(ctypes.byref(cfg), N.ptr(pool_t), N.ptr(idx_t), N.ptr(pos32_t), 1, npos,
                                      N.ptr(out), N.ptr(err), N.stream_handle(gpu)))
    assert np.array_equal(out.cpu().numpy(), io.glimpse(imgs, pos32, sensor, scale))


def test_glimpse_out_of_bounds_flags_like_scipy(gpu):
    import torch

    from ap_gym_amd import _native as N
    from oracle import image_oracle as io

    rng = np.random.default_rng(5)
    h = w = 16
    pool = _pool(rng, 2, h, w, 1, np.uint8)
    sensor, scale = (5, 5), 0.5  # scale < 1 lets the sensing points leave the image at |pos| = 1
    for pos, dim in (([[0.0, 1.0]], 0), ([[1.0, 0.0]], 1), ([[1.0, 1.0]], 0)):
        pos = np.array([pos])
        with pytest.raises(ValueError, match=f"dimension {dim}"):
            io.glimpse(io.images_f32(pool, 1)[:1], pos, sensor, scale)
        cfg = _cfg(N, 1, N.APG_IMAGE_CLASSIFY, h, w, 1, 1, sensor, scale, np.uint8, 2)
        out = torch.zeros((1, 1, 5, 5, 1), dtype=torch.float32, device=gpu)
        err = torch.zeros(1, dtype=torch.int32, device=gpu)
        keep = [_dev_pool(pool, gpu), torch.zeros(1, dtype=torch.int64, device=gpu),
                torch.as_tensor(pos, device=gpu)]  # device buffers must outlive the async launch
        N.check(N.lib().apg_image_glimpse(ctypes.byref(cfg), *[N.ptr(x) for x in keep], 0, 1, N.ptr(out), N.ptr(err),
                                          N.stream_handle(gpu)))
        bits = int(err.item())
        assert bits & (N.APG_ERR_OOB_Y if dim == 0 else N.APG_ERR_OOB_X)
        if dim == 1:
            assert not bits & N.APG_ERR_OOB_Y


# L = G*G*C: 25 and 108 (one leaf of numpy's pairwise sum), 432 (4 leaves), 300 (leaf tail), 4 (a leaf
# shorter than 8), 768 (deeper combine stack); knobs: the generic kernel, and few workgroups (env striding)
@pytest.mark.parametrize("h,w,c,sensor,n,knob", [(28, 28, 1, (5, 5), 24, None), (32, 32, 3, (6, 6), 6, None),
                                                 (64, 64, 3, (12, 12), 2, None), (32, 32, 3, (10, 10), 4, None),
                                                 (16, 16, 1, (2, 2), 3, None), (64, 64, 3, (16, 16), 2, None),
                                                 (64, 64, 3, (12, 12), 2, "APG_UNIQUE_GENERIC=1"),
                                                 (28, 28, 1, (5, 5), 24, "APG_UNIQUE_GRID=5")])
def test_unique_top_k_matches_oracle(gpu, h, w, c, sensor, n, knob, monkeypatch):
    import torch

    if knob:
        monkeypatch.setenv(*knob.split("="))

    from ap_gym_amd import _native as N
    from ap_gym_amd.image_env import unique_sampling_grid
    from oracle import image_oracle as io

    rng = np.random.default_rng(h + n)
    pool = _pool(rng, n, h, w, c, np.uint8)
    index = np.arange(n)
    grid, cell = unique_sampling_grid((h, w), sensor, 1.0)
    top, g_grid, g_cell, u = io.unique_top_k(io.images_f32(pool, c), sensor, 1.0, 10)
    assert np.array_equal(grid, g_grid) and np.array_equal(cell, g_cell)
    p = grid.shape[0]
    cfg = _cfg(N, n, N.APG_IMAGE_LOCALIZE, h, w, c, c, sensor, 1.0, np.uint8, n, top_k=10, points=p)
    top_d = torch.zeros((n, 10), dtype=torch.int32, device=gpu)
    uniq = torch.zeros((n, p), dtype=torch.float32, device=gpu)
    keep = [_dev_pool(pool, gpu)] + [torch.as_tensor(x, device=gpu) for x in (index, grid)]
    N.check(N.lib().apg_image_unique_top_k(ctypes.byref(cfg), *[N.ptr(x) for x in keep], p, 10, N.ptr(top_d),
                                           N.ptr(uniq), N.stream_handle(gpu)))
    assert np.array_equal(uniq.cpu().numpy().astype(np.float64), u)
    assert np.array_equal(top_d.cpu().numpy(), top)


# ---------------------------------------------------------------------------------------- losses
@pytest.mark.parametrize("k", [2, 10, 200, 1000])
def test_ce_loss_kernel_bit_exact(gpu, k):
    import scipy.special
    import torch

    from ap_gym_amd import _native as N

    rng = np.random.default_rng(k)
    n = 4099
    logits = (rng.standard_normal((n, k)) * 4).astype(np.float32)
    logits[0, 0] = -np.inf
    target = rng.integers(0, k, n).astype(np.int32)
    scale = 1 / np.log(k)
    out = torch.zeros(n, dtype=torch.float64, device=gpu)
    keep = [torch.as_tensor(x, device=gpu) for x in (logits, target)]
    N.check(N.lib().apg_loss_ce(*[N.ptr(x) for x in keep], n, k, float(scale), -0.0, N.ptr(out),
                                N.stream_handle(gpu)))
    want = -np.take_along_axis(scipy.special.log_softmax(logits, axis=-1), target[:, None], -1)[:, 0] * scale + -0.0
    assert np.array_equal(out.cpu().numpy(), want)


def test_ce_loss_kernel_exp_log_sweep(gpu):
    """numpy's float32 exp / log on the device over a million inputs: rows [0, -t] for t sampled across [0, 104]
    (every exp the log-softmax can underflow to), i.e. exp(-t) and log(1 + exp(-t)), and rows of K = 1000 equal
    logits but one (log of sums up to 1000)."""
    import scipy.special
    import torch

    from ap_gym_amd import _native as N

    t = np.linspace(0.0, 104.0, 1 << 20, dtype=np.float32)
    logits = np.stack([np.zeros_like(t), -t], axis=1)
    target = (np.arange(len(t)) % 2).astype(np.int32)
    rng = np.random.default_rng(7)
    wide = np.zeros((4096, 1000), np.float32)
    wide[:, 0] = rng.uniform(-20, 20, 4096).astype(np.float32)
    for lg, tg, k in ((logits, target, 2), (wide, rng.integers(0, 1000, 4096).astype(np.int32), 1000)):
        n = lg.shape[0]
        out = torch.zeros(n, dtype=torch.float64, device=gpu)
        keep = [torch.as_tensor(x, device=gpu) for x in (lg, tg)]
        N.check(N.lib().apg_loss_ce(*[N.ptr(x) for x in keep], n, k, 1.0, -0.0, N.ptr(out), N.stream_handle(gpu)))
        want = -np.take_along_axis(scipy.special.log_softmax(lg, axis=-1), tg[:, None], -1)[:, 0] * 1.0 + -0.0
        got = out.cpu().numpy()
        assert np.array_equal(got, want), int((got != want).sum())


@pytest.mark.parametrize("d", [1, 2, 7, 130])
def test_mse_loss_kernel_bit_exact(gpu, d):
    import torch

    from ap_gym_amd import _native as N

    rng = np.random.default_rng(d)
    n = 1000
    p, t = rng.standard_normal((2, n, d)).astype(np.float32)
    out = torch.zeros(n, dtype=torch.float32, device=gpu)
    keep = [torch.as_tensor(x, device=gpu) for x in (p, t)]
    N.check(N.lib().apg_loss_mse(*[N.ptr(x) for x in keep], n, d, 3.0, -0.0, N.ptr(out), N.stream_handle(gpu)))
    assert np.array_equal(out.cpu().numpy(), np.mean((p - t) ** 2, axis=-1) * 3.0 + -0.0)


# ---------------------------------------------------------------------------------------- envs
def _make_env(ap, g, backend="numpy", n=None, copy=False, log_stats=False, sparse=False):
    h, w, c, k, s0, s1, lim, inv, n_g, _ = (int(v) for v in g["config"])
    ds = ap.ArrayImageClassificationDataset(g["pool"], g["labels"], k, c)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(s0, s1), sensor_scale=float(g["sensor_scale"]),
                                   step_limit=lim, randomly_invert_labels=bool(inv))
    cls = ap.ImageClassificationVectorEnv if str(g["kind"]) == "cls" else ap.ImageLocalizationVectorEnv
    return cls(n or n_g, cfg, array_backend=backend, copy=copy, log_stats=log_stats, sparse=sparse)


def _assert_field(name, got, want, want_dtype, ce, key=None):
    got = np.asarray(got)
    assert str(got.dtype) == str(want_dtype), (name, got.dtype, want_dtype)
    if ce and (key or name) in ("loss", "reward"):
        np.testing.assert_allclose(got, want, rtol=CE_RTOL, atol=CE_ATOL, err_msg=name)  # NaN == NaN
    else:
        assert np.array_equal(got, want, equal_nan=got.dtype.kind == "f"), name


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_image_env_matches_reference_trace(gpu, name):
    import ap_gym_amd as ap

    g = golden(f"image_{name}.npz")
    env = _make_env(ap, g, log_stats=True, sparse=name.endswith("_sparse"))
    ce = str(g["kind"]) == "cls"
    obs, info = env.reset(seed=int(g["seed"]))
    for k, v in obs.items():
        _assert_field("reset_" + k, v, g["reset_" + k], g["reset_" + k].dtype, False)
    assert np.array_equal(info["index"], g["reset_index"])
    steps = int(g["config"][-1])
    for t in range(steps):
        obs, rew, term, trunc, info = env.step({"action": g["actions"][t], "prediction": g["predictions"][t]})
        tgt = info["prediction"]["target"]
        fields = dict(obs, reward=rew, terminated=term, truncated=trunc, index=info["index"],
                      base_reward=info["base_reward"], loss=info["prediction"]["loss"])
        if env.sparse:
            assert set(tgt) == {"target", "weight"}
            fields.update(target=tgt["target"], weight=tgt["weight"])
        else:
            fields["target"] = tgt
        assert set(fields) | {"stats_mask"} == {k[5:] for k in g.files if k.startswith("step_") and not k.endswith("_dtype")}
        for k, v in fields.items():
            _assert_field(f"step{t}_{k}", v, g["step_" + k][t], g["step_" + k + "_dtype"][t], ce, key=k)
        # vector log wrapper statistics (correct_label_prob uses the device exp: north-star tolerance)
        assert ("stats" in info) == bool(g["step_stats_mask"][t].any())
        if "stats" in info:
            check_image_stats(info["stats"], g, t, rtol=CE_RTOL if ce else 0.0)
    env.close()


@pytest.mark.parametrize("kind,n,shape,sensor,k,steps", [("cls", 2048, (28, 28), (5, 5), 10, 40),
                                                         ("cls", 256, (64, 64, 3), (10, 10), 200, 20),
                                                         ("loc", 48, (28, 28), (5, 5), 10, 36),
                                                         # k_image_env_cls1 / the fused step for K <= 16:
                                                         # the < 8 sequential sum, k % 8 == 0 without a
                                                         # tail, odd K (odd LDS stride), the K = 16 edge,
                                                         # and a partial last workgroup (n % 128 != 0)
                                                         ("cls", 2000, (28, 28), (5, 5), 2, 20),
                                                         ("cls", 2000, (28, 28), (5, 5), 3, 20),
                                                         ("cls", 2000, (28, 28), (5, 5), 8, 20),
                                                         ("cls", 2000, (28, 28), (5, 5), 13, 20),
                                                         ("cls", 2000, (28, 28), (5, 5), 16, 20)])
def test_image_env_matches_oracle_at_scale(gpu, kind, n, shape, sensor, k, steps):
    _env_vs_oracle(kind, n, shape, sensor, k, steps)


@pytest.mark.parametrize("kind,n,shape,sensor,k,steps,scale", [
    ("loc", 300, (33, 29, 3), (6, 6), 5, 20, 1.7),    # odd row pitch (87 B): per-row dword alignment of the box
    ("cls", 300, (31, 27), (5, 5), 10, 20, 1.3),      # grey, odd pitch
    ("cls", 200, (17, 19, 3), (5, 5), 4, 20, 2.0),    # box rows clipped to the image (min(h, ...))
    ("cls", 130, (12, 14), (4, 4), 5, 20, 3.0)])      # box rows = the whole image (h = 12)
def test_image_env_box_staging_edges(gpu, kind, n, shape, sensor, k, steps, scale):
    """The fused step's LDS box staging (u8 pools): odd pitches, scales != 1, boxes clipped at the image border;
    bit-exact vs the oracle like every other configuration."""
    _env_vs_oracle(kind, n, shape, sensor, k, steps, scale)


def _env_vs_oracle(kind, n, shape, sensor, k, steps, scale=1.0):
    import ap_gym_amd as ap
    from oracle import image_oracle as io

    rng = np.random.default_rng(n)
    pool = rng.integers(0, 256, (300, *shape), dtype=np.uint8)
    labels = rng.integers(0, k, 300)
    c = 1 if len(shape) == 2 else shape[-1]
    ds = ap.ArrayImageClassificationDataset(pool, labels, k, c)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=sensor, sensor_scale=scale, step_limit=16)
    env = (ap.ImageClassificationVectorEnv if kind == "cls" else ap.ImageLocalizationVectorEnv)(n, cfg)
    ref = io.ImageVectorEnvOracle(kind, pool, labels, k, c, n, sensor, scale, 16)
    obs, info = env.reset(seed=11)
    robs, rinfo = ref.reset(11)
    for key in robs:
        assert np.array_equal(obs[key], robs[key]), key
    arng = np.random.default_rng(3)
    for t in range(steps):
        a = arng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = (arng.standard_normal((n, k)) if kind == "cls" else arng.uniform(-1, 1, (n, 2))).astype(np.float32)
        got = env.step({"action": a, "prediction": p})
        want = ref.step(a, p)
        for key in want[0]:
            assert np.array_equal(got[0][key], want[0][key]), (t, key)
        for i, name in ((1, "reward"), (2, "terminated"), (3, "truncated")):
            _assert_field(name, got[i], want[i], want[i].dtype, kind == "cls")
        gi, wi = got[4], want[4]
        assert np.array_equal(gi["index"], wi["index"])
        _assert_field("base_reward", gi["base_reward"], wi["base_reward"], wi["base_reward"].dtype, False)
        _assert_field("target", gi["prediction"]["target"], wi["prediction"]["target"],
                      np.asarray(wi["prediction"]["target"]).dtype, False)
        _assert_field("loss", gi["prediction"]["loss"], wi["prediction"]["loss"], wi["prediction"]["loss"].dtype,
                      kind == "cls")
    env.close()


@pytest.mark.parametrize("via_op", [False, True], ids=["c_abi", "torch_op"])
@pytest.mark.parametrize("kind,sparse", [("cls", False), ("loc", False), ("cls", True), ("loc", True)])
def test_image_env_torch_backend_matches_numpy(gpu, kind, sparse, via_op):
    """The torch backend equals the numpy backend, with eager steps through the C ABI (default) and
    through torch.ops.apgym.image_step (use_torch_op)."""
    import torch

    import ap_gym_amd as ap

    if sparse:
        g = golden("image_cls_mnist_sparse.npz" if kind == "cls" else "image_loc_rect_sparse.npz")
    else:
        g = golden("image_cls_mnist.npz" if kind == "cls" else "image_loc_mnist.npz")
    e_np, e_t = _make_env(ap, g, sparse=sparse), _make_env(ap, g, backend="torch", copy=True, sparse=sparse)
    e_t.use_torch_op = via_op
    o1, _ = e_np.reset(seed=5)
    o2, _ = e_t.reset(seed=5)
    for k in o1:
        assert np.array_equal(o1[k], o2[k].cpu().numpy()), k
    for t in range(int(g["config"][-1])):
        act = {"action": g["actions"][t], "prediction": g["predictions"][t]}
        r1 = e_np.step(act)
        r2 = e_t.step(act)
        for k in r1[0]:
            assert np.array_equal(r1[0][k], r2[0][k].cpu().numpy()), (t, k)
        assert np.array_equal(r1[1].astype(np.float64), r2[1].cpu().numpy(), equal_nan=True)
        assert np.array_equal(r1[2], r2[2].cpu().numpy())
        assert np.array_equal(r1[4]["prediction"]["loss"], r2[4]["prediction"]["loss"].cpu().numpy())
        if sparse:
            w1, w2 = r1[4]["prediction"]["target"]["weight"], r2[4]["prediction"]["target"]["weight"]
            assert w2.dtype == torch.float32 and np.array_equal(w1, w2.cpu().numpy())
            assert np.array_equal(r1[4]["prediction"]["target"]["target"],
                                  r2[4]["prediction"]["target"]["target"].cpu().numpy())
    e_t.check_errors()


@pytest.mark.parametrize("kind", ["cls", "loc"])
def test_image_env_shards_equal_unsharded(gpu, kind):
    """Each shard draws the whole batch from the same streams and keeps its slice (ap_gym_amd.sharding)."""
    import ap_gym_amd as ap

    g = golden("image_cls_gray3_rect.npz" if kind == "cls" else "image_loc_mnist.npz")
    h, w, c, k, s0, s1, lim, inv, n, steps = (int(v) for v in g["config"])
    ds = ap.ArrayImageClassificationDataset(g["pool"], g["labels"], k, c)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(s0, s1), sensor_scale=float(g["sensor_scale"]),
                                   step_limit=lim, randomly_invert_labels=bool(inv))
    cls = ap.ImageClassificationVectorEnv if kind == "cls" else ap.ImageLocalizationVectorEnv
    full = cls(n, cfg)
    half = n // 2
    shards = [cls(half, cfg, num_envs_total=n, env_offset=r * half) for r in range(2)]
    outs = [e.reset(seed=3) for e in [full] + shards]
    for key in outs[0][0]:
        assert np.array_equal(outs[0][0][key], np.concatenate([outs[1][0][key], outs[2][0][key]])), key
    for t in range(steps):
        act = {"action": g["actions"][t], "prediction": g["predictions"][t]}
        f = full.step(act)
        parts = [e.step({kk: v[r * half:(r + 1) * half] for kk, v in act.items()}) for r, e in enumerate(shards)]
        for key in f[0]:
            assert np.array_equal(f[0][key], np.concatenate([p[0][key] for p in parts])), (t, key)
        for i in (1, 2, 3):
            assert np.array_equal(f[i], np.concatenate([p[i] for p in parts])), (t, i)
        for key in ("index", "base_reward"):
            assert np.array_equal(f[4][key], np.concatenate([p[4][key] for p in parts])), (t, key)
        for key in ("target", "loss"):
            assert np.array_equal(f[4]["prediction"][key], np.concatenate([p[4]["prediction"][key] for p in parts]))


def test_image_env_nan_errors(gpu):
    import ap_gym_amd as ap

    g = golden("image_cls_mnist.npz")
    for backend in ("numpy", "torch"):
        env = _make_env(ap, g, backend=backend)
        env.reset(seed=0)
        a = g["actions"][0].copy()
        p = g["predictions"][0].copy()
        a[3, 1] = np.nan
        with pytest.raises(ValueError, match="action"):
            env.step({"action": a, "prediction": p})
            env.check_errors()
        env.reset(seed=0)
        p[2, :] = -np.inf
        with pytest.raises(ValueError, match="prediction"):
            env.step({"action": g["actions"][0], "prediction": p})
            env.check_errors()
        env.close()


@pytest.mark.parametrize("gname", ["image_cls_mnist.npz"])
def test_image_numpy_vector_stats_array_mode(gpu, gname):
    """vector_stats="array" on the image envs: float32 row views holding the values of the reference's
    np.float32 lists (update_info_metrics_vec, util.py:68-77); anything else is a ValueError."""
    import ap_gym_amd as ap

    g = golden(gname)
    h, w, c, k, s0, s1, lim, inv, n_g, _ = (int(v) for v in g["config"])
    ds = ap.ArrayImageClassificationDataset(g["pool"], g["labels"], k, c)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(s0, s1), sensor_scale=float(g["sensor_scale"]),
                                   step_limit=lim, randomly_invert_labels=bool(inv))
    e1 = ap.ImageClassificationVectorEnv(n_g, cfg, log_stats=True)
    e2 = ap.ImageClassificationVectorEnv(n_g, cfg, log_stats=True, vector_stats="array")
    e1.reset(seed=0)
    e2.reset(seed=0)
    seen = 0
    for t in range(len(g["actions"])):
        act = {"action": g["actions"][t], "prediction": g["predictions"][t]}
        i1, i2 = e1.step(act)[4], e2.step(act)[4]
        assert ("stats" in i1) == ("stats" in i2)
        if "stats" in i1:
            for name, v1 in i1["stats"]["vector"].items():
                if name.startswith("_"):
                    continue
                v2 = i2["stats"]["vector"][name]
                for j in range(n_g):
                    assert isinstance(v1[j], list) and isinstance(v1[j][0], np.float32)
                    assert isinstance(v2[j], np.ndarray) and v2[j].dtype == np.float32
                    assert np.array_equal(np.array(v1[j], np.float32), v2[j], equal_nan=True)
                    seen += 1
    assert seen > 0
    e1.close()
    e2.close()
    with pytest.raises(ValueError):
        ap.ImageClassificationVectorEnv(n_g, cfg, vector_stats="bad")


def test_image_cls_full_size_properties(gpu):
    """BASELINE config 4 (MNIST-shaped classification, N = 65536, 5x5 glimpse): bounded glimpses,
    clipped positions, reset cadence, label targets from the pool."""
    import torch

    import ap_gym_amd as ap

    ds = ap.SyntheticImageClassificationDataset(60000, (28, 28), 10, seed=0)
    env = ap.ImageClassificationVectorEnv(65536, ap.ImagePerceptionConfig(dataset=ds), array_backend="torch")
    obs, info = env.reset(seed=0)
    pool_labels = torch.as_tensor(ds.device_pool()[1], device=gpu)
    g = torch.Generator(device=gpu).manual_seed(0)
    for t in range(40):
        a = torch.rand((65536, 2), generator=g, device=gpu) * 3 - 1.5
        p = torch.randn((65536, 10), generator=g, device=gpu)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        assert bool(((obs["glimpse"] >= 0) & (obs["glimpse"] <= 1)).all())
        assert bool((obs["glimpse_pos"].abs() <= 1).all())
        assert bool((info["prediction"]["target"] == pool_labels[info["index"]]).all())
        assert bool(term.all()) == (t % 17 == 15)
    env.check_errors()
    env.close()


def test_image_loc_full_size_cfg5(gpu):
    """BASELINE config 5 itself (TinyImageNetLoc shape: N = 32768, 64x64x3 pool of 100000, 12x12 glimpse,
    MSE) including the unique-sampler reset: reset targets in [-1, 1], glimpses in [0, 1]; for sampled
    envs the uniqueness ranking equals image_oracle.unique_top_k on their images, and their complete
    first episode (glimpse, glimpse_pos, target glimpse, reward, loss) equals an ImageVectorEnvOracle
    started from their reset state."""
    import torch

    import ap_gym_amd as ap
    from oracle import image_oracle as io

    n, sensor = 32768, (12, 12)
    ds = ap.SyntheticImageClassificationDataset(100000, (64, 64, 3), 200, 3, seed=0)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=sensor, step_limit=16)
    env = ap.ImageLocalizationVectorEnv(n, cfg, array_backend="torch")
    obs, info = env.reset(seed=0)
    T = env._t
    tgt = T["target"]
    assert bool(((tgt >= -1) & (tgt <= 1)).all())
    assert bool(((obs["glimpse"] >= 0) & (obs["glimpse"] <= 1)).all())
    assert bool(((obs["target_glimpse"] >= 0) & (obs["target_glimpse"] <= 1)).all())
    sample = np.sort(np.random.default_rng(5).choice(n, 6, replace=False))
    sel = torch.as_tensor(sample, device=gpu)
    pool, labels = ds.device_pool()
    idx = info["index"][sel].cpu().numpy()
    ref = io.ImageVectorEnvOracle("loc", pool, labels, 200, 3, len(sample), sensor, step_limit=16)
    ref.seed(0)  # the per-env state below replaces everything the batch-level streams would draw
    top_ref, _, _, _ = io.unique_top_k(ref.pool[idx], sensor, 1.0, int(cfg.unique_sampling_top_k))
    assert np.array_equal(T["top_k"][sel].cpu().numpy(), top_ref)
    ref.idx, ref.images, ref.cur_labels = idx, ref.pool[idx], ref.labels_pool[idx]
    ref.pos = T["pos"][sel].cpu().numpy().astype(np.float64)
    ref.target = tgt[sel].cpu().numpy().astype(np.float32)
    ref.t, ref.prev_done, ref.env_prev_done = 0, np.zeros(len(sample), bool), np.zeros(len(sample), bool)
    ref.hist, ref.log_prev_done = [[] for _ in sample], np.zeros(len(sample), bool)
    assert np.array_equal(obs["glimpse"][sel].cpu().numpy(), io.glimpse(ref.images, ref.pos, sensor, 1.0))
    g = torch.Generator(device=gpu).manual_seed(1)
    for t in range(1, 21):
        a = torch.rand((n, 2), generator=g, device=gpu) * 2 - 1
        p = torch.rand((n, 2), generator=g, device=gpu) * 2 - 1
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        assert bool(((obs["glimpse"] >= 0) & (obs["glimpse"] <= 1)).all())
        assert bool((obs["glimpse_pos"].abs() <= 1).all())
        assert bool(term.all()) == (t == 16)
        if t <= 16:  # the first episode of the sampled envs, step by step
            ro, rr, rt, _, ri = ref.step(a[sel].cpu().numpy(), p[sel].cpu().numpy())
            assert np.array_equal(obs["glimpse"][sel].cpu().numpy(), ro["glimpse"]), t
            assert np.array_equal(obs["glimpse_pos"][sel].cpu().numpy(), ro["glimpse_pos"]), t
            assert np.array_equal(obs["target_glimpse"][sel].cpu().numpy(), ro["target_glimpse"]), t
            assert np.array_equal(rew[sel].cpu().numpy(), np.asarray(rr, np.float64)), t
            assert np.array_equal(info["prediction"]["loss"][sel].cpu().numpy(), ri["prediction"]["loss"]), t
    env.check_errors()
    env.close()


@pytest.mark.parametrize("knobs", [{"APG_GLIMPSE_PPT": "9"}, {"APG_CLS_LANES8": "1"}, {"APG_IMAGE_UNFUSED": "1"},
                                   {"APG_GLIMPSE_PPT": "16", "APG_IMAGE_UNFUSED": "1"}, {"APG_IMAGE_ENV_WAVE": "0"},
                                   {"APG_IMAGE_ENV_WAVE": "1", "APG_GLIMPSE_PPT": "3"}])
def test_tuning_knobs_do_not_change_results(gpu, tmp_path, knobs):
    """The library reads its tuning knobs once per process, so each setting runs in a child process
    (tests/knob_child.py) and must reproduce the default-knob child bit for bit: another glimpse
    workgroup size, the 8-lane classification kernel for K <= 16, the two-launch step, the fused step with
    and without its env wave."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))

    def run(env_extra, name):
        env = {k: v for k, v in os.environ.items() if not k.startswith("APG_")}
        env.update(env_extra)
        out = tmp_path / name
        subprocess.run([sys.executable, os.path.join(here, "knob_child.py"), str(out)], env=env, check=True,
                       timeout=300)
        return np.load(out)

    base = run({}, "base.npz")
    got = run(knobs, "knob.npz")
    assert set(base.files) == set(got.files)
    for key in base.files:
        assert np.array_equal(base[key], got[key]), key


@pytest.mark.parametrize("kind,invert,backend,limit", [("cls", True, "torch", 5), ("loc", False, "torch", 5),
                                                       ("cls", False, "numpy", 5), ("loc", False, "numpy", 5),
                                                       ("cls", True, "torch", 1), ("loc", False, "numpy", 2)])
def test_draw_ahead_matches_drawing_at_the_autoreset(gpu, kind, invert, backend, limit):
    """The next batch's draws made ahead on the side stream (apg_image_draw_ahead, installed by the fused step
    kernel) give the outputs of drawing them in the autoreset step, across autoresets, a reset() (the streams are
    restored from before the draws made ahead) and a reset(seed); also with episodes of 1 and 2 steps."""
    import torch

    import ap_gym_amd as ap

    ch = 3 if kind == "loc" else 1
    ds = ap.SyntheticImageClassificationDataset(64, (32, 32, 3) if ch == 3 else (28, 28), 10, ch, seed=3)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(8, 8) if kind == "loc" else (5, 5), step_limit=limit,
                                   randomly_invert_labels=invert)
    cls = ap.ImageLocalizationVectorEnv if kind == "loc" else ap.ImageClassificationVectorEnv
    n = 300
    envs = [cls(n, cfg, array_backend=backend, draw_ahead=d) for d in (True, False)]
    assert envs[0]._ahead_stream is not None and envs[1]._ahead_stream is None
    rng = np.random.default_rng(6)

    def same(x, y, what):
        if isinstance(x, dict):
            assert x.keys() == y.keys(), what
            for k in x:
                same(x[k], y[k], f"{what}/{k}")
        elif isinstance(x, torch.Tensor):
            assert torch.equal(x.cpu(), y.cpu()), what
        else:
            assert np.array_equal(np.asarray(x), np.asarray(y), equal_nan=True), what

    def run(steps):
        for t in range(steps):
            a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
            p = (rng.standard_normal((n, 10)) if kind == "cls" else rng.uniform(-1, 1, (n, 2))).astype(np.float32)
            if backend == "torch":
                a, p = torch.from_numpy(a).to(gpu), torch.from_numpy(p).to(gpu)
            out = [e.step({"action": a, "prediction": p}) for e in envs]
            for i, what in enumerate(("obs", "reward", "terminated", "truncated", "info")):
                same(out[0][i], out[1][i], f"step {t} {what}")

    for e in envs:
        e.reset(seed=4)
    run(14)  # two batch autoresets
    outs = [e.reset() for e in envs]  # mid-episode reset(): the batch drawn from the restored streams
    same(outs[0][0], outs[1][0], "reset obs")
    same(outs[0][1], outs[1][1], "reset info")
    run(8)
    outs = [e.reset(seed=9) for e in envs]
    same(outs[0][0], outs[1][0], "reset(seed) obs")
    run(7)
    for e in envs:
        e.check_errors()
        e.close()


@pytest.mark.parametrize("snapshot", ["copy", "shared"])
def test_image_numpy_returned_arrays_are_writable(gpu, snapshot):
    """The reference computes every observation anew each step (image_localization.py:142-146, 170-174): a caller
    may write into them.  Writes into every returned array on consecutive steps (target glimpse included) leave the
    next steps' values unaffected (checked against the oracle across a batch change); obs_snapshot="shared" (opt-in)
    returns the target glimpse as a read-only array shared by a batch's steps."""
    import ap_gym_amd as ap
    from oracle import image_oracle as io

    n, k, sensor, shape = 96, 10, (5, 5), (28, 28)
    rng = np.random.default_rng(4)
    pool = rng.integers(0, 256, (64, *shape), dtype=np.uint8)
    labels = rng.integers(0, k, 64)
    ds = ap.ArrayImageClassificationDataset(pool, labels, k, 1)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=sensor, step_limit=4)
    env = ap.ImageLocalizationVectorEnv(n, cfg, obs_snapshot=snapshot)
    ref = io.ImageVectorEnvOracle("loc", pool, labels, k, 1, n, sensor, 1.0, 4)
    env.reset(seed=2)
    ref.reset(2)
    arng = np.random.default_rng(1)
    for t in range(11):  # two batch changes
        a = arng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = arng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        want = ref.step(a, p)
        for key in want[0]:
            assert np.array_equal(obs[key], want[0][key]), (t, key)
        assert np.array_equal(rew, want[1]), t
        for key, v in obs.items():
            if key == "target_glimpse" and snapshot == "shared":
                assert not v.flags.writeable
                continue
            v[...] = 5
        rew[...] = -1
        info["prediction"]["target"][...] = 9
    env.close()


@pytest.mark.parametrize("kind,shape,sensor,scale", [("loc", (64, 64, 3), (12, 12), 1.0),
                                                     ("cls", (33, 29, 3), (6, 6), 1.7),
                                                     ("loc", (17, 19, 3), (5, 5), 2.0)])
def test_tiled_rgb_pool_matches_row_major(gpu, monkeypatch, kind, shape, sensor, scale):
    """RGB u8 pools run as RGBX 8 x 4-pixel tiles (APG_POOL_U8_TILED) by default: every output of reset (the unique
    sampler's targets included) and of 40 steps across batch changes equals the row-major pool's (APG_IMAGE_TILED=0),
    which the oracle suites pin."""
    import torch

    import ap_gym_amd as ap
    from ap_gym_amd import _native as N

    rng = np.random.default_rng(7)
    pool = rng.integers(0, 256, (50, *shape), dtype=np.uint8)
    labels = rng.integers(0, 10, 50)
    envs = []
    for tiled in ("1", "0"):
        monkeypatch.setenv("APG_IMAGE_TILED", tiled)
        ds = ap.ArrayImageClassificationDataset(pool, labels, 10, 3)
        cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=sensor, sensor_scale=scale, step_limit=16)
        cls = ap.ImageClassificationVectorEnv if kind == "cls" else ap.ImageLocalizationVectorEnv
        envs.append(cls(512, cfg, array_backend="torch"))
    assert envs[0]._cfg.pool_dtype == N.APG_POOL_U8_TILED and envs[1]._cfg.pool_dtype == N.APG_POOL_U8
    outs = [e.reset(seed=3) for e in envs]
    for k in outs[0][0]:
        assert torch.equal(outs[0][0][k], outs[1][0][k]), k
    arng = np.random.default_rng(2)
    for t in range(40):
        a = torch.as_tensor(arng.uniform(-1.5, 1.5, (512, 2)).astype(np.float32), device=gpu)
        p = torch.as_tensor((arng.standard_normal((512, 10)) if kind == "cls" else arng.uniform(-1, 1, (512, 2)))
                            .astype(np.float32), device=gpu)
        r = [e.step({"action": a, "prediction": p}) for e in envs]
        for k in r[0][0]:
            assert torch.equal(r[0][0][k], r[1][0][k]), (t, k)
        assert torch.equal(r[0][1], r[1][1]), t
    for e in envs:
        e.check_errors()
        e.close()
