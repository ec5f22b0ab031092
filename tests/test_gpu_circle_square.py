"""GPU parity of the CircleSquare family: the device-rendered dataset pools (apg_circle_square_pool)
against the reference's renders (tests/golden/circle_square_data.npz) and the numpy oracle, the
registered ids end to end against reference traces (tests/golden/cs_env_*.npz), and the
hide-and-seek reward kernel (apg_hide_and_seek_reward) against the oracle at scale.

Bar: bit-exact, the cross-entropy-derived rewards of the prediction variants included (numpy's float32 exp / log
restated on the device; round 4 held them to |got - want| <= 1e-6 + 1e-6 |want|).
"""

import numpy as np
import pytest

from conftest import check_image_stats, golden
from test_oracle_golden import CS_DATA_CASES

pytestmark = pytest.mark.gpu

CE_TOL = 0.0  # (bit-exact: numpy's float32 exp / log restated on the device)


def _dataset(ap, name):
    kind, shape, ga, gb, ext = CS_DATA_CASES[name]
    if kind == "single":
        return ap.CircleSquareDataset(show_gradient=ga, image_shape=shape, object_extents=ext)
    return ap.DoubleCircleSquareDataset(ga, gb, image_shape=shape, object_extents=ext)


@pytest.mark.parametrize("name", sorted(CS_DATA_CASES))
def test_device_pool_matches_reference_renders(gpu, name):
    import ap_gym_amd as ap

    g = golden("circle_square_data.npz")
    ds = _dataset(ap, name)
    images, labels = ds.device_pool_tensors(gpu)  # the whole dataset, as the envs hold it
    assert images.shape[0] == int(g[f"{name}_len"])
    idx = g[f"{name}_idx"]
    sel = images[idx].cpu().numpy()
    assert sel.dtype == np.float32 and sel.shape == g[f"{name}_images"].shape
    assert np.array_equal(sel, g[f"{name}_images"])
    assert np.array_equal(labels[idx].cpu().numpy(), g[f"{name}_labels"])
    # the reference's dataset API (get_data_point_batch / __getitem__) renders the same points
    few = idx[:3]
    im, lb = ds.get_data_point_batch(few)
    assert np.array_equal(im, g[f"{name}_images"][:3]) and np.array_equal(lb, g[f"{name}_labels"][:3])


@pytest.mark.parametrize("name", ["cs28g", "cs20n", "csrect", "dcs15g", "dcs15n", "dcs15ab"])
def test_device_pool_matches_oracle_whole_dataset(gpu, name):
    import ap_gym_amd as ap
    from oracle import image_oracle as io

    kind, shape, ga, gb, ext = CS_DATA_CASES[name]
    ds = _dataset(ap, name)
    images, labels = ds.device_pool_tensors(gpu)
    want_i, want_l = io.circle_square_images(kind, shape, np.arange(len(ds)), ga, gb, ext)
    assert np.array_equal(images.cpu().numpy(), want_i)
    assert np.array_equal(labels.cpu().numpy(), want_l)


def test_double_circle_square_28_properties(gpu):
    """DoubleCircleSquare 28x28 (902 880 images, 2.8 GB): every image has pixels == 1 (the objects),
    all values lie in [0, 1], labels are 0/1/2 with the reference's pattern, and an index sample is
    bit-exact against the oracle."""
    import torch

    import ap_gym_amd as ap
    from oracle import image_oracle as io

    ds = ap.DoubleCircleSquareDataset(image_shape=(28, 28))
    images, labels = ds.device_pool_tensors(gpu)
    n = len(ds)
    assert images.shape == (n, 28, 28, 1)
    assert bool(((images >= 0) & (images <= 1)).all())
    assert bool((images.view(n, -1) == 1.0).any(dim=1).all())
    idx = torch.arange(n, device=gpu)
    want_l = torch.where((idx % 2) == ((idx // 2) % 2), idx % 2, torch.full_like(idx, 2)).to(torch.int32)
    assert torch.equal(labels, want_l)
    sample = np.random.default_rng(5).integers(0, n, 4096)
    want_i, _ = io.circle_square_images("double", (28, 28), sample, positions=ds.positions)
    assert np.array_equal(images[torch.as_tensor(sample, device=gpu)].cpu().numpy(), want_i)


ENV_TRACES = {  # golden: (env id, mask_prediction, sparse)
    "cs28": ("CircleSquare-v0", False, False),
    "csinv15n": ("CircleSquareInverted-s15-nograd-v0", False, False),
    "dcs15": ("DoubleCircleSquare-s15-v0", False, False),
    "hs28": ("CircleSquareHideAndSeek-v0", False, False),
    "hs28_sparse": ("CircleSquareHideAndSeek-sparse-v0", False, True),
}


def _check(name, got, want, want_dtype, tol):
    got = np.asarray(got)
    assert str(got.dtype) == str(want_dtype), (name, got.dtype, want_dtype)
    if tol:
        np.testing.assert_allclose(got, want, rtol=CE_TOL, atol=CE_TOL, err_msg=name)
    else:
        assert np.array_equal(got, want, equal_nan=got.dtype.kind == "f"), name


@pytest.mark.parametrize("name", sorted(ENV_TRACES))
def test_circle_square_ids_match_reference_trace(gpu, name):
    import ap_gym_amd as ap

    env_id, mask, sparse = ENV_TRACES[name]
    g = golden(f"cs_env_{name}.npz")
    lim, inv, n, steps, k = (int(v) for v in g["config"])
    env = ap.make_vec(env_id, num_envs=n)
    assert env.config.step_limit == lim and env.config.randomly_invert_labels == bool(inv)
    obs, info = env.reset(seed=int(g["seed"]))
    for key, v in obs.items():
        _check("reset_" + key, v, g["reset_" + key], g["reset_" + key].dtype, False)
    assert np.array_equal(info["index"], g["reset_index"])
    for t in range(steps):
        obs, rew, term, trunc, info = env.step({"action": g["actions"][t], "prediction": g["predictions"][t]})
        tgt = info["prediction"]["target"]
        fields = dict(obs, reward=rew, terminated=term, truncated=trunc, index=info["index"],
                      base_reward=info["base_reward"], loss=info["prediction"]["loss"])
        if sparse:
            fields.update(target=tgt["target"], weight=tgt["weight"])
        else:
            fields["target"] = tgt
        for key, v in fields.items():
            tol = key in ("loss", "reward")
            _check(f"step{t}_{key}", v, g["step_" + key][t], g["step_" + key + "_dtype"][t], tol)
        assert ("stats" in info) == bool(g["step_stats_mask"][t].any())
        if "stats" in info:
            check_image_stats(info["stats"], g, t, rtol=CE_TOL)
    env.close()


def test_hide_and_seek_no_prediction_reset_raises_like_reference(gpu):
    import ap_gym_amd as ap

    g = golden("cs_env_hs_noprediction_reset.npz")
    assert str(g["reset_error"]) == "KeyError:prediction"
    env = ap.make_vec("CircleSquareHideAndSeekNoPrediction-v0", num_envs=3)
    with pytest.raises(KeyError, match="prediction"):
        env.reset(seed=0)
    env.close()


@pytest.mark.parametrize("mask,sparse", [(False, False), (True, False), (False, True), (True, True)])
def test_hide_and_seek_matches_oracle_at_scale(gpu, mask, sparse):
    """4096 envs over two episodes (incl. the autoreset step): the wrapper's base_reward / reward
    equal the inner env's plus the oracle's additional reward, with the reference's dtypes."""
    import ap_gym_amd as ap
    from oracle import image_oracle as io

    n, steps = 4096, 36
    ds = ap.CircleSquareDataset(image_shape=(28, 28))
    cfg = ap.ImagePerceptionConfig(dataset=ds, step_limit=16)
    inner = ap.ImageClassificationVectorEnv(n, cfg)
    ref = ap.ImageClassificationVectorEnv(n, cfg)
    env = ap.CircleSquareHideAndSeekVectorWrapper(inner, mask_prediction=mask, sparse=sparse)
    if not mask:
        env.reset(seed=9)
    else:
        inner.reset(seed=9)
    ref.reset(seed=9)
    rng = np.random.default_rng(0)
    for t in range(steps):
        a = rng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = rng.standard_normal((n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": () if mask else p})
        robs, rrew, rterm, _, rinfo = ref.step({"action": a, "prediction": np.zeros((n, 2)) if mask else p})
        assert np.array_equal(obs["glimpse"], robs["glimpse"]) and np.array_equal(term, rterm)
        add = io.hide_and_seek_additional_reward(rinfo["index"], robs["glimpse_pos"], (28, 28), (5, 5), 1.0)
        base = rinfo["base_reward"].copy()
        base += add  # the reference's in-place update (float32 storage, float64 on the autoreset step)
        _check(f"t{t} base_reward", info["base_reward"], base, base.dtype, False)
        if mask:
            want = base
        elif sparse:
            want = base - rinfo["prediction"]["loss"] * np.full(n, bool(rterm[0]), dtype=np.float32)
        else:
            want = rrew + add
        _check(f"t{t} reward", rew, want, want.dtype, False)
        if sparse:
            assert np.array_equal(info["prediction"]["target"]["weight"], np.full(n, bool(rterm[0]), np.float32))
    env.close()
    ref.close()


def test_hide_and_seek_torch_backend_matches_numpy(gpu):
    import torch

    import ap_gym_amd as ap

    n = 512
    envs = [ap.make_vec("CircleSquareHideAndSeek-v0", num_envs=n, array_backend=b) for b in ("numpy", "torch")]
    outs = [e.reset(seed=4) for e in envs]
    assert np.array_equal(outs[0][0]["glimpse"], outs[1][0]["glimpse"].cpu().numpy())
    rng = np.random.default_rng(2)
    for t in range(40):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        p = rng.standard_normal((n, 2)).astype(np.float32)
        on = envs[0].step({"action": a, "prediction": p})
        ot = envs[1].step({"action": torch.as_tensor(a, device=gpu), "prediction": torch.as_tensor(p, device=gpu)})
        assert np.array_equal(on[1], ot[1].cpu().numpy()), t
        assert on[1].dtype == ot[1].cpu().numpy().dtype
        assert np.array_equal(on[4]["base_reward"], ot[4]["base_reward"].cpu().numpy()), t
    for e in envs:
        e.close()
