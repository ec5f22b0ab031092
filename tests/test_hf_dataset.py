"""HF data ingestion: ap_gym_amd.HuggingfaceImageClassificationDataset against the
reference's HuggingfaceImageClassificationDataset (huggingface_image_classification_dataset.py:12-80) on
small local datasets (tests/golden/hf_dataset.npz, make_golden.py `hf`): the same PNG-encoded parquet
directory is rebuilt here from the fixture's arrays and loaded offline with `datasets.load_dataset`.
Checks lengths, class counts, filter_labels remapping, processed batches and the device pool upload
arrays.  Host logic only (no GPU)."""

import os

import numpy as np
import pytest

from conftest import golden

NAMES = ["zero", "one", "two", "three", "four"]


def _write_parquet(root, images, labels):
    from datasets import ClassLabel, Dataset, Features, Image

    feats = Features({"image": Image(), "label": ClassLabel(names=NAMES)})
    os.makedirs(os.path.join(root, "data"), exist_ok=True)
    start = 0
    for split, n in (("train", 12), ("test", 6)):
        Dataset.from_dict({"image": [images[i] for i in range(start, start + n)],
                           "label": [int(v) for v in labels[start:start + n]]},
                          features=feats).to_parquet(os.path.join(root, "data", f"{split}-00000-of-00001.parquet"))
        start += n


@pytest.mark.parametrize("name", ["rgb", "grey", "grey_to_rgb"])
def test_hf_dataset_matches_reference(tmp_path, monkeypatch, name):
    pytest.importorskip("datasets")
    monkeypatch.setenv("HF_DATASETS_OFFLINE", "1")
    import ap_gym_amd as ap

    g = golden("hf_dataset.npz")
    root = str(tmp_path / name)
    _write_parquet(root, g[f"{name}_images"], g[f"{name}_labels"])
    channels = int(g[f"{name}_channels"])
    for split in ("train", "test"):
        for filt in (None, ["three", "one"]):
            key = f"{name}_{split}_{'filt' if filt else 'all'}"
            ds = ap.HuggingfaceImageClassificationDataset(root, channels=channels, split=split, filter_labels=filt)
            ds.load()
            assert len(ds) == int(g[key + "_len"]), key
            assert ds.num_classes == int(g[key + "_num_classes"]), key
            imgs, labs = ds.get_data_point_batch(g[key + "_idx"])
            assert np.array_equal(np.asarray(imgs), g[key + "_batch_images"]), key
            assert np.asarray(imgs).dtype == np.float32
            assert np.array_equal(np.asarray(labs), g[key + "_batch_labels"]), key
            # the device pool the envs upload: raw uint8 rows whose u8 -> f32 / 255 path gives the batches
            pool, pool_labels = ds.device_pool()
            order = g[key + "_idx"]
            vals = pool[order].astype(np.float32) / 255
            if vals.shape[-1] == 1 and channels == 3:
                vals = np.repeat(vals, 3, axis=-1)
            assert np.array_equal(vals, g[key + "_batch_images"]), key
            assert np.array_equal(pool_labels[order], g[key + "_batch_labels"]), key


@pytest.mark.gpu
def test_hf_dataset_drives_image_env(tmp_path, monkeypatch, gpu):
    """make_vec over a local HF dataset: the env's glimpses and labels equal those of the same pool
    given as arrays (the HF rows are uploaded once into the resident device pool)."""
    pytest.importorskip("datasets")
    monkeypatch.setenv("HF_DATASETS_OFFLINE", "1")
    import ap_gym_amd as ap

    g = golden("hf_dataset.npz")
    root = str(tmp_path / "rgb")
    _write_parquet(root, g["rgb_images"], g["rgb_labels"])
    hf = ap.HuggingfaceImageClassificationDataset(root, channels=3, split="train", filter_labels=["three", "one"])
    pool, labels = hf.device_pool()
    arr = ap.ArrayImageClassificationDataset(pool, labels, 2, 3)
    envs = [ap.ImageClassificationVectorEnv(4, ap.ImagePerceptionConfig(dataset=d, sensor_size=(3, 3)), device=gpu)
            for d in (hf, arr)]
    outs = [e.reset(seed=7) for e in envs]
    for k in outs[0][0]:
        assert np.array_equal(outs[0][0][k], outs[1][0][k]), k
    rng = np.random.default_rng(0)
    for _ in range(5):
        act = {"action": rng.uniform(-1, 1, (4, 2)).astype(np.float32),
               "prediction": rng.standard_normal((4, 2)).astype(np.float32)}
        a, b = (e.step(act) for e in envs)
        assert np.array_equal(a[0]["glimpse"], b[0]["glimpse"]) and np.array_equal(a[1], b[1])
        assert np.array_equal(a[4]["prediction"]["target"], b[4]["prediction"]["target"])
