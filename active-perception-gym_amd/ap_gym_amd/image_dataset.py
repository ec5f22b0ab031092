"""Image classification datasets (ap_gym/envs/image/image_classification_dataset.py, dataset/dataset.py).

Same interface as the reference (`len`, `num_classes`, `get_data_point[_batch]`, `__getitem__`,
`load`), plus `device_pool()`: the whole dataset as one array for the GPU envs, which keep it
resident in HBM and gather each env's image by index (the reference instead copies the drawn
batch through a prefetch thread, dataset_iterator.py:35-59, buffered_iterator.py).  Raw uint8
pools stay uint8 on the device (the u8 -> f32 / 255 conversion of `_process_imgs_np` happens in the
glimpse kernel); other dtypes are converted to float32 on the host like `_process_imgs_np`.

HuggingFace datasets cannot be downloaded here (no network); `ArrayImageClassificationDataset`
takes the same data as arrays, `SyntheticImageClassificationDataset` makes seeded uint8 pools of
the benchmark shapes.
"""

from __future__ import annotations

from typing import Sequence

import numpy as np


class ImageClassificationDataset:
    """Base class with the reference's processing rules (image_classification_dataset.py:12-98)."""

    def load(self):
        pass

    def _get_length(self) -> int:
        raise NotImplementedError

    def _get_num_classes(self) -> int:
        raise NotImplementedError

    def _get_num_channels(self) -> int:
        raise NotImplementedError

    def _get_data_point_batch(self, idx: np.ndarray):
        raise NotImplementedError

    def __len__(self):
        return self._get_length()

    @property
    def num_classes(self) -> int:
        return self._get_num_classes()

    @property
    def num_channels(self) -> int:
        return self._get_num_channels()

    def _process_imgs_np(self, imgs: np.ndarray) -> np.ndarray:
        if imgs.dtype == np.uint8:
            imgs = imgs.astype(np.float32) / 255
        elif imgs.dtype != np.float32:
            imgs = imgs.astype(np.float32)
        if imgs.ndim == 3:
            imgs = imgs[..., None]
        c = self._get_num_channels()
        if c not in (1, 3):
            raise ValueError(f"Target channels must be either 1 or 3 but is {c}.")
        if imgs.shape[-1] == 1 and c == 3:
            imgs = np.repeat(imgs, 3, axis=-1)
        if imgs.shape[-1] != c:
            raise ValueError(f"Invalid image format. Expected {c} channels but got {imgs.shape[-1]}")
        return imgs

    def get_data_point_batch(self, idx: Sequence[int] | np.ndarray):
        idx = np.asarray(idx)
        if idx.shape[0] == 0:
            raise ValueError("Empty index array")
        imgs, labels = self._get_data_point_batch(idx)
        imgs = np.stack([np.asarray(i) for i in imgs]) if not isinstance(imgs, np.ndarray) else imgs
        return self._process_imgs_np(imgs), np.asarray(labels).astype(np.int32)

    def get_data_point(self, idx: int):
        imgs, labels = self.get_data_point_batch(np.array([int(idx)]))
        return imgs[0], int(labels[0])

    def __getitem__(self, item):
        if isinstance(item, (Sequence, np.ndarray)):
            return self.get_data_point_batch(item)
        return self.get_data_point(item)

    def device_pool(self) -> tuple[np.ndarray, np.ndarray]:
        """(images [M, H, W, Cp] uint8 or float32, labels int32 [M]) of the whole dataset."""
        idx = np.arange(len(self))
        imgs, labels = self._get_data_point_batch(idx)
        imgs = np.stack([np.asarray(i) for i in imgs]) if not isinstance(imgs, np.ndarray) else np.asarray(imgs)
        if imgs.ndim == 3:
            imgs = imgs[..., None]
        if imgs.dtype != np.uint8:
            imgs = imgs.astype(np.float32)
        return np.ascontiguousarray(imgs), np.asarray(labels).astype(np.int32)


class ForeignDatasetView(ImageClassificationDataset):
    """Any object with the reference dataset interface (`load`, `__len__`, `num_classes`,
    `num_channels`, `_get_data_point_batch`) -- e.g. a subclass of the reference's own
    ImageClassificationDataset (image_classification_dataset.py:12-98) -- seen as a pool dataset:
    `device_pool()` fetches every data point once through its `_get_data_point_batch`, in chunks of
    FETCH_CHUNK indices, and freezes the result on the device.

    Static-pool assumption: the reference env fetches a data point every time it draws it, so a dataset
    whose `_get_data_point(_batch)` randomizes per fetch (augmentation) or that does not fit in memory
    behaves differently here (every draw of index i sees the same frozen image).  Such datasets are not
    supported: the view warns once, and parity for them is unpinned."""

    FETCH_CHUNK = 4096

    def __init__(self, inner):
        self.inner = inner
        import warnings

        warnings.warn(f"{type(inner).__name__} is used through ForeignDatasetView: its data points are fetched "
                      "once and frozen on the device (per-fetch randomization is not reproduced)", stacklevel=3)

    def device_pool(self) -> tuple[np.ndarray, np.ndarray]:
        n = len(self)
        imgs, labels = [], []
        for lo in range(0, n, self.FETCH_CHUNK):
            i, l = self._get_data_point_batch(np.arange(lo, min(n, lo + self.FETCH_CHUNK)))
            imgs.append(np.stack([np.asarray(x) for x in i]) if not isinstance(i, np.ndarray) else np.asarray(i))
            labels.append(np.asarray(l))
        im = np.concatenate(imgs)
        if im.ndim == 3:
            im = im[..., None]
        if im.dtype != np.uint8:
            im = im.astype(np.float32)
        return np.ascontiguousarray(im), np.concatenate(labels).astype(np.int32)

    def load(self):
        if hasattr(self.inner, "load"):
            self.inner.load()

    def _get_length(self):
        return len(self.inner)

    def _get_num_classes(self):
        return int(self.inner.num_classes)

    def _get_num_channels(self):
        return int(self.inner.num_channels)

    def _get_data_point_batch(self, idx):
        return self.inner._get_data_point_batch(idx)


def as_pool_dataset(ds):
    """`ds` itself when it can hand the envs its pool, else a ForeignDatasetView of it."""
    if hasattr(ds, "device_pool") or hasattr(ds, "device_pool_tensors"):
        return ds
    return ForeignDatasetView(ds)


class ArrayImageClassificationDataset(ImageClassificationDataset):
    """In-memory dataset: images [M, H, W] or [M, H, W, C] (uint8 or float), labels [M]."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, num_classes: int | None = None,
                 channels: int | None = None):
        self._images = np.asarray(images)
        self._labels = np.asarray(labels)
        if self._images.shape[0] != self._labels.shape[0]:
            raise ValueError("images and labels must have the same length")
        self._k = int(num_classes) if num_classes is not None else int(self._labels.max()) + 1
        src_c = 1 if self._images.ndim == 3 else self._images.shape[-1]
        self._c = int(channels) if channels is not None else src_c

    def _get_length(self):
        return self._images.shape[0]

    def _get_num_classes(self):
        return self._k

    def _get_num_channels(self):
        return self._c

    def _get_data_point_batch(self, idx):
        return self._images[idx], self._labels[idx]

    def device_pool(self):
        imgs = self._images if self._images.ndim == 4 else self._images[..., None]
        if imgs.dtype != np.uint8:
            imgs = imgs.astype(np.float32)
        return np.ascontiguousarray(imgs), self._labels.astype(np.int32)


class SyntheticImageClassificationDataset(ArrayImageClassificationDataset):
    """Seeded uint8 pool of a benchmark shape: uniform pixels 0..255, uniform labels."""

    def __init__(self, length: int, image_shape: tuple[int, ...], num_classes: int, channels: int | None = None,
                 seed: int = 0):
        rng = np.random.default_rng(seed)
        images = rng.integers(0, 256, (int(length), *image_shape), dtype=np.uint8)
        labels = rng.integers(0, num_classes, int(length))
        super().__init__(images, labels, num_classes, channels)


class HuggingfaceImageClassificationDataset(ImageClassificationDataset):
    """huggingface_image_classification_dataset.py:12-80 — usable where `datasets` can load the data
    (a local cache); this build has no network, so loading fails with the datasets library's error."""

    def __init__(self, dataset_name: str, channels: int = 3, split: str = "train", image_feature_name: str = "image",
                 label_feature_name: str = "label", filter_labels=None):
        self.dataset_name, self.split, self.channels = dataset_name, split, channels
        self.image_feature_name, self.label_feature_name = image_feature_name, label_feature_name
        self.filter_labels = None if filter_labels is None else list(filter_labels)
        self._data = self._train = None

    def load(self):
        if self._data is not None:
            return
        from datasets import load_dataset

        ds = load_dataset(self.dataset_name)
        self._data, self._train = ds[self.split], ds["train"]
        if self.filter_labels is not None:
            names = self._train.features[self.label_feature_name].names
            keep = [names.index(n) for n in self.filter_labels]
            remap = {v: i for i, v in enumerate(keep)}
            lab = np.asarray(self._data[self.label_feature_name])
            sel = np.nonzero(np.isin(lab, keep))[0]
            self._data = self._data.select(sel)
            self._remap = remap
        else:
            self._remap = None

    def _get_length(self):
        self.load()
        return len(self._data)

    def _get_num_classes(self):
        self.load()
        if self.filter_labels is not None:
            return len(self.filter_labels)
        return self._train.features[self.label_feature_name].num_classes

    def _get_num_channels(self):
        return self.channels

    def _get_data_point_batch(self, idx):
        self.load()
        rows = self._data[np.asarray(idx)]
        imgs = [np.asarray(im) for im in rows[self.image_feature_name]]
        labels = rows[self.label_feature_name]
        if self._remap is not None:
            labels = [self._remap[v] for v in labels]
        return imgs, labels
