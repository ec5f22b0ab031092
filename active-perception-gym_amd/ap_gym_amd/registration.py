"""Env ids of the hot path and make_vec (ap_gym/envs/registration.py:145-192, 319-512, 516-690, 753-767).

Only the ids whose step is accelerated by this backend are registered.  `make_vec(id, num_envs,
**kwargs)` accepts the same keyword overrides as the reference (dataset, lidar_beam_count,
lidar_range, static_map_index, image_perception_config, ...) plus backend options (device,
array_backend, copy, strict_errors, env_offset).

Image ids: the reference loads MNIST / CIFAR10 / Tiny ImageNet from the HuggingFace hub, which is
not reachable here; pass `dataset=` (e.g. ArrayImageClassificationDataset) to use local data.  The
registered sensor size / step limit / render options are kept.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable

from .floor_map import FloorMapDatasetMaze, FloorMapDatasetRooms


@dataclass
class EnvSpec:
    id: str
    vector_entry_point: Callable
    kwargs: dict = field(default_factory=dict)
    max_episode_steps: int | None = None


registry: dict[str, EnvSpec] = {}


def sparse_id(id: str) -> str:
    """parse_env_id / get_env_id as registration.py:115-118 use them: "<name>-v<ver>" ->
    "<name>-sparse-v<ver>" (namespace kept)."""
    name, sep, version = id.rpartition("-v")
    if not sep or not version.isdigit():
        raise ValueError(f"malformed env id {id!r}")
    return f"{name}-sparse-v{version}"


def register(id: str, vector_entry_point: Callable, kwargs: dict | None = None, max_episode_steps=None,
             register_sparse_version: bool = True):
    """registration.py:87-142: every id also gets a "-sparse" variant whose loss (and so reward) is
    masked to the last step of each episode (SparsifyVectorWrapper / SparsifyWrapper)."""
    registry[id] = EnvSpec(id, vector_entry_point, dict(kwargs or {}), max_episode_steps)
    if register_sparse_version:
        sid = sparse_id(id)
        registry[sid] = EnvSpec(sid, vector_entry_point, dict(kwargs or {}, sparse=True), max_episode_steps)


def _lidar(num_envs: int = 1, **kwargs):
    from .lidar_env import LIDARLocalization2DVectorEnv

    return LIDARLocalization2DVectorEnv(num_envs=num_envs, **kwargs)


def _image(kind: str):
    def entry(num_envs: int = 1, image_perception_config=None, dataset=None, dataset_factory=None,
              config_kwargs=None, **kwargs):
        from .image_env import ImageClassificationVectorEnv, ImageLocalizationVectorEnv, ImagePerceptionConfig

        if image_perception_config is None:
            if dataset is None:
                dataset = dataset_factory()
            image_perception_config = ImagePerceptionConfig(dataset=dataset, **(config_kwargs or {}))
        cls = ImageClassificationVectorEnv if kind == "cls" else ImageLocalizationVectorEnv
        kwargs.setdefault("log_stats", True)  # the vector log wrapper of the registered ids
        return cls(num_envs, image_perception_config, **kwargs)

    return entry


def _light_dark(num_envs: int = 1, **kwargs):
    from .light_dark_env import LightDarkVectorEnv

    return LightDarkVectorEnv(num_envs=num_envs, **kwargs)


def _hide_and_seek(mask_prediction: bool):
    """registration.py:471-512: CircleSquareHideAndSeekVectorWrapper(ImageClassificationVectorEnv), with the
    classification log wrapper outside it for the prediction variant only."""

    def entry(num_envs: int = 1, sparse: bool = False, **kwargs):
        from .circle_square import CircleSquareHideAndSeekVectorWrapper

        kwargs.setdefault("log_stats", not mask_prediction)
        inner = _image("cls")(num_envs=num_envs, **kwargs)
        return CircleSquareHideAndSeekVectorWrapper(inner, mask_prediction=mask_prediction, sparse=sparse)

    return entry


def _circle_square(double: bool, size: int, show_gradient: bool):
    def factory():
        from .circle_square import CircleSquareDataset, DoubleCircleSquareDataset

        if double:
            return DoubleCircleSquareDataset(image_shape=(size, size), show_gradient_a=show_gradient,
                                             show_gradient_b=show_gradient)
        return CircleSquareDataset(image_shape=(size, size), show_gradient=show_gradient)

    return factory


def _register_circle_square(size: int, show_gradient: bool, suffix: str, step_limit: int = 16):
    # register_circle_square (registration.py:358-406)
    cfg = dict(step_limit=step_limit)
    register(f"CircleSquare{suffix}-v0", _image("cls"),
             kwargs=dict(dataset_factory=_circle_square(False, size, show_gradient), config_kwargs=dict(cfg)))
    register(f"CircleSquareInverted{suffix}-v0", _image("cls"),
             kwargs=dict(dataset_factory=_circle_square(False, size, show_gradient),
                         config_kwargs=dict(cfg, randomly_invert_labels=True)))
    register(f"DoubleCircleSquare{suffix}-v0", _image("cls"),
             kwargs=dict(dataset_factory=_circle_square(True, size, show_gradient), config_kwargs=dict(cfg)))


def _hf(name: str, split: str, **kw):
    def factory():
        from .image_dataset import HuggingfaceImageClassificationDataset

        return HuggingfaceImageClassificationDataset(name, split=split, **kw)

    return factory


CIFAR10_CLASSES = ["airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck"]


def _register_image_ids(kind, name, factory, config_kwargs):
    # register_img_envs (registration.py:224-260): <name>-v0 and <name>-train-v0 use the train split
    for suffix, split in (("", "train"), ("-train", "train"), ("-test", "test")):
        register(f"{name}{suffix}-v0", _image(kind),
                 kwargs=dict(dataset_factory=factory(split), config_kwargs=dict(config_kwargs)))


def register_envs():
    # registration.py:640-690: maze maps default to 21x21, rooms maps to 32x32; TimeLimit(100)
    for name, ds, static in (("LIDARLocMazeStatic-v0", FloorMapDatasetMaze, True),
                             ("LIDARLocMaze-v0", FloorMapDatasetMaze, False),
                             ("LIDARLocRoomsStatic-v0", FloorMapDatasetRooms, True),
                             ("LIDARLocRooms-v0", FloorMapDatasetRooms, False)):
        # TimeLimit + ActiveRegressionLogWrapper (registration.py:348-355): episode stats on
        register(name, _lidar, kwargs=dict(dataset_factory=ds, static_map=static, log_stats=True),
                 max_episode_steps=100)
    # registration.py:640-647: TimeLimit(50) + ActiveRegressionLogWrapper over LightDarkEnv
    register("LightDark-v0", _light_dark, kwargs=dict(log_stats=True), max_episode_steps=50)
    # registration.py:409-512: the CircleSquare family (procedural datasets rendered on the device)
    for size, grad, suffix, limit in ((28, True, "", 16), (28, True, "-s28", 16), (20, True, "-s20", 16),
                                      (15, True, "-s15", 16), (28, False, "-nograd", 16),
                                      (20, False, "-s20-nograd", 16), (15, False, "-s15-nograd", 16),
                                      (28, True, "-t32", 32), (28, True, "-t64", 64)):
        _register_circle_square(size, grad, suffix, limit)
    for name, mask in (("CircleSquareHideAndSeek-v0", False), ("CircleSquareHideAndSeekNoPrediction-v0", True)):
        register(name, _hide_and_seek(mask),
                 kwargs=dict(dataset_factory=_circle_square(False, 28, True), config_kwargs=dict(step_limit=32)))
    render_kw = dict(render_unvisited_opacity=0.5, render_visited_opacity=0.25)
    _register_image_ids("cls", "MNIST", lambda split: _hf("mnist", split, channels=1), dict(step_limit=16))
    _register_image_ids("cls", "CIFAR10", lambda split: _hf("cifar10", split, image_feature_name="img"),
                        dict(step_limit=16, **render_kw))
    for i in range(2, 11):
        _register_image_ids("cls", f"CIFAR10-c{i}",
                            lambda split, i=i: _hf("cifar10", split, image_feature_name="img",
                                                   filter_labels=CIFAR10_CLASSES[:i]),
                            dict(step_limit=16, **render_kw))
    tin = lambda split: _hf("zh-plus/tiny-imagenet", split if split == "train" else "valid")  # noqa: E731
    _register_image_ids("cls", "TinyImageNet", tin, dict(step_limit=16, sensor_size=(10, 10), **render_kw))
    _register_image_ids("loc", "MNISTLoc", lambda split: _hf("mnist", split, channels=1),
                        dict(step_limit=16, **render_kw))
    _register_image_ids("loc", "CIFAR10Loc", lambda split: _hf("cifar10", split, image_feature_name="img"),
                        dict(step_limit=16, **render_kw))
    _register_image_ids("loc", "TinyImageNetLoc", tin, dict(step_limit=16, sensor_size=(10, 10), **render_kw))


def make_vec(id: str | EnvSpec, num_envs: int = 1, vectorization_mode: str | None = None,
             vector_kwargs: dict[str, Any] | None = None, wrappers=None, **kwargs):
    spec = id if isinstance(id, EnvSpec) else registry.get(id)
    if spec is None:
        raise KeyError(f"Environment id {id!r} is not provided by the MI355X backend. Known ids: {sorted(registry)}")
    mode = getattr(vectorization_mode, "value", vectorization_mode)  # gymnasium.VectorizeMode members too
    if mode not in (None, "vector_entry_point", "sync", "async"):
        raise ValueError(f"unknown vectorization_mode {vectorization_mode!r}")
    # "sync" / "async": gymnasium's SyncVectorEnv and AsyncVectorEnv return the same batches for the same
    # seeds (both autoreset NEXT_STEP); the batched env reproduces them, the worker processes are not needed
    if wrappers:
        raise NotImplementedError("per-sub-env wrappers are not supported by the batched backend")
    kw = dict(spec.kwargs)
    if "config_kwargs" in kw:  # image ids: the entry point builds the ImagePerceptionConfig
        kw["config_kwargs"] = dict(kw["config_kwargs"], **kwargs.pop("config_kwargs", {}))
    else:
        factory = kw.pop("dataset_factory", None)
        if "dataset" not in kwargs and factory is not None:
            kwargs["dataset"] = factory()
    if spec.max_episode_steps is not None:
        kw.setdefault("max_episode_steps", spec.max_episode_steps)
    kw.update(kwargs)
    kw.update(vector_kwargs or {})
    return spec.vector_entry_point(num_envs=num_envs, **kw)


register_envs()
