"""Reference-side drop-in: the batched MI355X envs under ap_gym's own env ids and `make_vec`.

`ap_gym.make_vec(id, N)` (ap_gym/envs/registration.py:753-767) calls `gymnasium.make_vec` and then
`ensure_active_perception_vector_env` (active_perception_vector_env.py:311-320), which accepts an
env as it is only if it is a `BaseActivePerceptionVectorEnv`; anything else is wrapped in
`ActivePerceptionVectorRestoreWrapper` / `PseudoActivePerceptionVectorWrapper`, which look for
`loss_fn` and the prediction spaces through `find_loss_and_pred_space_vec` (:215-251) and lose them
for a foreign class.  So the binding has two parts:

  * `vector_env_class(ap_gym)` — an adapter class derived from the reference's own
    `ap_gym.BaseActivePerceptionVectorEnv`, holding one ap_gym_amd env (`env_impl`) and exposing its
    `loss_fn`, prediction target spaces and reference-typed spaces (`ap_gym.ActivePerceptionActionSpace`,
    `ap_gym.ImageSpace`, `ap_gym.LogitSpace`, gymnasium spaces);
  * `register_with_ap_gym(ap_gym)` — re-registers every id the reference registered and this
    backend accelerates with a `vector_entry_point` that builds the adapter.  gymnasium refuses a
    vector entry point together with non-empty `additional_wrappers` (the reference notes this at
    registration.py:124-125), so the single-env entry point composes the spec's additional
    wrappers itself (TimeLimit + log wrapper of the LIDAR / LightDark ids, registration.py:319-356,
    640-647), exactly as the reference's own "-sparse" entry points do (:115-135), and the spec's
    `additional_wrappers` become empty.  The batched env folds TimeLimit (`max_episode_steps`), the
    log wrappers (`log_stats`) and SparsifyWrapper (`sparse`) into its kernels.

Usage (after the reference has registered its ids, i.e. at the end of ap_gym/__init__.py or in user
code after `import ap_gym`):

    import ap_gym
    import ap_gym_amd.integration as amd
    amd.register_with_ap_gym(ap_gym, device="cuda:0")
    env = ap_gym.make_vec("LIDARLocRooms-v0", num_envs=65536, lidar_beam_count=32,
                          dataset=ap_gym.envs.floor_map.FloorMapDatasetRooms(64, 64))

Reference dataset objects in the kwargs (FloorMapDatasetRooms/Maze, CircleSquareDataset,
DoubleCircleSquareDataset, any ImageClassificationDataset) are converted to their device-resident
equivalents (`convert_dataset`); reference `ImagePerceptionConfig`s to ap_gym_amd's.
"""

from __future__ import annotations

from dataclasses import fields
from typing import Any, Callable

import numpy as np

_ADAPTERS: dict[int, type] = {}


# ---------------------------------------------------------------------------------- spaces
def to_reference_space(space, ap_gym):
    """The same space built from the reference's / gymnasium's classes."""
    import gymnasium as gym

    from . import spaces as S

    name = type(space).__name__
    if isinstance(space, S.ActivePerceptionActionSpace) or name == "ActivePerceptionActionSpace":
        if isinstance(space, ap_gym.ActivePerceptionActionSpace):
            return space
        return ap_gym.ActivePerceptionActionSpace(to_reference_space(space["action"], ap_gym),
                                                  to_reference_space(space["prediction"], ap_gym))
    if isinstance(space, S.ImageSpace):
        return ap_gym.ImageSpace(space.width, space.height, space.channels, tuple(space.batch_shape), space.dtype,
                                 low=np.asarray(space.low), high=np.asarray(space.high))
    if isinstance(space, S.LogitSpace):
        return ap_gym.LogitSpace(np.asarray(space.low), np.asarray(space.high), space.shape, space.dtype)
    if isinstance(space, (gym.spaces.Box, gym.spaces.Discrete, gym.spaces.MultiDiscrete)):
        return space
    if isinstance(space, S.Dict) or isinstance(space, gym.spaces.Dict):
        return gym.spaces.Dict({k: to_reference_space(v, ap_gym) for k, v in space.spaces.items()})
    if isinstance(space, S.Tuple) or isinstance(space, gym.spaces.Tuple):
        return gym.spaces.Tuple([to_reference_space(v, ap_gym) for v in space.spaces])
    if isinstance(space, S.Box):
        return gym.spaces.Box(np.asarray(space.low), np.asarray(space.high), space.shape, space.dtype)
    if isinstance(space, S.Discrete):
        return gym.spaces.Discrete(space.n, start=space.start)
    if isinstance(space, S.MultiDiscrete):
        return gym.spaces.MultiDiscrete(space.nvec)
    raise TypeError(f"cannot convert space {space!r}")


# ---------------------------------------------------------------------------------- adapter
class _AdapterMixin:
    """Methods of the adapter; the class itself is created per reference package by
    `vector_env_class` so that it derives from that package's BaseActivePerceptionVectorEnv."""

    _ap_gym: Any = None

    def __init__(self, impl):
        import gymnasium as gym

        ap = self._ap_gym
        self.env_impl = impl
        self.num_envs = impl.num_envs
        self.metadata = dict(impl.metadata)
        autoreset = getattr(getattr(gym.vector, "AutoresetMode", None), "NEXT_STEP", None)
        if autoreset is not None:
            self.metadata["autoreset_mode"] = autoreset
        self.render_mode = impl.render_mode
        self.single_observation_space = to_reference_space(impl.single_observation_space, ap)
        self.observation_space = to_reference_space(impl.observation_space, ap)
        self.single_action_space = to_reference_space(impl.single_action_space, ap)
        self.action_space = to_reference_space(impl.action_space, ap)
        self.single_prediction_target_space = to_reference_space(impl.single_prediction_target_space, ap)
        self.prediction_target_space = to_reference_space(impl.prediction_target_space, ap)
        self.loss_fn = impl.loss_fn

    def reset(self, *, seed=None, options=None):
        return self.env_impl.reset(seed=seed, options=options)

    def step(self, actions):
        return self.env_impl.step(actions)

    def render(self):
        return self.env_impl.render()

    def close(self, **kwargs):
        impl = self.__dict__.get("env_impl")
        if impl is not None:
            impl.close(**kwargs)
        self.closed = True

    def __getattr__(self, name):  # backend extras: check_errors, device, array_backend, ...
        if name.startswith("__") or name == "env_impl":
            raise AttributeError(name)
        return getattr(self.env_impl, name)

    def __repr__(self):
        return f"<{type(self).__name__}{self.env_impl!r}>"


def vector_env_class(ap_gym) -> type:
    """Adapter class deriving from the given reference package's BaseActivePerceptionVectorEnv."""
    base = ap_gym.BaseActivePerceptionVectorEnv
    cls = _ADAPTERS.get(id(base))
    if cls is None:
        cls = type("ApGymAmdVectorEnv", (_AdapterMixin, base), {"_ap_gym": ap_gym, "__module__": __name__})
        _ADAPTERS[id(base)] = cls
    return cls


def wrap(ap_gym, impl):
    return vector_env_class(ap_gym)(impl)


# ---------------------------------------------------------------------------------- kwargs
def convert_dataset(ds):
    """Reference dataset object -> the ap_gym_amd dataset with the same parameters (by class name and
    the reference's attribute names); ap_gym_amd datasets and unknown image datasets pass through
    (the image envs read unknown ones once through their `_get_data_point_batch`)."""
    from . import circle_square as cs
    from . import floor_map as fm

    if ds is None or type(ds).__module__.startswith("ap_gym_amd"):
        return ds
    name = type(ds).__name__
    # FloorMapDatasetRooms / FloorMapDatasetMaze (floor_map_dataset_rooms.py:10-24, floor_map_dataset_maze.py:10-22)
    # and subclasses that keep their maps (found in the MRO): the device generators; other floor-map datasets are
    # read through ForeignFloorMapView by the env (a frozen pool or streamed per episode)
    proc = fm.procedural_equivalent(ds)
    if proc is not None:
        return proc
    if name == "CircleSquareDataset":  # circle_square_dataset.py:80-89
        return cs.CircleSquareDataset(show_gradient=ds._show_gradient, image_shape=tuple(ds._image_shape),
                                      object_extents=ds._object_extents)
    if name == "DoubleCircleSquareDataset":  # circle_square_dataset.py:114-125
        return cs.DoubleCircleSquareDataset(show_gradient_a=ds._show_gradient_a, show_gradient_b=ds._show_gradient_b,
                                            image_shape=tuple(ds._image_shape), object_extents=ds._object_extents)
    return ds


def convert_kwargs(kwargs: dict) -> dict:
    from .image_env import ImagePerceptionConfig

    kw = dict(kwargs)
    if "dataset" in kw:
        kw["dataset"] = convert_dataset(kw["dataset"])
    cfg = kw.get("image_perception_config")
    if cfg is not None and not isinstance(cfg, ImagePerceptionConfig):
        values = {f.name: getattr(cfg, f.name) for f in fields(ImagePerceptionConfig) if hasattr(cfg, f.name)}
        values["dataset"] = convert_dataset(values["dataset"])
        kw["image_perception_config"] = ImagePerceptionConfig(**values)
    return kw


# ---------------------------------------------------------------------------------- registration
def _single_entry(spec) -> Callable:
    """The spec's single-env entry point with its additional wrappers applied inside (the pattern of
    the reference's own sparse entry points, registration.py:124-135)."""
    from gymnasium.envs.registration import load_env_creator

    entry, wrappers = spec.entry_point, tuple(spec.additional_wrappers or ())
    if not wrappers:
        return entry

    def single(*args, **kwargs):
        env = load_env_creator(entry)(*args, **kwargs)
        for w in wrappers:
            env = load_env_creator(w.entry_point)(env=env, **w.kwargs)
        return env

    return single


def register_with_ap_gym(ap_gym, ids=None, make_impl: Callable | None = None, **backend_kwargs) -> list[str]:
    """Point the reference's registered ids at the batched backend; returns the ids switched.

    ids:        restrict to these ids (default: every id both the reference and ap_gym_amd know)
    make_impl:  factory (id, num_envs, **kwargs) -> batched env (default: ap_gym_amd.make_vec); tests
                pass an oracle-backed stand-in here
    backend_kwargs: forwarded to every env (device, array_backend, copy, strict_errors, ...)
    """
    import gymnasium as gym

    from .registration import make_vec as amd_make_vec
    from .registration import registry as amd_registry

    make_impl = make_impl or amd_make_vec
    switched = []
    for env_id in amd_registry:
        if ids is not None and env_id not in ids:
            continue
        spec = gym.registry.get(env_id)
        if spec is None:
            continue

        def vec(num_envs: int = 1, _id=env_id, **kwargs):
            kw = convert_kwargs(kwargs)
            kw.update(backend_kwargs)
            return wrap(ap_gym, make_impl(_id, num_envs=num_envs, **kw))

        gym.register(id=env_id, entry_point=_single_entry(spec) if spec.entry_point is not None else None,
                     reward_threshold=spec.reward_threshold, nondeterministic=spec.nondeterministic,
                     max_episode_steps=spec.max_episode_steps, order_enforce=spec.order_enforce,
                     disable_env_checker=spec.disable_env_checker, additional_wrappers=(),
                     vector_entry_point=vec, kwargs=dict(spec.kwargs or {}))
        switched.append(env_id)
    return switched
