"""Env ids of the hot path and make_vec (ap_gym/envs/registration.py:319-356, 640-690, 753-767).

Only the ids whose step is accelerated by this backend are registered.  `make_vec(id, num_envs,
**kwargs)` accepts the same keyword overrides as the reference (dataset, lidar_beam_count,
lidar_range, static_map_index, ...) plus backend options (device, array_backend, copy,
strict_errors, env_offset).
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


def register(id: str, vector_entry_point: Callable, kwargs: dict | None = None, max_episode_steps=None):
    registry[id] = EnvSpec(id, vector_entry_point, dict(kwargs or {}), max_episode_steps)


def _lidar(num_envs: int = 1, **kwargs):
    from .lidar_env import LIDARLocalization2DVectorEnv

    return LIDARLocalization2DVectorEnv(num_envs=num_envs, **kwargs)


def register_envs():
    # registration.py:640-690: maze maps default to 21x21, rooms maps to 32x32; TimeLimit(100)
    for name, ds, static in (("LIDARLocMazeStatic-v0", FloorMapDatasetMaze, True),
                             ("LIDARLocMaze-v0", FloorMapDatasetMaze, False),
                             ("LIDARLocRoomsStatic-v0", FloorMapDatasetRooms, True),
                             ("LIDARLocRooms-v0", FloorMapDatasetRooms, False)):
        register(name, _lidar, kwargs=dict(dataset_factory=ds, static_map=static), max_episode_steps=100)


def make_vec(id: str | EnvSpec, num_envs: int = 1, vectorization_mode: str | None = None,
             vector_kwargs: dict[str, Any] | None = None, wrappers=None, **kwargs):
    spec = id if isinstance(id, EnvSpec) else registry.get(id)
    if spec is None:
        raise KeyError(f"Environment id {id!r} is not provided by the MI355X backend. Known ids: {sorted(registry)}")
    if vectorization_mode not in (None, "vector_entry_point", "sync"):
        raise ValueError("the MI355X backend always runs the batched vector env (vectorization_mode=None)")
    if wrappers:
        raise NotImplementedError("per-sub-env wrappers are not supported by the batched backend")
    kw = dict(spec.kwargs)
    factory = kw.pop("dataset_factory", None)
    if "dataset" not in kwargs and factory is not None:
        kwargs["dataset"] = factory()
    if spec.max_episode_steps is not None:
        kw.setdefault("max_episode_steps", spec.max_episode_steps)
    kw.update(kwargs)
    kw.update(vector_kwargs or {})
    return spec.vector_entry_point(num_envs=num_envs, **kw)


register_envs()
