"""gymnasium.envs.registration restated (registry, register, make_vec) for the build container.

Only what the reference's registration.py and the drop-in test (tests/test_integration.py) exercise:
  * register(id, entry_point, vector_entry_point, additional_wrappers, kwargs, ...) into `registry`
  * make_vec(id, num_envs, vectorization_mode, vector_kwargs, wrappers, **kwargs), gymnasium >= 1.1:
    the spec's kwargs are updated with the call's kwargs; with a vector entry point (chosen by
    default when the spec has one) a non-empty `additional_wrappers` or a `wrappers` argument is an
    error, else the entry point is called as vector_entry_point(num_envs=num_envs, **kwargs);
    without one, SyncVectorEnv over `make(spec)` with the additional wrappers applied in order.
"""

from __future__ import annotations

import copy
import importlib
from dataclasses import dataclass, field
from typing import Any, Callable


class Error(Exception):
    pass


@dataclass
class WrapperSpec:
    name: str
    entry_point: str
    kwargs: dict = field(default_factory=dict)


@dataclass
class EnvSpec:
    id: str = ""
    entry_point: Any = None
    reward_threshold: Any = None
    nondeterministic: bool = False
    max_episode_steps: Any = None
    order_enforce: bool = True
    disable_env_checker: bool = False
    kwargs: dict = field(default_factory=dict)
    additional_wrappers: tuple = ()
    vector_entry_point: Any = None


EnvCreator = Callable
VectorEnvCreator = Callable

registry: dict[str, EnvSpec] = {}


def parse_env_id(env_id):
    name, version = env_id.rsplit("-v", 1)
    return None, name, int(version)


def get_env_id(ns, name, version):
    return f"{name}-v{version}"


def load_env_creator(entry_point):
    if callable(entry_point):
        return entry_point
    mod_name, attr = entry_point.split(":")
    return getattr(importlib.import_module(mod_name), attr)


def register(id: str, entry_point=None, reward_threshold=None, nondeterministic=False, max_episode_steps=None,
             order_enforce=True, disable_env_checker=False, additional_wrappers=(), vector_entry_point=None,
             kwargs=None, **_ignored):
    if entry_point is None and vector_entry_point is None:
        raise Error("Either entry_point or vector_entry_point must be provided")
    registry[id] = EnvSpec(id=id, entry_point=entry_point, reward_threshold=reward_threshold,
                           nondeterministic=nondeterministic, max_episode_steps=max_episode_steps,
                           order_enforce=order_enforce, disable_env_checker=disable_env_checker,
                           kwargs=dict(kwargs or {}), additional_wrappers=tuple(additional_wrappers),
                           vector_entry_point=vector_entry_point)


def make(id, max_episode_steps=None, disable_env_checker=None, **kwargs):
    spec = registry[id] if isinstance(id, str) else id
    if spec.entry_point is None:
        raise Error(f"{spec.id} registered but entry_point is not specified")
    kw = dict(copy.deepcopy(spec.kwargs), **kwargs)
    env = load_env_creator(spec.entry_point)(**kw)
    for w in spec.additional_wrappers:
        env = load_env_creator(w.entry_point)(env=env, **w.kwargs)
    return env


def make_vec(id, num_envs: int = 1, vectorization_mode=None, vector_kwargs=None, wrappers=None, **kwargs):
    from .. import VectorizeMode
    from ..vector import SyncVectorEnv

    spec = copy.deepcopy(registry[id] if isinstance(id, str) else id)
    env_kwargs = copy.deepcopy(spec.kwargs)
    env_kwargs.update(kwargs)
    mode = vectorization_mode
    if isinstance(mode, str):
        mode = VectorizeMode(mode)
    if mode is None:
        mode = VectorizeMode.VECTOR_ENTRY_POINT if spec.vector_entry_point is not None else VectorizeMode.SYNC
    if mode == VectorizeMode.VECTOR_ENTRY_POINT:
        if len(spec.additional_wrappers) > 0:
            raise Error("Cannot use `vector_entry_point` vectorization mode with the additional_wrappers parameter "
                        f"in spec being not empty, {spec.additional_wrappers}.")
        if wrappers is not None:
            raise Error("Cannot use `vector_entry_point` vectorization mode with the wrappers argument.")
        if spec.vector_entry_point is None:
            raise Error(f"Cannot create vectorized environment for {spec.id} because it doesn't have a vector entry "
                        "point defined.")
        env = load_env_creator(spec.vector_entry_point)(num_envs=num_envs, **env_kwargs)
    elif mode == VectorizeMode.SYNC:
        def one():
            env = make(spec, **env_kwargs)
            for w in wrappers or ():
                env = w(env)
            return env

        env = SyncVectorEnv([one] * num_envs, **(vector_kwargs or {}))
    else:
        raise Error(f"unsupported vectorization mode {mode}")
    env.spec = spec
    return env
