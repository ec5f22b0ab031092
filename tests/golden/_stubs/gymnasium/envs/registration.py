from dataclasses import dataclass, field
from typing import Any, Callable


@dataclass
class EnvSpec:
    id: str = ""
    entry_point: Any = None
    max_episode_steps: Any = None
    kwargs: dict = field(default_factory=dict)


@dataclass
class WrapperSpec:
    name: str
    entry_point: str
    kwargs: dict = field(default_factory=dict)


EnvCreator = Callable
VectorEnvCreator = Callable


def parse_env_id(env_id):
    name, version = env_id.rsplit("-v", 1)
    return None, name, int(version)


def get_env_id(ns, name, version):
    return f"{name}-v{version}"


def load_env_creator(entry_point):
    raise NotImplementedError
