"""Base class of the batched envs: gymnasium.vector.VectorEnv when gymnasium is importable.

The reference's vector envs are `gymnasium.vector.VectorEnv` subclasses
(ap_gym/active_perception_vector_env.py:40-66), and gymnasium tooling (wrappers, `make_vec`,
`isinstance` checks) relies on that.  The GPU box has no gymnasium, so there the same attributes
come from a minimal stand-in (num_envs, metadata, render_mode, spec, closed, unwrapped, context
manager).
"""

from __future__ import annotations

from typing import Any

try:  # pragma: no cover - gymnasium is absent in the build image
    import gymnasium as _gym

    VectorEnv = _gym.vector.VectorEnv
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class VectorEnv:  # type: ignore[no-redef]
        """The attribute surface of gymnasium.vector.VectorEnv (gymnasium >= 1.1) the envs use."""

        metadata: dict[str, Any] = {}
        spec = None
        render_mode: str | None = None
        closed: bool = False
        num_envs: int

        def reset(self, *, seed=None, options=None):
            raise NotImplementedError

        def step(self, actions):
            raise NotImplementedError

        def render(self):
            raise NotImplementedError

        def close(self, **kwargs):
            self.closed = True

        @property
        def unwrapped(self):
            return self

        def __enter__(self):
            return self

        def __exit__(self, *args):
            self.close()
            return False
