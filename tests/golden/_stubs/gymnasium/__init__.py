"""Minimal gymnasium (>=1.1) restatement used ONLY to execute the reference's own ap_gym modules in
the build container when generating golden fixtures (gymnasium is not installed here).

Restated behaviour that affects values (everything else is a no-op placeholder):
  * Env.reset(seed) -> np_random = Generator(PCG64(SeedSequence(seed)))   (gymnasium/utils/seeding.py)
  * Wrapper forwarding of reset/step/spaces/np_random                    (gymnasium/core.py)
  * register / make / make_vec with gymnasium's vector-entry-point rules     (gymnasium/envs/registration.py)
  * SyncVectorEnv with NEXT_STEP autoreset, seed+i per sub-env, info merging with `_key` masks,
    float64 rewards / bool flags                                          (gymnasium/vector/sync_vector_env.py)
"""

from __future__ import annotations

import enum

import numpy as np

from . import spaces, utils, vector, envs  # noqa: F401
from .core import Env, Wrapper  # noqa: F401
from .spaces import Space  # noqa: F401


class VectorizeMode(enum.Enum):
    ASYNC = "async"
    SYNC = "sync"
    VECTOR_ENTRY_POINT = "vector_entry_point"


from .envs.registration import make, make_vec, register, registry  # noqa: E402,F401
