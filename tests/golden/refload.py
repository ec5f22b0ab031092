"""Load modules of the reference (/root/reference, ap_gym 0.5.0) by file path.

TEST INFRASTRUCTURE, build container only: /root/reference does not exist on the GPU box and
nothing under tests/ that runs there imports this module (only tests/golden/make_golden.py does).

`ap_gym/__init__.py` and `ap_gym/envs/__init__.py` import shapely, gymnasium and `datasets`
(absent here), so those two package modules are replaced by empty namespace modules whose
`__path__` points at the reference directories; every *leaf* module that is loaded is the
reference's own file, executed unmodified.  Third-party modules the image lacks (gymnasium,
shapely) are provided by tests/golden/_stubs (a minimal gymnasium restatement and an
exact-rational GEOS line∩polygon model) -- see DESIGN.md §Oracle for what that pins and what
it does not.
"""

from __future__ import annotations

import importlib
import os
import sys
import types

REF_ROOT = os.environ.get("APG_REFERENCE_ROOT", "/root/reference")
STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_stubs")


def reference_available() -> bool:
    return os.path.isfile(os.path.join(REF_ROOT, "ap_gym", "envs", "lidar_localization2d.py"))


def _ns(name: str, path: str) -> types.ModuleType:
    mod = sys.modules.get(name)
    if mod is None:
        mod = types.ModuleType(name)
        mod.__path__ = [path]
        mod.__package__ = name
        sys.modules[name] = mod
    return mod


def install_stubs() -> None:
    if STUBS not in sys.path:
        sys.path.insert(0, STUBS)


def load(modname: str):
    """Import `ap_gym.<modname>` from the reference tree without running the package inits."""
    if not reference_available():
        raise RuntimeError("reference tree not available at %s" % REF_ROOT)
    _ns("ap_gym", os.path.join(REF_ROOT, "ap_gym"))
    _ns("ap_gym.envs", os.path.join(REF_ROOT, "ap_gym", "envs"))
    return importlib.import_module("ap_gym." + modname)


def load_core():
    """Populate the `ap_gym` namespace with the names lidar_localization2d.py imports from it
    (`from ap_gym import ActiveRegressionEnv, ImageSpace, idoc`), using the reference's files."""
    install_stubs()
    pkg = _ns("ap_gym", os.path.join(REF_ROOT, "ap_gym"))
    util = load("util")
    types_ = load("types")
    loss_fn = load("loss_fn")
    image_space = load("image_space")
    ape = load("active_perception_env")
    apve = load("active_perception_vector_env")
    are = load("active_regression_env")
    ace = load("active_classification_env")
    for m in (util, types_, loss_fn, image_space, ape, apve, are, ace):
        for k, v in vars(m).items():
            if not k.startswith("_"):
                setattr(pkg, k, v)
    tl = load("time_limit")
    pkg.TimeLimit = tl.TimeLimit
    return pkg
