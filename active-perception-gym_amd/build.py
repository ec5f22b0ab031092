"""Build the gfx950 shared library (no GPU needed: hipcc cross-compiles).

    python active-perception-gym_amd/build.py [--force] [--verbose]

Output: active-perception-gym_amd/ap_gym_amd/_lib/libapgym_hip.so (git-ignored; travels to the
GPU box with the gpurun snapshot).
"""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "ap_gym_amd", "_lib")
OUT = os.path.join(OUT_DIR, "libapgym_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
SOURCES = ["apg_lidar.hip", "apg_image.hip", "apg_circle_square.hip", "apg_light_dark.hip"]
HEADERS = ["apg_device.hpp", "apg_maps.hpp", "apg_scan.hpp", "apg_rng.hpp", "apg_host.hpp", "apg_pairwise.hpp",
           "apg_ziggurat.hpp"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # exactness: the kernels restate numpy/GEOS float arithmetic operation by operation
    "-ffp-contract=off",
    "-fno-fast-math",
    "-fno-gpu-flush-denormals-to-zero",
]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "apgym_capi.h"),
                                                                  os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, extra_flags=(), out: str | None = None) -> str:
    """Build the library; `extra_flags`/`out` make tuning variants (e.g. -DAPG_STEP_PROFILE into tune/)."""
    os.makedirs(OUT_DIR, exist_ok=True)
    variant = out is not None
    out = out or OUT
    if not force and not variant and not _stale():
        return OUT
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    cmd = [HIPCC, *FLAGS, *extra_flags, "-I", INCLUDE, "-o", out + ".tmp", *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    out_arg = next((a.split("=", 1)[1] for a in args if a.startswith("--out=")), None)
    defs = [a for a in args if a.startswith("-D")]
    print(build(force="--force" in args, verbose="--verbose" in args, extra_flags=defs, out=out_arg))
