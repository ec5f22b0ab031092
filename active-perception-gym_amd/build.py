"""Build the gfx950 shared library (no GPU needed: hipcc cross-compiles).

    python active-perception-gym_amd/build.py [--force] [--verbose]

Outputs (git-ignored; they travel to the GPU box with the gpurun snapshot):
  active-perception-gym_amd/ap_gym_amd/_lib/libapgym_hip.so    the gfx950 kernels + C ABI
  active-perception-gym_amd/ap_gym_amd/_lib/libapgym_torch.so  TORCH_LIBRARY(apgym) ops over that C ABI
"""

from __future__ import annotations

import hashlib
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
           "apg_ziggurat.hpp", "apg_maze.hpp", "apg_binom_table.hpp"]

# per-source compiler options, each measured: k_lidar_step's latency-bound phases schedule better under the
# memory-clause strategy (same-box A/B over six interleaved pairs of 300-step runs: median 32.53 -> 32.35 us, mean
# 36.27 -> 36.05 us, profiles/r06/ab/lidar_sched_strategy.txt; max-ilp measured slower).  bench.kernel_source_sha
# hashes these with the sources, so tables collected under other options are not used.
SOURCE_FLAGS = {"apg_lidar.hip": ("-mllvm", "-amdgpu-sched-strategy=max-memory-clause")}

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
    # every build (tuning variants included) answers to libapgym_hip.so: a variant loaded first through
    # APG_LIBRARY then also serves libapgym_torch.so's dependency, so the torch ops run it too
    "-Wl,-soname,libapgym_hip.so",
]


TORCH_OUT = os.path.join(OUT_DIR, "libapgym_torch.so")
TORCH_SRC = os.path.join(CSRC, "apg_torch_ops.cpp")


def _torch_stale() -> bool:
    if not os.path.exists(TORCH_OUT):
        return True
    t = os.path.getmtime(TORCH_OUT)
    return any(os.path.getmtime(d) > t for d in (TORCH_SRC, OUT, os.path.join(INCLUDE, "apgym_capi.h"),
                                                  os.path.abspath(__file__)))


def build_torch_ops(force: bool = False) -> str:
    """Host-only C++ against torch's headers (hipcc for the HIP stream API), linked to
    libapgym_hip.so next to it ($ORIGIN) and to torch's libraries."""
    if not force and not _torch_stale():
        return TORCH_OUT
    import torch
    from torch.utils import cpp_extension as ce

    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=apgym_torch",
           *[f"-I{p}" for p in ce.include_paths(device_type="cuda")], "-I", INCLUDE,
           "-o", TORCH_OUT + ".tmp", TORCH_SRC,
           f"-L{OUT_DIR}", "-lapgym_hip", f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch",
           "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{torch_lib}"]
    subprocess.run(cmd, check=True)
    os.replace(TORCH_OUT + ".tmp", TORCH_OUT)
    return TORCH_OUT


FAST_SRC = os.path.join(CSRC, "apg_pyfast.cpp")


def fast_module_path() -> str:
    import sysconfig

    return os.path.join(OUT_DIR, "_apgfast" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_fast_module(force: bool = False) -> str:
    """The CPython fast-call entry points of the per-step C-ABI calls (csrc/apg_pyfast.cpp): g++ against the
    interpreter's headers, linked to libapgym_hip.so next to it ($ORIGIN)."""
    import sysconfig

    out = fast_module_path()
    deps = (FAST_SRC, OUT, os.path.join(INCLUDE, "apgym_capi.h"), os.path.abspath(__file__))
    if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    tmp = f"{out}.{os.getpid()}.tmp"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{sysconfig.get_paths()['include']}",
                    "-I", INCLUDE, "-o", tmp, FAST_SRC, f"-L{OUT_DIR}", "-lapgym_hip", "-Wl,-rpath,$ORIGIN"],
                   check=True)
    os.replace(tmp, out)
    return out


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "apgym_capi.h"),
                                                                  os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


OBJ_DIR = os.path.join(HERE, "build_obj")  # per-source objects (git- and gpurun-ignored)


def _closure(path: str) -> list[str]:
    """The source and every file of its quoted #include closure (an object is stale once any is newer)."""
    import re

    todo, seen = [path], set()
    while todo:
        p = os.path.normpath(todo.pop())
        if p in seen:
            continue
        seen.add(p)
        with open(p) as fh:
            todo += [os.path.join(os.path.dirname(p), inc) for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', fh.read(), re.M)]
    return sorted(seen)


def build(force: bool = False, verbose: bool = False, extra_flags=(), out: str | None = None, only=None) -> str:
    """Build the library; `extra_flags`/`out` make tuning variants (e.g. -DAPG_STEP_PROFILE into tune/).
    Each source compiles to its own object in parallel (the kernels are independent translation units), and only
    objects older than their source or a shared header are rebuilt; then one link.  `only` (variants): the sources
    that take `extra_flags`; the others link their default objects."""
    os.makedirs(OUT_DIR, exist_ok=True)
    variant = out is not None
    out = out or OUT
    if not force and not variant and not _stale():
        return OUT
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    tag = "" if not extra_flags else "_" + hashlib.sha1(" ".join(extra_flags).encode()).hexdigest()[:10]
    odir = os.path.join(OBJ_DIR, "default" + tag)
    os.makedirs(odir, exist_ok=True)
    compile_flags = [f for f in FLAGS if f != "-shared" and not f.startswith("-Wl,")]
    procs, objs = [], []
    for src in SOURCES:
        spath = os.path.join(CSRC, src)
        flags = extra_flags if only is None or src in only else ()
        sdir = odir if flags else os.path.join(OBJ_DIR, "default")
        os.makedirs(sdir, exist_ok=True)
        obj = os.path.join(sdir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(
                os.path.getmtime(d) for d in _closure(spath) + [os.path.abspath(__file__)]):
            continue
        tmp = f"{obj}.{os.getpid()}.tmp"  # concurrent builds never share a temporary
        cmd = [HIPCC, *compile_flags, *SOURCE_FLAGS.get(src, ()), *flags, "-I", INCLUDE, "-c", "-o", tmp, spath]
        if verbose:
            cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), obj, tmp))
    failed = [obj for p, obj, _ in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc -c ({', '.join(os.path.basename(f) for f in failed)})")
    for _, obj, tmp in procs:
        os.replace(tmp, obj)
    link = [HIPCC, *[f for f in FLAGS if f in ("--offload-arch=gfx950", "-fPIC", "-shared") or f.startswith("-Wl,")],
            "-o", out + ".tmp", *objs]
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_all(force: bool = False) -> tuple[str, str, str]:
    return build(force=force), build_torch_ops(force=force), build_fast_module(force=force)


if __name__ == "__main__":
    args = sys.argv[1:]
    out_arg = next((a.split("=", 1)[1] for a in args if a.startswith("--out=")), None)
    defs = [a for a in args if a.startswith("-D")]
    only = next((a.split("=", 1)[1].split(",") for a in args if a.startswith("--only=")), None)
    print(build(force="--force" in args, verbose="--verbose" in args, extra_flags=defs, out=out_arg, only=only))
    if out_arg is None:
        print(build_torch_ops(force="--force" in args))
        print(build_fast_module(force="--force" in args))
