"""Throughput benchmark of the north-star hot path: LIDARLocRooms-v0 vectorized step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]              # 1 GPU
    python bench.py --gpus N [--steps K] [--warmup W]          # N GPUs: bench.py starts the N ranks itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W        # the same under torchrun

Workload (BASELINE.json configs[1]): LIDARLocRooms-v0, num_envs = 65536 per GPU, 32 beams,
64x64 procedurally generated rooms maps, TimeLimit(100) with NEXT_STEP autoreset (so the timed
steps include the map-generation reset bursts at the reference's 1-in-101 rate).  A "step" is one
`env.step({"action", "prediction"})` over the whole batch with inputs already resident in HBM
(synthetic actions/predictions, uniform(-1, 1), pre-generated on device).  Multi-GPU: weak
scaling, each rank owns an independent env shard (seed offset rank*N), no data-path collective
(--gather adds the optional RCCL all-gather of the step outputs and reports its time separately).

Prints ONE JSON line on rank 0 (value = env-steps/s summed over all GPUs).

`--workload mnist` / `--workload tinyimagenet-loc` measure the image glimpse path on BASELINE.json
configs 4 and 5 instead (synthetic uint8 pools of the datasets' shapes; same JSON contract, the
timed region is the whole device step between HIP events).
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
sys.path.insert(0, ROOT)

BYTES_PER_ENV_STEP = lambda beams: 228 + 4 * beams  # noqa: E731  SURVEY §8(d): compulsory bytes per env-step
MAP_OBS_BYTES = lambda m: 4 * m * m  # noqa: E731  f32 map observation written on an env's autoreset step
EPISODE_PERIOD = 101  # TimeLimit(100) + the NEXT_STEP autoreset step: every env resets on steps 101, 202, ...
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


class HipEvents:
    """hipEvent_t pairs created through libamdhip64 (the runtime torch already loaded)."""

    def __init__(self, n: int):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self.hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = []
        for _ in range(2 * n):
            e = ctypes.c_void_p()
            if self.hip.hipEventCreate(ctypes.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev.append(e)

    def pair(self, i):
        return self.ev[2 * i], self.ev[2 * i + 1]

    def elapsed_ms(self, i) -> float:
        ms = ctypes.c_float()
        if self.hip.hipEventElapsedTime(ctypes.byref(ms), self.ev[2 * i], self.ev[2 * i + 1]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(e)


def cpu_threads() -> int:
    """Host cores this process may use (the GPU box's share: OMP_NUM_THREADS, CPU affinity)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp)) if omp and omp.isdigit() else n)


def cpu_baseline(beams: int, size: int, kind: str, num_envs: int | None, steps: int, threads: int | None) -> dict:
    """The C oracle (a port of the reference path, bit-identical outputs) on this host: reset, then
    `steps` steps (one autoreset burst in 101), once with `threads` OpenMP threads over the sub-envs
    (the reported row) and once with 1 thread (`single_thread`, the reference's own single-core shape)."""
    import numpy as np

    from oracle import oracle

    oracle.build()
    threads = threads or cpu_threads()
    per_env = 1.0 if kind == "rooms" else 4.0  # 127x127 mazes with 64 beams cost about 4x per env-step
    rows = {}
    for th, envs in ((threads, num_envs or int(8192 * min(threads, 16) / per_env)), (1, int(8192 / per_env))):
        env = oracle.OracleLidarVectorEnv(envs, kind, size, False, 0, beams)
        env.reset(0)
        rng = np.random.default_rng(1)
        acts = rng.uniform(-1, 1, (steps, envs, 2)).astype(np.float32)
        preds = rng.uniform(-1, 1, (steps, envs, 2)).astype(np.float32)
        t0 = time.perf_counter()
        for t in range(steps):
            env.step(acts[t], preds[t], threads=th)
        dt = time.perf_counter() - t0
        env.close()
        rows[th] = {"value": envs * steps / dt, "unit": "env-steps/s", "cores": th, "kind": "port",
                    "sample": f"oracle/liboracle.so C port ({'OpenMP, ' + str(th) + ' threads' if th > 1 else '1 thread'}), "
                              f"LIDARLoc {kind} {size}x{size} {beams} beams, {envs} envs x {steps} steps after "
                              f"reset(seed=0) incl. one autoreset burst ({dt:.1f} s)"}
    out = dict(rows[threads])
    if threads > 1:
        out["single_thread"] = rows[1]
    return out


# image workloads (BASELINE.json configs 4, 5): per-GPU envs, pool, classes, sensor, kind
IMAGE_WORKLOADS = {
    "mnist": dict(name="MNIST-v0 ImageClassificationVectorEnv", kind="cls", envs=65536, shape=(28, 28),
                  pool=60000, classes=10, sensor=(5, 5)),  # BASELINE config 4: 65536 envs on one GPU (weak)
    # BASELINE config 5: 32768 envs in total, sharded over the GPUs (strong, like the maze config)
    "tinyimagenet-loc": dict(name="TinyImageNetLoc-v0 ImageLocalizationVectorEnv", kind="loc", envs_total=32768,
                             shape=(64, 64, 3), pool=100000, classes=200, sensor=(12, 12)),
}


def image_bytes_per_env_step(kind: str, k: int, g: tuple, c: int) -> int:
    """Compulsory HBM bytes of one env-step of the image path: reads pos f64,
    action, prediction, label/target, data-point index, the (G+1)^2 C u8 bilinear taps; writes the glimpse
    (f32), glimpse_pos, pos, reward (f64), base_reward, loss, target, time_step."""
    taps = (g[0] + 1) * (g[1] + 1) * c
    glimpse = 4 * g[0] * g[1] * c
    if kind == "cls":
        return (16 + 8 + 4 * k + 4 + 8 + taps) + (glimpse + 8 + 16 + 8 + 4 + 8 + 4 + 4)
    return (16 + 8 + 8 + 8 + 8 + taps) + (glimpse + 8 + 16 + 8 + 4 + 4 + 8 + 4)


def image_cpu_baseline(w: dict, pool: np.ndarray, labels: np.ndarray, c: int, num_envs: int, steps: int) -> dict:
    from oracle import image_oracle as io

    env = io.ImageVectorEnvOracle(w["kind"], pool, labels, w["classes"], c, num_envs, w["sensor"])
    env.reset(0)
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1, 1, (steps, num_envs, 2)).astype(np.float32)
    preds = (rng.standard_normal((steps, num_envs, w["classes"])) if w["kind"] == "cls"
             else rng.uniform(-1, 1, (steps, num_envs, 2))).astype(np.float32)
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(acts[t], preds[t])
    dt = time.perf_counter() - t0
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/image_oracle.py numpy port (1 thread), {w['name']}, {num_envs} envs x {steps} steps "
                      f"after reset(seed=0) (reset untimed) incl. one autoreset ({dt:.1f} s)"}


def run_image(args, world, rank, dev):
    import torch
    import torch.distributed as dist

    import ap_gym_amd as apg

    w = IMAGE_WORKLOADS[args.workload]
    plan = shard_plan(args, world)
    n_local, n_total = plan["num_envs_per_gpu"], plan["num_envs_total"]
    log_stats = not args.no_log_stats
    c = 1 if len(w["shape"]) == 2 else w["shape"][-1]
    pool_len = args.pool_len or w["pool"]
    ds = apg.SyntheticImageClassificationDataset(pool_len, w["shape"], w["classes"], c, seed=0)
    cfg = apg.ImagePerceptionConfig(dataset=ds, sensor_size=w["sensor"], step_limit=16)
    cls = apg.ImageClassificationVectorEnv if w["kind"] == "cls" else apg.ImageLocalizationVectorEnv
    from ap_gym_amd.sharding import ShardedVectorEnv

    # (**kw: packed_outputs=True when gathering: the step kernel writes the all-gather's rows itself)
    senv = ShardedVectorEnv(lambda num_envs, env_offset, **kw: cls(num_envs, cfg, device=dev, array_backend="torch",
                                                                   num_envs_total=n_total, env_offset=env_offset,
                                                                   log_stats=log_stats, **kw),
                            n_total, rank, world, gather=args.gather, time_gather=True, sub_batches=args.sub_batches)
    env = senv.env
    ring = 17
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    acts = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    if w["kind"] == "cls":
        preds = torch.randn((ring, n_local, w["classes"]), generator=g, device=dev)
    else:
        preds = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    inputs = [{"action": acts[k], "prediction": preds[k]} for k in range(ring)]  # prepared up front
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    (senv if senv.sub_batches > 1 else env).reset(seed=0)  # (every sub-batch's env resets)
    torch.cuda.synchronize(dev)
    reset_ms = (time.perf_counter() - t0) * 1e3
    for t in range(args.warmup):
        senv.step(inputs[t % ring])
    senv.gather_ms()
    ev = HipEvents(args.steps)
    stepper = senv.step if senv.gather else env.step
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # the timed window (`value`): K plain steps, no hipEvents between the launches (nor around the all-gathers)
    senv.time_gather = False
    t0 = time.perf_counter()
    for t in range(args.steps):
        stepper(inputs[(args.warmup + t) % ring])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    senv.check_errors()
    # the kernel-time pass (roofline and gather_ms, not `value`): K more steps, hipEvents right around the step's
    # kernel launches (inside env.step) on every event_every-th, and around every all-gather
    senv.time_gather = True
    timed = [t for t in range(args.steps) if t % args.event_every == args.event_every - 1]  # steps with hipEvents
    for t in range(args.steps):
        if t % args.event_every == args.event_every - 1:
            env.set_kernel_timing_events(*ev.pair(t))
            stepper(inputs[(args.warmup + args.steps + t) % ring])
            env.set_kernel_timing_events(None)
        else:
            stepper(inputs[(args.warmup + args.steps + t) % ring])
    env.set_kernel_timing_events(None)
    torch.cuda.synchronize(dev)
    senv.check_errors()
    step_ms = sum(ev.elapsed_ms(i) for i in timed) / len(timed)
    gather_ms = senv.gather_ms() or 0.0
    ev.close()
    if world > 1:
        tt = torch.tensor([elapsed, step_ms, reset_ms, gather_ms], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, step_ms, reset_ms, gather_ms = (float(x) for x in tt)
    if rank == 0:
        bpe = image_bytes_per_env_step(w["kind"], w["classes"], w["sensor"], c)
        shape = {"num_envs": n_local, "sensor": list(w["sensor"]), "classes": w["classes"], "log_stats": log_stats}
        # the step kernel's time: the rocprof duration table of these sources at this shape when there is one
        # (the events around a launch the GPU is not backed up behind include the host's launch latency, and
        # then exceed the wall time per step), else the events
        dj, dpath = newest_table("durations", args.workload, "image", shape, lambda t: "step" in t.get("per_class", {}))
        events_ms = step_ms
        if dj is not None:
            step_ms = dj["per_class"]["step"]["median_us"] / 1e3
        achieved = bpe * (n_local // args.sub_batches) / (step_ms * 1e-3) / 1e9  # (the timed launch: sub-batch 0's)
        tj, tpath = pmc_table(args.workload, "image", shape)
        traffic = issue = traffic_cal = None
        if tj is not None:
            traffic = tj["hbm_bytes_per_launch"]["step"]
            issue = issue_fractions(tj["per_launch"]["step"], step_ms)
            issue["source"] = tpath
            # u8 tap rows: dword gathers in 64-B runs; f32 glimpse / output stores
            traffic_cal = calibrated_traffic(tj["per_launch"]["step"], "k_seg64_4", "k_store4")
        bound, basis = derive_bound(achieved / HBM_PEAK_GBS, issue)
        out = {
            "metric": "env-steps/sec (vectorized step) at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": n_total * args.steps / elapsed, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": plan["scaling"], "vs_baseline": None, "dtype": "f64 bilinear / f32 outputs",
            "data": f"synthetic uint8 pool {pool_len}x{'x'.join(map(str, w['shape']))} (default_rng(0)); "
                    "uniform actions, normal logits / uniform predictions generated on device",
            "config": {"workload": w["name"], "num_envs_per_gpu": n_local, "num_envs_total": n_total,
                       "sensor": list(w["sensor"]), "classes": w["classes"], "step_limit": 16,
                       "log_stats": log_stats,
                       "reset_ms": reset_ms, "parallelism": f"env-shard x{world}" + (" + all-gather" if senv.gather
                                                                                        else ""),
                       "packed_rows": bool(senv._packed),
                       "gather_ms": gather_ms if senv.gather else None},
            "roofline": {"bound": bound, "bound_basis": basis, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_calibrated": traffic_cal, "traffic_source": tpath,
                         "kernel": "k_image_step_fused" if dj else "image step (all kernels, HIP events around the "
                                                                   "step's launches)",
                         "kernel_ms": step_ms, "kernel_ms_source": dpath or "hip events",
                         "kernel_ms_events": events_ms,
                         "launches_timed": len(timed), "event_every": args.event_every,
                         "bytes_per_launch": bpe * (n_local // args.sub_batches), "issue": issue},
        }
        if world == 1 and not args.no_cpu_baseline:
            pool, labels = ds.device_pool()
            n_cpu, s_cpu = (65536, 170) if w["kind"] == "cls" else (256, 2040)  # about 10 s of CPU work each
            out["cpu_baseline"] = image_cpu_baseline(w, pool, labels, c, n_cpu, s_cpu)
        print(json.dumps(out), flush=True)
    env.close()
    if dist.is_initialized():
        dist.destroy_process_group()


# LIDAR workloads (BASELINE.json configs 2 and 3)
LIDAR_WORKLOADS = {
    "lidar": dict(env_id="LIDARLocRooms-v0", kind="rooms", map=64, beams=32, envs=65536, scaling="weak",
                  note="BASELINE config 2: 65536 envs per GPU"),
    "maze127": dict(env_id="LIDARLocMaze-v0", kind="maze", map=127, beams=64, envs_total=262144, scaling="strong",
                    note="BASELINE config 3: 262144 envs in total, split over the GPUs (127x127: the reference "
                         "maze needs odd sizes, SURVEY §0.6)"),
}
KERNEL_ROOTS = {"lidar": "apg_lidar.hip", "image": "apg_image.hip"}  # the kernel family's translation unit
HIP_CLOCK_HZ = 2.4e9  # MI355X max engine clock (MI355X_MICROARCH.md); capacity of the issue fractions
SIMDS, CUS = 1024, 256


def kernel_sources(family: str) -> list[str]:
    """Every file the family's translation unit compiles: its .hip and the closure of its quoted #includes
    (csrc headers and include/apgym_capi.h), as sorted paths."""
    import re

    todo = [os.path.join(ROOT, "active-perception-gym_amd", "csrc", KERNEL_ROOTS[family])]
    seen = set()
    while todo:
        path = os.path.normpath(todo.pop())
        if path in seen:
            continue
        seen.add(path)
        with open(path) as fh:
            for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', fh.read(), re.M):
                todo.append(os.path.join(os.path.dirname(path), inc))
    return sorted(seen)


def kernel_source_sha(family: str) -> str:
    """Hash of the kernel sources a PMC table was collected with (a stale table is never used): the translation
    unit, every header it includes and its per-source compiler options (build.SOURCE_FLAGS)."""
    import hashlib

    import build  # active-perception-gym_amd/build.py: the per-source compiler options

    h = hashlib.sha256()
    for path in kernel_sources(family):
        h.update(os.path.relpath(path, ROOT).encode())
        with open(path, "rb") as fh:
            h.update(fh.read())
    opts = build.SOURCE_FLAGS.get(KERNEL_ROOTS[family])
    if opts:  # (a family compiled without extra options keeps its sources-only hash)
        h.update(" ".join(opts).encode())
    return h.hexdigest()[:16]


def pmc_table(workload: str, family: str, shape: dict):
    """The newest profiles/r*/pmc_<workload>.json collected (tools/collect_pmc.sh) from these kernel
    sources at this run shape, or (None, None)."""
    import glob

    sha = kernel_source_sha(family)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{workload}.json")), reverse=True):
        with open(path) as f:
            tj = json.load(f)
        if (tj.get("source_sha") == sha and tj.get("shape") == shape and "step" in tj.get("per_launch", {})
                and tj.get("hbm_bytes_per_launch", {}).get("step") is not None):
            return tj, os.path.relpath(path, ROOT)
    return None, None


def newest_table(kind: str, workload: str, family: str, shape: dict, need=lambda tj: True):
    """The newest profiles/r*/<kind>_<workload>.json collected from these kernel sources at this run shape,
    or (None, None)."""
    import glob

    sha = kernel_source_sha(family)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{kind}_{workload}.json")), reverse=True):
        with open(path) as f:
            tj = json.load(f)
        if tj.get("source_sha") == sha and tj.get("shape") == shape and need(tj):
            return tj, os.path.relpath(path, ROOT)
    return None, None


def fetch_calibration():
    """Newest profiles/r*/fetch_calibration.json (tools/fetch_calib.hip + tools/fetch_calib.py): bytes per
    counted FETCH_SIZE / WRITE_SIZE byte for each measured access pattern, or (None, None)."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "fetch_calibration.json")), reverse=True)
    if not paths:
        return None, None
    with open(paths[0]) as f:
        return json.load(f)["patterns"], os.path.relpath(paths[0], ROOT)


def calibrated_traffic(per_launch: dict, read_pattern: str, write_pattern: str):
    """HBM bytes per launch from the raw FETCH_SIZE / WRITE_SIZE (KiB) scaled by the calibration factors of
    the access patterns the kernel's reads / writes follow; None without counters or calibration."""
    cal, path = fetch_calibration()
    if cal is None or "FETCH_SIZE" not in per_launch or "WRITE_SIZE" not in per_launch:
        return None
    rf, wf = cal[read_pattern]["read_factor"], cal[write_pattern]["write_factor"]
    if rf is None or wf is None:
        return None
    return {"bytes": 1024.0 * (per_launch["FETCH_SIZE"] * rf + per_launch["WRITE_SIZE"] * wf),
            "read_pattern": read_pattern, "read_factor": rf, "write_pattern": write_pattern, "write_factor": wf,
            "calibration": path}


def derive_bound(frac: float, issue: dict | None):
    """roofline.bound from the measurement instead of a label: "hbm" only when the algorithmic bytes move at
    >= 50 % of the HBM peak; otherwise the kernel is issue/latency bound, with the PMC issue block's figures."""
    if frac >= 0.5:
        return "hbm", f"algorithmic bytes at {frac:.0%} of the HBM peak"
    if not issue:
        return "issue/latency", f"algorithmic bytes at {frac:.1%} of the HBM peak (no PMC table for these sources)"
    parts = [f"HBM at {frac:.1%} of peak"]
    for k, lab in (("valu_frac", "VALU issue"), ("lds_frac", "LDS issue"), ("wait_any_frac", "waves waiting")):
        if issue.get(k) is not None:
            parts.append(f"{lab} {issue[k]:.0%}")
    return "issue/latency", ", ".join(parts)


def issue_fractions(per_launch: dict, kernel_ms: float) -> dict:
    """Issue-rate roofline beside the HBM one: VALU wave-instructions x 2 cycles (wave64 on SIMD-32)
    over the SIMDs' cycles, and LDS array cycles (2 per ds_read_b32 wave-instruction + the counted
    bank-conflict cycles) over the CUs' LDS cycles, at the 2.4 GHz max clock."""
    cyc = kernel_ms * 1e-3 * HIP_CLOCK_HZ
    valu = per_launch.get("SQ_INSTS_VALU")
    lds = per_launch.get("SQ_INSTS_LDS")
    conf = per_launch.get("SQ_LDS_BANK_CONFLICT")
    out = {"valu_insts": valu, "lds_insts": lds, "lds_bank_conflict_cycles": conf,
           "valu_frac": 2.0 * valu / (SIMDS * cyc) if valu is not None else None,
           "lds_frac": (2.0 * lds + (conf or 0.0)) / (CUS * cyc) if lds is not None else None}
    if per_launch.get("SQ_WAIT_ANY") and per_launch.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = per_launch["SQ_WAIT_ANY"] / per_launch["SQ_WAVE_CYCLES"]
    if per_launch.get("SQ_THREAD_CYCLES_VALU") and per_launch.get("SQ_ACTIVE_INST_VALU"):
        out["valu_lane_util"] = per_launch["SQ_THREAD_CYCLES_VALU"] / (64.0 * per_launch["SQ_ACTIVE_INST_VALU"])
    return out


def run_lidar(args, world, rank, dev):
    import statistics

    import torch
    import torch.distributed as dist

    import ap_gym_amd as apg
    from ap_gym_amd.sharding import ShardedVectorEnv

    w = LIDAR_WORKLOADS[args.workload]
    beams = args.beams or w["beams"]
    msize = args.map_size or w["map"]
    if args.num_envs:
        n_local = args.num_envs
    elif "envs_total" in w:
        n_local = w["envs_total"] // world
    else:
        n_local = w["envs"]
    n_total = n_local * world
    ds = (apg.FloorMapDatasetRooms(msize, msize) if w["kind"] == "rooms" else apg.FloorMapDatasetMaze(msize, msize))

    def make_local(num_envs, env_offset, **kw):  # kw: packed_outputs=True when gathering
        if args.array_backend == "numpy":
            kw["obs_snapshot"] = args.obs_snapshot
        return apg.make_vec(w["env_id"], num_envs=num_envs, lidar_beam_count=beams, dataset=ds, device=dev,
                            array_backend=args.array_backend, env_offset=env_offset, **kw)

    senv = ShardedVectorEnv(make_local, n_total, rank, world, beams, gather=args.gather, time_gather=True,
                            sub_batches=args.sub_batches, gather_lag=args.gather_lag)
    env = senv.env
    ring = 128  # distinct synthetic action/prediction batches, cycled
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    acts = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    preds = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    if args.array_backend == "numpy":  # the default drop-in mode: host arrays in and out of every step
        acts, preds = acts.cpu().numpy(), preds.cpu().numpy()
    # the per-step input batches prepared up front, as a policy hands them over (no indexing in the loop)
    inputs = [{"action": acts[k], "prediction": preds[k]} for k in range(ring)]
    steps_done = 0

    def step(ev=None):
        nonlocal steps_done
        if ev is not None:
            env.set_kernel_timing_events(*ev)  # (None, None): no events on this step
        senv.step(inputs[steps_done % ring])
        steps_done += 1

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    senv.reset(seed=0)
    torch.cuda.synchronize(dev)
    reset_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(args.warmup):
        step()
    senv.gather_ms()
    ev = HipEvents(args.steps + EPISODE_PERIOD)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # the timed window (`value`): K plain steps, no hipEvents between the launches (nor around the all-gathers)
    senv.time_gather = False
    t0 = time.perf_counter()
    first_timed = steps_done + 1
    for t in range(args.steps):
        step()
    if senv.gather_lag:  # (the last step's all-gather, returned one call late, is part of the window)
        senv.flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    senv.check_errors()
    # the kernel-time pass (roofline and gather_ms, not `value`): K more steps, hipEvents around the step's
    # launches on every event_every-th (an event pair adds stream packets and +6..9 us of wall to its step) and
    # around every all-gather
    senv.time_gather = True
    first_ev = steps_done + 1
    timed = [t for t in range(args.steps) if t % args.event_every == args.event_every - 1]  # steps with hipEvents
    for t in range(args.steps):
        step(ev.pair(t) if t % args.event_every == args.event_every - 1 else (None, None))
    torch.cuda.synchronize(dev)
    env.set_kernel_timing_events(None)
    senv.check_errors()
    per_step = [ev.elapsed_ms(i) for i in timed]
    gather_ms = senv.gather_ms() or 0.0
    kernel_ms = sum(per_step) / len(per_step)
    median_ms = statistics.median(per_step)
    # reset steps (1-based step index t with t % 101 == 0: synchronized episodes) in the timed window
    reset_steps = sum(1 for t in range(first_timed, first_timed + args.steps) if t % EPISODE_PERIOD == 0)

    # one whole episode after the timed region (untimed for `value`): 100 steps + the autoreset step
    episode = None
    if not args.no_episode:
        while steps_done % EPISODE_PERIOD:
            step()
        torch.cuda.synchronize(dev)
        te = time.perf_counter()
        # events on every event_every-th step and on the autoreset step (the last)
        ep_t = [t for t in range(EPISODE_PERIOD)
                if t % args.event_every == args.event_every - 1 or t == EPISODE_PERIOD - 1]
        for t in range(EPISODE_PERIOD):
            step(ev.pair(args.steps + t) if t in ep_t else (None, None))
        if senv.gather_lag:
            senv.flush()
        torch.cuda.synchronize(dev)
        ep_s = time.perf_counter() - te
        env.set_kernel_timing_events(None)
        senv.check_errors()
        ep = [ev.elapsed_ms(args.steps + t) for t in ep_t]
        # mean kernel time of the episode: the ordinary steps' sampled mean over 100 steps + the reset step
        ep_mean = (statistics.mean(ep[:-1]) * (EPISODE_PERIOD - 1) + ep[-1]) / EPISODE_PERIOD
        episode = [ep_s, ep[-1], statistics.median(ep[:-1]), ep_mean]
    ev.close()

    if world > 1:
        tt = torch.tensor([elapsed, kernel_ms, median_ms, reset_ms, gather_ms] + (episode or [0.0] * 4),
                          dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        vals = [float(x) for x in tt]
        elapsed, kernel_ms, median_ms, reset_ms, gather_ms = vals[:5]
        episode = vals[5:] if episode else None

    if rank == 0:
        value = n_total * args.steps / elapsed
        step_b = BYTES_PER_ENV_STEP(beams) * (n_local // args.sub_batches)  # (the timed launch: sub-batch 0's)
        # a reset step also writes each env's map obs (f32) and its bit-packed occupancy rows
        reset_b = step_b + (MAP_OBS_BYTES(msize) + msize * ((msize + 63) // 64) * 8) * (n_local // args.sub_batches)
        # the launches the kernel time averages over: the kernel-time pass's steps that carried events
        reset_ev = sum(1 for t in timed if (first_ev + t) % EPISODE_PERIOD == 0)
        bytes_per_launch = (step_b * (len(timed) - reset_ev) + reset_b * reset_ev) / len(timed)
        achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
        shape = {"num_envs": n_local, "beams": beams, "map": msize}
        tj, tpath = pmc_table(args.workload, "lidar", shape)
        traffic = issue = traffic_cal = None
        if tj is not None:
            hb = tj["hbm_bytes_per_launch"]
            reset_b_pmc = hb.get("reset_step") or hb["step"]  # a table without a reset step: no reset in the window
            traffic = (hb["step"] * (len(timed) - reset_ev) + reset_b_pmc * reset_ev) / len(timed)
            issue = issue_fractions(tj["per_launch"]["step"], median_ms)
            issue["source"] = tpath
            # state / action loads and the 32-row occupancy windows: 8-B lanes in 256-B runs; 4-B output stores
            traffic_cal = calibrated_traffic(tj["per_launch"]["step"], "k_seg256_8", "k_store4")
        dj, dpath = newest_table("durations", args.workload, "lidar", shape, lambda t: "step" in t.get("per_class", {}))
        bound, basis = derive_bound(achieved / HBM_PEAK_GBS, issue)
        out = {
            "metric": "env-steps/sec (vectorized step) at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": w["scaling"],
            "vs_baseline": None,
            "dtype": "f32 (f64 exact geometry predicates)",
            "data": "synthetic (uniform(-1,1) actions/predictions generated on device; maps generated on device)"
                    + ("; array_backend=numpy: host arrays in/out of every step (PCIe included)"
                       if args.array_backend == "numpy" else ""),
            "config": {"workload": w["env_id"], "array_backend": args.array_backend,
                       "obs_snapshot": args.obs_snapshot if args.array_backend == "numpy" else None,
                       "num_envs_per_gpu": n_local,
                       "num_envs_total": n_total,
                       "beams": beams, "map": f"{msize}x{msize} {w['kind']}", "max_episode_steps": 100,
                       "reset_ms": reset_ms, "note": w["note"], "gather_ms": gather_ms if senv.gather else None,
                       "packed_rows": bool(senv._packed), "gather_lag": senv.gather_lag,
                       "parallelism": f"env-shard x{world}" + (" + all-gather" if senv.gather else "") + (
                           " (pipelined: step t's batch returned with step t+1)" if senv.gather_lag else "")},
            "roofline": {"bound": bound, "bound_basis": basis, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_calibrated": traffic_cal,
                         "kernel": "k_lidar_step" + (" (+ k_maze_stream, k_maze, k_maze_paint: workgroups that exit at "
                                                     "once on ordinary steps)" if w["kind"] == "maze" else ""),
                         "kernel_ms": kernel_ms, "median_kernel_ms": median_ms,
                         "kernel_ms_rocprof": ({c: v["median_us"] / 1e3 for c, v in dj["per_class"].items()}
                                               if dj else None), "durations_source": dpath,
                         "bytes_per_launch": bytes_per_launch, "reset_steps_timed": reset_steps,
                         "launches_timed": len(timed), "event_every": args.event_every,
                         "traffic_source": tpath, "issue": issue},
        }
        if episode:
            ep_s, reset_step_ms, ep_median, ep_mean = episode
            out["episode"] = {
                "steps": EPISODE_PERIOD, "env_steps_per_s": n_total * EPISODE_PERIOD / ep_s,
                "ms_per_step": ep_s * 1e3 / EPISODE_PERIOD, "reset_step_kernel_ms": reset_step_ms,
                "median_kernel_ms": ep_median, "mean_kernel_ms": ep_mean,
                "note": "one synchronized episode after the timed steps: 100 steps + the NEXT_STEP autoreset step "
                        "(map generation of every env + map obs), wall clock"}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(beams, msize, w["kind"], args.cpu_envs, args.cpu_steps,
                                               args.cpu_threads)
        print(json.dumps(out), flush=True)
    senv.close()
    if dist.is_initialized():
        dist.destroy_process_group()


class stdout_to_stderr:
    """File descriptor 1 pointed at stderr inside the block (native libraries write there directly)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(n: int) -> None:
    """Start `n` rank processes of this same command line (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    rendezvous on 127.0.0.1) as children, wait for all of them and exit with the first non-zero status.
    Rank 0 prints the JSON line; the other ranks print nothing on stdout."""
    import subprocess

    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # rank 0's stdout is filtered below; the others' goes to stderr (libraries print there, e.g. gloo)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    for line in procs[0].stdout:  # only the JSON line reaches our stdout
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    if bad:
        raise SystemExit(bad[0])


def shard_plan(args, world: int) -> dict:
    """The per-rank work of a workload at `world` ranks, as run_lidar / run_image size it: envs per rank, total
    envs, the scaling mode, and with --gather the packed output row every rank all-gathers per step (the row
    layouts the step kernels write: lidar_env.lidar_output_row_layout / image_env.image_output_row_layout)."""
    from ap_gym_amd import _native as N

    if args.workload in IMAGE_WORKLOADS:
        from ap_gym_amd.image_env import image_output_row_layout

        w = IMAGE_WORKLOADS[args.workload]
        c = 1 if len(w["shape"]) == 2 else w["shape"][-1]
        kind = N.APG_IMAGE_CLASSIFY if w["kind"] == "cls" else N.APG_IMAGE_LOCALIZE
        row = image_output_row_layout(kind, w["sensor"], c, not args.no_log_stats)[1]
        name = w["name"]
    else:
        from ap_gym_amd.lidar_env import lidar_output_row_layout

        w = LIDAR_WORKLOADS[args.workload]
        row = lidar_output_row_layout(args.beams or w["beams"], True)[1]  # make_vec logs stats
        name = w["env_id"]
    if args.num_envs:
        n_local = args.num_envs
    elif "envs_total" in w:
        if w["envs_total"] % world:
            raise SystemExit(f"{args.workload}: {w['envs_total']} envs do not split over {world} ranks")
        n_local = w["envs_total"] // world
    else:
        n_local = w["envs"]
    return {"workload": name, "num_envs_per_gpu": n_local, "num_envs_total": n_local * world,
            "scaling": "strong" if "envs_total" in w else "weak", "row_bytes": row if args.gather else None,
            "gather_bytes_per_rank_step": row * n_local * (world - 1) if args.gather else 0,
            "sub_batches": args.sub_batches, "gather_lag": args.gather_lag,
            "parallelism": f"env-shard x{world}" + (" + all-gather" if args.gather else "") + (
                f" in {args.sub_batches} overlapped sub-batches" if args.sub_batches > 1 else "") + (
                " (pipelined: step t's batch returned with step t+1)" if args.gather_lag else "")}


def run_dry(args, world, rank):
    """--dry-run: the multi-rank plumbing of the bench over gloo on CPU, without envs or a GPU: rendezvous, the
    workload's shard plan (envs per rank, seed offsets, packed row size), barrier-bracketed timing of `steps`
    rounds, max over ranks, one JSON line from rank 0.  With --gather every round all-gathers the full-size
    [envs per rank, row] byte buffers the step kernels would write and checks every rank's block arrived."""
    import torch
    import torch.distributed as dist

    plan = shard_plan(args, world)
    n_local = plan["num_envs_per_gpu"]
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    S = args.sub_batches
    if n_local % S:
        raise SystemExit(f"{n_local} envs per rank do not split into {S} sub-batches")
    m = n_local // S
    sends = parts = None
    if args.gather:  # sub-batch h of rank r: global envs [(h*W + r)*m, +m) (ShardedVectorEnv's layout)
        sends = []
        for h in range(S):
            snd = torch.empty((m, plan["row_bytes"]), dtype=torch.uint8)
            snd[:, 0] = rank
            snd[:, 8:16].view(torch.int64)[:, 0] = torch.arange((h * world + rank) * m, (h * world + rank + 1) * m)
            sends.append(snd)
        parts = [[torch.empty_like(sends[0]) for _ in range(world)] for _ in range(S)]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if args.gather:
            for h in range(S):
                if world > 1:
                    dist.all_gather(parts[h], sends[h])
                else:
                    parts[h][0].copy_(sends[h])
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if args.gather:
        got = torch.cat([p for ps in parts for p in ps])
        ok = bool((got[:, 0] == torch.arange(world).repeat_interleave(m).repeat(S)).all()) and bool(
            (got[:, 8:16].contiguous().view(torch.int64)[:, 0] == torch.arange(world * n_local)).all())
        if not ok:
            raise SystemExit(f"rank {rank}: gathered rows out of order")
    tt = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": args.steps / float(tt[0]), "unit": "steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": float(tt[0]) * 1e3 / args.steps, "higher_is_better": True,
                          "scaling": plan["scaling"], "vs_baseline": None, "dtype": "none",
                          "data": "none (gloo on CPU)", "config": dict(plan, ranks=world)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=505)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="lidar", choices=[*LIDAR_WORKLOADS, *IMAGE_WORKLOADS])
    ap.add_argument("--num-envs", type=int, default=None, help="envs per GPU (default: the workload's)")
    ap.add_argument("--pool-len", type=int, default=None, help="image pool size (image workloads)")
    ap.add_argument("--beams", type=int, default=None)
    ap.add_argument("--map-size", type=int, default=None)
    ap.add_argument("--gather", action="store_true", help="all-gather step outputs across ranks (RCCL)")
    ap.add_argument("--sub-batches", type=int, default=1,
                    help="with --gather: each rank's envs in S sub-batches whose all-gathers are issued right after "
                         "their steps, so RCCL gathers sub-batch h while sub-batch h+1 steps (ShardedVectorEnv)")
    ap.add_argument("--gather-lag", type=int, default=0, choices=[0, 1],
                    help="with --gather (LIDAR): 1 = pipelined all-gather, step t's gathered batch returned with step "
                         "t+1's call (two send / receive buffers), so RCCL moves step t's rows while step t+1 runs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-episode", action="store_true", help="skip the one-episode measurement after the timed steps")
    ap.add_argument("--cpu-envs", type=int, default=None)
    ap.add_argument("--cpu-steps", type=int, default=101)
    ap.add_argument("--cpu-threads", type=int, default=None, help="OpenMP threads of the multi-thread CPU row")
    ap.add_argument("--event-every", type=int, default=4,
                    help="kernel-time pass after the timed window: record the kernel's hipEvents on every N-th "
                         "step (steps N-1, 2N-1, ...: not the first launch after the synchronize); the timed "
                         "window itself carries no events (an event pair adds two stream packets between kernels, "
                         "+6..9 us of wall per step on MI355X, tools/host_overhead.py)")
    ap.add_argument("--array-backend", default="torch", choices=["torch", "numpy"],
                    help="LIDAR workloads: torch = device tensors in/out (the hot path, default); numpy = the "
                         "drop-in default of make_vec (host arrays, one packed D2H copy per step)")
    ap.add_argument("--obs-snapshot", default="copy", choices=["copy", "shared"],
                    help="--array-backend numpy: obs['map'] as the caller's own writable copy per step (copy: "
                         "SyncVectorEnv(copy=True), the default) or one read-only snapshot shared until a reset")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend of multi-rank runs (nccl = RCCL; gloo for rehearsals with "
                         "several ranks on one GPU)")
    ap.add_argument("--no-log-stats", action="store_true",
                    help="image workloads: the bare env class without the episode statistics make_vec's log "
                         "wrapper adds (the default measures the drop-in make_vec configuration, log_stats=True)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks rendezvous over gloo, time a barrier, rank 0 prints "
                         "the JSON line")
    args = ap.parse_args()
    args.event_every = max(1, min(args.event_every, args.steps))  # at least one timed launch carries events

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # started as `python bench.py --gpus N`: launch the N ranks ourselves (fresh processes, before anything
        # here touches a GPU), like torch.distributed.run would, and exit with the worst rank's status
        return self_launch(args.gpus)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.sub_batches > 1 and not args.gather:
        raise SystemExit("--sub-batches overlaps the all-gather with the steps: it needs --gather")
    if args.gather_lag and (not args.gather or args.sub_batches > 1 or args.workload in IMAGE_WORKLOADS):
        raise SystemExit("--gather-lag 1 pipelines the LIDAR all-gather: it needs --gather and --sub-batches 1")
    if args.dry_run:
        return run_dry(args, world, rank)
    # one rank per GPU; with fewer visible GPUs than ranks (rehearsals with --dist-backend gloo) ranks share them
    ndev = max(1, torch.cuda.device_count())  # counting devices does not initialise HIP
    torch.cuda.set_device(local_rank % ndev)
    dev = torch.device("cuda", local_rank % ndev)
    if world == 1 and args.gather:  # one GPU: a one-rank group still runs the all-gather's collective code path
        os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    if world > 1 or args.gather:
        # RCCL prints its version banner on stdout when the communicator comes up (eagerly here: device_id):
        # keep stdout for the one JSON line
        with stdout_to_stderr():
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
                dist.barrier()
            else:
                dist.init_process_group("gloo")
    if args.workload in IMAGE_WORKLOADS:
        return run_image(args, world, rank, dev)
    return run_lidar(args, world, rank, dev)


if __name__ == "__main__":
    main()
