"""Throughput benchmark of the north-star hot path: LIDARLocRooms-v0 vectorized step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]              # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W        # N GPUs, one rank per GPU

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


def cpu_baseline(beams: int, size: int, num_envs: int, steps: int) -> dict:
    """The C oracle (a 1-thread port of the reference path) on this host: reset + `steps` steps."""
    import numpy as np

    from oracle import oracle

    oracle.build()
    env = oracle.OracleLidarVectorEnv(num_envs, "rooms", size, False, 0, beams)
    env.reset(0)
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1, 1, (steps, num_envs, 2)).astype(np.float32)
    preds = rng.uniform(-1, 1, (steps, num_envs, 2)).astype(np.float32)
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(acts[t], preds[t])
    dt = time.perf_counter() - t0
    env.close()
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/liboracle.so C port, 1 thread, LIDARLocRooms {size}x{size} {beams} beams, "
                      f"{num_envs} envs x {steps} steps after reset(seed=0) incl. one autoreset burst "
                      f"({dt:.1f} s)"}


# image workloads (BASELINE.json configs 4, 5): per-GPU envs, pool, classes, sensor, kind
IMAGE_WORKLOADS = {
    "mnist": dict(name="MNIST-v0 ImageClassificationVectorEnv", kind="cls", envs=65536, shape=(28, 28),
                  pool=60000, classes=10, sensor=(5, 5)),
    "tinyimagenet-loc": dict(name="TinyImageNetLoc-v0 ImageLocalizationVectorEnv", kind="loc", envs=32768,
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
    n_local = args.num_envs or w["envs"]
    n_total = n_local * world
    c = 1 if len(w["shape"]) == 2 else w["shape"][-1]
    pool_len = args.pool_len or w["pool"]
    ds = apg.SyntheticImageClassificationDataset(pool_len, w["shape"], w["classes"], c, seed=0)
    cfg = apg.ImagePerceptionConfig(dataset=ds, sensor_size=w["sensor"], step_limit=16)
    cls = apg.ImageClassificationVectorEnv if w["kind"] == "cls" else apg.ImageLocalizationVectorEnv
    env = cls(n_local, cfg, device=dev, array_backend="torch", num_envs_total=n_total, env_offset=rank * n_local)
    ring = 17
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    acts = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    if w["kind"] == "cls":
        preds = torch.randn((ring, n_local, w["classes"]), generator=g, device=dev)
    else:
        preds = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    env.reset(seed=0)
    torch.cuda.synchronize(dev)
    reset_ms = (time.perf_counter() - t0) * 1e3
    for t in range(args.warmup):
        env.step({"action": acts[t % ring], "prediction": preds[t % ring]})
    ev = HipEvents(args.steps)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ev.hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for t in range(args.steps):
        b, e = ev.pair(t)
        k = (args.warmup + t) % ring
        ev.hip.hipEventRecord(b, stream)
        env.step({"action": acts[k], "prediction": preds[k]})
        ev.hip.hipEventRecord(e, stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    env.check_errors()
    step_ms = sum(ev.elapsed_ms(i) for i in range(args.steps)) / args.steps
    ev.close()
    if world > 1:
        tt = torch.tensor([elapsed, step_ms, reset_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, step_ms, reset_ms = (float(x) for x in tt)
    if rank == 0:
        bpe = image_bytes_per_env_step(w["kind"], w["classes"], w["sensor"], c)
        achieved = bpe * n_local / (step_ms * 1e-3) / 1e9
        out = {
            "metric": "env-steps/sec (vectorized step) at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": n_total * args.steps / elapsed, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64 bilinear / f32 outputs",
            "data": f"synthetic uint8 pool {pool_len}x{'x'.join(map(str, w['shape']))} (default_rng(0)); "
                    "uniform actions, normal logits / uniform predictions generated on device",
            "config": {"workload": w["name"], "num_envs_per_gpu": n_local, "num_envs_total": n_total,
                       "sensor": list(w["sensor"]), "classes": w["classes"], "step_limit": 16,
                       "reset_ms": reset_ms, "parallelism": f"env-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "image step (all kernels, HIP events around env.step)", "kernel_ms": step_ms,
                         "bytes_per_launch": bpe * n_local},
        }
        if world == 1 and not args.no_cpu_baseline:
            pool, labels = ds.device_pool()
            n_cpu, s_cpu = (65536, 170) if w["kind"] == "cls" else (256, 2040)  # about 10 s of CPU work each
            out["cpu_baseline"] = image_cpu_baseline(w, pool, labels, c, n_cpu, s_cpu)
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=505)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="lidar", choices=["lidar", *IMAGE_WORKLOADS])
    ap.add_argument("--num-envs", type=int, default=None, help="envs per GPU (default: the workload's)")
    ap.add_argument("--pool-len", type=int, default=None, help="image pool size (image workloads)")
    ap.add_argument("--beams", type=int, default=32)
    ap.add_argument("--map-size", type=int, default=64)
    ap.add_argument("--gather", action="store_true", help="all-gather step outputs across ranks (RCCL)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-envs", type=int, default=8192)
    ap.add_argument("--cpu-steps", type=int, default=101)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import ap_gym_amd as apg
    from ap_gym_amd.sharding import ShardedVectorEnv

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.workload != "lidar":
        return run_image(args, world, rank, dev)

    n_local = args.num_envs or 65536
    n_total = n_local * world

    def make_local(num_envs, env_offset):
        return apg.make_vec("LIDARLocRooms-v0", num_envs=num_envs, lidar_beam_count=args.beams,
                            dataset=apg.FloorMapDatasetRooms(args.map_size, args.map_size), device=dev,
                            array_backend="torch", env_offset=env_offset)

    senv = ShardedVectorEnv(make_local, n_total, rank, world, args.beams, gather=args.gather and world > 1)
    env = senv.env
    ring = 128  # distinct synthetic action/prediction batches, cycled
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    acts = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1
    preds = torch.rand((ring, n_local, 2), generator=g, device=dev) * 2 - 1

    senv.reset(seed=0)
    for t in range(args.warmup):
        senv.step({"action": acts[t % ring], "prediction": preds[t % ring]})
    ev = HipEvents(args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for t in range(args.steps):
        b, e = ev.pair(t)
        env.set_kernel_timing_events(b, e)
        k = (args.warmup + t) % ring
        senv.step({"action": acts[k], "prediction": preds[k]})
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    env.set_kernel_timing_events(None)
    env.check_errors()
    kernel_ms = sum(ev.elapsed_ms(i) for i in range(args.steps)) / args.steps
    ev.close()

    if world > 1:
        tt = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(tt[0]), float(tt[1])

    if rank == 0:
        value = n_total * args.steps / elapsed
        # algorithmic bytes of the timed k_lidar_step launches: the per-env-step bytes every step, plus
        # the map observation on the autoreset steps (all envs reset together: synchronized episodes)
        reset_steps = sum(1 for t in range(args.steps) if (args.warmup + t + 1) % EPISODE_PERIOD == 0)
        bytes_total = (BYTES_PER_ENV_STEP(args.beams) * n_local * args.steps
                       + MAP_OBS_BYTES(args.map_size) * n_local * reset_steps)
        bytes_per_launch = bytes_total / args.steps
        achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic_lidar_step.json")
        if os.path.exists(tpath):
            with open(tpath) as f:
                tj = json.load(f)
            if tj.get("num_envs") == n_local and tj.get("beams") == args.beams:
                traffic = tj.get("hbm_bytes_per_launch")
        out = {
            "metric": "env-steps/sec (vectorized step) at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (f64 exact geometry predicates)",
            "data": "synthetic (uniform(-1,1) actions/predictions generated on device; maps generated on device)",
            "config": {"workload": "LIDARLocRooms-v0", "num_envs_per_gpu": n_local, "num_envs_total": n_total,
                       "beams": args.beams, "map": f"{args.map_size}x{args.map_size} rooms",
                       "max_episode_steps": 100, "parallelism": f"env-shard x{world}" + (" + all-gather" if args.gather
                                                                                         and world > 1 else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_lidar_step", "kernel_ms": kernel_ms,
                         "bytes_per_launch": bytes_per_launch, "reset_steps_timed": reset_steps},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.beams, args.map_size, args.cpu_envs, args.cpu_steps)
        print(json.dumps(out), flush=True)
    senv.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
