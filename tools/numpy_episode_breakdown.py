"""Where the numpy backend's episode-end step goes (make_vec's drop-in default, cfg 2: LIDARLocRooms-v0,
65536 envs, 32 beams, 64x64): one synchronized episode (100 steps + the autoreset step), with the reset step
split into its host parts by timing the env's methods:
  rows      the packed output rows D2H (one pinned copy + synchronize)
  map       the map observation mirror refresh (1 GB D2H at a full reset) + the copy=True snapshot
  stats     info["stats"]: scalar arrays and the per-env metric histories (lists of np.float32, the
            reference's ActiveRegressionLogWrapper lists; vector_stats="array" returns float32 rows instead)
  other     the rest of step() (launch, info assembly)
Prints one JSON object per vector_stats mode.
    python tools/numpy_episode_breakdown.py [num_envs]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
import ap_gym_amd as ap  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda:0")


def timed(obj, name, acc):
    f = getattr(obj, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
        return r

    setattr(obj, name, w)


for mode in ("list", "array"):
    env = ap.make_vec("LIDARLocRooms-v0", num_envs=n, lidar_beam_count=32, dataset=ap.FloorMapDatasetRooms(64, 64),
                      device=dev, array_backend="numpy", vector_stats=mode)
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1, 1, (4, n, 2)).astype(np.float32)
    env.reset(seed=0)
    for t in range(101):  # one whole episode first (warm: pinned buffers, snapshot, the first autoreset)
        env.step({"action": acts[t % 4], "prediction": acts[(t + 1) % 4]})
    acc: dict = {}
    for name in ("_host_rows", "_map_refresh", "_numpy_stats"):
        timed(env, name, acc)
    per = []
    t_ep = time.perf_counter()
    for t in range(101):
        a0 = dict(acc)
        t0 = time.perf_counter()
        _, _, term, trunc, info = env.step({"action": acts[t % 4], "prediction": acts[(t + 1) % 4]})
        dt = time.perf_counter() - t0
        per.append((dt, {k: acc.get(k, 0.0) - a0.get(k, 0.0) for k in acc}))
    t_ep = time.perf_counter() - t_ep
    ends = [i for i, (dt, _) in enumerate(per) if dt == max(d for d, _ in per)]
    dt, parts = per[ends[0]]
    ordinary = [d for i, (d, _) in enumerate(per) if i != ends[0]]
    out = {"vector_stats": mode, "num_envs": n, "episode_s": t_ep, "episode_env_steps_per_s": n * 101 / t_ep,
           "ordinary_step_ms_median": 1e3 * float(np.median(ordinary)), "end_step": ends[0],
           "end_step_ms": 1e3 * dt,
           "end_step_parts_ms": {"rows": 1e3 * parts.get("_host_rows", 0.0),
                                 "map": 1e3 * parts.get("_map_refresh", 0.0),
                                 "stats": 1e3 * parts.get("_numpy_stats", 0.0)},
           "np_float32_objects": 2 * n * 100 if mode == "list" else 0,
           "torch_threads": torch.get_num_threads()}
    out["end_step_parts_ms"]["other"] = out["end_step_ms"] - sum(out["end_step_parts_ms"].values())
    print(json.dumps(out), flush=True)
    env.close()
