"""Where an ordinary step of the numpy backend goes (make_vec's drop-in default, cfg 2: LIDARLocRooms-v0, 65536
envs, 32 beams, 64x64, log_stats): the step split into
  host_in     numpy inputs -> NaN checks -> pinned staging (host)
  h2d         the staged inputs' H2D copy (device, events)
  kernel      the fused step kernel (device, events)
  d2h         the output block's D2H copy into pinned memory (device, events)
  sync_wait   host time blocked in the synchronize after the D2H was enqueued (kernel + copies not yet done)
  host_out    field copies, info dict (host)
Medians over the episode's ordinary steps.  Prints one JSON object.
    python tools/numpy_step_breakdown.py [num_envs] [steps]
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
from ap_gym_amd import _native as N  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
dev = torch.device("cuda:0")
env = ap.make_vec("LIDARLocRooms-v0", num_envs=n, lidar_beam_count=32, dataset=ap.FloorMapDatasetRooms(64, 64),
                  device=dev, array_backend="numpy")
rng = np.random.default_rng(1)
acts = rng.uniform(-1, 1, (4, n, 2)).astype(np.float32)
env.reset(seed=0)
for t in range(5):
    env.step({"action": acts[t % 4], "prediction": acts[(t + 1) % 4]})

marks = {}
ev = {k: torch.cuda.Event(enable_timing=True) for k in ("h2d0", "k0", "k1", "d0", "d1")}
orig_launch, orig_rows = env._launch_step, env._host_rows


def launch(a_t, p_t):
    marks["launch"] = time.perf_counter()
    ev["k0"].record()
    orig_launch(a_t, p_t)
    ev["k1"].record()


def host_rows():  # LIDARLocalization2DVectorEnv._host_rows with events around the D2H copy
    from ap_gym_amd.lidar_env import block_views, row_views_np

    src = env.output_rows if env._out_block is None else env._out_block
    blk_t, blk_np = env._host_block()
    ev["d0"].record()
    blk_t.copy_(src, non_blocking=True)
    env._err_host.copy_(env._t["err"], non_blocking=True)
    ev["d1"].record()
    t0 = time.perf_counter()
    torch.cuda.current_stream(dev).synchronize()
    marks["sync"] = time.perf_counter() - t0
    marks["rows_done"] = time.perf_counter()
    env._err_pending = False
    return (row_views_np(blk_np, env.output_layout) if env._out_block is None
            else block_views(blk_np, env._block_layout))


env._launch_step = launch
env._host_rows = host_rows


rows = []
for t in range(steps):
    a, p = acts[t % 4], acts[(t + 1) % 4]
    torch.cuda.synchronize()
    ev["h2d0"].record()
    t0 = time.perf_counter()
    _, _, term, trunc, info = env.step({"action": a, "prediction": p})
    t1 = time.perf_counter()
    if env._autoreset_host.any() or "map_idx" in info:
        continue  # episode ends / autoresets: not ordinary
    rows.append(dict(total=1e3 * (t1 - t0), host_in=1e3 * (marks["launch"] - t0),
                     h2d=ev["h2d0"].elapsed_time(ev["k0"]), kernel=ev["k0"].elapsed_time(ev["k1"]),
                     d2h=ev["d0"].elapsed_time(ev["d1"]), sync_wait=1e3 * marks["sync"],
                     host_out=1e3 * (t1 - marks["rows_done"])))
med = {k: float(np.median([r[k] for r in rows])) for k in rows[0]}
block = (env._out_block if env._out_block is not None else env.output_rows).numel()
out = {"num_envs": n, "ordinary_steps": len(rows), "ms_median": med,
       "env_steps_per_s": n / (med["total"] * 1e-3), "d2h_bytes": int(block), "h2d_bytes": int(2 * n * 2 * 4),
       "d2h_GBps": block / (med["d2h"] * 1e-3) / 1e9, "torch_threads": torch.get_num_threads(),
       "copy": env.copy, "host_blocks": len(env._ring), "ring_copy_fallback": env._ring_copy}
print(json.dumps(out), flush=True)
env.close()
