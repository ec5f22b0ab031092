"""Host time of the image env's torch-backend step (bench.py's MNIST / TinyImageNetLoc configuration): per-call host
durations of env.step without synchronizing (is the loop host- or GPU-bound?), the wall per step, and a cProfile of
the host side.
    python tools/image_host_time.py [mnist|tinyimagenet-loc] [steps]
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
sys.path.insert(0, ROOT)
import ap_gym_amd as apg  # noqa: E402
from bench import IMAGE_WORKLOADS  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "mnist"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 340
w = IMAGE_WORKLOADS[wl]
dev = torch.device("cuda:0")
n = w.get("envs", w.get("envs_total"))
c = 1 if len(w["shape"]) == 2 else w["shape"][-1]
ds = apg.SyntheticImageClassificationDataset(w["pool"], w["shape"], w["classes"], c, seed=0)
cfg = apg.ImagePerceptionConfig(dataset=ds, sensor_size=w["sensor"], step_limit=16)
cls = apg.ImageClassificationVectorEnv if w["kind"] == "cls" else apg.ImageLocalizationVectorEnv
env = cls(n, cfg, device=dev, array_backend="torch", log_stats=True)
ring = 17
g = torch.Generator(device=dev).manual_seed(1)
acts = torch.rand((ring, n, 2), generator=g, device=dev) * 2 - 1
preds = (torch.randn((ring, n, w["classes"]), generator=g, device=dev) if w["kind"] == "cls"
         else torch.rand((ring, n, 2), generator=g, device=dev) * 2 - 1)
inputs = [{"action": acts[k], "prediction": preds[k]} for k in range(ring)]
env.reset(seed=0)
for t in range(5):
    env.step(inputs[t % ring])
torch.cuda.synchronize()

host, kinds = [], []
t0 = time.perf_counter()
for t in range(steps):
    resetting = env._prev_done
    a = time.perf_counter()
    env.step(inputs[t % ring])
    host.append(time.perf_counter() - a)
    kinds.append(resetting)
t_sub = time.perf_counter() - t0
torch.cuda.synchronize()
wall = time.perf_counter() - t0
host = np.array(host) * 1e6
kinds = np.array(kinds)
pr = cProfile.Profile()
pr.enable()
for t in range(steps):
    env.step(inputs[t % ring])
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
out = {"workload": wl, "steps": steps, "wall_us_per_step": wall / steps * 1e6,
       "submit_us_per_step": t_sub / steps * 1e6,
       "host_us_ordinary": {"median": float(np.median(host[~kinds])), "mean": float(host[~kinds].mean()),
                            "p90": float(np.percentile(host[~kinds], 90))},
       "host_us_reset_step": {"median": float(np.median(host[kinds])), "max": float(host[kinds].max()),
                              "count": int(kinds.sum())}}
print(json.dumps(out), flush=True)
print(s.getvalue())
env.close()
