"""Wall time of the image envs' numpy backend (make_vec's drop-in default: host arrays in and out, log_stats on) at
the bench's MNIST / TinyImageNetLoc configurations: ms per step over `steps` steps (batch autoresets included).
    python tools/image_numpy_step.py [mnist|tinyimagenet-loc] [steps] [list|array]
(the last argument is the env's vector_stats: form of the episode-end info["stats"]["vector"] entries).
"""
import json
import os
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
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 68
vstats = sys.argv[3] if len(sys.argv) > 3 else "list"
w = IMAGE_WORKLOADS[wl]
n = w.get("envs", w.get("envs_total"))
c = 1 if len(w["shape"]) == 2 else w["shape"][-1]
ds = apg.SyntheticImageClassificationDataset(w["pool"], w["shape"], w["classes"], c, seed=0)
cfg = apg.ImagePerceptionConfig(dataset=ds, sensor_size=w["sensor"], step_limit=16)
cls = apg.ImageClassificationVectorEnv if w["kind"] == "cls" else apg.ImageLocalizationVectorEnv
env = cls(n, cfg, device=torch.device("cuda:0"), array_backend="numpy", log_stats=True,
          vector_stats=vstats)
rng = np.random.default_rng(1)
acts = rng.uniform(-1, 1, (4, n, 2)).astype(np.float32)
preds = (rng.standard_normal((4, n, w["classes"])) if w["kind"] == "cls" else rng.uniform(-1, 1, (4, n, 2))).astype(
    np.float32)
env.reset(seed=0)
for t in range(4):
    env.step({"action": acts[t % 4], "prediction": preds[t % 4]})
per = []
t0 = time.perf_counter()
for t in range(steps):
    a = time.perf_counter()
    env.step({"action": acts[t % 4], "prediction": preds[t % 4]})
    per.append(time.perf_counter() - a)
dt = time.perf_counter() - t0
per = np.array(per) * 1e3
print(json.dumps({"workload": wl, "num_envs": n, "vector_stats": vstats, "steps": steps,
                  "ms_per_step": dt / steps * 1e3,
                  "ms_median": float(np.median(per)), "ms_max": float(per.max()),
                  "env_steps_per_s": n * steps / dt}), flush=True)
env.close()
