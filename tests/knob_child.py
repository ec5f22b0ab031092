"""Child process of tests/test_gpu_image.py::test_tuning_knobs_do_not_change_results: runs one small
image env trace with whatever APG_* tuning knobs its environment sets (the library reads them once per
process) and saves every output to the .npz named by argv[1]."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
import ap_gym_amd as ap  # noqa: E402


def trace(kind: str, k: int, n: int, steps: int) -> dict:
    rng = np.random.default_rng(k + n)
    shape = (28, 28) if kind == "cls" else (32, 32, 3)
    pool = rng.integers(0, 256, (200, *shape), dtype=np.uint8)
    labels = rng.integers(0, k, 200)
    ds = ap.ArrayImageClassificationDataset(pool, labels, k, 1 if len(shape) == 2 else 3)
    cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(5, 5) if kind == "cls" else (7, 7), step_limit=6)
    env = (ap.ImageClassificationVectorEnv if kind == "cls" else ap.ImageLocalizationVectorEnv)(n, cfg)
    out = {}
    obs, _ = env.reset(seed=3)
    out["reset_glimpse"] = obs["glimpse"]
    arng = np.random.default_rng(7)
    for t in range(steps):
        a = arng.uniform(-1.5, 1.5, (n, 2)).astype(np.float32)
        p = (arng.standard_normal((n, k)) if kind == "cls" else arng.uniform(-1, 1, (n, 2))).astype(np.float32)
        obs, rew, term, trunc, info = env.step({"action": a, "prediction": p})
        out[f"{t}_glimpse"] = obs["glimpse"]
        out[f"{t}_pos"] = obs["glimpse_pos"]
        out[f"{t}_reward"] = np.asarray(rew, np.float64)
        out[f"{t}_loss"] = np.asarray(info["prediction"]["loss"], np.float64)
    env.close()
    return out


if __name__ == "__main__":
    res = {}
    for kind, k, n in (("cls", 3, 300), ("cls", 13, 300), ("loc", 2, 300)):
        for key, v in trace(kind, k, n, 14).items():
            res[f"{kind}{k}_{key}"] = v
    np.savez(sys.argv[1], **res)
