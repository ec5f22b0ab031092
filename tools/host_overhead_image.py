"""Where the per-step wall time of the MNIST image step goes beyond the kernel (tuning aid): env.step
submission rate (host only) and wall, and the host cost of its pieces (input normalisation, the torch op,
the output dicts), each timed in a loop of its own."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
import ap_gym_amd as ap  # noqa: E402

n, K = 65536, 400
dev = torch.device("cuda:0")
ds = ap.SyntheticImageClassificationDataset(60000, (28, 28), 10, 1, seed=0)
cfg = ap.ImagePerceptionConfig(dataset=ds, sensor_size=(5, 5), step_limit=16)
env = ap.ImageClassificationVectorEnv(n, cfg, device=dev, array_backend="torch", log_stats="--no-stats" not in sys.argv)
env.reset(seed=0)
acts = torch.rand((8, n, 2), device=dev) * 2 - 1
preds = torch.randn((8, n, 10), device=dev)
for t in range(20):
    env.step({"action": acts[t % 8], "prediction": preds[t % 8]})
torch.cuda.synchronize()


def loop(label, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(K):
        fn(t)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"{label:28s} host {th / K * 1e6:6.1f} us/step  wall {tw / K * 1e6:6.1f} us/step", flush=True)


import ctypes  # noqa: E402

from ap_gym_amd import _native as N  # noqa: E402

L = N.lib()
stream = N.stream_handle(dev)
cfg_p, st_p, out_p = ctypes.byref(env._cfg), ctypes.byref(env._state), ctypes.byref(env._out)
a_ptr, p_ptr = [N.ptr(acts[t]) for t in range(8)], [N.ptr(preds[t]) for t in range(8)]
for _ in range(2):
    loop("raw op .default", lambda t: env._step_op(env._h, acts[t % 8], preds[t % 8], 1, 0))
    loop("C ABI via ctypes", lambda t: L.apg_image_step(cfg_p, st_p, a_ptr[t % 8], p_ptr[t % 8], 1, 0, out_p, stream))
for _ in range(2):
    loop("env.step", lambda t: env.step({"action": acts[t % 8], "prediction": preds[t % 8]}))
    loop("as_tensor+reshape+contig x2", lambda t: (
        torch.as_tensor(acts[t % 8], dtype=torch.float32, device=dev).reshape(n, 2).contiguous(),
        torch.as_tensor(preds[t % 8], dtype=torch.float32, device=dev).reshape(n, 10).contiguous()))
    loop("raw op", lambda t: env._ops.image_step(env._h, acts[t % 8], preds[t % 8], 1, 0))
    loop("_torch_step", lambda t: env._torch_step(False, False))
    loop("check_errors(block=False)", lambda t: env.check_errors(block=False))
print("ok")

if "--profile" in sys.argv:  # where env.step's host time goes, by function (prebuilt inputs, as bench.py)
    import cProfile
    import pstats

    inputs = [{"action": acts[t], "prediction": preds[t]} for t in range(8)]
    loop("env.step (prebuilt inputs)", lambda t: env.step(inputs[t % 8]))
    pr = cProfile.Profile()
    pr.enable()
    for t in range(2000):
        env.step(inputs[t % 8])
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
