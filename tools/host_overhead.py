"""Where the per-step wall time goes beyond the kernel (tuning aid): submission rate of env.step
(host only), wall per step with and without per-step hipEvents, and a CUDA-graph replay of the op."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
sys.path.insert(0, ROOT)
import ap_gym_amd as ap  # noqa: E402
from bench import HipEvents  # noqa: E402

n, K = 65536, 200
dev = torch.device("cuda:0")
env = ap.make_vec("LIDARLocRooms-v0", num_envs=n, lidar_beam_count=32, dataset=ap.FloorMapDatasetRooms(64, 64),
                  device=dev, array_backend="torch")
env.reset(seed=0)
acts = torch.rand((8, n, 2), device=dev) * 2 - 1
for t in range(5):
    env.step({"action": acts[t % 8], "prediction": acts[t % 8]})
torch.cuda.synchronize()


def run(label, events):
    ev = HipEvents(K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(K):
        if events:
            env.set_kernel_timing_events(*ev.pair(t))
        env.step({"action": acts[t % 8], "prediction": acts[t % 8]})
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    env.set_kernel_timing_events(None)
    k = sum(ev.elapsed_ms(i) for i in range(K)) / K if events else float("nan")
    ev.close()
    print(f"{label:24s} host {t_host / K * 1e6:6.1f} us/step  wall {t_wall / K * 1e6:6.1f} us/step  kernel {k * 1e3:6.1f} us")


run("events every step", True)
run("no events", False)
run("events every step", True)
run("no events", False)
ops = ap._native.torch_ops()
a0 = acts[0].contiguous()
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(K):
    ops.lidar_step(env._h, a0, a0)
th = time.perf_counter() - t0
torch.cuda.synchronize()
print(f"{'raw op loop':24s} host {th / K * 1e6:6.1f} us/step  wall {(time.perf_counter() - t0) / K * 1e6:6.1f} us/step")
g = env.capture_step_graph(a0, a0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(K):
    g.replay()
th = time.perf_counter() - t0
torch.cuda.synchronize()
print(f"{'graph replay (1 step)':24s} host {th / K * 1e6:6.1f} us/step  wall {(time.perf_counter() - t0) / K * 1e6:6.1f} us/step")
# a graph of 10 steps
g10 = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side), torch.cuda.graph(g10, stream=side):
    for t in range(10):
        ops.lidar_step(env._h, acts[t % 8], acts[t % 8])
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(K // 10):
    g10.replay()
th = time.perf_counter() - t0
torch.cuda.synchronize()
print(f"{'graph replay (10 steps)':24s} host {th / K * 1e6:6.1f} us/step  wall {(time.perf_counter() - t0) / K * 1e6:6.1f} us/step")
