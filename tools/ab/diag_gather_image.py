"""Which torch ops run per gathered TinyImageNetLoc step (one-rank RCCL group): torch.profiler op table."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import ap_gym_amd as apg  # noqa: E402
from ap_gym_amd.sharding import ShardedVectorEnv  # noqa: E402

os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(bench.free_port()))
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
with bench.stdout_to_stderr():
    dist.init_process_group("nccl", device_id=dev)
w = bench.IMAGE_WORKLOADS["tinyimagenet-loc"]
n = 32768
ds = apg.SyntheticImageClassificationDataset(100000, w["shape"], w["classes"], 3, seed=0)
cfg = apg.ImagePerceptionConfig(dataset=ds, sensor_size=w["sensor"], step_limit=16)
senv = ShardedVectorEnv(lambda num_envs, env_offset, **kw: apg.ImageLocalizationVectorEnv(
    num_envs, cfg, device=dev, array_backend="torch", num_envs_total=n, env_offset=env_offset, log_stats=True, **kw),
    n, 0, 1, gather=True)
print("packed", senv._packed, flush=True)
acts = torch.rand((4, n, 2), device=dev) * 2 - 1
inputs = [{"action": acts[k], "prediction": acts[(k + 1) % 4]} for k in range(4)]
senv.reset(seed=0)
for t in range(20):
    senv.step(inputs[t % 4])
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU], record_shapes=False) as prof:
    for t in range(34):
        senv.step(inputs[t % 4])
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="count", row_limit=30), flush=True)
dist.destroy_process_group()
