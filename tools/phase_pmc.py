"""Phase split of k_lidar_step's instruction mix (tuning aid).  Run under rocprofv3 --pmc with a
library built with -DAPG_STEP_STOP=k (returns after phase k) in $APG_LIBRARY; the fused step kernel is
launched through that library's C ABI (the torch ops link the default library).

    APG_LIBRARY=.../libstop2.so rocprofv3 --pmc SQ_INSTS_VALU ... -- python3 tools/phase_pmc.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
import ap_gym_amd as ap  # noqa: E402
from ap_gym_amd import _native as N  # noqa: E402

n = int(os.environ.get("NENV", 65536))
env = ap.make_vec("LIDARLocRooms-v0", num_envs=n, lidar_beam_count=32, dataset=ap.FloorMapDatasetRooms(64, 64),
                  array_backend="torch")
env.reset(seed=0)
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(int(os.environ.get("STEPS", 20))):
    a = torch.rand((n, 2), device="cuda", generator=g) * 2 - 1
    N.check(N.lib().apg_lidar_step(ctypes.byref(env._cfg), ctypes.byref(env._state), N.ptr(a), N.ptr(a),
                                   ctypes.byref(env._out), N.stream_handle(a.device)), "apg_lidar_step")
torch.cuda.synchronize()
print("ok")
