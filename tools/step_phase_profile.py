"""Phase timeline of k_lidar_step (tuning aid): needs a library built with -DAPG_STEP_PROFILE, e.g.

    python active-perception-gym_amd/build.py -DAPG_STEP_PROFILE --out=tune/libprof.so
    APG_LIBRARY=tune/libprof.so python tools/step_phase_profile.py

Marks per workgroup (s_memrealtime, 100 MHz): 0 start, 1 windows staged, 2 move phase done,
3 beam pre-test done, 4 queued walks done, 5 end; slot 6 = queued walks.  WARM=100 profiles the rooms
autoreset step (marks 8 phase R start, 10 / 11 wave 0's generation / paint done, 12 phase-R barrier).
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))
import ap_gym_amd as ap  # noqa: E402
from ap_gym_amd import _native as N  # noqa: E402

n = int(os.environ.get("NENV", 65536))
M = int(os.environ.get("MAP", 64))  # bench.py's workload: BASELINE config 2 (64x64 rooms, 32 beams)
KIND = os.environ.get("KIND", "rooms")  # maze: BASELINE config 3 (MAP=127 BEAMS=64 NENV=262144)
B = int(os.environ.get("BEAMS", 32))
ds = ap.FloorMapDatasetRooms(M, M) if KIND == "rooms" else ap.FloorMapDatasetMaze(M, M)
env = ap.make_vec("LIDARLocRooms-v0" if KIND == "rooms" else "LIDARLocMaze-v0", num_envs=n, lidar_beam_count=B,
                  dataset=ds, array_backend="torch")
env.reset(seed=0)
g = torch.Generator(device="cuda")
g.manual_seed(0)
for t in range(int(os.environ.get("WARM", 30))):
    a = torch.rand((n, 2), device="cuda", generator=g) * 2 - 1
    env.step({"action": a, "prediction": a})
torch.cuda.synchronize()
if not hasattr(N.lib(), "apg_debug_step_profile"):
    sys.exit("library built without -DAPG_STEP_PROFILE: only the warm-up steps ran")
N.lib().apg_debug_step_profile.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
for rep in range(3):
    a = torch.rand((n, 2), device="cuda", generator=g) * 2 - 1
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    # through the ctypes C ABI of $APG_LIBRARY (the torch ops link the default library)
    N.check(N.lib().apg_lidar_step(ctypes.byref(env._cfg), ctypes.byref(env._state), N.ptr(a), N.ptr(a),
                                   ctypes.byref(env._out), N.stream_handle(a.device)), "apg_lidar_step")
    ev1.record()
    torch.cuda.synchronize()
    print(f"rep {rep}: events around env.step {ev0.elapsed_time(ev1) * 1000:.1f} us")
    epb = int(os.environ.get("APG_STEP_EPB") or (256 if n >= 256 * 256 else 64))
    nwg = (n + epb - 1) // epb
    buf = np.zeros((16384, 16), np.uint64)
    assert N.lib().apg_debug_step_profile(buf.ctypes.data, buf.nbytes) == 0
    b = buf[:nwg].astype(np.int64)
    t0 = b[:, 0].min()

    def us(x):
        return x * 0.01  # 100 MHz ticks -> us

    off = b[:, 0] - t0
    print(f"rep {rep}: kernel span {us(b[:, 5].max() - t0):.1f} us; WG start offsets p50/p99/max "
          f"{us(np.percentile(off, 50)):.1f}/{us(np.percentile(off, 99)):.1f}/{us(off.max()):.1f}; "
          f"WG end p50/max {us(np.percentile(b[:, 5] - t0, 50)):.1f}/{us((b[:, 5] - t0).max()):.1f}")
    if b[:, 10].any():  # a rooms autoreset step: 10 generation done, 11 maps painted (wave 0), 12 phase-R barrier
        for nm, k0, k1 in (("  launch -> R start", 0, 8), ("  R1 generate (wave 0)", 8, 10),
                           ("  R2 paint (wave 0)", 10, 11), ("  R3 + R barrier", 11, 12),
                           ("  windows reloaded", 12, 9), ("  stored -> barrier", 9, 1)):
            d = us(b[:, k1] - b[:, k0])
            print(f"   {nm:22s} p50 {np.percentile(d, 50):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f}")
    elif b[:, 8].any() and b[:, 9].any():  # sub-marks of the staging phase: 8 phase-R barrier, 9 windows in LDS
        for nm, k0, k1 in (("  launch -> R barrier", 0, 8), ("  R barrier -> stored", 8, 9), ("  stored -> barrier", 9, 1)):
            d = us(b[:, k1] - b[:, k0])
            print(f"   {nm:22s} p50 {np.percentile(d, 50):6.2f}  p90 {np.percentile(d, 90):6.2f}")
    if b[:, 10].any() and hasattr(N.lib(), "apg_debug_step_profile_waves"):  # per-wave R1 / R2 ends (lane 0)
        wv = np.zeros((16384, 16, 2), np.uint64)
        N.lib().apg_debug_step_profile_waves.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        assert N.lib().apg_debug_step_profile_waves(wv.ctypes.data, wv.nbytes) == 0
        w = wv[:nwg].astype(np.int64)
        r0 = b[:, 8][:, None]
        g1 = us(w[:, :, 0] - r0)  # R start -> wave's generation done
        p2 = us(w[:, :, 1] - w[:, :, 0])  # wave's paint
        e2 = us(w[:, :, 1] - r0)  # R start -> wave's paint done
        for nm, d in (("R1 generate, per wave", g1), ("R2 paint, per wave", p2), ("R start -> R2 done, per wave", e2)):
            print(f"   {nm:30s} all-wave p50 {np.percentile(d, 50):6.1f} p90 {np.percentile(d, 90):6.1f}  "
                  f"per-WG max: p50 {np.percentile(d.max(1), 50):6.1f} max {d.max():6.1f}")
        slow = np.argmax(e2, axis=1)
        print(f"   slowest wave of a WG: its R1 p50 {np.percentile(g1[np.arange(nwg), slow], 50):.1f}, "
              f"its R2 p50 {np.percentile(p2[np.arange(nwg), slow], 50):.1f} us")
    names = ["stage windows", "move (phase 1)", "pre-test (2a)", "walks (2b)", "store"]
    for k in range(5):
        d = us(b[:, k + 1] - b[:, k])
        print(f"   {names[k]:16s} p50 {np.percentile(d, 50):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
    mhz = np.median(b[:, 7] / np.maximum(b[:, 5] - b[:, 0], 1)) * 100
    print(f"   shader clock / realtime x 100 MHz: {mhz:.0f} MHz")
    q = b[:, 6]
    print(f"   queued walks per WG: mean {q.mean():.0f} p90 {np.percentile(q, 90):.0f} max {q.max()}")
    end = us(b[:, 5] - t0)
    print(f"   WG end percentiles p10/p25/p50/p75/p90/p99/max: " +
          "/".join(f"{np.percentile(end, p):.1f}" for p in (10, 25, 50, 75, 90, 99)) + f"/{end.max():.1f}")
    print(f"   corr(queued walks, WG end) = {np.corrcoef(q, end)[0, 1]:.2f}")
