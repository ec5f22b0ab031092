"""Wall time of reset(seed) of LIDARLocMaze at BASELINE config 3 (262144 envs, 127 x 127, 64 beams): k_maze
(every env's maze + map obs + start cell) and the observation pass.  Tuning A/B driver (APG_MAZE_LANES=...).

    python tools/maze_reset_time.py [num_envs] [size]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "active-perception-gym_amd"))


def main():
    import torch

    import ap_gym_amd as ap

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 127
    env = ap.make_vec("LIDARLocMaze-v0", num_envs=n, lidar_beam_count=64, dataset=ap.FloorMapDatasetMaze(size, size),
                      device="cuda:0", array_backend="torch")
    ts = []
    for seed in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.reset(seed=seed)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    env.check_errors()
    print(f"APG_MAZE_LANES={os.environ.get('APG_MAZE_LANES', 'default')} n={n} size={size} reset ms: "
          + " ".join(f"{t:.2f}" for t in ts), flush=True)


if __name__ == "__main__":
    main()
