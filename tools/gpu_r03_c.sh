#!/bin/bash
# round 3 (c): maze generator A/B — standalone halves, then parity (maze tests), then the cfg-3 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/maze_bench 262144 127 64 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lidar.py -x -q --timeout 300 --timeout-method thread -k "maze" \
  > gpurun_out/t_maze.log 2>&1 || { echo "maze tests failed"; tail -30 gpurun_out/t_maze.log; exit 1; }
tail -2 gpurun_out/t_maze.log
timeout -k 10 300 python -u bench.py --workload maze127 --steps 20 --warmup 3 --no-cpu-baseline \
  > gpurun_out/b_maze.json 2> gpurun_out/b_maze.err || { echo "bench failed"; tail -20 gpurun_out/b_maze.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b_maze.json'));print(d['value'],d['config']['reset_ms'],d['episode'])"
