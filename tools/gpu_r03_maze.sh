#!/bin/bash
# round 3: LIDAR tests (maze DFS rewrite, packed rows, numpy path), launcher + sharding tests, then the cfg-3
# bench with its episode leg and a rocprofv3 kernel trace of the same command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_lidar.py tests/test_gpu_sharding.py tests/test_bench_launcher.py}
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/t_r03.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_r03.log; exit 1; }
tail -3 gpurun_out/t_r03.log
timeout -k 10 300 python -u bench.py --workload maze127 --steps 20 --warmup 3 --no-cpu-baseline \
  > gpurun_out/b_maze.json 2> gpurun_out/b_maze.err || { echo "bench failed"; tail -20 gpurun_out/b_maze.err; exit 1; }
cat gpurun_out/b_maze.json
rm -rf gpurun_out/prof_maze
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_maze" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload maze127 --steps 20 --warmup 3 --no-cpu-baseline \
  > "$GRAFT_REPO_ROOT/gpurun_out/b_maze_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/b_maze_prof.err" || { echo "prof failed"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 tools/rocpd_stats.py gpurun_out/prof_maze --csv gpurun_out/prof_maze_stats.csv | cut -c1-150 | head -8
timeout -k 10 300 python -u bench.py --workload lidar --steps 20 --warmup 3 --no-cpu-baseline --array-backend numpy --no-episode \
  > gpurun_out/b_numpy.json 2> gpurun_out/b_numpy.err || { echo "numpy bench failed"; tail -20 gpurun_out/b_numpy.err; exit 1; }
cat gpurun_out/b_numpy.json
for L in 64 32 16; do
  APG_MAZE_LANES=$L timeout -k 10 200 python tools/maze_reset_time.py || exit 1
done
