# Precomputed-stream maze: tool timing, maze parity tests (incl. branching and the stream overflow), the
# maze env tests, then a cfg-3 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mzs
mkdir -p $O
timeout -k 10 120 tools/maze_bench 262144 127 64 > $O/maze_bench.json 2> $O/maze_bench.err || { echo "maze_bench failed"; cat $O/maze_bench.err; exit 1; }
cat $O/maze_bench.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_lidar.py -x -v --timeout 240 --timeout-method thread -k "maze or Maze" > $O/pytest_maze.log 2>&1 || { echo "maze tests failed"; grep -E "PASS|FAIL|Error|error" $O/pytest_maze.log | tail -30; exit 1; }
grep -cE "PASSED" $O/pytest_maze.log; tail -1 $O/pytest_maze.log
timeout -k 10 400 python bench.py --workload maze127 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_maze127.json 2> $O/bench_maze127.err || { echo "bench failed"; tail -5 $O/bench_maze127.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/bench_maze127.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'episode', d.get('episode'), 'reset_ms', d['config'].get('reset_ms'))"
