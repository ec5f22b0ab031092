# maze A/B bench + all maze / lidar env GPU tests + the maze127 episode profile (tools/gpu_maze_prof.sh)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/maze_bench 262144 127 64 > gpurun_out/r04/maze_bench_ab.json 2>&1 || { cat gpurun_out/r04/maze_bench_ab.json; exit 1; }
cat gpurun_out/r04/maze_bench_ab.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_lidar.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r04/t_lidar.log 2>&1
rc=$?; tail -n 4 gpurun_out/r04/t_lidar.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_maze_prof.sh
