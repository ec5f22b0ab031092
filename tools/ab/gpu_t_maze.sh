set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_lidar.py -x -q -m gpu --timeout 600 --timeout-method thread -k "maze" > gpurun_out/r04/t_maze.log 2>&1
rc=$?; tail -n 4 gpurun_out/r04/t_maze.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_maze_prof.sh
