# maze maps past 255 (k_maze_big) and rooms maps past 255 / max_rooms past 32: map parity and the vector-env parity
# runs, then the image batch
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_lidar.py -x -v -m gpu --timeout 300 --timeout-method thread -k "maze_branching or (vector_env_matches_oracle and maze) or rooms_parameters or large_rooms" > gpurun_out/r04/t_bigmaps.log 2>&1
rc=$?; tail -n 5 gpurun_out/r04/t_bigmaps.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_batch2.sh
