# LIDAR map / env parity subset, then an interleaved A/B of the in-tree library against variants
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_lidar.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/t_lidar.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04/t_lidar.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab/gpu_ab.sh lidar 300 default "$@"
