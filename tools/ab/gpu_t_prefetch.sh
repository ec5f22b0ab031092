set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_lidar.py -x -v --timeout 300 --timeout-method thread -m gpu -k "prefetch or maze or copy_semantics or vector_stats or graph" > gpurun_out/r04/t_prefetch.log 2>&1
rc=$?; tail -n 30 gpurun_out/r04/t_prefetch.log; exit $rc
