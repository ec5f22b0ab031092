# image + sharding GPU suites, one-rank RCCL gather lines -> gpurun_out/r04/
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_sharding.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r04/t_image.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04/t_image.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_gather1.sh || exit 1
