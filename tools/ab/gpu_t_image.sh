set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1200 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_sharding.py tests/test_gpu_circle_square.py tests/test_gpu_render.py -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/r04/t_image.log 2>&1
rc=$?; tail -n 25 gpurun_out/r04/t_image.log; exit $rc
