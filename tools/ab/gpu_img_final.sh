# image + sharding + circle-square suites, then the round's final MNIST / TinyImageNetLoc measurement sets
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_sharding.py tests/test_gpu_circle_square.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/t_img_final.log 2>&1
rc=$?; tail -n 1 gpurun_out/r04/t_img_final.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04_final.sh mnist || exit 1
bash tools/gpu_r04_final.sh tinyimagenet-loc || exit 1
bash tools/ab/gpu_image_long.sh
