#!/bin/bash
# Image parity tests of the working tree (image, CircleSquare, sharding), then interleaved A/Bs against HEAD's
# kernels (tools/ab/ab_prev.sh) on MNIST and TinyImageNetLoc
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
timeout -k 10 700 python -u -m pytest tests/test_gpu_image.py tests/test_gpu_circle_square.py tests/test_gpu_sharding.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/image_test.log 2>&1 \
  || { echo IMAGE TESTS FAIL; tail -30 gpurun_out/r03/image_test.log; exit 1; }
tail -1 gpurun_out/r03/image_test.log
V=active-perception-gym_amd/ap_gym_amd/_lib/variants/prev.so
timeout -k 10 400 bash tools/ab/gpu_ab.sh mnist 200 default $V || exit 1
timeout -k 10 400 bash tools/ab/gpu_ab.sh tinyimagenet-loc 200 default $V
