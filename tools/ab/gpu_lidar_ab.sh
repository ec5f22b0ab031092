#!/bin/bash
# LIDAR parity tests of the working tree, then an interleaved A/B against HEAD's kernels (tools/ab/ab_prev.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
timeout -k 10 700 python -u -m pytest tests/test_gpu_lidar.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03/lidar_test.log 2>&1 || { echo LIDAR TESTS FAIL; tail -30 gpurun_out/r03/lidar_test.log; exit 1; }
tail -1 gpurun_out/r03/lidar_test.log
timeout -k 10 500 bash tools/ab/gpu_ab.sh ${1:-lidar} ${2:-300} default active-perception-gym_amd/ap_gym_amd/_lib/variants/prev.so
