# LIDAR parity tests ON A VARIANT library, then an interleaved A/B of the in-tree library against it:
#   bash tools/ab/gpu_variant_ab.sh <variant.so> [steps]
set -o pipefail
mkdir -p gpurun_out/r04
APG_LIBRARY=$PWD/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_lidar.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/t_variant.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04/t_variant.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab/gpu_ab.sh lidar ${2:-300} default $1
