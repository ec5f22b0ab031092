set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_image.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/img_test.log 2>&1 || { echo IMGTEST FAIL; tail -30 gpurun_out/r03/img_test.log; exit 1; }
tail -2 gpurun_out/r03/img_test.log
V=active-perception-gym_amd/ap_gym_amd/_lib/variants/lut.so
timeout -k 10 400 bash tools/gpu_ab.sh mnist 200 default $V || exit 1
timeout -k 10 400 bash tools/gpu_ab.sh tinyimagenet-loc 200 default $V || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharding.py -x -q --timeout 240 --timeout-method thread -k rccl > gpurun_out/r03/rccl_test.log 2>&1 || { echo RCCL FAIL; tail -30 gpurun_out/r03/rccl_test.log; exit 1; }
tail -2 gpurun_out/r03/rccl_test.log
timeout -k 10 200 python bench.py --gather --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03/bench_lidar_gather_rccl1.json 2> gpurun_out/r03/bench_lidar_gather_rccl1.err || { tail -5 gpurun_out/r03/bench_lidar_gather_rccl1.err; exit 1; }
tail -c 300 gpurun_out/r03/bench_lidar_gather_rccl1.json
