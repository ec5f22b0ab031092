set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharding.py tests/test_gpu_lidar.py -x -v -m gpu --timeout 600 --timeout-method thread -k "sharding or gather or packed or copy_semantics or vector_stats or full_size" > gpurun_out/r04/t_shard.log 2>&1
rc=$?; tail -n 25 gpurun_out/r04/t_shard.log; exit $rc
