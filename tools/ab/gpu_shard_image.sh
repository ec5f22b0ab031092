#!/bin/bash
# sharding + image full-size tests, then the image benches
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharding.py "tests/test_gpu_image.py::test_image_cls_full_size_properties" "tests/test_gpu_image.py::test_image_loc_full_size_cfg5" > gpurun_out/pt_shard.log 2>&1 || { tail -40 gpurun_out/pt_shard.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pt_shard.log | tail -8
