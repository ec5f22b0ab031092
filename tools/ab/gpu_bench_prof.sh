#!/bin/bash
# GPU tests, then the default bench under a rocprofv3 kernel trace (per-kernel durations) and plain.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pb
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pb -o pb -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/pb.log 2>&1
cd $R
for k in k_lidar_step k_lidar_reset; do python3 tools/durations.py $(find gpurun_out/pb -name "*kernel_trace.csv") $k; done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
cat gpurun_out/bench.log | grep metric
