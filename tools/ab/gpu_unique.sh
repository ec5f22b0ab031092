#!/bin/bash
# image GPU tests, then the localization bench under a kernel trace: k_unique* durations
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_image.py > gpurun_out/pt_img.log 2>&1 || { tail -30 gpurun_out/pt_img.log; exit 1; }
tail -1 gpurun_out/pt_img.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pi -o pi -- python3 $R/bench.py --workload tinyimagenet-loc --no-cpu-baseline --steps 50 > $R/gpurun_out/pi.log 2>&1
cd $R
python3 tools/durations.py $(find gpurun_out/pi -name "*kernel_trace.csv") k_unique
