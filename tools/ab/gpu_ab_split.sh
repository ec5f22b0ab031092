set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_lidar.py tests/test_gpu_render.py > gpurun_out/pt_def.log 2>&1 || { tail -30 gpurun_out/pt_def.log; exit 1; }
echo "default: $(tail -1 gpurun_out/pt_def.log)"
APG_LIBRARY=$PWD/active-perception-gym_amd/ap_gym_amd/_lib/variants/split1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_lidar.py > gpurun_out/pt_split.log 2>&1 || { tail -30 gpurun_out/pt_split.log; exit 1; }
echo "split1: $(tail -1 gpurun_out/pt_split.log)"
timeout -k 10 400 bash tools/ab/gpu_variants.sh > gpurun_out/var1.log 2>&1; cat gpurun_out/var1.log | grep median
timeout -k 10 400 bash tools/ab/gpu_variants.sh > gpurun_out/var2.log 2>&1; cat gpurun_out/var2.log | grep median
