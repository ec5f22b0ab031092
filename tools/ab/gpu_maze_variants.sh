#!/bin/bash
# LIDAR GPU tests on the default library, then the maze127 bench (reset(seed) time, fused autoreset
# step, ordinary step) for the default library and each variant in _lib/variants
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_lidar.py > gpurun_out/pt_lidar.log 2>&1 || { tail -30 gpurun_out/pt_lidar.log; exit 1; }
tail -1 gpurun_out/pt_lidar.log
for lib in default $(ls active-perception-gym_amd/ap_gym_amd/_lib/variants/*.so 2>/dev/null); do
  if [ $lib = default ]; then unset APG_LIBRARY; name=default; else export APG_LIBRARY=$PWD/$lib; name=$(basename $lib .so); fi
  if [ $name != default ]; then
    timeout -k 10 200 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_lidar.py -k "maze or cfg3" > gpurun_out/pt_$name.log 2>&1 || { tail -30 gpurun_out/pt_$name.log; exit 1; }
    echo "$name tests: $(tail -1 gpurun_out/pt_$name.log)"
  fi
  timeout -k 10 300 python bench.py --workload maze127 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bm_$name.json 2> gpurun_out/bm_$name.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/bm_$name.json').read().strip().splitlines()[-1]); r=d['roofline']; e=d.get('episode',{})
print('$name', '%.4g env-steps/s' % d['value'], 'kernel median %.1f us' % (r['median_kernel_ms']*1e3), 'episode %.4g reset-step %.1f ms' % (e.get('env_steps_per_s',0), e.get('reset_step_kernel_ms',0)), 'reset_ms %.1f' % d['config']['reset_ms'])"
done
