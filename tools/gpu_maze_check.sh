set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_lidar.py > gpurun_out/pt_full.log 2>&1 || { tail -30 gpurun_out/pt_full.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pt_full.log | tail -4
timeout -k 10 300 python bench.py --workload maze127 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/b_maze.json 2> gpurun_out/b_maze.err
python3 -c "
import json; d=json.loads(open('gpurun_out/b_maze.json').read().strip().splitlines()[-1]); r=d['roofline']; e=d.get('episode',{})
print('maze127', '%.4g env-steps/s' % d['value'], 'wall %.1f us/step' % (d['ms_per_step']*1e3), 'kernel mean %.1f median %.1f us' % (r['kernel_ms']*1e3, r['median_kernel_ms']*1e3), 'episode %.4g reset-step %.1f ms' % (e.get('env_steps_per_s',0), e.get('reset_step_kernel_ms',0)), 'reset_ms %.1f' % d['config']['reset_ms'])"
