#!/bin/bash
# LIDAR iteration loop on the GPU box: parity tests, benches (default EPB and APG_STEP_EPB=64), a kernel trace.
#   bash tools/ab/gpu_lidar_iter.sh [pytest selection]
set -e
mkdir -p gpurun_out
SEL=${1:-tests/test_gpu_lidar.py tests/test_gpu_render.py}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $SEL > gpurun_out/pt_lidar.log 2>&1 || { tail -40 gpurun_out/pt_lidar.log; exit 1; }
tail -1 gpurun_out/pt_lidar.log
summ() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; e=d.get('episode',{})
print(sys.argv[2], '%.4g env-steps/s' % d['value'], 'wall %.1f us/step' % (d['ms_per_step']*1e3), 'kernel mean %.1f median %.1f us' % (r['kernel_ms']*1e3, r['median_kernel_ms']*1e3), 'frac %.4f' % r['frac'], 'episode %.4g env-steps/s reset-step %.1f us' % (e.get('env_steps_per_s',0), e.get('reset_step_kernel_ms',0)*1e3), 'reset_ms %.1f' % d['config']['reset_ms'])
" $1 $2; }
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 5 > gpurun_out/b_default.json 2> gpurun_out/b_default.err
summ gpurun_out/b_default.json default
for e in ${EPBS:-64 128}; do
  APG_STEP_EPB=$e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 5 > gpurun_out/b_epb$e.json 2> gpurun_out/b_epb$e.err
  summ gpurun_out/b_epb$e.json epb$e
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt -o kt -- python3 $R/bench.py --no-cpu-baseline --steps 120 --warmup 0 > $R/gpurun_out/kt.log 2>&1
cd $R
python3 tools/durations.py $(find gpurun_out/kt -name "*kernel_trace.csv") k_lidar_step
python3 tools/durations.py $(find gpurun_out/kt -name "*kernel_trace.csv") k_lidar_reset
