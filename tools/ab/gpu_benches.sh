#!/bin/bash
# bench lines of every workload with the current bench.py (after the PMC tables are current):
# LIDAR driver shape + default, maze127 (PMC table refreshed first), MNIST, TinyImageNetLoc
set -e
R=$PWD
O=$R/gpurun_out/benches
mkdir -p $O $R/profiles/r02
if [ "${MAZE_PMC:-1}" = 1 ]; then
  bash tools/collect_pmc.sh maze127 > $O/pmc_maze127.log 2>&1
  cp gpurun_out/pmc_maze127.json profiles/r02/pmc_maze127.json
  cp gpurun_out/pmc_maze127.json $O/
fi
run() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err
  python3 -c "
import json; d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1]); r=d['roofline']; e=d.get('episode') or {}
print('$name', '%.4g' % d['value'], 'wall %.1f us' % (d['ms_per_step']*1e3), 'kernel %.1f us' % (r['kernel_ms']*1e3), 'frac %.3f' % r['frac'], 'traffic', r.get('traffic'), 'episode %.4g' % e.get('env_steps_per_s', 0))"
}
run lidar_driver_shape --steps 20 --warmup 5
run maze127_driver_shape --workload maze127 --steps 20 --warmup 5
run mnist_driver_shape --workload mnist --steps 20 --warmup 5
run tinyimagenet-loc_driver_shape --workload tinyimagenet-loc --steps 20 --warmup 5
run default
