#!/bin/bash
# EPB A/B through APG_STEP_EPB (same library): bash tools/ab/gpu_epb_env_ab.sh <workload> <steps> <epb>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
WL=$1; STEPS=$2; shift 2
for round in 1 2; do
  for E in "$@"; do
    if [ "$E" = default ]; then unset APG_STEP_EPB; else export APG_STEP_EPB=$E; fi
    timeout -k 10 300 python bench.py --workload $WL --steps $STEPS --warmup 10 --no-cpu-baseline --no-episode \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "ab $E failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('epb $E', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step kernel(ev)', round(r.get('median_kernel_ms', 0)*1e3,2))"
  done
done
unset APG_STEP_EPB
