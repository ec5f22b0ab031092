#!/bin/bash
# Tuning-knob A/B through environment variables (same library), two interleaved rounds:
#   bash tools/ab/gpu_env_ab.sh <workload> <steps> "<VAR=value ...>" ...   ("-" = no variables)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
WL=$1; STEPS=$2; shift 2
for round in 1 2; do
  for V in "$@"; do
    if [ "$V" = - ]; then VARS=""; else VARS="$V"; fi
    env $VARS timeout -k 10 300 python bench.py --workload $WL --steps $STEPS --warmup 10 --no-cpu-baseline --no-episode \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "ab $V failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$V', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
