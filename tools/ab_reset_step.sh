#!/bin/bash
# Reset-step A/B at cfg 2 (on the GPU box): per variant and round, the bench line's synchronized episode (100 steps +
# the NEXT_STEP autoreset step) under a rocprof kernel trace: its reset_step_kernel_ms (hipEvents around the step
# call: every launch of the reset step) and env-steps/s, and the traced k_lidar_step / k_map_obs_deferred durations.
#   bash tools/ab_reset_step.sh <default|env:NAME=VALUE|variant.so>...       outputs under gpurun_out/ab/
set -o pipefail
R=$PWD
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for V in "$@"; do
    unset APG_LIBRARY
    case "$V" in
      default) tag=reset_default_$round; ENVSET="" ;;
      env:*) ENVSET=${V#env:}; tag=reset_$(echo $ENVSET | tr '=' '_')_$round ;;
      *) export APG_LIBRARY=$R/$V; ENVSET=""; tag=reset_$(basename $V .so)_$round ;;
    esac
    rm -rf $O/kt_$tag
    [ -n "$ENVSET" ] && export "$ENVSET"
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$tag -o run -- python3 $R/bench.py \
      --steps 20 --warmup 5 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { echo "ab $V failed"; tail -5 $O/$tag.err; exit 1; }
    [ -n "$ENVSET" ] && unset "${ENVSET%%=*}"
    f=$(find $O/kt_$tag -name "*kernel_trace.csv" | head -1)
    echo "$tag $(python3 -c "
import json; d=json.load(open('$O/$tag.json')); e=d['episode']
print('episode', round(e['env_steps_per_s']/1e6,1), 'M/s reset_step', round(e['reset_step_kernel_ms']*1e3,1), 'us')")"
    echo "   step: $(python3 $R/tools/durations.py $f 'k_lidar_step')"
    echo "   deferred: $(python3 $R/tools/durations.py $f 'k_map_obs_deferred' 2>&1)"
  done
done
