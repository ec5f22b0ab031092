#!/bin/bash
# Interleaved A/B of library variants (rocprof kernel-trace medians + the bench line), on the GPU box:
#   bash tools/ab_trace.sh <workload> <steps> <kernel-regex> <variant.so|default|env:NAME=VALUE>...
# (env:NAME=VALUE: the in-tree library with that tuning variable set)
# Two rounds; per variant and round: the bench value / wall ms per step, and the median / mean duration of the
# dispatches matching <kernel-regex> (durations.py).  Outputs under gpurun_out/ab/.
set -o pipefail
R=$PWD
O=$R/gpurun_out/ab
mkdir -p $O
WL=$1; STEPS=$2; KR=$3; shift 3
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for V in "$@"; do
    unset APG_LIBRARY
    case "$V" in
      default) tag=default_$round; ENVSET="" ;;
      env:*) ENVSET=${V#env:}; tag=$(echo $ENVSET | tr '=' '_')_$round ;;
      *) export APG_LIBRARY=$R/$V; ENVSET=""; tag=$(basename $V .so)_$round ;;
    esac
    rm -rf $O/kt_$tag
    [ -n "$ENVSET" ] && export "$ENVSET"
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$tag -o run -- python3 $R/bench.py --workload $WL \
      --steps $STEPS --warmup 20 --no-cpu-baseline --no-episode > $O/$tag.json 2> $O/$tag.err || { echo "ab $V failed"; tail -5 $O/$tag.err; exit 1; }
    [ -n "$ENVSET" ] && unset "${ENVSET%%=*}"
    f=$(find $O/kt_$tag -name "*kernel_trace.csv" | head -1)
    echo "$tag $(python3 -c "import json;d=json.load(open('$O/$tag.json'));print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')") $(python3 $R/tools/durations.py $f "$KR")"
  done
done
