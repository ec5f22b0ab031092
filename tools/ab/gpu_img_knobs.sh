#!/bin/bash
# Image fused-step knob sweep: for each workload and each "NAME=VAL[,NAME=VAL]" setting (or "default"), a
# rocprofv3 kernel trace of a 200-step bench run and the fused step's duration.
#   bash tools/ab/gpu_img_knobs.sh "<workloads>" <setting>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/img_knobs
mkdir -p $O
WLS=$1; shift
for WL in $WLS; do
  for SET in "$@"; do
    TAG=$(echo "$SET" | tr ',=' '__')
    ENVS=""
    [ "$SET" != default ] && ENVS=$(echo "$SET" | tr ',' ' ')
    cd /tmp
    rm -rf $O/tr_${WL}_$TAG
    env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_${WL}_$TAG -o run -- \
      python3 $R/bench.py --workload $WL --steps 200 --warmup 20 --no-cpu-baseline --no-episode \
      > $O/b_${WL}_$TAG.json 2> $O/b_${WL}_$TAG.err || { echo "trace $WL $SET failed"; tail -5 $O/b_${WL}_$TAG.err; exit 1; }
    cd $R
    python3 tools/rocpd_stats.py $O/tr_${WL}_$TAG > $O/stats_${WL}_$TAG.txt && rm -rf $O/tr_${WL}_$TAG
    python3 -c "
import csv, json, re
d = json.load(open('$O/b_${WL}_$TAG.json'))
ks = []
for r in csv.DictReader(open('$O/stats_${WL}_$TAG.txt')):
    if int(r['calls']) >= 150:
        ks.append(re.sub(r'\(.*', '', r['kernel'].replace('(anonymous namespace)::', '')).split('::')[-1][:40] + ' ' + r['median_us'])
print('$WL', '$SET', '| wall', round(d['ms_per_step'] * 1e3, 2), 'us/step |', '; '.join(ks))"
  done
done
