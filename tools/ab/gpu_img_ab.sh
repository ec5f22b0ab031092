#!/bin/bash
# Image step A/B: staged tap windows (default) vs direct tap loads (APG_GLIMPSE_NO_WINDOW), interleaved, with a
# rocprofv3 kernel trace of each for the fused step's duration.  bash tools/ab/gpu_img_ab.sh [workloads...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/img_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_image.log 2>&1 || { echo "image tests failed"; tail -20 $O/pytest_image.log; exit 1; }
tail -1 $O/pytest_image.log
for WL in ${@:-mnist tinyimagenet-loc}; do
  for V in win direct; do
    if [ $V = direct ]; then export APG_GLIMPSE_NO_WINDOW=1; else unset APG_GLIMPSE_NO_WINDOW; fi
    cd /tmp
    rm -rf $O/tr_${WL}_$V
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_${WL}_$V -o run -- \
      python3 $R/bench.py --workload $WL --steps 200 --warmup 20 --no-cpu-baseline --no-episode \
      > $O/b_${WL}_$V.json 2> $O/b_${WL}_$V.err || { echo "trace $WL $V failed"; tail -5 $O/b_${WL}_$V.err; exit 1; }
    cd $R
    python3 tools/rocpd_stats.py $O/tr_${WL}_$V > $O/stats_${WL}_$V.txt
    echo "== $WL $V"
    python3 -c "
import csv
for r in csv.DictReader(open('$O/stats_${WL}_$V.txt')):
    if 'k_image_step_fused' in r['kernel']: print('   fused', r['calls'], 'calls avg', r['avg_us'], 'median', r['median_us'], 'min', r['min_us'])"
    python3 -c "import json;d=json.load(open('$O/b_${WL}_$V.json'));print('  ', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
unset APG_GLIMPSE_NO_WINDOW
