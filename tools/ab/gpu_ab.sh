#!/bin/bash
# A/B of library variants on one workload, interleaved: bash tools/ab/gpu_ab.sh <workload> <steps> <variant.so>...
# ("default" = the in-tree library).  Prints value and ms_per_step of each run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
WL=$1; STEPS=$2; shift 2
for round in 1 2; do
  for V in "$@"; do
    if [ "$V" = default ]; then unset APG_LIBRARY; else export APG_LIBRARY=$PWD/$V; fi
    if [ $round = 1 ]; then  # the libraries the process maps (the torch ops must use the variant too)
      python3 -c "import sys; sys.path.insert(0, 'active-perception-gym_amd'); import ap_gym_amd._native as N; N.torch_ops(); print('$V maps', sorted({l.split()[-1].split('/')[-1] for l in open('/proc/self/maps') if 'apgym' in l or 'variants' in l}))"
    fi
    timeout -k 10 300 python bench.py --workload $WL --steps $STEPS --warmup 20 --no-cpu-baseline --no-episode \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "ab $V failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$V', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step kernel(ev)', round(r.get('median_kernel_ms', r.get('kernel_ms_events', 0))*1e3,2))"
  done
done
unset APG_LIBRARY
