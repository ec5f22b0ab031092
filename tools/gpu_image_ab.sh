#!/bin/bash
# Image step A/B (tuning aid): bench kernel time of every library in _lib/variants (loaded through
# APG_LIBRARY; the torch ops follow it by SONAME) and of the default one with glimpse knob settings.
set -e
shopt -s nullglob
R=$PWD
V=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants
O=$R/gpurun_out/image_ab
rm -rf $O; mkdir -p $O
one() {
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 200 > $O/${tag}_$w.json 2> $O/${tag}_$w.err
  python3 -c "import json;d=json.loads(open('$O/${tag}_$w.json').read().strip().splitlines()[-1]);print('%-22s %-18s %6.1f us/step  kernel %6.1f us  median %6.1f us' % ('$tag', '$w', d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, (d['roofline'].get('median_kernel_ms') or 0)*1e3))"
}
# two interleaved rounds: box-to-box and run-order drift shows up as round-to-round differences
for round in 1 2; do
  for w in mnist tinyimagenet-loc; do
    one default $w A=1
    for p in ${PPTS:-}; do one ppt$p $w APG_GLIMPSE_PPT=$p; done
    for lib in $V/*.so; do one $(basename $lib .so) $w APG_LIBRARY=$lib; done
  done
done
