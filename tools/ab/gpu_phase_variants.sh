#!/bin/bash
# Phase timeline of every APG_STEP_PROFILE variant library in _lib/variants (tuning aid).
set -e
R=$PWD
V=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants
O=$R/gpurun_out/phase_variants
rm -rf $O; mkdir -p $O
for lib in $V/libprof*.so; do
  name=$(basename $lib .so)
  APG_LIBRARY=$lib timeout -k 10 120 python tools/step_phase_profile.py > $O/$name.log 2>&1
  echo "== $name"; grep -A6 "rep 2: kernel span" $O/$name.log
done
