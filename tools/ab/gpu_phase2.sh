#!/bin/bash
# Phase timeline (APG_STEP_PROFILE variants) + SQ counters of the stop variants vs the full kernel.
set -e
R=$PWD
V=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants
O=$R/gpurun_out/phase2
rm -rf $O; mkdir -p $O
for lib in prof; do
  APG_LIBRARY=$V/lib$lib.so timeout -k 10 120 python tools/step_phase_profile.py > $O/$lib.log 2>&1
  echo "$lib ok"
done
cd /tmp && export TMPDIR=/tmp
for v in stop2 stop3 full; do
  if [ $v = full ]; then unset APG_LIBRARY; else export APG_LIBRARY=$V/lib$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex k_lidar_step -d $O/${v}_256 -o run --output-format csv -- python3 $R/tools/phase_pmc.py > $O/${v}_256.log 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${v}_256 -o run -- python3 $R/tools/phase_pmc.py > $O/kt_${v}_256.log 2>&1
  echo "$v ok"
done
cd $R
python3 tools/phase_pmc_summary.py $O
