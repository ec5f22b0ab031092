#!/bin/bash
# Round-5 phase split of k_lidar_step at cfg 2 (rooms 64x64, 32 beams, 65536 envs), on the GPU box:
#   1. per-workgroup phase timeline (s_memrealtime marks; -DAPG_STEP_PROFILE build, tools/step_phase_profile.py)
#   2. SQ counters + kernel trace of the APG_STEP_STOP=k builds (the kernel returns after phase k) and the full one
# Variants in _lib/variants: libprof.so, libstop{1..4}.so (build.py -D... --only=apg_lidar.hip --out=...).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r05/phase
mkdir -p $O
V=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants
APG_LIBRARY=$V/libprof.so timeout -k 10 150 python tools/step_phase_profile.py > $O/timeline_rooms64.log 2>&1 || exit $?
tail -n 14 $O/timeline_rooms64.log
cd /tmp && export TMPDIR=/tmp
export APG_STEP_EPB=256
for v in stop1 stop2 stop3 stop4 full; do
  if [ $v = full ]; then unset APG_LIBRARY; else export APG_LIBRARY=$V/lib$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT --kernel-include-regex k_lidar_step -d $O/${v} -o run --output-format csv -- python3 $R/tools/phase_pmc.py > $O/${v}.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${v} -o run -- python3 $R/tools/phase_pmc.py > $O/kt_${v}.log 2>&1 || exit $?
  echo "$v ok"
done
unset APG_LIBRARY
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 --kernel-include-regex k_lidar_step -d $O/f64 -o run --output-format csv -- python3 $R/tools/phase_pmc.py > $O/f64.log 2>&1 || exit $?
cd $R
python3 tools/phase_pmc_summary.py $O | tee $O/summary.txt
