#!/bin/bash
# Phase split of k_lidar_step: PMC + kernel trace of the APG_STEP_STOP variants (tools/phase_pmc.py)
set -e
R=$PWD
O=$R/gpurun_out/phase_pmc
rm -rf $O; mkdir -p $O
V=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants
cd /tmp && export TMPDIR=/tmp
for epb in ${EPBS:-256 64}; do
  for v in stop1 stop2 stop3 stop4 full; do
    if [ $v = full ]; then unset APG_LIBRARY; else export APG_LIBRARY=$V/lib$v.so; fi
    export APG_STEP_EPB=$epb
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex k_lidar_step -d $O/${v}_$epb -o run --output-format csv -- python3 $R/tools/phase_pmc.py > $O/${v}_$epb.log 2>&1
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${v}_$epb -o run -- python3 $R/tools/phase_pmc.py > $O/kt_${v}_$epb.log 2>&1
    echo "$v $epb ok"
  done
done
unset APG_LIBRARY; export APG_STEP_EPB=256
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 --kernel-include-regex k_lidar_step -d $O/f64_256 -o run --output-format csv -- python3 $R/tools/phase_pmc.py > $O/f64_256.log 2>&1
cd $R
python3 tools/phase_pmc_summary.py $O
