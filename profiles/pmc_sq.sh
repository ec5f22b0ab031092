#!/bin/bash
# SQ instruction-mix / stall counters of k_lidar_step (one rocprofv3 --pmc pass per counter group,
# kernel-filtered, no tracing domains).  Run from the repo root on the GPU box:
#   bash profiles/pmc_sq.sh <tag>     -> gpurun_out/pmc_<tag>/{list.txt, <group>/...csv}
set -e
TAG=${1:-sq}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/list.txt 2>&1 || true
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex k_lidar_step -d $O/$name -o run --output-format csv -- \
    python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/$name.log 2>&1
}
run mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run stall SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run f32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT
run f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64
