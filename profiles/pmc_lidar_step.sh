#!/bin/bash
# PMC passes for k_lidar_step (run on the GPU box from the repo root; one rocprofv3 pass per counter
# group, --pmc never combined with tracing domains).  Output: gpurun_out/pmc_<pass>/
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
run() { timeout -k 10 240 rocprofv3 --pmc $2 --kernel-include-regex k_lidar_step -d $R/gpurun_out/pmc_$1 -o run --output-format csv -- $B > $R/gpurun_out/pmc_$1.log 2>&1; }
run A "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES"
run B "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_WAIT_INST_ANY SQ_WAIT_ANY"
run C "FETCH_SIZE"
run D "WRITE_SIZE"
run E "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS"
