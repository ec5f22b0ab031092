#!/bin/bash
# maze_bench timing + PMC passes on its kernels (k_stream, k_dfs, k_paint): bash tools/ab/gpu_maze_pmc.sh <outdir>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 120 tools/maze_bench 262144 127 64 | tee $O/maze_bench.json || exit 1
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$name" -o run --output-format csv -- "$R/tools/maze_bench" 262144 127 64 \
    > "$O/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$O/$name.log"; exit 1; }
  echo "pass $name ok"
}
pass mz_mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
pass mz_wait SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM
pass mz_fetch FETCH_SIZE
pass mz_write WRITE_SIZE
