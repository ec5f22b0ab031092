#!/bin/bash
# round 3 (b): maze generator halves in isolation + PMC passes on them, FETCH/WRITE_SIZE calibration, full GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03b
mkdir -p $O
timeout -k 10 120 tools/maze_bench 262144 127 64 || exit 1
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
"$R/tools/fetch_calib" > $O/calib_known.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal_fetch -o run --output-format csv -- "$R/tools/fetch_calib" > $O/cal_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/cal_write -o run --output-format csv -- "$R/tools/fetch_calib" > $O/cal_write.log 2>&1 || exit 1
cd $R && python3 tools/fetch_calib.py $O/calib_known.json $O/cal_fetch $O/cal_write > $O/fetch_calibration.json && cat $O/fetch_calibration.json | head -60
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
