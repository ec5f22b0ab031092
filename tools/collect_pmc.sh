#!/bin/bash
# PMC passes over bench.py's step kernel(s) for one workload, each counter group in its own
# rocprofv3 run (no tracing domains), then tools/pmc_tables.py -> gpurun_out/pmc_<workload>.json
# (copy it to profiles/<round>/: bench.py reads traffic and issue counters from there when the
# kernel sources hash the same).  Run from the repo root on the GPU box:
#   bash tools/collect_pmc.sh <workload> [extra bench.py args]
set -e
WL=$1
shift
R=$PWD
O=$R/gpurun_out/pmc_$WL
rm -rf "$O"
mkdir -p "$O"
case $WL in
  lidar | maze127) REGEX="k_lidar_step|k_maze" ;;
  *) REGEX='k_glimpse|k_image_env|k_image_step|k_fill|k_unique|k_loc_target' ;;
esac
# 110 steps from reset(seed=0): step 101 is the synchronized autoreset step
ARGS=(--workload "$WL" --no-cpu-baseline --steps 110 --warmup 0 --no-episode "$@")
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1
  shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$REGEX" -d "$O/$name" -o run --output-format csv \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$O/$name.log" 2>&1
  echo "pass $name ok"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
pass wait SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
cd "$R"
python3 tools/pmc_tables.py "$O" "$WL" > "gpurun_out/pmc_$WL.json"
echo "wrote gpurun_out/pmc_$WL.json"
