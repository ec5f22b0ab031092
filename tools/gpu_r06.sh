#!/bin/bash
# Round-6 GPU steps (run from the repo root on the box; outputs under gpurun_out/r06):
#   bash tools/gpu_r06.sh tests [pytest -k expr]   GPU suite (optionally a subset)
#   bash tools/gpu_r06.sh smoke                    __graft_entry__.smoke()
#   bash tools/gpu_r06.sh ab <wl> <steps> <regex> <variants...>   tools/ab_trace.sh
#   bash tools/gpu_r06.sh fetch <wl> <tag> [ENV=VAL]              one FETCH_SIZE + WRITE_SIZE pass pair (per-kernel MB)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06
mkdir -p $O
case $1 in
  tests)
    K=${2:-}
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
      > $O/pytest_gpu${K:+_sub}.log 2>&1 || { echo "GPU tests failed"; tail -40 $O/pytest_gpu${K:+_sub}.log; exit 1; }
    tail -3 $O/pytest_gpu${K:+_sub}.log
    ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
      || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log
    ;;
  ab)
    shift
    timeout -k 10 1000 bash tools/ab_trace.sh "$@"
    ;;
  fetch)
    WL=$2; TAG=$3; [ -n "$4" ] && export "$4"
    case $WL in lidar | maze127) REGEX="k_lidar_step|k_maze" ;; *) REGEX='k_image_step|k_glimpse|k_unique' ;; esac
    R=$PWD
    cd /tmp
    rm -rf $O/pmc_$TAG && mkdir -p $O/pmc_$TAG
    for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"; do
      D=$O/pmc_$TAG/$(echo $C | cut -d' ' -f1)
      timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "$REGEX" -d $D -o run \
        --output-format csv -- python3 $R/bench.py --workload $WL --no-cpu-baseline --steps 60 --warmup 0 --no-episode \
        > $D.log 2>&1 || { echo "pmc $C failed"; tail -5 $D.log; exit 1; }
    done
    cd $R
    python3 tools/pmc_by_kernel.py $O/pmc_$TAG 2>&1 | tee $O/pmc_${TAG}.txt
    ;;
esac
