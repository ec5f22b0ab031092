#!/bin/bash
# Round-5 GPU runs (from the repo root on the GPU box; outputs under gpurun_out/r05/):
#   bash tools/gpu_r05.sh tests                 the whole GPU suite + smoke
#   bash tools/gpu_r05.sh t <name> <pytest args> a pytest selection -> gpurun_out/r05/t_<name>.log
#   bash tools/gpu_r05.sh bench <wl> [..]       a driver-shaped bench line (+ extra bench args) of one workload
#   bash tools/gpu_r05.sh episode <wl> [..]     a 300-step bench with episodes (no CPU baseline)
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
case "$1" in
  tests)
    timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
    rc=$?; tail -n 5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; cat $O/smoke.log; exit $rc ;;
  t)
    N=$2; shift 2
    timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread "$@" > $O/t_$N.log 2>&1
    rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_$N.log | tail -n 40; [ $rc -eq 0 ] || tail -n 60 $O/t_$N.log; exit $rc ;;
  bench)
    WL=$2; shift 2
    timeout -k 10 600 python bench.py --workload $WL --steps 20 --warmup 5 "$@" > $O/bench_$WL.json 2> $O/bench_$WL.err
    rc=$?; tail -c 1500 $O/bench_$WL.json; [ $rc -eq 0 ] || tail -n 20 $O/bench_$WL.err; exit $rc ;;
  episode)
    WL=$2; shift 2
    timeout -k 10 600 python bench.py --workload $WL --steps 300 --warmup 20 --no-cpu-baseline "$@" > $O/ep_$WL.json 2> $O/ep_$WL.err
    rc=$?; tail -c 1500 $O/ep_$WL.json; [ $rc -eq 0 ] || tail -n 20 $O/ep_$WL.err; exit $rc ;;
esac
