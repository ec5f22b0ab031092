#!/bin/bash
# Round-5 final measurement set, in parts (each well inside one gpurun call):
#   bash tools/gpu_r05_final.sh tests     full GPU suite + smoke
#   bash tools/gpu_r05_final.sh lidar     collect_r05 lidar + the --gather (gloo, 2 ranks on 1 GPU) and numpy lines
#   bash tools/gpu_r05_final.sh <wl>      collect_r05 <wl> (maze127, mnist, tinyimagenet-loc)
# Outputs under gpurun_out/r05 (collect_r05 copies its profiles/r05 files to gpurun_out/r05/profiles).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05
mkdir -p $O
case $1 in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
      || { echo "GPU tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
    tail -1 $O/pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
      || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log
    ;;
  lidar)
    timeout -k 10 1000 bash tools/collect_round.sh r05 lidar || { echo "collect lidar failed"; exit 1; }
    timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --gather --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_lidar_gather_gloo2.json 2> $O/bench_lidar_gather_gloo2.err || { echo "gather line failed"; tail -5 $O/bench_lidar_gather_gloo2.err; exit 1; }
    tail -1 $O/bench_lidar_gather_gloo2.json | cut -c1-300
    timeout -k 10 300 python bench.py --array-backend numpy --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_lidar_numpy.json 2> $O/bench_lidar_numpy.err || { echo "numpy line failed"; tail -5 $O/bench_lidar_numpy.err; exit 1; }
    tail -1 $O/bench_lidar_numpy.json | cut -c1-300
    timeout -k 10 300 python bench.py --gather --steps 300 --warmup 20 --no-cpu-baseline --no-episode \
      > $O/bench_lidar_gather_rccl1.json 2> $O/bench_lidar_gather_rccl1.err || { echo "rccl gather line failed"; exit 1; }
    ;;
  *)
    timeout -k 10 1000 bash tools/collect_round.sh r05 $1 || { echo "collect $1 failed"; exit 1; }
    if [ "$1" = tinyimagenet-loc ]; then
      timeout -k 10 300 python bench.py --workload $1 --gather --steps 300 --warmup 20 --no-cpu-baseline \
        > $O/bench_${1}_gather_rccl1.json 2> $O/bench_${1}_gather_rccl1.err || { echo "rccl gather line failed"; exit 1; }
    fi
    ;;
esac
