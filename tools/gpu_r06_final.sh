#!/bin/bash
# Round-6 final measurement set, in parts (each inside one gpurun call; outputs under gpurun_out/r06):
#   bash tools/gpu_r06_final.sh lidar     collect_round r06 lidar + numpy lines (copy / shared) + gathered lines
#   bash tools/gpu_r06_final.sh <wl>      collect_round r06 <wl> (maze127, mnist, tinyimagenet-loc)
#   bash tools/gpu_r06_final.sh default   the default `python bench.py` line (505 steps incl. 5 autoresets)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06
mkdir -p $O
case $1 in
  lidar)
    timeout -k 10 1000 bash tools/collect_round.sh r06 lidar || { echo "collect lidar failed"; exit 1; }
    timeout -k 10 300 python bench.py --array-backend numpy --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_lidar_numpy.json 2> $O/bench_lidar_numpy.err || { echo "numpy line failed"; tail -5 $O/bench_lidar_numpy.err; exit 1; }
    tail -1 $O/bench_lidar_numpy.json | cut -c1-300
    timeout -k 10 300 python bench.py --array-backend numpy --obs-snapshot shared --steps 20 --warmup 5 \
      --no-cpu-baseline > $O/bench_lidar_numpy_shared.json 2> $O/bench_lidar_numpy_shared.err \
      || { echo "numpy shared line failed"; tail -5 $O/bench_lidar_numpy_shared.err; exit 1; }
    tail -1 $O/bench_lidar_numpy_shared.json | cut -c1-300
    timeout -k 10 300 python bench.py --gather --steps 300 --warmup 20 --no-cpu-baseline --no-episode \
      > $O/bench_lidar_gather_rccl1.json 2> $O/bench_lidar_gather_rccl1.err || { echo "rccl gather line failed"; exit 1; }
    timeout -k 10 300 python bench.py --gather --gather-lag 1 --steps 300 --warmup 20 --no-cpu-baseline --no-episode \
      > $O/bench_lidar_gather_lag_rccl1.json 2> $O/bench_lidar_gather_lag_rccl1.err || { echo "lag gather line failed"; exit 1; }
    for f in gather_rccl1 gather_lag_rccl1; do tail -1 $O/bench_lidar_$f.json | cut -c1-200; done
    ;;
  default)
    timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; exit 1; }
    tail -1 $O/bench_default.json | cut -c1-400
    ;;
  *)
    timeout -k 10 1000 bash tools/collect_round.sh r06 $1 || { echo "collect $1 failed"; exit 1; }
    ;;
esac
