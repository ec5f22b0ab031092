#!/bin/bash
# Round-2 measurement set (run from the repo root on the GPU box; outputs under gpurun_out/r02/):
#   bash tools/collect_r02.sh lidar    PMC tables of the LIDAR step (tools/collect_pmc.sh) ->
#                                      profiles/r02/pmc_lidar.json (in the box's tree, so the benches below
#                                      pick up traffic and issue counters for this exact kernel source),
#                                      rocprofv3 --kernel-trace --stats of the driver-shaped bench, the
#                                      driver-shaped bench and the default bench (CPU baselines)
#   bash tools/collect_r02.sh others   the same PMC tables, kernel stats and bench lines for maze127,
#                                      mnist and tinyimagenet-loc
set -e
R=$PWD
O=$R/gpurun_out/r02
mkdir -p $O $R/profiles/r02
if [ "$1" = lidar ]; then WLS=lidar; else WLS="maze127 mnist tinyimagenet-loc"; fi
for WL in $WLS; do
  bash tools/collect_pmc.sh $WL
  cp gpurun_out/pmc_$WL.json profiles/r02/pmc_$WL.json
  cp gpurun_out/pmc_$WL.json $O/
  cd /tmp && export TMPDIR=/tmp
  rm -rf $O/stats_$WL
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$WL -o run --output-format csv -- \
    python3 $R/bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline > $O/stats_$WL.json 2> $O/stats_$WL.err
  cd $R
  timeout -k 10 300 python bench.py --workload $WL --steps 20 --warmup 5 > $O/bench_${WL}_driver_shape.json \
    2> $O/bench_${WL}_driver_shape.err
  tail -1 $O/bench_${WL}_driver_shape.json
done
if [ "$1" = lidar ]; then
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
  tail -1 $O/bench_default.json
fi
