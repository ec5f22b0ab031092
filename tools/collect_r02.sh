#!/bin/bash
# Round-2 measurement set (run from the repo root on the GPU box; outputs under gpurun_out/r02/):
#   1. PMC tables of the LIDAR step (tools/collect_pmc.sh) -> profiles/r02/pmc_lidar.json (in the box's tree,
#      so the benches below pick up traffic and issue counters for this exact kernel source)
#   2. rocprofv3 --kernel-trace --stats of the driver-shaped bench (--steps 20 --warmup 5)
#   3. the driver-shaped bench and the default bench (505 steps, CPU baselines) as JSON lines
set -e
R=$PWD
O=$R/gpurun_out/r02
mkdir -p $O $R/profiles/r02
bash tools/collect_pmc.sh lidar
cp gpurun_out/pmc_lidar.json profiles/r02/pmc_lidar.json
cp gpurun_out/pmc_lidar.json $O/
cd /tmp && export TMPDIR=/tmp
rm -rf $O/stats_driver
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_driver -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/stats_driver.json 2> $O/stats_driver.err
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver_shape.json 2> $O/bench_driver_shape.err
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_driver_shape.json
