#!/bin/bash
# Measurement set of round RND for one workload (run from the repo root on the GPU box; outputs under gpurun_out/$RND/
# and profiles/$RND/ of the box's tree, so the bench run at the end already reads them):
#   PMC tables (tools/collect_pmc.sh)                      -> profiles/$RND/pmc_<wl>.json
#   rocprofv3 --kernel-trace of a 110-step run from reset -> profiles/$RND/durations_<wl>.json (per-class kernel
#                                                             durations, source-hash keyed) + kernel_stats_<wl>.csv
#   the driver-shaped bench line (CPU baseline included)   -> gpurun_out/$RND/bench_<wl>.json
#   bash tools/collect_round.sh <round, e.g. r04> <workload> [extra bench args for the final bench line]
set -e
RND=$1
WL=$2
shift 2
R=$PWD
O=$R/gpurun_out/$RND
mkdir -p $O $R/profiles/$RND
timeout -k 10 900 bash tools/collect_pmc.sh $WL
cp gpurun_out/pmc_$WL.json profiles/$RND/pmc_$WL.json
cd /tmp && export TMPDIR=/tmp
rm -rf $O/trace_$WL
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$WL -o run -- \
  python3 $R/bench.py --workload $WL --steps 110 --warmup 0 --no-cpu-baseline --no-episode \
  > $O/trace_$WL.json 2> $O/trace_$WL.err
cd $R
python3 tools/durations_table.py $O/trace_$WL $WL $O/trace_$WL.json > profiles/$RND/durations_$WL.json
python3 tools/rocpd_stats.py $O/trace_$WL --csv profiles/$RND/kernel_stats_$WL.csv > /dev/null
timeout -k 10 400 python3 bench.py --workload $WL --steps 20 --warmup 5 "$@" > $O/bench_$WL.json 2> $O/bench_$WL.err
cp $O/bench_$WL.json profiles/$RND/bench_${WL}_driver_shape.json
# profiles/ of the box's tree does not travel back: copies under gpurun_out/$RND/profiles
mkdir -p $O/profiles && cp profiles/$RND/*_$WL* $O/profiles/
tail -1 $O/bench_$WL.json | cut -c1-400
