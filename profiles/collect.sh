#!/bin/bash
# Round profile collection on the GPU box (run from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the default bench (per-kernel average durations)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over k_lidar_step, each its own run, no tracing domains
#   3. profiles/traffic.py turns the PMC CSVs into profiles/traffic_lidar_step.json
# Outputs land in gpurun_out/prof_<round>/; copy the summaries into profiles/<round>/.
set -e
RND=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$RND
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
  python $R/bench.py --no-cpu-baseline > $O/bench_stats.json 2> $O/bench_stats.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex k_lidar_step -d $O/pmc_$c -o run --output-format csv -- \
    python $R/bench.py --no-cpu-baseline > $O/pmc_$c.log 2>&1
done
python $R/profiles/traffic.py $O > $O/traffic_lidar_step.json
# image workloads (BASELINE configs 4, 5): kernel stats of the benches
for w in mnist tinyimagenet-loc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$w -o run --output-format csv -- \
    python $R/bench.py --workload $w --no-cpu-baseline > $O/bench_stats_$w.json 2> $O/bench_stats_$w.err
done
