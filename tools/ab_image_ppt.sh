#!/bin/bash
# A/B of the fused image step's glimpse units per workgroup (APG_GLIMPSE_PPT: pixels per glimpse thread, 8 by default
# for the env-wave instances; upb = min(64, ceil(ppt * 256 / (G0*G1)))) on a workload, interleaved rounds, rocprof
# kernel-trace medians of k_image_step_fused.   bash tools/ab_image_ppt.sh tinyimagenet-loc "8 16 12"
set -o pipefail
R=$PWD
WL=${1:-tinyimagenet-loc}
VALS=${2:-"8 16 12"}
O=$R/gpurun_out/r05/ab_ppt_$WL
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for p in $VALS; do
    rm -rf $O/kt_${p}_$round
    APG_GLIMPSE_PPT=$p timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${p}_$round -o run -- \
      python3 $R/bench.py --workload $WL --steps 150 --warmup 10 --no-cpu-baseline --no-episode \
      > $O/b_${p}_$round.json 2> $O/b_${p}_$round.err || { tail -n 20 $O/b_${p}_$round.err; exit 1; }
    f=$(find $O/kt_${p}_$round -name "*kernel_trace.csv" | head -1)
    echo "round $round ppt $p: $(python3 $R/tools/durations.py $f k_image_step_fused)"
  done
done
