#!/bin/bash
# A/B of the image step between the in-tree library ("tree") and a variant build ("<name>": _lib/variants/lib<name>.so,
# loaded through APG_LIBRARY): the image parity suite on the tree, then interleaved rounds of rocprof kernel-trace
# medians of k_image_step_fused per workload.     bash tools/ab_image_lib.sh narrow "tinyimagenet-loc mnist"
set -o pipefail
R=$PWD
VAR=$1
WLS=${2:-"tinyimagenet-loc mnist"}
O=$R/gpurun_out/r05/ab_$VAR
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_image.py \
  > $O/t_image.log 2>&1 || { tail -n 40 $O/t_image.log; exit 1; }
tail -n 1 $O/t_image.log
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for WL in $WLS; do
    for arm in tree $VAR; do
      if [ $arm = tree ]; then unset APG_LIBRARY; else export APG_LIBRARY=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants/lib$arm.so; fi
      rm -rf $O/kt_${WL}_${arm}_$round
      timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${WL}_${arm}_$round -o run -- \
        python3 $R/bench.py --workload $WL --steps 150 --warmup 10 --no-cpu-baseline --no-episode \
        > $O/b_${WL}_${arm}_$round.json 2> $O/b_${WL}_${arm}_$round.err || { tail -n 20 $O/b_${WL}_${arm}_$round.err; exit 1; }
      f=$(find $O/kt_${WL}_${arm}_$round -name "*kernel_trace.csv" | head -1)
      echo "round $round $WL $arm: $(python3 $R/tools/durations.py $f k_image_step_fused)"
    done
  done
done
unset APG_LIBRARY
