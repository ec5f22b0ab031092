#!/bin/bash
# Round-5 image checks on the GPU box: the image parity suites, then for MNIST / TinyImageNetLoc the driver-shaped
# bench line (20 steps after 5 warm-up) and a 340-step kernel trace (durations per kernel, durations.py)
set -o pipefail
R=$PWD
O=$R/gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_image.py \
  tests/test_gpu_circle_square.py tests/test_gpu_light_dark.py > $O/t_image.log 2>&1
rc=$?; tail -n 3 $O/t_image.log; [ $rc -eq 0 ] || { tail -n 40 $O/t_image.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for WL in mnist tinyimagenet-loc; do
  timeout -k 10 300 python $R/bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${WL}_driver.json 2> $O/bench_${WL}_driver.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_${WL}_driver.json'));print('$WL driver', round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step')"
  rm -rf $O/kt_$WL
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/bench.py --workload $WL \
    --steps 340 --warmup 20 --no-cpu-baseline --no-episode > $O/bench_${WL}_340.json 2> $O/bench_${WL}_340.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_${WL}_340.json'));print('$WL 340', round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step')"
  f=$(find $O/kt_$WL -name "*kernel_trace.csv" | head -1)
  for k in k_image_step_fused k_fill_count k_fill_write k_fill_uniform k_fill_finish k_fill_uniform_finish; do
    echo "  $k $(python3 $R/tools/durations.py $f $k 2>&1)"
  done
done
