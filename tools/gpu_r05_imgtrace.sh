#!/bin/bash
# Round-5 image step: the image parity suite, then MNIST (config 4) in the driver's shape and over 340 steps under a
# kernel + HIP API trace (where the wall time between fused step kernels goes: host submission, markers, fills).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r05
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_image.py > $O/t_image_only.log 2>&1
rc=$?; tail -n 3 $O/t_image_only.log; [ $rc -eq 0 ] || { tail -n 40 $O/t_image_only.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp
WL=${WL:-mnist}
timeout -k 10 300 python $R/bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${WL}_driver.json 2> $O/bench_${WL}_driver.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_${WL}_driver.json'));print('$WL driver', round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step')"
rm -rf $O/ht_$WL
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/ht_$WL -o run -- python3 $R/bench.py --workload $WL \
  --steps 340 --warmup 20 --no-cpu-baseline --no-episode > $O/bench_${WL}_340h.json 2> $O/bench_${WL}_340h.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_${WL}_340h.json'));print('$WL 340 (traced)', round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step')"
f=$(find $O/ht_$WL -name "*kernel_trace.csv" | head -1)
for k in k_image_step_fused k_fill_count k_fill_write k_fill_uniform; do
  echo "  $k $(python3 $R/tools/durations.py $f $k 2>&1)"
done
