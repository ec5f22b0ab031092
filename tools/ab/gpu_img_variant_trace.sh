# image GPU suite on the in-tree library, then rocprof k_image_step_fused durations (110-step runs) of the in-tree
# library and of each variant:  WL=mnist bash tools/ab/gpu_img_variant_trace.sh <variant.so>...
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_image.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/t_img_v.log 2>&1
rc=$?; tail -n 1 $O/t_img_v.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for V in default "$@"; do
    if [ "$V" = default ]; then unset APG_LIBRARY; else export APG_LIBRARY=$R/$V; fi
    cd /tmp && export TMPDIR=/tmp
    rm -rf $O/trace_v
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_v -o run -- \
      python3 $R/bench.py --workload ${WL:-mnist} --steps 110 --warmup 0 --no-cpu-baseline --no-episode > $O/trace_v.json 2> $O/trace_v.err || exit 1
    cd $R
    echo "$V $(python3 tools/rocpd_stats.py $O/trace_v | grep k_image_step_fused | awk -F, '{print $(NF-5), $(NF-2)}')"
  done
done
unset APG_LIBRARY
