# rocprof k_image_step_fused durations (110-step runs) under environment settings, interleaved:
#   WL=tinyimagenet-loc bash tools/ab/gpu_img_env_trace.sh "" "APG_IMAGE_ENV_WAVE=1" ...
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
for round in 1 2; do
  for E in "$@"; do
    cd /tmp && export TMPDIR=/tmp
    rm -rf $O/trace_e
    env $E timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_e -o run -- \
      python3 $R/bench.py --workload ${WL:-mnist} --steps 110 --warmup 0 --no-cpu-baseline --no-episode > $O/trace_e.json 2> $O/trace_e.err || exit 1
    cd $R
    echo "[$E] $(python3 tools/rocpd_stats.py $O/trace_e | grep k_image_step_fused | awk -F, '{print $(NF-5), $(NF-2)}')"
  done
done
