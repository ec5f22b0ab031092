# rocprof kernel durations of the MNIST fused step with APG_IMAGE_GT=448 and 256 (110-step runs)
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
for gt in 448 256; do
  cd /tmp && export TMPDIR=/tmp
  rm -rf $O/trace_gt$gt
  APG_IMAGE_GT=$gt timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_gt$gt -o run -- \
    python3 $R/bench.py --workload ${WL:-mnist} --steps 110 --warmup 0 --no-cpu-baseline --no-episode > $O/trace_gt$gt.json 2> $O/trace_gt$gt.err || exit 1
  cd $R
  python3 tools/rocpd_stats.py $O/trace_gt$gt | grep k_image_step_fused | cut -c1-40,200-
done
