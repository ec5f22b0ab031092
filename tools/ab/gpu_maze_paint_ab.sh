# maze parity subset on each variant, then rocprof k_maze_paint / k_pf_paint durations of maze127 runs (reset(seed)
# + 110 steps), interleaved:  bash tools/ab/gpu_maze_paint_ab.sh <variant.so>...
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
for V in "$@"; do
  APG_LIBRARY=$R/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_lidar.py -x -q -m gpu -k "maze" --timeout 300 --timeout-method thread > $O/t_mp.log 2>&1
  rc=$?; echo "$V $(tail -n 1 $O/t_mp.log)"; [ $rc -eq 0 ] || exit $rc
done
unset APG_LIBRARY
for round in 1 2; do
  for V in default "$@"; do
    if [ "$V" = default ]; then unset APG_LIBRARY; else export APG_LIBRARY=$R/$V; fi
    cd /tmp && export TMPDIR=/tmp
    rm -rf $O/trace_mp
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_mp -o run -- \
      python3 $R/bench.py --workload maze127 --steps 110 --warmup 0 --no-cpu-baseline --no-episode > $O/trace_mp.json 2> $O/trace_mp.err || exit 1
    cd $R
    echo "$V $(python3 tools/rocpd_stats.py $O/trace_mp | grep -E 'k_maze_paint|k_pf_paint' | awk -F, '{print $1, $(NF-5), $(NF-2)}' | sed 's/(anonymous namespace):://g' | cut -c1-200 | tr '\n' ' ')"
  done
done
unset APG_LIBRARY
