# one-rank RCCL gathered vs ungathered step (bench.py --gather at N = 1) for LIDAR and TinyImageNetLoc, then a
# kernel trace of the gathered LIDAR run -> gpurun_out/r04/gather1_*.json, trace_gather_lidar/
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
for WL in lidar tinyimagenet-loc; do
  timeout -k 10 200 python3 bench.py --workload $WL --steps 300 --warmup 20 --no-cpu-baseline --no-episode \
    > $O/gather1_${WL}_plain.json 2> $O/gather1_${WL}_plain.err || exit 1
  timeout -k 10 200 python3 bench.py --workload $WL --steps 300 --warmup 20 --no-cpu-baseline --no-episode --gather \
    > $O/gather1_${WL}.json 2> $O/gather1_${WL}.err || exit 1
done
[ -n "$TRACE" ] || exit 0
cd /tmp && export TMPDIR=/tmp
for WL in lidar tinyimagenet-loc; do
  rm -rf $O/trace_gather_$WL
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace_gather_$WL -o run -- \
    python3 $R/bench.py --workload $WL --steps 100 --warmup 10 --no-cpu-baseline --no-episode --gather \
    > $O/trace_gather_$WL.json 2> $O/trace_gather_$WL.err || exit 1
done
