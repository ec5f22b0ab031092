# rocprofv3 kernel trace of a 110-step bench run per workload -> gpurun_out/r04/trace_<wl>/ + stats print
#   bash tools/ab/gpu_trace.sh <wl> [<wl> ...]
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04
mkdir -p $O
for WL in "$@"; do
  cd /tmp && export TMPDIR=/tmp
  rm -rf $O/trace_$WL
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$WL -o run -- \
    python3 $R/bench.py --workload $WL --steps 110 --warmup 0 --no-cpu-baseline --no-episode $TRACE_ARGS \
    > $O/trace_$WL.json 2> $O/trace_$WL.err || exit 1
  cd $R
  python3 tools/rocpd_stats.py $O/trace_$WL | python3 -c "
import sys,csv
r=csv.reader(sys.stdin); next(r)
for row in r:
    name=row[0].replace('(anonymous namespace)::','').split('(')[0][:44]
    if 'at::native' in row[0]: continue
    print(f'{name:46s}', ' '.join(f'{x:>10s}' for x in row[1:]))
"
done
