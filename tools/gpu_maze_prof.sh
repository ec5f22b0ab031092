#!/bin/bash
# rocprofv3 kernel trace + stats of a maze127 episode (bench.py --workload maze127, 101 steps + reset) -> gpurun_out/r04/
set -o pipefail
O=$PWD/gpurun_out/r04
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof_maze
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_maze -o run -- python3 $R/bench.py --workload maze127 --steps 101 --warmup 0 --no-cpu-baseline --no-episode > $O/prof_maze.json 2> $O/prof_maze.err
rc=$?
cd $R
f=$(find $O/prof_maze -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp $f $O/kernel_stats_maze127.csv && cut -d, -f1-8 $O/kernel_stats_maze127.csv | head -20
exit $rc
