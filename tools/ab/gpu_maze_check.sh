# maze parity tests + a kernel trace of the cfg-3 bench (per-kernel durations) + the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/mzc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lidar.py -x -q --timeout 240 --timeout-method thread -k "maze or Maze" > $O/pytest_maze.log 2>&1 || { echo "maze tests failed"; tail -30 $O/pytest_maze.log; exit 1; }
tail -1 $O/pytest_maze.log
for SET in default "$@"; do
echo "== $SET"
ENVS=""; [ "$SET" != default ] && ENVS=$(echo "$SET" | tr ',' ' ')
cd /tmp
rm -rf $O/tr
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 $R/bench.py --workload maze127 --steps 30 --warmup 2 --no-cpu-baseline > $O/tr.json 2> $O/tr.err || { echo "trace failed"; tail -5 $O/tr.err; exit 1; }
cd $R
python3 tools/rocpd_stats.py $O/tr > $O/stats.txt && rm -rf $O/tr
python3 - <<'PY'
import csv, re
for r in csv.DictReader(open("gpurun_out/mzc/stats.txt")):
    n = re.sub(r"\(.*", "", r["kernel"].replace("(anonymous namespace)::", "")).split("::")[-1][:40]
    if float(r["total_us"]) > 200 or 'maze' in n:
        print(f"{n:40s} calls {r['calls']:>4s} avg {r['avg_us']:>9s} med {r['median_us']:>9s} max {r['max_us']:>9s} tot {r['total_us']}")
PY
done
timeout -k 10 400 python bench.py --workload maze127 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/bench.json'))
e = d['episode']; print('value %.4g ms/step %.4f episode %.4g reset_step_kernel_ms %.2f reset_ms %.1f' % (d['value'], d['ms_per_step'], e['env_steps_per_s'], e['reset_step_kernel_ms'], d['config']['reset_ms']))"
