# LIDAR parity tests + a kernel trace of the cfg-2 bench (per-kernel durations) + the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/lc
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lidar.py tests/test_gpu_sharding.py tests/test_gpu_render.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "lidar tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
rm -rf $O/tr
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 $R/bench.py --workload lidar --steps 200 --warmup 20 --no-cpu-baseline --no-episode > $O/tr.json 2> $O/tr.err || { echo "trace failed"; tail -5 $O/tr.err; exit 1; }
cd $R
python3 tools/rocpd_stats.py $O/tr > $O/stats.txt && rm -rf $O/tr
python3 - <<'PY'
import csv, re
for r in csv.DictReader(open("gpurun_out/lc/stats.txt")):
    n = re.sub(r"\(.*", "", r["kernel"].replace("(anonymous namespace)::", "")).split("::")[-1][:40]
    if int(r["calls"]) > 100:
        print(f"{n:40s} calls {r['calls']:>4s} avg {r['avg_us']:>9s} med {r['median_us']:>9s} min {r['min_us']:>9s}")
PY
timeout -k 10 400 python bench.py --workload lidar --steps 500 --warmup 50 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/bench.json'))
print('value %.4g ms/step %.4f kernel_ms %s' % (d['value'], d['ms_per_step'], d['roofline'].get('median_kernel_ms')))"
