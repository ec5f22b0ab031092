#!/bin/bash
# image GPU tests, then the mnist and tinyimagenet-loc benches (plain, then under a kernel trace)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_image.py tests/test_gpu_circle_square.py > gpurun_out/pt_img.log 2>&1 || { tail -30 gpurun_out/pt_img.log; exit 1; }
tail -1 gpurun_out/pt_img.log
R=$PWD
for w in mnist tinyimagenet-loc; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_$w.log').read().strip().splitlines()[-1]);print('$w', '%.3g env-steps/s' % d['value'], '%.1f us/step' % (d['ms_per_step']*1e3), 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'reset_ms %.0f' % d['config']['reset_ms'])"
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/pk_$w
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pk_$w -o pk -- python3 $R/bench.py --workload $w --no-cpu-baseline --steps 100 > $R/gpurun_out/pk_$w.log 2>&1
  cd $R
  python3 - $w <<'PY'
import csv, glob, sys
for r in list(csv.DictReader(open(glob.glob(f"gpurun_out/pk_{sys.argv[1]}/*kernel_stats.csv")[0])))[:4]:
    print("   ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
