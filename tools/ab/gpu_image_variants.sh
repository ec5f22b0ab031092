#!/bin/bash
# image parity tests, then the image benches with and without the fused step (tuning)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_image.py tests/test_gpu_circle_square.py tests/test_gpu_sharding.py > gpurun_out/pt_img.log 2>&1 || { tail -30 gpurun_out/pt_img.log; exit 1; }
tail -1 gpurun_out/pt_img.log
run() {
  local tag=$1; shift
  for w in mnist tinyimagenet-loc; do
    env "$@" timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 200 > gpurun_out/bv_${tag}_$w.json 2> gpurun_out/bv.err
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/bv_${tag}_$w.json').read().strip().splitlines()[-1]);print('$tag $w', '%.1f us/step' % (d['ms_per_step']*1e3), 'kernel %.1f us' % (d['roofline']['kernel_ms']*1e3))"
  done
}
run fused A=1
run unfused APG_IMAGE_UNFUSED=1
