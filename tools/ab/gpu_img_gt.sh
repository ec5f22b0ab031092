# image GPU suite, then MNIST over 340 steps with APG_IMAGE_GT=448 (default) vs 256, interleaved
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_image.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/t_img_gt.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04/t_img_gt.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for gt in 448 256; do
    APG_IMAGE_GT=$gt timeout -k 10 300 python bench.py --workload ${WL:-mnist} --steps 340 --warmup 34 --no-cpu-baseline > gpurun_out/gt.json 2> gpurun_out/gt.err || { echo "gt $gt failed"; tail -5 gpurun_out/gt.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/gt.json').read().strip().splitlines()[-1]);r=d['roofline'];print('GT $gt', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step kernel(ev)', round(r.get('kernel_ms_events', r['kernel_ms'])*1e3,2))"
  done
done
