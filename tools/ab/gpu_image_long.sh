# image bench lines over whole episodes (340 steps = 20 MNIST / TinyImageNetLoc batch episodes after 34 warmup)
set -o pipefail
mkdir -p gpurun_out/r04
for wl in mnist tinyimagenet-loc; do
  timeout -k 10 300 python bench.py --workload $wl --steps 340 --warmup 34 --no-cpu-baseline > gpurun_out/r04/bench_${wl}_340.json 2> gpurun_out/r04/bench_${wl}_340.err || { echo "$wl failed"; tail -5 gpurun_out/r04/bench_${wl}_340.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r04/bench_${wl}_340.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$wl', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(r['kernel_ms']*1e3,2), r.get('kernel_ms_source'))"
done
