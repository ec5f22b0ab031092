#!/bin/bash
# Round-5 gathered step on one GPU (a one-rank RCCL group: the all-gather is RCCL's local copy), without and with
# two overlapped sub-batches (bench.py --sub-batches), for LIDAR config 2 and TinyImageNetLoc (config 5 shape).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r05/gather
mkdir -p $O
for WL in lidar tinyimagenet-loc; do
  for S in 1 2; do
    timeout -k 10 300 python bench.py --workload $WL --gather --sub-batches $S --steps 200 --warmup 20 --no-cpu-baseline \
      --no-episode > $O/${WL}_sub$S.json 2> $O/${WL}_sub$S.err || { tail -n 30 $O/${WL}_sub$S.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${WL}_sub$S.json'));c=d['config'];print('$WL sub $S', round(d['ms_per_step']*1e3,2),'us/step gathered; gather span', c.get('gather_ms'))"
  done
  timeout -k 10 300 python bench.py --workload $WL --steps 200 --warmup 20 --no-cpu-baseline --no-episode \
    > $O/${WL}_nogather.json 2> $O/${WL}_nogather.err || exit 1
  python3 -c "import json;d=json.load(open('$O/${WL}_nogather.json'));print('$WL no gather', round(d['ms_per_step']*1e3,2),'us/step')"
done
