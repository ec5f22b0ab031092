# LIDAR GPU suite, one-rank RCCL gather lines, maze127 episode bench -> gpurun_out/r04/
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_lidar.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r04/t_lidar.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04/t_lidar.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/gpu_gather1.sh || exit 1
timeout -k 10 300 python -u bench.py --workload maze127 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/r04/ep_maze127.json 2> gpurun_out/r04/ep_maze127.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r04/ep_maze127.json')); print('maze127', d['value'], d['episode'])"
