# final tree: full GPU suite + smoke, then the LIDAR and maze127 measurement sets (source hash changed)
set -o pipefail
bash tools/gpu_r04_final.sh tests || exit 1
bash tools/gpu_r04_final.sh lidar || exit 1
bash tools/gpu_r04_final.sh maze127 || exit 1
