set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/img_knobs
timeout -k 10 300 env APG_GLIMPSE_PIPE=1 python -u -m pytest tests/test_gpu_image.py -x -q --timeout 120 --timeout-method thread > gpurun_out/img_knobs/pytest_image.log 2>&1 || { echo "image tests failed"; tail -30 gpurun_out/img_knobs/pytest_image.log; exit 1; }
tail -1 gpurun_out/img_knobs/pytest_image.log
bash tools/ab/gpu_img_knobs.sh "mnist tinyimagenet-loc" APG_GLIMPSE_PPT=8 APG_GLIMPSE_PPT=8,APG_GLIMPSE_PIPE=1 APG_IMAGE_ENV_WAVE=0 APG_IMAGE_ENV_WAVE=0,APG_GLIMPSE_PIPE=1 APG_IMAGE_ENV_WAVE=0,APG_GLIMPSE_PIPE=1,APG_GLIMPSE_PPT=6
