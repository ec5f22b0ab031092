#!/bin/bash
# A/B of the working tree's kernels against a commit's (tuning aid): builds REV's (default HEAD) csrc into
# _lib/variants/prev.so:  bash tools/ab/ab_prev.sh [REV]
set -e
R=$(git rev-parse --show-toplevel)
T=$(mktemp -d)
mkdir -p $T/a/csrc $T/include
for f in $(git -C $R ls-tree -r --name-only ${1:-HEAD} active-perception-gym_amd/csrc); do git -C $R show ${1:-HEAD}:$f > $T/a/csrc/$(basename $f); done
cp $R/include/*.h $T/include/
V=$R/active-perception-gym_amd/ap_gym_amd/_lib/variants
mkdir -p $V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -fno-gpu-flush-denormals-to-zero -Wl,-soname,libapgym_hip.so -o $V/prev.so $T/a/csrc/apg_lidar.hip $T/a/csrc/apg_image.hip \
  $T/a/csrc/apg_circle_square.hip $T/a/csrc/apg_light_dark.hip 2>&1 | grep -v hip-link || true
rm -rf $T
# The soname matters: libapgym_torch.so (the reset/step torch ops) resolves libapgym_hip.so by soname, so a variant
# without it would leave the ops on the in-tree library while ctypes calls use the variant.
