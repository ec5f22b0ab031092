#!/bin/bash
# Round-4 phase timeline of k_lidar_step (tools/step_phase_profile.py, -DAPG_STEP_PROFILE build in _lib/variants)
set -e
O=gpurun_out/r04
mkdir -p $O
export APG_LIBRARY=$PWD/active-perception-gym_amd/ap_gym_amd/_lib/variants/libprof.so
timeout -k 10 150 python tools/step_phase_profile.py > $O/phase_rooms64.log 2>&1
KIND=maze MAP=127 BEAMS=64 NENV=262144 WARM=10 timeout -k 10 240 python tools/step_phase_profile.py > $O/phase_maze127.log 2>&1
tail -n 14 $O/phase_rooms64.log $O/phase_maze127.log
