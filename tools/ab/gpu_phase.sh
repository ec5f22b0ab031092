set -e
export APG_LIBRARY=$PWD/active-perception-gym_amd/ap_gym_amd/_lib/variants/libprof.so
timeout -k 10 120 python tools/step_phase_profile.py > gpurun_out/phase256.log 2>&1; cat gpurun_out/phase256.log
APG_STEP_EPB=64 timeout -k 10 120 python tools/step_phase_profile.py > gpurun_out/phase64.log 2>&1; cat gpurun_out/phase64.log
