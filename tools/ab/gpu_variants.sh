#!/bin/bash
# kernel-trace median of k_lidar_step for each variant library in _lib/variants (tools/phase_pmc.py workload)
set -e
R=$PWD
O=$R/gpurun_out/variants
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in default $(ls $R/active-perception-gym_amd/ap_gym_amd/_lib/variants/*.so); do
  if [ $lib = default ]; then unset APG_LIBRARY; name=default; else export APG_LIBRARY=$lib; name=$(basename $lib .so); fi
  STEPS=80 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o run -- python3 $R/tools/phase_pmc.py > $O/$name.log 2>&1
  python3 - $O/$name <<'PY'
import csv, glob, sys, numpy as np
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_lidar_step" in r["Kernel_Name"] and "true" in r["Kernel_Name"]]
print(f"{sys.argv[1].split('/')[-1]:24s} n={len(d)} median {np.median(d):.1f} max {max(d):.1f} us")
PY
done
