#!/bin/bash
# k_lidar_step kernel-trace medians for each workgroup size (APG_STEP_EPB), two interleaved rounds
set -e
R=$PWD
O=$R/gpurun_out/epb_ab
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for epb in ${EPBS:-256 128 64}; do
    export APG_STEP_EPB=$epb
    STEPS=80 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/${epb}_$round -o run -- python3 $R/tools/phase_pmc.py > $O/${epb}_$round.log 2>&1
    python3 - $O/${epb}_$round <<'PY'
import csv, glob, sys, numpy as np
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_lidar_step" in r["Kernel_Name"] and "true" in r["Kernel_Name"]]
print(f"EPB {sys.argv[1].split('/')[-1]:8s} n={len(d)} median {np.median(d):.1f} min {min(d):.1f} max {max(d):.1f} us")
PY
  done
done
