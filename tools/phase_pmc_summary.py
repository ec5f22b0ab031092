"""Summarise tools/gpu_phase_pmc.sh: per variant, median over the fused k_lidar_step dispatches."""
import collections
import csv
import glob
import os
import sys

import numpy as np

d = sys.argv[1]
for run in sorted(os.listdir(d)):
    p = os.path.join(d, run)
    if not os.path.isdir(p):
        continue
    if run.startswith("kt_"):
        f = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
        rows = [r for r in csv.DictReader(open(f[0])) if "k_lidar_step" in r["Kernel_Name"] and "true" in r["Kernel_Name"]]
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        print(f"{run:16s} dispatches {len(dur)} median {np.median(dur):.1f} us")
        continue
    f = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f[0])):
        if "true" not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    med = {c: float(np.median(list(v.values()))) for c, v in per.items()}
    s = " ".join(f"{c.replace('SQ_INSTS_', '').replace('SQ_', '')}={v / 1e6:.3f}M" for c, v in sorted(med.items()))
    print(f"{run:16s} {s}")
