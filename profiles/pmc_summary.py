"""Summarise profiles/pmc_sq.sh output: per-dispatch totals of each SQ counter of k_lidar_step
(median over dispatches) plus derived ratios.  python profiles/pmc_summary.py gpurun_out/pmc_<tag>"""

import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    med = {}
    for p in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(p)):
            if "k_lidar_step" in r["Kernel_Name"]:
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for name, by in per.items():
            v = sorted(by.values())
            med[name] = v[len(v) // 2]
    waves = med.get("SQ_WAVES", 1.0)
    out = {"kernel": "k_lidar_step", "median_per_dispatch": med,
           "valu_insts_per_wave": med.get("SQ_INSTS_VALU", 0) / waves,
           "salu_insts_per_wave": med.get("SQ_INSTS_SALU", 0) / waves,
           "valu_lane_utilisation": (med["SQ_THREAD_CYCLES_VALU"] / (64.0 * med["SQ_ACTIVE_INST_VALU"])
                                     if med.get("SQ_ACTIVE_INST_VALU") else None),
           "wait_any_over_wave_cycles": (med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"]
                                         if med.get("SQ_WAVE_CYCLES") else None)}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
