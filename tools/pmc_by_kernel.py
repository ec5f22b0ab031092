"""Per-kernel PMC averages of rocprofv3 --pmc CSV passes (tuning aid): counters summed over a dispatch's rows,
averaged over the dispatches of each kernel name.
    python tools/pmc_by_kernel.py <dir with pass subdirs> [name-filter]"""
import collections
import csv
import glob
import os
import sys

root, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    per = collections.defaultdict(float)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            key = (row["Dispatch_Id"], row["Counter_Name"])
            per[key] += float(row["Counter_Value"])
            names[row["Dispatch_Id"]] = row["Kernel_Name"]
    for (disp, cname), v in per.items():
        k = names[disp].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if filt in k:
            acc[k][cname].append(v)
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")
