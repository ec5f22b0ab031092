"""Per-dispatch counter sums of rocprofv3 --pmc CSV directories (one line per kernel dispatch):
python3 tools/pmc_summary.py <dir>..."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(f[0])):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0][:28])
        agg.setdefault(k, collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
    print("==", d)
    for (i, n), c in agg.items():
        print(i, n, " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
