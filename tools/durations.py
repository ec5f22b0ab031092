"""Per-dispatch durations (us) of kernels matching argv[2] in a rocprofv3 kernel_trace.csv (argv[1])."""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
if not rows:
    sys.exit(f"no dispatches of {sys.argv[2]}")
d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows])
print(f"{len(d)} dispatches: mean {d.mean():.1f} median {np.median(d):.1f} min {d.min():.1f} max {d.max():.1f} us")
if "-v" in sys.argv:
    print(" ".join(f"{x:.0f}" for x in d))
