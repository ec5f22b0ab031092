"""PMC CSVs of profiles/collect.sh -> HBM traffic per k_lidar_step launch (JSON on stdout).

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch.  Per MI355X_MICROARCH.md (HBM section),
gfx950's FETCH_SIZE tallies 128-B read requests at 64 B, so it is doubled; WRITE_SIZE is taken as is.
Both raw values are kept in the JSON.
"""

import csv
import glob
import json
import os
import sys


def per_launch(d, counter):
    vals = []
    for p in glob.glob(os.path.join(d, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == counter and "k_lidar_step" in r["Kernel_Name"]:
                vals.append((float(r["Counter_Value"]) * 1024.0, int(r["Grid_Size"])))
    if not vals:
        raise SystemExit(f"no {counter} rows under {d}")
    return sum(v for v, _ in vals) / len(vals), len(vals), vals[0][1]


def main():
    d = sys.argv[1]
    fetch, nf, grid = per_launch(d, "FETCH_SIZE")
    write, nw, _ = per_launch(d, "WRITE_SIZE")
    num_envs = grid // 4  # 256-thread workgroups of 64 envs
    print(json.dumps({
        "kernel": "k_lidar_step", "num_envs": num_envs, "beams": 32, "launches": [nf, nw],
        "fetch_bytes_raw": fetch, "write_bytes_raw": write,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "note": "FETCH_SIZE doubled per the gfx950 correction; averaged over all launches incl. post-reset ones",
    }))


if __name__ == "__main__":
    main()
