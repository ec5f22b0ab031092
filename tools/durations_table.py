"""rocprofv3 kernel trace (rocpd SQLite) of a bench.py run -> per-class kernel durations (JSON on stdout), keyed
like the PMC tables by the kernel-source hash and the run shape, for bench.py's roofline.kernel_ms.

    python tools/durations_table.py <trace dir or .db> <workload> <bench JSON line file>

Classes as in tools/pmc_tables.py (LIDAR: reset_pass / step / reset_step of k_lidar_step, maze_* of k_maze;
image: the kernel name, and "step" = the ordinary step's k_image_step_fused).
"""
import collections
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import rocpd_stats  # noqa: E402
from pmc_tables import lidar_class, lidar_family  # noqa: E402


def main():
    src, wl, line_file = sys.argv[1], sys.argv[2], sys.argv[3]
    db = src if src.endswith(".db") else glob.glob(src + "/**/*.db", recursive=True)[0]
    b = [json.loads(x) for x in open(line_file).read().splitlines() if x.startswith("{")][-1]
    cfg = b["config"]
    acc = {}
    ordinal = collections.Counter()
    for name, s, e, g, w in rocpd_stats.load(db):
        us = (e - s) / 1e3
        if wl in bench.LIDAR_WORKLOADS:
            if "k_lidar_step" in name or "k_maze" in name:
                fam, prefix = lidar_family(name)
                cls = lidar_class(ordinal[fam], prefix)
                ordinal[fam] += 1
            else:
                continue
        else:
            if not re.search(r"k_(glimpse|image|fill|unique|loc_target)", name):
                continue
            cls = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
        acc.setdefault(cls, []).append(us)
    if wl not in bench.LIDAR_WORKLOADS:
        fused = [c for c in acc if c.startswith("k_image_step_fused")]
        if fused:
            acc["step"] = acc[fused[0]]
    per = {c: {"calls": len(v), "avg_us": sum(v) / len(v), "median_us": statistics.median(v), "min_us": min(v),
               "max_us": max(v)} for c, v in acc.items()}
    if wl in bench.LIDAR_WORKLOADS:
        family = "lidar"
        shape = {"num_envs": cfg["num_envs_per_gpu"], "beams": cfg["beams"], "map": int(cfg["map"].split("x")[0])}
    else:
        family = "image"
        shape = {"num_envs": cfg["num_envs_per_gpu"], "sensor": cfg["sensor"], "classes": cfg["classes"],
                 "log_stats": cfg.get("log_stats", False)}
    print(json.dumps({"workload": wl, "kernel_family": family, "source_sha": bench.kernel_source_sha(family),
                      "shape": shape, "per_class": per, "bench_cmd_shape": {"steps": b["steps"], "warmup": b["warmup"]},
                      "note": "rocprofv3 --kernel-trace dispatch durations (end - start) per class"}, indent=1,
                     sort_keys=True))


if __name__ == "__main__":
    main()
