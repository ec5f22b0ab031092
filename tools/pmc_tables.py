"""PMC CSVs of tools/collect_pmc.sh -> per-launch counter table (JSON on stdout) for bench.py.

    python tools/pmc_tables.py gpurun_out/pmc_<workload> <workload>

LIDAR workloads: every k_lidar_step dispatch is classified by the bench's step order (the first is
reset(seed)'s observation pass; dispatch k is env step t = k, and t % 101 == 0 is the synchronized
autoreset step), and each counter is averaged per class: "step" (ordinary steps), "reset_step" and
"reset_pass"; mazes also launch k_maze before every step (classes "maze_reset" for reset(seed), then
"maze_step" / "maze_reset_step": a no-op wave exit, or every env's maze).  Image workloads: per kernel name, and
"step" = the ordinary step's k_image_step_fused launch (else the sum over the kernels launched on
every step).

FETCH_SIZE / WRITE_SIZE are KiB per dispatch; hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE in
bytes (MI355X_MICROARCH.md, HBM: gfx950's FETCH_SIZE tallies 128-B read requests at 64 B).  The table
carries the kernel-source hash and run shape bench.py checks before using it.
"""

from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (kernel_source_sha, EPISODE_PERIOD)

PASSES = ("fetch", "write", "mix", "wait")


def read_pass(d: str, name: str):
    """{dispatch_id: (kernel_name, {counter: value summed over the CSV's dimension rows})}"""
    out: dict[int, tuple[str, dict]] = {}
    for p in glob.glob(os.path.join(d, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            did = int(r["Dispatch_Id"])
            kname, vals = out.setdefault(did, (r["Kernel_Name"], collections.defaultdict(float)))
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def bench_line(d: str) -> dict:
    for name in PASSES:
        p = os.path.join(d, f"{name}.log")
        if os.path.exists(p):
            for line in reversed(open(p).read().strip().splitlines()):
                if line.startswith("{"):
                    return json.loads(line)
    raise SystemExit(f"no bench JSON line under {d}")


def lidar_family(kname: str):
    """(kernel family, class prefix) of a LIDAR-workload dispatch: the step kernel, or one of the three maze
    reset kernels (each launched once per step, exiting at once on steps without autoresets)."""
    for fam, prefix in (("k_maze_stream", "maze_stream_"), ("k_maze_paint", "maze_paint_")):
        if fam in kname:
            return fam, prefix
    if re.search(r"k_maze<", kname):
        return "k_maze", "maze_"
    return "k_lidar_step", ""


def lidar_class(ordinal: int, prefix: str = "") -> str:
    if ordinal == 0:
        return prefix + "reset_pass" if not prefix else prefix + "reset"
    return prefix + ("reset_step" if ordinal % bench.EPISODE_PERIOD == 0 else "step")


def main():
    d, wl = sys.argv[1], sys.argv[2]
    b = bench_line(d)
    cfg = b["config"]
    acc: dict[str, dict[str, list[float]]] = collections.defaultdict(lambda: collections.defaultdict(list))
    for name in PASSES:
        rows = read_pass(d, name)
        ordinal = collections.Counter()
        for did in sorted(rows):
            kname, vals = rows[did]
            if wl in bench.LIDAR_WORKLOADS:
                fam, prefix = lidar_family(kname)
                cls = lidar_class(ordinal[fam], prefix)
                ordinal[fam] += 1
            else:
                cls = kname.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
            for c, v in vals.items():
                acc[cls][c].append(v)
    per = {cls: {c: sum(v) / len(v) for c, v in cs.items()} for cls, cs in acc.items()}
    counts = {cls: max(len(v) for v in cs.values()) for cls, cs in acc.items()}

    def hbm(p):
        if "FETCH_SIZE" not in p or "WRITE_SIZE" not in p:
            return None
        return 1024.0 * (2.0 * p["FETCH_SIZE"] + p["WRITE_SIZE"])

    if wl in bench.LIDAR_WORKLOADS:
        family = "lidar"
        shape = {"num_envs": cfg["num_envs_per_gpu"], "beams": cfg["beams"], "map": int(cfg["map"].split("x")[0])}
        hbm_b = {cls: hbm(p) for cls, p in per.items()}
    else:
        family = "image"
        shape = {"num_envs": cfg["num_envs_per_gpu"], "sensor": cfg["sensor"], "classes": cfg["classes"],
                 "log_stats": cfg.get("log_stats", False)}
        steps = b["steps"]
        fused = [cls for cls in counts if cls.startswith("k_image_step_fused")]
        # an ordinary step is one k_image_step_fused launch; otherwise the kernels launched on every step
        every = fused if fused else [cls for cls, n in counts.items() if n >= steps]
        step = collections.defaultdict(float)
        for cls in every:
            for c, v in per[cls].items():
                step[c] += v
        per["step"] = dict(step)
        counts["step"] = counts[fused[0]] if fused else steps
        hbm_b = {cls: hbm(p) for cls, p in per.items()}
    print(json.dumps({"workload": wl, "kernel_family": family, "source_sha": bench.kernel_source_sha(family),
                      "shape": shape, "launches": counts, "per_launch": per, "hbm_bytes_per_launch": hbm_b,
                      "bench_cmd_shape": {"steps": b["steps"], "warmup": b["warmup"]},
                      "note": "counters summed over the CSV's rows per dispatch, averaged per class; "
                              "hbm bytes = 1024 * (2 * FETCH_SIZE + WRITE_SIZE)"}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
