"""Per-kernel duration stats (and optionally the dispatch sequence) from a rocprofv3 rocpd SQLite database.

    python tools/rocpd_stats.py <run_results.db> [--seq KERNEL_SUBSTR] [--csv out.csv]
"""
import argparse
import glob
import sqlite3
import statistics


def load(db):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = c.execute(f"select s.display_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x from {kd} d "
                     f"join {ks} s on d.kernel_id = s.id order by d.start").fetchall()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--seq", default=None, help="print the dispatch sequence of kernels matching this substring")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    db = a.db if a.db.endswith(".db") else glob.glob(a.db + "/**/*.db", recursive=True)[0]
    rows = load(db)
    by = {}
    for name, s, e, g, w in rows:
        by.setdefault(name, []).append((e - s) / 1e3)
    lines = ["kernel,calls,total_us,avg_us,median_us,min_us,max_us"]
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"\"{name}\",{len(d)},{sum(d):.1f},{sum(d) / len(d):.2f},{statistics.median(d):.2f},"
                     f"{min(d):.2f},{max(d):.2f}")
    print("\n".join(lines))
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")
    if a.seq:
        prev_end = None
        for name, s, e, g, w in rows:
            if a.seq in name:
                gap = (s - prev_end) / 1e3 if prev_end is not None else float("nan")
                print(f"{name[:60]:60s} dur {(e - s) / 1e3:10.2f} us  gap_before {gap:8.2f} us  grid {g} wg {w}")
            prev_end = e


if __name__ == "__main__":
    main()
