#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite *.db or *_kernel_stats.csv) into
a per-kernel CSV: name, calls, total_us, avg_us, pct.  Usage: rocprof_summary.py <db|csv> [out.csv]
[--by-grid]  (--by-grid: one row per (kernel, grid size, workgroup size), so the launches of one
symbol at different shapes get their own average duration)"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    db = sqlite3.connect(path)
    q = "select name, total_calls, total_duration, average, percentage from top_kernels order by total_duration desc"
    return [(n, int(c), t, a, p) for n, c, t, a, p in db.execute(q)]  # top_kernels reports microseconds


def rows_by_grid(path):
    db = sqlite3.connect(path)
    q = ("select name, grid_x, grid_y, grid_z, workgroup_x, count(*), sum(duration), avg(duration) from kernels "
         "group by name, grid_x, grid_y, grid_z, workgroup_x order by sum(duration) desc")
    rows = list(db.execute(q))
    tot = sum(r[6] for r in rows) or 1.0
    return [(f"{n} grid=({gx},{gy},{gz}) wg={wx}", int(c), t / 1e3, a / 1e3, 100.0 * t / tot)
            for n, gx, gy, gz, wx, c, t, a in rows]                    # kernels.duration is in ns


def main():
    by_grid = "--by-grid" in sys.argv
    argv = [a for a in sys.argv[1:] if a != "--by-grid"]
    src = argv[0]
    out = argv[1] if len(argv) > 1 else None
    rows = rows_by_grid(src) if by_grid else rows_from_db(src)
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f)
    w.writerow(["name", "calls", "total_us", "avg_us", "pct"])
    for n, c, t, a, p in rows:
        if len(n) > 200:
            n = n[:160] + "..." + n[n.rfind(" grid="):] if " grid=" in n else n[:200] + "..."
        w.writerow([n, c, f"{t:.3f}", f"{a:.3f}", f"{p:.2f}"])
    if out:
        f.close()


if __name__ == "__main__":
    main()
