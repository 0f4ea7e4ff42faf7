#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite *.db or *_kernel_stats.csv) into
a per-kernel CSV: name, calls, total_us, avg_us, pct.  Usage: rocprof_summary.py <db|csv> [out.csv]"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    db = sqlite3.connect(path)
    q = "select name, total_calls, total_duration, average, percentage from top_kernels order by total_duration desc"
    return [(n, int(c), t, a, p) for n, c, t, a, p in db.execute(q)]  # top_kernels reports microseconds


def main():
    src = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    rows = rows_from_db(src)
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f)
    w.writerow(["name", "calls", "total_us", "avg_us", "pct"])
    for n, c, t, a, p in rows:
        w.writerow([n if len(n) < 200 else n[:200] + "...", c, f"{t:.3f}", f"{a:.3f}", f"{p:.2f}"])
    if out:
        f.close()


if __name__ == "__main__":
    main()
