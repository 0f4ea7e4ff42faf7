#!/usr/bin/env python3
"""Per-kernel HBM bandwidth report: PMC traffic (tools/pmc_traffic.py json: FETCH / WRITE passes,
gfx950-corrected) divided by the kernel's average duration from the rocprofv3 --stats summary of the
same workload (tools/rocprof_summary.py csv).  Peak: 8 TB/s HBM3E (MI355X_MICROARCH.md).

    python tools/hbm_report.py <pmc.json> <stats.csv> <out.json> [label] [--algo 'substr=bytes' ...]

``--algo`` adds an algorithmic byte count per launch for kernels whose name contains ``substr``
(traffic well above it means re-reads)."""
import csv
import json
import sys

PEAK = 8.0e12


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--algo")]
    algo = {}
    for a in sys.argv[1:]:
        if a.startswith("--algo="):
            k, v = a[len("--algo="):].rsplit("=", 1)
            algo[k] = float(v)
    pmc_path, stats_path, out_path = args[:3]
    label = args[3] if len(args) > 3 else ""
    pmc = json.load(open(pmc_path))["kernels"]
    stats = {r["name"]: r for r in csv.DictReader(open(stats_path))}
    rows = []
    for name, st in stats.items():
        p = pmc.get(name)
        if p is None:
            continue
        us = float(st["avg_us"])
        b = p["bytes_per_launch"]
        row = {"kernel": name, "calls": int(st["calls"]), "avg_us": round(us, 3), "pct_time": float(st["pct"]),
               "bytes_per_launch": b, "achieved_GBps": round(b / (us * 1e-6) / 1e9, 1),
               "frac_of_8TBps": round(b / (us * 1e-6) / PEAK, 4)}
        for k, v in algo.items():
            if k in name:
                row["algorithmic_bytes_per_launch"] = v
                row["algorithmic_GBps"] = round(v / (us * 1e-6) / 1e9, 1)
        rows.append(row)
    rows.sort(key=lambda r: -r["pct_time"])
    doc = {"label": label, "peak_Bps": PEAK,
           "method": "bytes = PMC 1024*(2*FETCH_SIZE+WRITE_SIZE) per launch (eager pass); avg_us = rocprofv3 --stats "
                     "of the benchmarked (graph-replayed) run", "kernels": rows}
    json.dump(doc, open(out_path, "w"), indent=1)
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>9s} {'MB/launch':>10s} {'GB/s':>8s} {'frac':>6s}")
    for r in rows[:25]:
        print(f"{r['kernel'][:70]:70s} {r['calls']:6d} {r['avg_us']:9.1f} {r['bytes_per_launch'] / 1e6:10.2f} "
              f"{r['achieved_GBps']:8.0f} {r['frac_of_8TBps']:6.3f}")


if __name__ == "__main__":
    main()
