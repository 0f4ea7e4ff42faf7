#!/usr/bin/env python3
"""HBM traffic per kernel launch from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot
share a pass on gfx950: MI355X_MICROARCH.md §rocprofv3 PMC slots).

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE / WRITE_SIZE are in
KiB, and on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so

    bytes per launch = 1024 * (2 * FETCH_SIZE + WRITE_SIZE)

averaged over the launches of each kernel symbol.

Usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> [label]
(each dir is a rocprofv3 ``--output-format csv -d`` directory; every *counter_collection.csv under
it is read).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(root, counter):
    vals = {}
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {root}")
    for path in files:
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                key = (path, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                dur = (float(row.get("End_Timestamp") or 0) - float(row.get("Start_Timestamp") or 0)) / 1e3
                vals[key] = (row["Kernel_Name"], float(row["Counter_Value"]) + vals.get(key, ("", 0.0))[1],
                             row.get("Grid_Size", ""), dur)
    return vals


def summarise(fetch_dir, write_dir):
    agg = defaultdict(lambda: {"fetch_kib": 0.0, "write_kib": 0.0, "fetch_n": 0, "write_n": 0, "us": 0.0})
    for (_, _), (name, v, grid, dur) in per_dispatch(fetch_dir, "FETCH_SIZE").items():
        for k in (name, f"{name} grid={grid}"):
            agg[k]["fetch_kib"] += v
            agg[k]["fetch_n"] += 1
            agg[k]["us"] += dur
    for (_, _), (name, v, grid, _) in per_dispatch(write_dir, "WRITE_SIZE").items():
        for k in (name, f"{name} grid={grid}"):
            agg[k]["write_kib"] += v
            agg[k]["write_n"] += 1
    out = {}
    for name, a in agg.items():
        if not a["fetch_n"] or not a["write_n"]:
            continue
        f = a["fetch_kib"] / a["fetch_n"]
        w = a["write_kib"] / a["write_n"]
        out[name] = {"launches": a["fetch_n"], "fetch_kib_raw": round(f, 3), "write_kib": round(w, 3),
                     "bytes_per_launch": round(1024 * (2 * f + w)), "pass_us": round(a["us"], 1)}
    return out


def main():
    fetch_dir, write_dir, out_path = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    kern = summarise(fetch_dir, write_dir)
    doc = {"label": label,
           "formula": "bytes = 1024 * (2 * FETCH_SIZE + WRITE_SIZE) per launch, averaged per kernel symbol "
                      "and per (symbol, grid) ('<symbol> grid=<work-items>'; pass_us = the launches' summed "
                      "duration in this PMC pass) (gfx950 FETCH_SIZE half-count correction, MI355X_MICROARCH.md §HBM)",
           "per_launch_bytes": {k: v["bytes_per_launch"] for k, v in kern.items() if " grid=" not in k},
           "per_grid": {k: {"bytes_per_launch": v["bytes_per_launch"], "launches": v["launches"], "pass_us": v["pass_us"]}
                        for k, v in kern.items() if " grid=" in k},
           "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["bytes_per_launch"] * kv[1]["launches"]))}
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in list(doc["kernels"].items())[:15]:
        print(f"{v['bytes_per_launch'] / 1e6:10.2f} MB/launch x{v['launches']:4d}  {k[:110]}")


if __name__ == "__main__":
    main()
