#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 ``--pmc ... --output-format csv`` runs.

    pmc_counters.py <dir> [<dir> ...] [--match SUBSTR] [--grid WORK_ITEMS] [--out file.json]

``--grid``: only dispatches of that total grid size (work-items), i.e. one launch shape of the symbol.

Each dir is one pass's ``-d`` directory; counters of the same kernel symbol are averaged over its
dispatches and merged across passes.  Derived, when the inputs are present (MI355X_MICROARCH.md
§rocprofv3 / cycle constants: SQ_* wave counters count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES counts
cycles, GRBM_GUI_ACTIVE sums the 8 XCDs):
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 * SQ_BUSY_CU_CYCLES)   (per-SIMD matrix-pipe utilisation)
  wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES, valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match, out, grid = "", "", None
    if "--match" in args:
        i = args.index("--match"); match = args[i + 1]; del args[i:i + 2]
    if "--grid" in args:
        i = args.index("--grid"); grid = args[i + 1]; del args[i:i + 2]
    if "--out" in args:
        i = args.index("--out"); out = args[i + 1]; del args[i:i + 2]
    acc = defaultdict(lambda: defaultdict(list))
    for d in args:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            names = {}
            with open(path, newline="") as f:
                for row in csv.DictReader(f):
                    if grid is not None and str(row.get("Grid_Size", "")).split(".")[0] != grid:
                        continue
                    key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Counter_Name"])
                    per[key] += float(row["Counter_Value"])
                    names[key[0]] = row["Kernel_Name"]
            for (disp, cname), v in per.items():
                acc[names[disp]][cname].append(v)
    res = {}
    for k, cs in acc.items():
        if match and match not in k:
            continue
        r = {c: sum(v) / len(v) for c, v in cs.items()}
        r["dispatches"] = max(len(v) for v in cs.values())
        if "SQ_VALU_MFMA_BUSY_CYCLES" in r and r.get("SQ_BUSY_CU_CYCLES"):
            r["mfma_busy"] = r["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * r["SQ_BUSY_CU_CYCLES"])
        if "SQ_WAIT_ANY" in r and r.get("SQ_WAVE_CYCLES"):
            r["wait_frac"] = r["SQ_WAIT_ANY"] / r["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_INST_ANY" in r and r.get("SQ_WAVE_CYCLES"):
            r["wait_inst_frac"] = r["SQ_WAIT_INST_ANY"] / r["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in r and r.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = r["SQ_INSTS_VALU"] / r["SQ_INSTS_MFMA"]
            # SQ_INSTS_VALU counts the MFMAs too (MI355X_MICROARCH.md): the non-MFMA vector work per MFMA
            r["nonmfma_valu_per_mfma"] = (r["SQ_INSTS_VALU"] - r["SQ_INSTS_MFMA"]) / r["SQ_INSTS_MFMA"]
        if "FETCH_SIZE" in r or "WRITE_SIZE" in r:
            # gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM / rocprofv3); both in KiB
            r["counter_bytes"] = 1024 * (2 * r.get("FETCH_SIZE", 0.0) + r.get("WRITE_SIZE", 0.0))
        res[k] = r
    for k, r in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(k[:120])
        print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(r.items())))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
