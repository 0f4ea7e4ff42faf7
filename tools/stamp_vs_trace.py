#!/usr/bin/env python3
"""The headline roofline's in-kernel stamps against rocprofv3's kernel trace of the SAME process
(VERDICT r04 item 2): bench.py --dump-stamps under rocprofv3 --kernel-trace.

For every launch of the dominant symbol's headline shape (its FLOPs per launch), in launch order, the
trace's (start, end) and the stamps' (first block start, last block end, s_memrealtime 100 MHz) are paired;
the stamp clock is mapped onto the trace clock by a least-squares fit of the launch midpoints (slope ~10 ns
per tick).  Per launch: trace duration, stamped duration, and the trace's extra time split into the part
before the first block starts (dispatch -> first wave) and after the last block ends (last wave -> the
completion signal).  Usage: stamp_vs_trace.py <run_results.db> <stamps.json> [out.json]"""
import json
import sqlite3
import sys


def main():
    db_path, st_path = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else ""
    st = json.load(open(st_path))
    sym = st["kernel"]
    recs = st["launches"].get(sym, [])
    if not recs:
        raise SystemExit(f"no stamped launches of {sym}")
    groups = {}
    for r, slot, s0, s1, fl in recs:
        groups.setdefault(round(fl), []).append((r, slot, s0, s1))
    fl_head, head = max(groups.items(), key=lambda kv: sum(s1 - s0 for _, _, s0, s1 in kv[1]))
    head.sort()
    db = sqlite3.connect(db_path)
    cols = [c[1] for c in db.execute("pragma table_info(kernels)")]
    s_col = "start" if "start" in cols else "start_ns"
    e_col = "end" if "end" in cols else "end_ns"
    name = sym.split("(")[0]
    rows = list(db.execute(f"select name, {s_col}, {e_col}, grid_x, grid_y, grid_z from kernels order by {s_col}"))
    rows = [r for r in rows if r[0].split("(")[0] == name]
    # the headline shape's grid: the grid whose launch count per replay matches and whose total time is largest
    by_grid = {}
    for n, a, b, gx, gy, gz in rows:
        by_grid.setdefault((gx, gy, gz), []).append((a, b))
    nrep = len({r for r, _, _, _ in head})
    per_rep = len(head) // max(1, nrep)
    cand = [(g, v) for g, v in by_grid.items() if len(v) >= len(head)]
    grid, tr = max(cand, key=lambda gv: sum(b - a for a, b in gv[1][-len(head):]))
    tr = tr[-len(head):]                     # the timed replays are the last launches of that grid
    tick = 1e9 / st["clock_hz"]
    # least squares: trace midpoint = off + k * stamp midpoint (ns)
    xs = [(s0 + s1) / 2 for _, _, s0, s1 in head]
    ys = [(a + b) / 2 for a, b in tr]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    k = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / max(1e-30, sum((x - mx) ** 2 for x in xs))
    off = my - k * mx
    per = []
    for (r, slot, s0, s1), (a, b) in zip(head, tr):
        t0, t1 = off + k * s0, off + k * s1
        per.append({"replay": r, "trace_us": (b - a) / 1e3, "stamp_us": (s1 - s0) * tick / 1e3,
                    "head_us": (t0 - a) / 1e3, "tail_us": (b - t1) / 1e3,
                    "fit_resid_us": ((a + b) / 2 - (off + k * (s0 + s1) / 2)) / 1e3})
    avg = lambda key: sum(p[key] for p in per) / len(per)  # noqa: E731
    res = {"kernel": sym, "flops_per_launch": fl_head, "grid": list(grid), "launches": len(per),
           "launches_per_replay": per_rep, "clock_ns_per_tick_fit": k, "trace_us": avg("trace_us"),
           "stamp_us": avg("stamp_us"), "gap_us": avg("trace_us") - avg("stamp_us"),
           "gap_pct": 100.0 * (avg("trace_us") - avg("stamp_us")) / avg("stamp_us"),
           "gap_min_us": min(p["trace_us"] - p["stamp_us"] for p in per),
           "gap_max_us": max(p["trace_us"] - p["stamp_us"] for p in per),
           "fit_resid_max_us": max(abs(p["fit_resid_us"]) for p in per), "per_launch": per}
    print(json.dumps({k2: v for k2, v in res.items() if k2 != "per_launch"}, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
