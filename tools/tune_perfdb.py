#!/usr/bin/env python3
"""Measure the split-precision conv perf-db (speech-to-video-mpp_amd/perfdb_mi355x.json) on an MI355X.

Runs one eager forward of each bench.py workload named on the command line with ops.TUNE set: every
conv launch ops.conv_key() covers (split precision, no forced configuration, no conv group, no grid
cap) whose planner choice is a one-block-per-tile ``conv_igemm_x3`` tile is timed against every other
tile (force_tile 1..11, or --tiles) and split-K factor, each candidate as a HIP graph of REPS back-to-back launches
(its splitk_reduce launch included), best of ROUNDS replays.  Keys seen before are not re-measured.
The output is restored after the candidates ran (in-place residuals), so the forward continues on the
planner's result.  A key is written to the table only when its best candidate beats the planner's
choice by more than 3 %.

    python tools/tune_perfdb.py lnet lipsync dnet [--out speech-to-video-mpp_amd/perfdb_mi355x.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402

TILES = range(1, 12)
SPLITS = (1, 2, 3, 4, 6, 8, 12, 16)
REPS, ROUNDS = 8, 3
GAIN = 0.97


def graph_us(fn):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()                                   # sizes the workspace outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(REPS):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    best = 1e30
    for _ in range(ROUNDS):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / REPS)
    del g
    return best


class Tuner:
    def __init__(self):
        self.seen = {}

    def __call__(self, ctx, key, relaunch, plan_of, yv, resv):
        if key in self.seen:
            return
        plan0 = plan_of(0, 0)
        sym0 = ops.plan_symbol(plan0)
        if not sym0.startswith("void s2v::conv_igemm_x3<"):
            self.seen[key] = None
            return
        torch.cuda.synchronize()
        saved = yv.clone()
        t0 = time.time()
        res = {"planner": {"symbol": sym0, "splits": plan0[5], "us": graph_us(lambda: relaunch(0, 0))}}
        cands = []
        for t in TILES:
            for s in SPLITS:
                try:
                    p = plan_of(t, s)
                except (RuntimeError, ops._lib.S2VError):
                    continue
                if p[5] != s:                      # split factor clamped to the K tiles: seen already
                    continue
                try:
                    us = graph_us(lambda t=t, s=s: relaunch(t, s))
                except (RuntimeError, ops._lib.S2VError):
                    continue
                cands.append({"tile": t, "splits": s, "us": us, "symbol": ops.plan_symbol(p)})
        yv.copy_(saved)
        f = ctx.range_flag()
        if f is not None:
            f.zero_()                              # candidates re-accumulating an in-place residual
        torch.cuda.synchronize()
        best = min(cands, key=lambda c: c["us"]) if cands else None
        res["best"] = best
        res["candidates"] = len(cands)
        self.seen[key] = res
        b = f"{best['us']:8.1f} us tile {best['tile']:2d} splits {best['splits']:2d} {best['symbol'][10:40]}" if best else "-"
        print(f"{key}: planner {res['planner']['us']:8.1f} us {sym0[10:40]} s{plan0[5]} | best {b} "
              f"({len(cands)} cands, {time.time() - t0:.1f} s)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="+", choices=("lnet", "lipsync", "dnet", "pipeline", "enhance"))
    ap.add_argument("--out", default=ops.PERFDB_PATH)
    ap.add_argument("--raw", default="", help="also write every measured key (planner, best) here")
    ap.add_argument("--merge", action="store_true", help="keep the entries of --out for keys not measured here")
    ap.add_argument("--tiles", default="", help="comma list of force_tile values (default 1..11); r05: 1..15 adds "
                    "the deep-stage 4-wave tiles")
    a = ap.parse_args()
    global TILES
    if a.tiles:
        TILES = [int(t) for t in a.tiles.split(",")]
    sys.argv = [sys.argv[0]]
    bargs = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ops.PERFDB = {}                                # the planner's own choices are the baseline
    from s2v_amd.engine import enet as _enet, lnet as _lnet
    _lnet.BRANCHES = _enet.OVERLAP = False         # one stream: the candidates run alone
    tuner = Tuner()
    for w in a.workloads:
        wl = bench.WORKLOADS[w](bargs, dev, 0, 1)
        with torch.no_grad():
            wl.forward()                           # calibration forward (range guard)
            torch.cuda.synchronize()
            ops.TUNE = tuner
            try:
                wl.forward()
            finally:
                ops.TUNE = None
            torch.cuda.synchronize()
        print(f"== {w} done: {sum(1 for v in tuner.seen.values() if v)} keys measured", flush=True)
    entries, wls = {}, list(a.workloads)
    if a.merge and os.path.exists(a.out):
        with open(a.out) as f:
            old = json.load(f)
        entries = {k: v for k, v in old["entries"].items() if k not in tuner.seen}
        wls = sorted(set(old.get("workloads", [])) | set(wls))
    for k, v in tuner.seen.items():
        if v and v["best"] and v["best"]["us"] < GAIN * v["planner"]["us"]:
            b = v["best"]
            entries[k] = {"tile": b["tile"], "splits": b["splits"], "us": round(b["us"], 2),
                          "planner_us": round(v["planner"]["us"], 2), "planner": v["planner"]["symbol"][10:],
                          "planner_splits": v["planner"]["splits"], "symbol": b["symbol"][10:]}
    props = torch.cuda.get_device_properties(dev)
    out = {"device": torch.cuda.get_device_name(dev), "workloads": wls,
           "arch": props.gcnArchName.split(":")[0], "cus": props.multi_processor_count,
           "how": f"tools/tune_perfdb.py: each candidate a HIP graph of {REPS} launches, best of {ROUNDS} replays; "
                  f"kept when < {GAIN} x the planner's choice",
           "entries": entries}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    if a.raw:
        with open(a.raw, "w") as f:
            json.dump({k: v for k, v in tuner.seen.items() if v}, f, indent=1, sort_keys=True)
    tot_p = sum(v["planner"]["us"] for v in tuner.seen.values() if v)
    tot_b = sum(min(v["planner"]["us"], v["best"]["us"]) for v in tuner.seen.values() if v and v["best"])
    print(f"{len(entries)} entries written to {a.out}; per-key sum planner {tot_p:.0f} us -> tuned {tot_b:.0f} us")


if __name__ == "__main__":
    main()
