#!/usr/bin/env python3
"""Per-kernel HBM roofline report on ALGORITHMIC bytes.

For every HBM-bound kernel with a known launch shape in the workload (ALGO below: the bytes a launch
must move at least — its inputs read once and its outputs written once), the report gives

  * algorithmic bytes per launch and the achieved rate = algorithmic bytes / average duration
    (rocprofv3 --kernel-trace --stats of the benchmarked, graph-replayed run: tools/rocprof_summary.py csv);
  * ``frac`` = that rate / 8 TB/s (HBM3E peak, MI355X_MICROARCH.md);
  * the PMC counter bytes per launch (tools/pmc_traffic.py json: 2 x FETCH_SIZE + WRITE_SIZE of an eager
    pass, gfx950 FETCH correction) and their ratio to the algorithmic bytes.  Counter bytes are
    L2-miss traffic: FETCH_SIZE also counts Infinity-Cache (MALL) hits and the x2 correction is
    calibrated for wide streaming reads only, so they are an upper bound on HBM traffic, not HBM bytes;
    a ratio well above 1 means lines fetched more than once (re-reads across blocks / XCDs).

Kernels without an ALGO entry are listed with their counter rate only (no fraction).

    python tools/hbm_report.py <pmc.json | -> <stats.csv> <out.json> <label>
"""
import csv
import json
import sys

PEAK = 8.0e12
F = 4  # fp32


def _b(*terms):
    return int(sum(terms))


# (kernel substring, algorithmic bytes per launch, shape) per workload label; B = 16 frames (lipsync,
# lnet, dnet, pipeline), B = 4 faces (enhance)
_DNET = [
    ("conv_head_x3<1, 3, 7, 2>", _b(16 * 256 * 256 * 64 * F, 16 * 256 * 256 * 3 * F),
     "DNet 7x7 64->3 tanh head (DNet.py:77-86): in 16x256^2x64, out 16x256^2x3"),
    ("conv_halo_small<3, 7>", _b(16 * 256 * 256 * 64 * F, 16 * 256 * 256 * 3 * F),
     "DNet 7x7 64->3 tanh head, fp32 VALU form"),
    ("conv_head_x3<1, 2, 7,", _b(16 * 64 * 64 * 256 * F, 16 * 64 * 64 * 2 * F),
     "DNet 7x7 256->2 flow head (DNet.py:77-82), split-K over channel groups: in 16x64^2x256, out 16x64^2x2"),
    ("conv_halo_small<2, 7>", _b(16 * 64 * 64 * 256 * F, 16 * 64 * 64 * 2 * F),
     "DNet 7x7 256->2 flow head (DNet.py:77-82): in 16x64^2x256, out 16x64^2x2"),
    ("flow_warp_kernel<true>", _b(16 * 3 * 256 * 256 * F, 16 * 64 * 64 * 2 * F, 16 * 256 * 256 * 6 * F),
     "flow_util warp + cat (flow_util.py:3-56, DNet.py:114-115): src 16x3x256^2, flow 16x64^2x2, "
     "out 16x256^2x6"),
    ("flow_warp_kernel<false>", _b(16 * 3 * 256 * 256 * F, 16 * 64 * 64 * 2 * F, 16 * 256 * 256 * 3 * F),
     "flow_util warp: src 16x3x256^2, flow 16x64^2x2, out 16x256^2x3"),
]
_LNET = [
    ("conv_head_x3<1, 4, 7, 2>", _b(16 * 96 * 96 * 64 * F, 16 * 96 * 96 * 4 * F),
     "LNet 7x7 64->3 sigmoid head (LNet.py:77), Cout carried as 4: in 16x96^2x64, out 16x96^2x4"),
    ("conv_head_x3<1, 3, 7, 2>", _b(16 * 96 * 96 * 64 * F, 16 * 96 * 96 * 3 * F),
     "LNet 7x7 64->3 sigmoid head (LNet.py:77): in 16x96^2x64, out 16x96^2x3"),
]
_ENET = [
    ("conv_k4_mfma<1,", _b(16 * 256 * 256 * 4 * F, 16 * 256 * 256 * 256 * F),
     "ENet conv_body_first 1x1 4->256 (ENet.py:94), exact fp32 MFMA: in 16x256^2x4, out 16x256^2x256"),
    ("conv_k4_mfma<9,", _b(16 * 200 * 200 * 4 * F, 16 * 200 * 200 * F, 16 * 200 * 200 * 256 * F),
     "ENet first StyleConv 3x3 4->256 at 200^2 (ENet.py:122), exact fp32 MFMA: in 16x200^2x4, noise 16x200^2, "
     "out 16x200^2x256"),
    ("torgb_up2_kernel<8, 4>", _b(16 * 400 * 400 * 128 * F, 16 * 200 * 200 * 4 * F, 16 * 400 * 400 * 4 * F),
     "ENet 400^2 ToRGB + x2 skip (base_blocks.py:540-554): x 16x400^2x128, skip 16x200^2x4, out 16x400^2x4"),
    ("torgb_up2_kernel<8, 2>", _b(16 * 200 * 200 * 256 * F, 16 * 100 * 100 * 4 * F, 16 * 200 * 200 * 4 * F),
     "ENet 200^2 ToRGB + x2 skip: x 16x200^2x256, skip 16x100^2x4, out 16x200^2x4"),
]
ALGO = {
    "dnet": _DNET,
    "lnet": _LNET,
    "lipsync": _LNET + _ENET,
    "pipeline": _DNET + _ENET + [k for k in _LNET if "<1, 4," in k[0]],
}


def main():
    pmc_path, stats_path, out_path = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    pmc = json.load(open(pmc_path))["kernels"] if pmc_path != "-" else {}
    stats = {r["name"]: r for r in csv.DictReader(open(stats_path))}
    rows = []
    for name, st in stats.items():
        us = float(st["avg_us"])
        if us <= 0:
            continue
        row = {"kernel": name, "calls": int(st["calls"]), "avg_us": round(us, 3), "pct_time": float(st["pct"])}
        algo = next(((b, d) for k, b, d in ALGO.get(label, []) if k in name), None)
        p = pmc.get(name)
        if algo is None and p is None:
            continue
        if algo is not None:
            b, d = algo
            row.update({"shape": d, "algorithmic_bytes_per_launch": b,
                        "achieved_GBps": round(b / (us * 1e-6) / 1e9, 1),
                        "frac_of_8TBps": round(b / (us * 1e-6) / PEAK, 4)})
        if p is not None:
            cb = p["bytes_per_launch"]
            row.update({"counter_bytes_per_launch": cb, "counter_GBps": round(cb / (us * 1e-6) / 1e9, 1)})
            if algo is not None:
                row["counter_over_algorithmic"] = round(cb / algo[0], 2)
        rows.append(row)
    rows.sort(key=lambda r: (("frac_of_8TBps" not in r), -r["pct_time"]))
    doc = {"label": label, "peak_Bps": PEAK,
           "method": "achieved / frac: ALGORITHMIC bytes per launch (inputs read once, outputs written once; "
                     "shape per row) / rocprofv3 --stats average of the benchmarked graph-replayed run; "
                     "counter bytes: PMC 2*FETCH_SIZE + WRITE_SIZE per launch of an eager pass = L2-miss traffic "
                     "(FETCH_SIZE counts Infinity-Cache hits; the x2 gfx950 correction holds for wide streaming "
                     "reads), reported beside, not as HBM bytes", "kernels": rows}
    json.dump(doc, open(out_path, "w"), indent=1)
    print(f"{'kernel':60s} {'calls':>5s} {'avg_us':>8s} {'algo MB':>8s} {'GB/s':>7s} {'frac':>6s} {'ctr MB':>8s} {'ctr/algo':>8s}")
    for r in rows[:30]:
        print(f"{r['kernel'][:60]:60s} {r['calls']:5d} {r['avg_us']:8.1f} "
              f"{r.get('algorithmic_bytes_per_launch', 0) / 1e6:8.2f} {r.get('achieved_GBps', 0):7.0f} "
              f"{r.get('frac_of_8TBps', 0):6.3f} {r.get('counter_bytes_per_launch', 0) / 1e6:8.2f} "
              f"{r.get('counter_over_algorithmic', 0):8.2f}")


if __name__ == "__main__":
    main()
