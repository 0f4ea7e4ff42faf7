#!/usr/bin/env python3
"""Benchmark of the per-frame lip-sync hot path on MI355X (BASELINE.json metric).

Workload (one "step"): ENet(+LNet) forward — models/ENet.py:82-139 — on one batch of B=16
synthetic 256x256 face crops + 16 mel windows [1,80,16] (inference.py:393-399 batching,
LNet_batch_size 16), weights from the portable synthetic checkpoint (s2v_amd.synth), inputs
resident in HBM.  The whole forward is one HIP-graph replay; with ``--lanes L`` (default 1) the steps
alternate between L captured lanes (runtime.LaneRunner: separate buffers, workspaces and streams,
shared read-only weights), so batch k+1's latency-bound LNet head overlaps batch k's MFMA-bound
StyleConv tail.  Every step still runs the whole forward of its own batch.

Multi-GPU: one process per GPU.  Under torchrun (the driver's N > 1 launch) the ranks come from the
environment; ``python bench.py --gpus N`` without it spawns N fresh worker processes itself (before
anything touches a GPU).  Frames shard across ranks with no data-path collective (weak scaling:
every rank runs its own B-frame batches); the timed region is bracketed by a barrier and synchronize
on every rank and the max over ranks is reported.  ``--workload clip`` is the strong-scaling form
(BASELINE configs[3]): one step = a whole 1000-frame clip sharded over the ranks, with the RCCL
broadcast of the per-clip host data and the uint8 gather to rank 0 inside the step.

Prints ONE JSON line on rank 0 with the live roofline of the dominant kernel (HIP events on the
stream the kernels run on) and, at N=1, the CPU baseline (oracle restatement on host cores).

Other workloads (not the headline metric):
  --workload pipeline   one step = 16 frames through DNet -> uint8 ref -> ENet(+LNet) -> uint8
                        384x384 frames (s2v_amd.pipeline.LipSyncPipeline.run_batch), plus the
                        host precompute of a 1000-frame clip timed once;
  --workload enhance    one step = B 512x512 faces through GFPGANv1Clean and GPEN-512;
  --workload lnet       one step = LNet forward alone on B=16 (BASELINE configs[1]): 256x256 crops
                        bilinear-resized to 96x96 as ENet.py:104 does, then models/LNet.py:122-139;
  --workload dnet       one step = DNet forward alone on B=16 256x256 source crops + coefficient windows
                        (the pipeline's DNet phase, models/DNet.py:20-28);
  --workload mouth      one step = B 720x720 frames through the mouth-region post-process
                        (FaceParse-512 mask of the face box + 10-level Laplacian blend,
                        inference.py:302-313, s2v_amd.post.MouthBlend);
  --workload sr         one step = B 720x720 uint8 frames through RealESRNet x2 (SURVEY.md §8f(2):
                        FaceEnhancement's srmodel.process on every full frame, s2v_amd.sr);
  --workload gpen2048   one step = B 2048x2048 faces through GPEN-BFR-2048 (the CLI's enhancer GAN);
  --workload clip       one step = the 1000-frame clip of configs[3] through pipeline.run_sharded: broadcast
                        of wav / semantic / expression, mel + windows, coefficient windows, DNet -> ENet ->
                        uint8 on each rank's contiguous frame range (HIP-graph replay per 16-frame batch),
                        gather of the uint8 frames to rank 0;
  --workload selftest   (tests only, --device cpu) the launcher / timing / JSON path on the gloo backend.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import s2v_import  # noqa: E402,F401

METRIC = "synthesized 256×256 frames/sec/GPU (LNet+ENet path); 1/2/4/8-GPU scaling"
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (spec)
# split-fp32 kernels issue 3 dense 16-bit MFMAs (bf16 / f16: 2.5 PF/s dense, MI355X_MICROARCH.md) per
# fp32 MAC, so their ceiling in algorithmic (fp32-equivalent) FLOP/s is a third of that peak
X3_PEAK_TFLOPS = 2500.0 / 3
REF_GFLOP_PER_FRAME = 407.46       # ENet+LNet algorithmic GFLOP/frame (2*MAC)
# ENet's StyleConv NoiseInjection strength in the timed lipsync / pipeline / clip weights (non-zero,
# as in a trained checkpoint): every step draws four N(0,1) noise planes (base_blocks.py:528-531)
NOISE_W = 0.1
NOISE_DESC = (f"on: NoiseInjection weight {NOISE_W} on all four StyleConvs, fresh N(0,1) planes drawn "
              "on the device every step and added in the conv epilogues")


ARITH = {"f16x3": "f16x3: fp32 tensors, conv products as split-fp32 hi*hi+hi*lo+lo*hi on f16 MFMA "
                   "(22 significant bits per operand, <= 3*2^-22 per product), fp32 accumulate; 4-channel-input convs and "
                   "Cout <= 4 VALU heads in exact fp32; all other ops fp32",
         "bf16x3": "bf16x3: fp32 tensors, conv products as split-fp32 hi*hi+hi*lo+lo*hi on bf16 MFMA "
                    "(16 significant bits per operand), fp32 accumulate; 4-channel-input convs and Cout <= 4 VALU heads in "
                    "exact fp32; all other ops fp32",
         "f32": "f32: exact fp32 MFMA (v_mfma_f32_32x32x2_f32) convs; all other ops fp32"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=tuple(WORKLOADS), default="lipsync")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="0 = the workload's default (16, or 4 for enhance)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--lanes", type=int, default=1,
                    help="execution lanes: consecutive steps replay captured graphs on this many lanes, each on its "
                         "own stream (runtime.LaneRunner); 1 = every step on one stream")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--frames", type=int, default=1000, help="clip workload: frames in the clip")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda", help="cpu: launcher self-test only")
    ap.add_argument("--precision", choices=("f16x3", "bf16x3", "f32"), default="f16x3",
                    help="conv arithmetic (s2v_amd.ops.set_precision)")
    ap.add_argument("--no-alt", action="store_true", help="skip the timing of the other conv arithmetic")
    ap.add_argument("--dump-stamps", default="",
                    help="write every stamped launch of the timed replays (raw s_memrealtime ticks, per symbol, "
                         "replay and launch slot, with its FLOPs) to this JSON file (tools/stamp_vs_trace.py)")
    return ap.parse_args()


def make_inputs(batch, size, device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    mel = torch.rand((batch, 1, 80, 16), generator=g, device=device) * 8 - 4
    face = torch.rand((batch, 6, size, size), generator=g, device=device)
    face[:, :3, size // 2:] = 0.0                      # masked lower half (inference.py:397)
    gt = face[:, 3:].clone()
    return mel, face, gt


def live_roofline(forward, workload="lipsync"):
    """One un-graphed ``forward()`` with every conv/GEMM launch bracketed by HIP events on its
    stream; per kernel symbol: sum of algorithmic FLOPs / sum of durations.  The dominant symbol's
    durations are then re-measured with each launch repeated back to back (second pass)."""
    from s2v_amd import ops
    recs = []
    grids = {}      # round(flops) -> {symbol: grid work-items} (to find a launch shape's PMC row)

    def hook(ctx, p, flops, launch):
        sym = ops.conv_symbol(ctx, p)
        splits = ops.conv_splits(ctx, p)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        recs.append((sym, flops, splits, s, e, (p.n, p.h, p.w, p.cin, p.oh, p.ow, p.cout, p.kh, p.kw,
                                                p.in_scale, p.nc_scale, p.pix_add, p.res)))
        pl = p.plan     # [bm, bn, wm, amode, b_kn, splits, prec, nw, ...]: the launch's work-items
        if pl[0] > 0 and pl[1] > 0:
            grids.setdefault(round(flops), {})[sym] = (-(-p.n * p.oh * p.ow // pl[0]) * -(-p.cout // pl[1]) *
                                                       max(1, pl[5]) * 64 * max(1, pl[7]))

    # per-kernel durations are measured with the side-stream branches serialised (engine.lnet
    # BRANCHES, engine.enet OVERLAP), so concurrent kernels do not inflate each other's time
    from s2v_amd.engine import enet as _enet, lnet as _lnet
    saved = (_lnet.BRANCHES, _enet.OVERLAP)
    _lnet.BRANCHES = _enet.OVERLAP = False
    # one unhooked forward first: a kernel's first launch in the process also loads its code object
    # (HIP loads kernels lazily), which made a 28 us conv the "dominant" symbol of a cold pre-pass
    with torch.no_grad():
        forward()
    torch.cuda.synchronize()
    ops.CONV_HOOK = hook
    try:
        with torch.no_grad():
            forward()
        torch.cuda.synchronize()
    finally:
        ops.CONV_HOOK = None
        _lnet.BRANCHES, _enet.OVERLAP = saved
    per = {}
    if os.environ.get("S2V_BENCH_VERBOSE") == "2":
        for sym, flops, splits, s, e, shp in recs:
            ms = s.elapsed_time(e)
            print(f"  {ms * 1e3:9.1f} us {flops / max(ms, 1e-9) / 1e9:7.2f} TF/s splits={splits} "
                  f"n,h,w,cin,oh,ow,cout,kh,kw,ins,ncs,pix,res={shp} {sym[11:40]}", file=sys.stderr)
    for sym, flops, splits, s, e, _ in recs:
        d = per.setdefault(sym, {"flops": 0.0, "ms": 0.0, "launches": 0, "split_launches": 0})
        d["flops"] += flops
        d["ms"] += s.elapsed_time(e)
        d["launches"] += 1
        d["split_launches"] += int(splits > 1)
    dom = max(per, key=lambda k: per[k]["ms"])
    if os.environ.get("S2V_BENCH_VERBOSE"):
        for k in sorted(per, key=lambda k: -per[k]["ms"]):
            v = per[k]
            tf = v["flops"] / max(v["ms"], 1e-9) / 1e9
            print(f"  {v['ms']:9.3f} ms  {v['launches']:4d} launches  {tf:7.2f} TF/s  {k}", file=sys.stderr)
    d = per[dom]
    # second pass for the dominant symbol: each of its launches repeated REPS times back to back
    # between one event pair (a single short launch between two events also times the event
    # overhead: LNet's ~20 us 64x64 tiles read ~36 us that way); launches that accumulate into
    # their own output (res == y) run once
    REPS = 5
    rep = {"ms": 0.0, "n": 0}

    def hook2(ctx, p, flops, launch):
        if ops.conv_symbol(ctx, p) != dom:
            launch()
            return
        reps = 1 if p.res_is_y else REPS
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            launch()
        e.record()
        rep_recs.append((s, e, reps))

    rep_recs = []
    _lnet.BRANCHES = _enet.OVERLAP = False
    ops.CONV_HOOK = hook2
    try:
        with torch.no_grad():
            forward()
        torch.cuda.synchronize()
    finally:
        ops.CONV_HOOK = None
        _lnet.BRANCHES, _enet.OVERLAP = saved
    for s, e, reps in rep_recs:
        rep["ms"] += s.elapsed_time(e) / reps
        rep["n"] += 1
    if rep["n"] == d["launches"] and rep["ms"] > 0:
        d = dict(d, ms=rep["ms"])
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    peak = _peak(dom)
    total_ms = sum(v["ms"] for v in per.values())
    total_flops = sum(v["flops"] for v in per.values())
    # HBM bytes per launch of the same symbol from the PMC passes of this workload (tools/gpu_profile.sh:
    # separate FETCH_SIZE / WRITE_SIZE runs of this bench command; the newest round's file wins)
    traffic, traffic_src = pmc_traffic(workload, dom)
    return {
        "bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": traffic_src,
        "kernel": dom, "launches": d["launches"], "avg_launch_us": round(1e3 * d["ms"] / d["launches"], 2),
        "flops_per_launch": d["flops"] / d["launches"],
        "conv_family": {"achieved": round(total_flops / (total_ms * 1e-3) / 1e12, 2),
                        "ms_per_step": round(total_ms, 3), "symbols": len(per)},
        "per_kernel": per,
        "_grids": grids,
        "_workload": workload,
    }


class Stamper:
    """In-kernel launch timer of a set of kernel symbols in captured, replayed steps (ops.STAMP /
    s2v_conv_params.stamps): per lane a replay counter (bumped by the first kernel of every replay)
    and, per symbol, a [reps, launches, 2] buffer of (first block start, last block end) device
    real-time clock values (s_memrealtime, 100 MHz) per launch of that symbol in that replay, plus the
    algorithmic FLOPs of each launch slot.  ``kernels``: {symbol: max launches per step}."""

    CLOCK_HZ = 100e6

    def __init__(self, kernels, reps, device):
        self.kernels = dict(kernels)
        self.reps, self.device = reps, device
        self.lanes = {}
        self.cur = None

    def begin(self, lane):
        """Start of one forward of ``lane`` (eager warm-up or capture): bump its replay counter
        (captured as the graph's first kernel) and restart the launch numbering."""
        from s2v_amd import ops
        if lane not in self.lanes:
            self.lanes[lane] = {"ctr": torch.zeros(1, dtype=torch.int64, device=self.device), "n": {},
                                "buf": {k: torch.zeros((self.reps, m, 2), dtype=torch.int64, device=self.device)
                                        for k, m in self.kernels.items()},
                                "flops": {k: [0.0] * m for k, m in self.kernels.items()}}
        L = self.lanes[lane]
        L["n"] = {}
        self.cur = L
        ops.S2V.counter_add_(L["ctr"], 1)

    def __call__(self, info, flops):
        from s2v_amd import ops
        sym = ops.plan_symbol(info.plan)
        if self.cur is None or sym not in self.kernels:
            return None
        L = self.cur
        slot = L["n"].get(sym, 0)
        L["n"][sym] = slot + 1
        stride = self.kernels[sym]
        if slot >= stride:
            return None
        L["flops"][sym][slot] = flops
        return L["buf"][sym], L["ctr"], [slot, stride, self.reps]

    def arm(self):
        torch.cuda.synchronize()
        for L in self.lanes.values():
            for buf in L["buf"].values():
                buf[..., 0] = -1              # uint64 max: atomic min start
                buf[..., 1] = 0
            L["c0"] = int(L["ctr"].item())

    def raw(self):
        """{symbol: [[replay, slot, s0, s1, flops], ...]} of the timed replays, in replay / slot order."""
        torch.cuda.synchronize()
        out = {}
        for L in self.lanes.values():
            c1 = int(L["ctr"].item())
            for sym, buf in L["buf"].items():
                b = buf.cpu()
                for r in range(L["c0"] + 1, c1 + 1):
                    for slot, (s0, s1) in enumerate(b[r % self.reps].tolist()):
                        if s0 != -1 and s1 > 0:
                            out.setdefault(sym, []).append([r, slot, s0, s1, L["flops"][sym][slot]])
        return out

    def launches(self):
        """{symbol: [(duration us, flops), ...]} of every stamped launch of the timed replays."""
        torch.cuda.synchronize()
        out = {}
        self.replays = 0
        for L in self.lanes.values():
            c1 = int(L["ctr"].item())
            self.replays += c1 - L["c0"]
            for sym, buf in L["buf"].items():
                b = buf.cpu()
                for r in range(L["c0"] + 1, c1 + 1):
                    for slot, (s0, s1) in enumerate(b[r % self.reps].tolist()):
                        if s0 != -1 and s1 > 0:
                            out.setdefault(sym, []).append(((s1 - s0) / self.CLOCK_HZ * 1e6, L["flops"][sym][slot]))
        return out


X3_KERNELS = ("conv_igemm_x3", "conv_glds_x3", "conv_x3_nar", "conv_x3_halo")   # split-precision families


def _peak(sym):
    return X3_PEAK_TFLOPS if any(k in sym for k in X3_KERNELS) else FP32_MFMA_PEAK_TFLOPS


PMC_ROUND = "r06"     # only this round's PMC passes describe the current build


def pmc_traffic(workload, sym, grid=None):
    """HBM bytes per launch of ``sym`` from this round's PMC passes of the workload
    (profiles/pmc_<round>_<workload>.json, tools/pmc_traffic.py): the (symbol, grid) row nearest to
    ``grid`` work-items when given, else the symbol's average; (None, None) without a file."""
    pmc = os.path.join(ROOT, "profiles", f"pmc_{PMC_ROUND}_{workload}.json")
    if not os.path.exists(pmc):
        return None, None
    with open(pmc) as f:
        doc = json.load(f)
    src = os.path.relpath(pmc, ROOT)
    rows = {int(k.rsplit("grid=", 1)[1]): v for k, v in doc.get("per_grid", {}).items()
            if k.startswith(sym + " grid=") and k.rsplit("grid=", 1)[1].isdigit()}
    if grid and rows:
        g = min(rows, key=lambda r: abs(r - grid) / max(r, grid))
        if abs(g - grid) <= 0.05 * max(g, grid):
            return rows[g]["bytes_per_launch"], f"{src} [grid={g}]"
    t = doc.get("per_launch_bytes", {}).get(sym)
    return (t, src + " (symbol average)") if t is not None else (None, None)


def replay_roofline(pre, stamper):
    """roofline of the dominant kernel from the timed (graph-replayed, overlapped) launches, plus
    the same figure for every other stamped kernel symbol (``by_kernel``): the style encoder's
    persistent launches (conv_igemm_x3_persist, half the chip by design) are their own entry."""
    st = stamper.launches() if stamper is not None else {}
    r = dict(pre)
    iso = {"avg_launch_us": pre["avg_launch_us"], "frac": pre["frac"], "achieved": pre["achieved"],
           "how": "un-graphed pass, side branches serialised, each launch repeated back to back between HIP events"}
    by = {}
    for sym, recs in sorted(st.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
        us = sum(d for d, _ in recs)
        fl = sum(f for _, f in recs)
        ach = fl / (us * 1e-6) / 1e12
        by[sym] = {"launches": len(recs), "avg_launch_us": round(us / len(recs), 2),
                   "flops_per_launch": fl / len(recs), "achieved": round(ach, 2), "peak": round(_peak(sym), 1),
                   "frac": round(ach / _peak(sym), 4)}
        if "_persist<" in sym and pre.get("grid_cap_blocks"):
            # persistent launches hold grid_cap_blocks CUs by design (one 512-thread block per CU): their rate
            # against the chip's peak and against the share of the peak those CUs carry
            held = pre["grid_cap_blocks"]
            by[sym].update(held_cus=held, cus=pre.get("cus", 256),
                           frac_of_held=round(ach / (_peak(sym) * held / pre.get("cus", 256)), 4))
    d = st.get(pre["kernel"], [])
    if not d:
        r["timing"] = "isolated (no stamped launches in the timed run)"
    else:
        # the dominant symbol's launches grouped by problem (FLOPs per launch): the headline entry is the
        # group with the most stamped time — one launch shape, so one grid, as rocprof's by-grid rows
        # (a symbol-wide average also counts the symbol's small launches of other layers, e.g. LNet
        # convs the perf-db puts on the same tile); the symbol-wide figure stays in by_kernel
        groups = {}
        for du, fl in d:
            groups.setdefault(round(fl), []).append(du)
        shapes = []
        for fl, ds in groups.items():
            us = sum(ds)
            ach = fl * len(ds) / (us * 1e-6) / 1e12
            shapes.append({"flops_per_launch": fl, "launches": len(ds), "avg_launch_us": round(us / len(ds), 2),
                           "achieved": round(ach, 2), "frac": round(ach / _peak(pre["kernel"]), 4), "_us": us})
        shapes.sort(key=lambda g: -g["_us"])
        for g in shapes:
            g.pop("_us")
        e = shapes[0]
        grid = pre.get("_grids", {}).get(e["flops_per_launch"], {}).get(pre["kernel"])
        tr, src = pmc_traffic(pre.get("_workload", ""), pre["kernel"], grid)
        reps = max(1, getattr(stamper, "replays", 0))
        r.update(symbol_launches_per_forward=r.pop("launches", None),
                 launches=round(e["launches"] / reps, 2),      # launches of THIS shape per step (avg_launch_us's set)
                 achieved=e["achieved"], frac=e["frac"], avg_launch_us=e["avg_launch_us"], timed_launches=e["launches"],
                 flops_per_launch=e["flops_per_launch"], traffic=tr, traffic_source=src,
                 timing="in-kernel clock stamps (s_memrealtime, first block start to last block end) of every launch "
                        "of this kernel and launch shape in the timed, graph-replayed steps",
                 shape_groups=shapes[:6], isolated=iso)
    if by:
        r["by_kernel"] = by
        # the stamped symbol with the most kernel time in the timed steps (the lipsync step's persistent
        # style-encoder launches), as a first-class entry beside the headline launch shape
        top = max(st.items(), key=lambda kv: sum(d for d, _ in kv[1]))[0]
        r["time_dominant"] = dict(by[top], kernel=top,
                                  ms_per_step=round(sum(d for d, _ in st[top]) / 1e3 / max(1, getattr(stamper, "replays", 1)), 3))
    return r


def host_threads():
    """The host cores this job may use: OMP_NUM_THREADS when the launcher set it (the GPU box sets
    the per-GPU CPU share there), else the CPU affinity set of this process."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _timed_cpu(fn, units_per_call, seconds, max_calls):
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            fn()
            n += units_per_call
            el = time.perf_counter() - t0
            if el >= seconds or n >= max_calls * units_per_call:
                return n, el


# ----------------------------------------------------------------------------- workloads
class Workload:
    """name, metric, unit, per-step units, GFLOP per unit, graph-captured step, un-graphed forward
    (for the roofline), CPU baseline."""
    metric = METRIC
    unit = "frames/s"
    gflop_per_unit = REF_GFLOP_PER_FRAME
    graphable = True          # the step is one HIP-graph replay of ``fn(*inputs)``
    scaling = "weak"

    def units_per_step(self, world):
        return world * self.batch


class SelfTest(Workload):
    """Launcher / timing / JSON self-test on the CPU (gloo): each rank sums its shard of a broadcast
    vector; no GPU work."""
    metric = "bench launcher self-test (CPU, gloo)"
    unit = "items/s"
    gflop_per_unit = 0.0
    graphable = False

    def __init__(self, args, dev, rank, world):
        self.batch = args.batch or 4
        self.world = world
        self.inputs = []
        self.config = {"workload": "selftest"}

    def step(self):
        import torch.distributed as dist
        v = torch.arange(64, dtype=torch.float32) if self.world == 1 or dist.get_rank() == 0 else torch.empty(64)
        if self.world > 1:
            dist.broadcast(v, 0)
        return v.sum()

    forward = step


class LipSync(Workload):
    def __init__(self, args, dev, rank, world=1):
        from s2v_amd import models, synth
        from s2v_amd.models import arch
        self.batch = args.batch or 16
        # StyleConv noise ON: NoiseInjection weight 0.1 on every StyleConv (real checkpoints carry
        # non-zero strengths; base_blocks.py:528-531 draws fresh N(0,1) noise per call), so every timed
        # step draws its noise planes and adds them in the conv epilogues
        self.sd = synth.synth_torch_state_dict(arch.ENetParams(lnet=arch.LNetParams()), noise_weight=NOISE_W)
        self.model = models.ENet()
        self.model.load_state_dict(self.sd)
        self.model.eval()
        self.size = args.size
        self.inputs = make_inputs(self.batch, args.size, dev, 1000 + rank)
        self.fn = lambda m, f, g: self.model(m, f, g)  # noqa: E731
        self.fn_lane = lambda lane, m, f, g: self.model(m, f, g, lane=lane)  # noqa: E731
        self.config = {"workload": f"ENet(+LNet) forward, B={self.batch} synthetic {args.size}x{args.size} crops "
                                   f"+ [1,80,16] mel windows -> 384x384 (models/ENet.py:82-139)",
                       "crop": args.size, "styleconv_noise": NOISE_DESC}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import nets
        torch.set_num_threads(threads)
        mel, face, gt = make_inputs(2, self.size, "cpu", 1234)

        def fwd():             # fresh StyleConv noise per call, as the timed GPU step draws it
            noises = [torch.randn(2, 1, s, s) for s in (200, 200, 400, 400)]
            return nets.enet_forward(self.sd, mel, face, gt, noises=noises)
        n, el = _timed_cpu(fwd, 2, seconds, 8)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} frames (2-frame batches) of the same ENet(+LNet) {self.size}x{self.size} workload "
                          f"in {el:.1f}s, torch CPU fp32, {threads} threads"}


class LNetOnly(Workload):
    metric = "LNet-only frames/sec/GPU (B=16 synthetic 256x256 crops -> 96x96 LNet, BASELINE configs[1])"
    gflop_per_unit = 56.14

    def __init__(self, args, dev, rank, world=1):
        from s2v_amd import models, ops, synth
        from s2v_amd.models import arch
        self.batch = args.batch or 16
        self.sd = synth.synth_torch_state_dict(arch.LNetParams())
        self.model = models.LNet()
        self.model.load_state_dict(self.sd)
        self.model.eval()
        self.size = args.size
        mel, face, _ = make_inputs(self.batch, args.size, dev, 5000 + rank)
        self.inputs = [mel, face]
        self.x96 = [torch.empty((self.batch, 6, 96, 96), device=dev) for _ in range(max(1, args.lanes))]
        ctx = ops.Ctx(dev)

        def step(lane, m, f):
            # F.interpolate(face, (96, 96), mode='bilinear') (ENet.py:104) on the device, then LNet
            x = self.x96[lane]
            ops.resize(ctx, f, 0, tuple(f.shape), f.stride(), x, 0, (96, 96), x.stride())
            return self.model(m, x, lane=lane)
        self.fn = lambda m, f: step(0, m, f)  # noqa: E731
        self.fn_lane = step
        self.config = {"workload": f"LNet forward, B={self.batch} synthetic {args.size}x{args.size} 6-channel crops "
                                   "(lower half of the masked half zeroed) bilinear-resized to 96x96 + [1,80,16] mel "
                                   "windows (models/LNet.py:122-139)", "crop": args.size}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        import torch.nn.functional as F
        from oracle import nets
        torch.set_num_threads(threads)
        mel, face, _ = make_inputs(2, self.size, "cpu", 1234)
        f96 = F.interpolate(face, (96, 96), mode="bilinear", align_corners=False)
        n, el = _timed_cpu(lambda: nets.lnet_forward(self.sd, mel, f96), 2, seconds, 64)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} frames (2-frame batches) of LNet at 96x96 in {el:.1f}s, torch CPU fp32, {threads} threads"}


class DNetOnly(Workload):
    """The pipeline's DNet phase alone (DNet.py:20-28 on B 256x256 source crops + coefficient windows),
    graph-replayed: its FLOP rate is the DNet-phase roofline (101.45 GFLOP/frame)."""
    metric = "DNet frames/sec/GPU (B=16 256x256 source crops + [73, 26] coefficient windows)"
    gflop_per_unit = 101.45

    def __init__(self, args, dev, rank, world=1):
        import numpy as np
        from s2v_amd import models, pipeline, synth
        from s2v_amd.models import arch
        self.batch = args.batch or 16
        self.sd = synth.synth_torch_state_dict(arch.DNetParams())
        self.model = models.DNet()
        self.model.load_state_dict(self.sd)
        self.model.eval()
        rng = np.random.default_rng(1)
        semantic = rng.standard_normal((self.batch + 40, 262)).astype(np.float32)
        semantic[:, -3] = 1.0 + 0.1 * rng.random(semantic.shape[0])
        coeffs = pipeline.dnet_coefficients(semantic, rng.standard_normal(64).astype(np.float32))
        g = torch.Generator(device=dev)
        g.manual_seed(3000 + rank)
        self.inputs = [torch.rand((self.batch, 3, 256, 256), generator=g, device=dev) * 2 - 1,
                       torch.from_numpy(coeffs[: self.batch]).to(dev)]
        self.fn = lambda s, c: self.model(s, c)  # noqa: E731
        self.fn_lane = lambda lane, s, c: self.model(s, c, lane=lane)  # noqa: E731
        self.config = {"workload": f"DNet forward, B={self.batch} synthetic 256x256 source crops + coefficient windows "
                                   f"{tuple(self.inputs[1].shape[1:])} (models/DNet.py:20-28)"}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import nets
        torch.set_num_threads(threads)
        s, c = (t[:2].cpu() for t in self.inputs)
        n, el = _timed_cpu(lambda: nets.dnet_forward(self.sd, s, c), 2, seconds, 8)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} frames (2-frame batches) of DNet at 256x256 in {el:.1f}s, torch CPU fp32, "
                          f"{threads} threads"}


class Pipeline(Workload):
    metric = "full DNet->LNet->ENet frames/sec/GPU (uint8 384x384 output)"
    gflop_per_unit = 508.91            # ENet+LNet 407.46 + DNet 101.45 (live)

    def __init__(self, args, dev, rank, world=1):
        import numpy as np
        from s2v_amd import audio, models, pipeline, synth
        from s2v_amd.models import arch
        self.batch = args.batch or 16
        self.sd_d = synth.synth_torch_state_dict(arch.DNetParams())
        self.sd_e = synth.synth_torch_state_dict(arch.ENetParams(lnet=arch.LNetParams()), noise_weight=NOISE_W)
        dnet, enet = models.DNet(), models.ENet()
        dnet.load_state_dict(self.sd_d)
        enet.load_state_dict(self.sd_e)
        self.pipe = pipeline.LipSyncPipeline(dnet.eval(), enet.eval(), dev, batch=self.batch)
        # host precompute of a 1000-frame clip (SURVEY.md §8d config 3 inputs), timed once
        rng = np.random.default_rng(0)
        t = np.arange(640000) / 16000.0
        wav = (0.1 * rng.standard_normal(t.size) + 0.2 * (np.sin(2 * np.pi * 220 * t) + np.sin(2 * np.pi * 440 * t)
                                                          + np.sin(2 * np.pi * 1000 * t))).astype(np.float32)
        semantic = rng.standard_normal((1000, 262)).astype(np.float32)
        semantic[:, -3] = 1.0 + 0.1 * rng.random(1000)
        expression = rng.standard_normal(64).astype(np.float32)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mel = audio.melspectrogram(torch.from_numpy(wav).to(dev))
        chunks = audio.mel_chunks(mel)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        coeffs = pipeline.dnet_coefficients(semantic, expression)
        t2 = time.perf_counter()
        self.host = {"clip_frames": 1000, "mel_chunks": int(chunks.shape[0]), "mel_ms": round(1e3 * (t1 - t0), 2),
                     "coeff_windows_ms": round(1e3 * (t2 - t1), 2)}
        g = torch.Generator(device=dev)
        g.manual_seed(2000 + rank)
        b = self.batch
        self.inputs = [chunks[:b].contiguous(), torch.rand((b, 3, 256, 256), generator=g, device=dev) * 2 - 1,
                       torch.from_numpy(coeffs[:b]).to(dev)]
        self.outs = [torch.empty((b, 3, 384, 384), dtype=torch.uint8, device=dev) for _ in range(max(1, args.lanes))]
        self.fn = lambda m, s, c: self.pipe.run_batch(m, s, c, self.outs[0])  # noqa: E731
        self.fn_lane = lambda lane, m, s, c: self.pipe.run_batch(m, s, c, self.outs[lane], lane=lane)  # noqa: E731
        self.config = {"workload": f"DNet -> uint8 ref -> ENet(+LNet) -> uint8, B={b} frames per step "
                                   "(inference.py:259-288, facing.py:176-191), 256x256 DNet/ENet crops",
                       "host_precompute": self.host, "styleconv_noise": NOISE_DESC}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import pipeline as OP
        torch.set_num_threads(threads)
        m, s, c = (t[:2].cpu() for t in self.inputs)
        n, el = _timed_cpu(lambda: OP.lipsync_frames(self.sd_d, self.sd_e, m, s, c), 2, seconds, 8)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} frames (2-frame batches) DNet->ENet->uint8 in {el:.1f}s, torch CPU fp32, "
                          f"{threads} threads"}


class Enhance(Workload):
    metric = "enhanced 512x512 faces/sec/GPU (GFPGANv1Clean + GPEN-512, both per face)"
    unit = "faces/s"
    gflop_per_unit = 395.5 + 276.2

    def __init__(self, args, dev, rank, world=1):
        from s2v_amd import models, synth
        from s2v_amd.models import enhancer_arch as ea
        kw = dict(out_size=512, num_style_feat=512, channel_multiplier=2, decoder_load_path=None, fix_decoder=False,
                  num_mlp=8, input_is_latent=True, different_w=True, narrow=1, sft_half=True)
        self.batch = args.batch or 4
        self.sd_g = synth.synth_torch_state_dict(ea.GFPGANv1CleanParams(**kw), **synth.GFPGAN_SYNTH)
        self.sd_p = synth.synth_torch_state_dict(ea.FullGeneratorParams(512, 512, 8, 2), **synth.GPEN_SYNTH)
        self.gfpgan = models.GFPGANv1Clean(**kw)
        self.gfpgan.load_state_dict(self.sd_g)
        self.gpen = models.FullGenerator(512, 512, 8, 2)
        self.gpen.load_state_dict(self.sd_p)
        g = torch.Generator(device=dev)
        g.manual_seed(3000 + rank)
        self.inputs = [torch.rand((self.batch, 3, 512, 512), generator=g, device=dev) * 2 - 1]
        self.fn = lambda x: (self.gfpgan(x, return_rgb=False)[0], self.gpen(x)[0])  # noqa: E731
        self.config = {"workload": f"GFPGANv1Clean(return_rgb=False, randomize_noise=True) + GPEN FullGenerator-512 "
                                   f"on B={self.batch} synthetic 512x512 faces per step (gfpgan/utils.py:120, "
                                   "face_gan.py:42)"}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import enhancers
        torch.set_num_threads(threads)
        x = self.inputs[0][:1].cpu()

        def one():
            enhancers.gfpgan_forward(self.sd_g, x, return_rgb=False)
            enhancers.gpen_forward(self.sd_p, x)
        n, el = _timed_cpu(one, 1, seconds, 8)
        return {"value": round(n / el, 4), "unit": "faces/s", "cores": threads, "kind": "port",
                "sample": f"{n} faces through GFPGAN + GPEN (oracle restatement) in {el:.1f}s, torch CPU fp32, "
                          f"{threads} threads"}


class Mouth(Workload):
    metric = "mouth-region post-process frames/sec/GPU (FaceParse-512 mouth mask + 10-level Laplacian blend)"
    gflop_per_unit = 468.08            # ParseNet-512 mask path, 2*MAC (469 GF/face)
    FRAME = 720

    def __init__(self, args, dev, rank, world=1):
        from s2v_amd import models, post, synth
        from s2v_amd.models import parse_arch
        self.batch = args.batch or 8
        cfg = parse_arch.face_parse_net(512)
        self.sd = synth.synth_torch_state_dict(parse_arch.ParseNetParams(**cfg), **synth.PARSENET_SYNTH)
        net = models.ParseNet(**cfg)
        net.load_state_dict(self.sd)
        self.mb = post.MouthBlend(post.FaceParse(device=dev, net=net.eval()))
        b, S = self.batch, self.FRAME
        g = torch.Generator(device=dev)
        g.manual_seed(4000 + rank)
        self.inputs = [torch.randint(0, 256, (b, S, S, 3), generator=g, device=dev, dtype=torch.uint8)
                       for _ in range(2)]
        self.coords = [(190 + 4 * i, 510 + 4 * i, 170 + 2 * i, 530 + 2 * i) for i in range(b)]   # face boxes
        self.out = torch.empty((b, S, S, 3), dtype=torch.uint8, device=dev)
        self.fn = lambda r, f: self.mb.run_batch(r, f, self.coords, self.out)  # noqa: E731
        self.config = {"workload": f"MouthBlend.run_batch on B={b} synthetic {S}x{S} uint8 frames (GFPGAN-restored + "
                                   "original) with ~320x360 face boxes: box resize to 512, FaceParse ParseNet-512 "
                                   "mask, mask paste, three 512 resizes, 10-level Laplacian blend, clip, resize back "
                                   "(inference.py:302-313)"}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        import numpy as np
        from oracle import parse as OPARSE
        from oracle import post as OP
        torch.set_num_threads(threads)
        r, f = (t[:1].cpu().numpy() for t in self.inputs)
        y1, y2, x1, x2 = self.coords[0]

        def one():
            im = OP.resize_linear(np.ascontiguousarray(r[0, y1:y2, x1:x2]), (512, 512))
            tmp = OP.tenor2mask(OPARSE.mask_logits(self.sd, im).numpy(), OP.MOUTH_MM)[0]
            OP.blend_frame(r[0], f[0], OP.mouth_mask_full(tmp, r.shape[1:3], self.coords[0]))
        n, el = _timed_cpu(one, 1, seconds, 4)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} frames through the oracle restatement (torch CPU ParseNet + NumPy blend) in "
                          f"{el:.1f}s, {threads} threads"}


class SuperRes(Workload):
    metric = "super-resolved 720x720 -> 1440x1440 frames/sec/GPU (RealESRNet x2, RRDBNet nf=32, 23 blocks)"
    FRAME = 720

    def __init__(self, args, dev, rank, world=1):
        from s2v_amd import models, synth
        from s2v_amd.models import sr_arch
        from s2v_amd.sr import RealESRNet
        self.batch = args.batch or 2
        self.gflop_per_unit = round(sr_arch.rrdb_gflop(self.FRAME, self.FRAME, 2), 2)
        self.sd = synth.synth_torch_state_dict(sr_arch.RRDBNetParams(3, 3, scale=2, num_feat=32), **synth.RRDB_SYNTH)
        net = models.RRDBNet(3, 3, scale=2, num_feat=32, num_block=23, num_grow_ch=32)
        net.load_state_dict(self.sd)
        self.sr = RealESRNet(scale=2, device=dev, net=net)
        b, S = self.batch, self.FRAME
        g = torch.Generator(device=dev)
        g.manual_seed(5000 + rank)
        self.inputs = [torch.randint(0, 256, (b, S, S, 3), generator=g, device=dev, dtype=torch.uint8)]
        self.out = torch.empty((b, 2 * S, 2 * S, 3), dtype=torch.uint8, device=dev)
        self.fn = lambda f: self.sr.process_device(f, self.out)  # noqa: E731
        self.config = {"workload": f"RealESRNet.process (scale 2, sr_model=None: realesrnet_x2, num_feat 32, 23 RRDB) "
                                   f"on B={b} synthetic {S}x{S} uint8 BGR frames -> {2 * S}x{2 * S} uint8 "
                                   "(face_enhancement.py:102-105, real_esrnet.py:99-137)"}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import sr as OSR
        torch.set_num_threads(threads)
        img = self.inputs[0][0].cpu().numpy()
        n, el = _timed_cpu(lambda: OSR.realesrnet_process(self.sd, img, 2), 1, seconds, 4)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} {self.FRAME}x{self.FRAME} frames through the oracle restatement (torch CPU RRDBNet "
                          f"+ NumPy uint8 ends) in {el:.1f}s, {threads} threads"}


class GPEN2048(Workload):
    metric = "enhanced 2048x2048 faces/sec/GPU (GPEN-BFR-2048 FullGenerator, the CLI enhancer face GAN)"
    unit = "faces/s"
    gflop_per_unit = 419.97            # torch FlopCounterMode on oracle.enhancers.gpen_forward at 2048 (2*MAC)

    def __init__(self, args, dev, rank, world=1):
        from s2v_amd import models, synth
        from s2v_amd.models import enhancer_arch as ea
        self.batch = args.batch or 2
        self.sd = synth.synth_torch_state_dict(ea.FullGeneratorParams(2048, 512, 8, 2), **synth.GPEN_SYNTH)
        self.gpen = models.FullGenerator(2048, 512, 8, 2)
        self.gpen.load_state_dict(self.sd)
        g = torch.Generator(device=dev)
        g.manual_seed(6000 + rank)
        self.inputs = [torch.rand((self.batch, 3, 2048, 2048), generator=g, device=dev) * 2 - 1]
        self.fn = lambda x: self.gpen(x)[0]  # noqa: E731
        self.config = {"workload": f"GPEN FullGenerator(2048, 512, 8, 2) on B={self.batch} synthetic 2048x2048 faces "
                                   "per step (FaceGAN(in_size=2048) of inference.py:228-231, face_gan.py:26-42)"}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import enhancers
        torch.set_num_threads(threads)
        x = self.inputs[0][:1].cpu()
        n, el = _timed_cpu(lambda: enhancers.gpen_forward(self.sd, x), 1, seconds, 3)
        return {"value": round(n / el, 4), "unit": "faces/s", "cores": threads, "kind": "port",
                "sample": f"{n} 2048x2048 faces through GPEN-2048 (oracle restatement) in {el:.1f}s, torch CPU fp32, "
                          f"{threads} threads"}


class Face3D(Workload):
    """facing.py:100-130 face_3dmm_extraction on B frames per step: the PIL
    bicubic resize + 224 crop of every frame (one s2v_pil_resize_crop launch) and ReconNetWrapper
    (ResNet-50 + 257-coefficient head).  The per-frame POS fits (host, like NMS) and the box upload
    are precomputed once for the clip, outside the timed step."""
    metric = "3DMM coefficient frames/sec/GPU (align_img resize+crop + ReconNetWrapper resnet50, facing.py:100-130)"
    gflop_per_unit = 8.175             # torch FlopCounterMode on oracle.face3d.recon_forward at 224x224 (2*MAC)
    FRAME = 700                        # examples/face/1.mp4 is 700x700

    def __init__(self, args, dev, rank, world=1):
        import numpy as np
        from s2v_amd import face3d, models, ops, synth
        from s2v_amd.models.face3d_arch import ReconNetWrapperParams
        from s2v_amd.ops import NHWC
        self.batch = b = args.batch or 64
        self.sd = synth.synth_torch_state_dict(ReconNetWrapperParams(), **synth.RETINA_SYNTH)
        self.net = models.ReconNetWrapper()
        self.net.load_state_dict(self.sd)
        self.net.eval()
        S = self.FRAME
        lm3d = np.array([[-0.31, 0.29, 0.41], [0.31, 0.29, 0.41], [0.0, 0.0, 0.65], [-0.25, -0.36, 0.44],
                         [0.25, -0.36, 0.44]])
        rng = np.random.default_rng(8000 + rank)
        t0 = time.perf_counter()
        boxes = []
        for i in range(b):             # a face of ~220-300 px eye-to-mouth scale drifting over the frame
            d = 180 + 60 * rng.random()
            cx, cy = S / 2 + 40 * rng.standard_normal(2)
            base = np.array([[-0.5, 0.45], [0.5, 0.45], [0.0, 0.0], [-0.42, -0.62], [0.42, -0.62]])
            lm5 = base * d + np.array([cx, S - 1 - cy]) + rng.standard_normal((5, 2))
            _, box, _ = face3d.align_params(S, S, lm5.astype(np.float32), lm3d)
            boxes.append(box)
        self.host = {"pos_fits_ms": round(1e3 * (time.perf_counter() - t0), 2)}
        g = torch.Generator(device=dev)
        g.manual_seed(8000 + rank)
        frames = torch.randint(0, 256, (b, S, S, 3), generator=g, device=dev, dtype=torch.uint8)
        self.params = face3d.box_params(boxes, S, S, dev)
        self.x4 = NHWC.empty(b, 224, 224, 4, dev)
        self.out = torch.empty((b, 257), device=dev)
        self.boxes = boxes
        ctx = ops.Ctx(dev)

        def step(f):
            face3d.resize_crop_params(ctx, f, self.params, self.x4)
            self.out.copy_(self.net.forward_nhwc(self.x4))
            return self.out
        self.inputs = [frames]
        self.fn = step
        self.config = {"workload": f"face_3dmm_extraction on B={b} synthetic {S}x{S} uint8 RGB frames per step: "
                                   "PIL bicubic resize + 224x224 crop (s2v_pil_resize_crop) -> ReconNetWrapper "
                                   "resnet50 -> [B, 257] coefficients", "host_precompute": self.host}

    def forward(self):
        return self.fn(*self.inputs)

    def cpu(self, threads, seconds):
        from oracle import face3d as O3
        torch.set_num_threads(threads)
        frames = self.inputs[0][:4].cpu().numpy()

        def one(i=[0]):
            k = i[0] % 4
            i[0] += 1
            im = O3.pil_resize_crop(frames[k], self.boxes[k])
            x = torch.tensor(im / 255., dtype=torch.float32).permute(2, 0, 1)[None]
            O3.recon_forward(self.sd, x)
        n, el = _timed_cpu(one, 1, seconds, 64)
        return {"value": round(n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": f"{n} {self.FRAME}x{self.FRAME} frames through the oracle restatement (NumPy Pillow "
                          f"resample + crop, torch CPU ResNet-50) in {el:.1f}s, {threads} threads"}


class Clip(Pipeline):
    """BASELINE configs[3] (configs[2] at N = 1): the 1000-frame clip sharded over the ranks by
    pipeline.run_sharded — RCCL broadcast of the per-clip host data, device mel + windows, host
    coefficient windows, DNet -> ENet(+LNet) -> uint8 per rank (graph replay per 16-frame batch),
    gather of the uint8 frames to rank 0.  Total work per step is fixed (strong scaling)."""
    metric = "full-clip lip-sync frames/sec (1000-frame clip sharded over the GPUs, DNet->LNet->ENet->uint8)"
    graphable = False
    scaling = "strong"

    def __init__(self, args, dev, rank, world=1):
        import numpy as np
        from s2v_amd import pipeline
        super().__init__(args, dev, rank, world)
        self.pipe.graph = not args.no_graph
        self.pipe.lanes = max(1, args.lanes)
        n = args.frames
        rng = np.random.default_rng(0)
        t = np.arange(n * 640) / 16000.0                      # 40 s of 16 kHz audio per 1000 frames at 25 fps
        wav = (0.1 * rng.standard_normal(t.size) + 0.2 * (np.sin(2 * np.pi * 220 * t) + np.sin(2 * np.pi * 440 * t)
                                                          + np.sin(2 * np.pi * 1000 * t))).astype(np.float32)
        sem = rng.standard_normal((n, 262)).astype(np.float32)
        sem[:, -3] = 1.0 + 0.1 * rng.random(n)
        expr = rng.standard_normal(64).astype(np.float32)
        self.host = (wav, sem, expr) if rank == 0 else (None, None, None)
        self.n = n
        s0, s1 = pipeline.shard_range(n, rank, world)
        g = torch.Generator(device=dev)
        g.manual_seed(7000 + rank)
        self.src = torch.rand((s1 - s0, 3, 256, 256), generator=g, device=dev) * 2 - 1   # resident before timing
        self.result = None
        self.config = {"workload": f"run_sharded over a {n}-frame clip (40 ms of 16 kHz audio per frame): broadcast "
                                   "wav/semantic/expression, mel + 16-column windows, coefficient windows, "
                                   "DNet -> uint8 ref -> ENet(+LNet) -> uint8 384x384 per rank, gather to rank 0 "
                                   "(inference.py:204-288, facing.py:176-191)", "clip_frames": n,
                       "styleconv_noise": NOISE_DESC}

    def units_per_step(self, world):
        # the clip's mel windows (inference.py:209-222: 997 for 40 s); only rank 0 holds the frames
        return int(self.result.shape[0]) if self.result is not None else 0

    def step(self):
        from s2v_amd import pipeline
        self.result = pipeline.run_sharded(self.pipe, *self.host, lambda s, e: self.src[: e - s])
        return self.result


WORKLOADS = {"lipsync": LipSync, "lnet": LNetOnly, "dnet": DNetOnly, "pipeline": Pipeline, "enhance": Enhance, "mouth": Mouth,
             "sr": SuperRes, "gpen2048": GPEN2048, "face3d": Face3D, "clip": Clip, "selftest": SelfTest}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawned(rank, args, port):
    """Entry of a worker started by ``launch`` (a fresh interpreter: nothing has touched a GPU)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    worker(args)


def launch(args):
    """``bench.py --gpus N`` outside torchrun: start N fresh worker processes (spawn, one per GPU)
    and wait for them; this process never touches a device."""
    import torch.multiprocessing as mp
    mp.start_processes(_spawned, args=(args, _free_port()), nprocs=args.gpus, join=True, start_method="spawn")


def main():
    args = parse()
    if args.device == "cpu" and args.workload != "selftest":
        raise SystemExit("--device cpu runs only the launcher self-test (--workload selftest)")
    if "WORLD_SIZE" in os.environ:                 # torchrun (the driver's N > 1 launch)
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; using WORLD_SIZE",
                  file=sys.stderr)
        return worker(args)
    if args.gpus > 1:
        return launch(args)
    return worker(args)


def worker(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = args.device == "cuda"
    if cuda:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    world_seen = 1
    if world > 1:
        import torch.distributed as dist
        if cuda:
            dist.init_process_group("nccl", device_id=dev)     # RCCL
        else:
            dist.init_process_group("gloo")
        world_seen = dist.get_world_size()
    from s2v_amd.runtime import GraphRunner, LaneRunner

    from s2v_amd import ops
    wl = WORKLOADS[args.workload](args, dev, rank, world)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        if cuda:
            torch.cuda.synchronize()

    def capture(fn_lane, stamper):
        """The step as captured lanes (or one graph); with ``stamper`` every launch of the dominant
        kernel records its in-kernel clock stamps (ops.STAMP) into the stamper's per-lane buffers."""
        def wrap(lane, *x):
            if stamper is not None:
                stamper.begin(lane)
            return fn_lane(lane, *x)
        ops.STAMP = stamper
        try:
            if args.lanes > 1 and hasattr(wl, "fn_lane"):
                return LaneRunner(wrap, list(wl.inputs), lanes=args.lanes, warmup=1)
            return GraphRunner(lambda *x: wrap(0, *x), list(wl.inputs), warmup=1)
        finally:
            ops.STAMP = None

    def timed(prec, stamper=None):
        """Capture (or not) the step in conv arithmetic ``prec``, warm up, time args.steps steps
        between barriers; returns the max over ranks of the elapsed seconds."""
        ops.set_precision(prec)
        if not wl.graphable:
            step = wl.step
            for _ in range(max(1, args.warmup)):
                step()
        elif args.no_graph:
            step = wl.forward
            for _ in range(max(1, args.warmup)):
                step()
        else:
            fn_lane = wl.fn_lane if hasattr(wl, "fn_lane") else (lambda lane, *x: wl.fn(*x))
            runner = capture(fn_lane, stamper)
            step = runner.replay
            for _ in range(max(args.warmup, args.lanes)):
                step()
        if stamper is not None:
            stamper.arm()                      # counters read and stamp slots cleared before the timed region
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        return el

    # roofline pre-pass (rank 0, un-graphed, launches serialised): the dominant kernel symbol, its
    # algorithmic FLOPs per launch and its isolated duration; the timed run below then stamps that
    # kernel's launches in-kernel, so the reported duration is the one of the benchmarked,
    # graph-replayed, overlapped launches (what rocprofv3 --kernel-trace sees for the same command)
    pre, stamper = None, None
    if rank == 0 and not args.no_roofline and cuda and wl.graphable:
        ops.set_precision(args.precision)
        pre = live_roofline(wl.forward, args.workload)
        if not args.no_graph:
            # the dominant symbol, the next three by time and the persistent form of the dominant one
            # (the style encoder's grid-capped launches, which the serialised pre-pass does not make)
            ks = {k: v["launches"] for k, v in pre["per_kernel"].items()}
            top = sorted(pre["per_kernel"], key=lambda k: -pre["per_kernel"][k]["ms"])[:4]
            kern = {k: ks[k] + 4 for k in top}
            if "conv_igemm_x3<" in pre["kernel"]:
                kern[pre["kernel"].replace("conv_igemm_x3<", "conv_igemm_x3_persist<")] = ks[pre["kernel"]] + 4
            stamper = Stamper(kern, args.warmup + args.steps + 2 * args.lanes + 4, dev)
    elapsed = timed(args.precision, stamper)
    if args.dump_stamps and stamper is not None:
        with open(args.dump_stamps, "w") as f:
            json.dump({"clock_hz": Stamper.CLOCK_HZ, "kernel": pre["kernel"], "launches": stamper.raw()}, f)
    if cuda:
        ops.check_all_ranges(args.workload)     # f16x3 range guard: raises if a timed launch overflowed
    units = wl.units_per_step(world) * args.steps
    value = units / elapsed
    config = dict(wl.config)
    config.update({"global_batch": wl.units_per_step(world), "batch_per_gpu": wl.batch,
                   "parallelism": f"frame-shard x{world} (no data-path collective)", "graph": not args.no_graph,
                   "lanes": args.lanes if (wl.graphable and not args.no_graph and hasattr(wl, "fn_lane")) else 1,
                   "world_size_seen": world_seen,
                   "achieved_tflops_algorithmic": round(value * wl.gflop_per_unit / 1e3, 2),
                   "gflop_per_unit": wl.gflop_per_unit})
    if args.workload == "clip":
        config["parallelism"] = (f"frame-shard x{world}: RCCL broadcast of the clip inputs + gather of the uint8 "
                                 "frames to rank 0 inside the step" if world > 1 else "single GPU")
    result = {
        "metric": wl.metric, "value": round(value, 3), "unit": wl.unit, "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": wl.scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic", "config": config,
    }
    config["conv_arith"] = ARITH[args.precision]
    if pre is not None:
        from s2v_amd.engine import enet as _enet
        if args.workload in ("lipsync", "pipeline", "clip") and _enet.OVERLAP and _enet.style_grid(dev):
            pre["grid_cap_blocks"] = _enet.style_grid(dev)
            pre["cus"] = torch.cuda.get_device_properties(dev).multi_processor_count
        result["roofline"] = replay_roofline(pre, stamper)
        for k in ("per_kernel", "_grids", "_workload", "grid_cap_blocks", "cus"):
            result["roofline"].pop(k, None)
        if args.workload in ("lipsync", "pipeline", "clip") and _enet.OVERLAP and _enet.style_grid(dev):
            result["roofline"]["grid_cap"] = (
                f"the style encoder's launches of the 256x256 tile (beside LNet) run as {_enet.style_grid(dev)} "
                "persistent blocks on half the CUs (conv_igemm_x3_persist, s2v_conv_params.grid_cap): reported "
                "separately under by_kernel; the headline entry is the full-grid launches only")
    elif rank == 0 and not args.no_roofline and cuda:
        result["roofline"] = live_roofline(wl.forward, args.workload)
        for k in ("per_kernel", "_grids", "_workload"):
            result["roofline"].pop(k, None)
    if world == 1 and not args.no_alt and cuda and wl.graphable:
        result["alt_precision"] = {}
        for other in ARITH:
            if other == args.precision:
                continue
            el = timed(other)
            result["alt_precision"][other] = {"value": round(units / el, 3),
                                              "ms_per_step": round(1e3 * el / args.steps, 3)}
        ops.set_precision(args.precision)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cuda:
        result["cpu_baseline"] = wl.cpu(args.cpu_threads or host_threads(), args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
