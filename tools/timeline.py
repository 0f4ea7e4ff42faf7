#!/usr/bin/env python3
"""Phase timeline of graph-replayed ENet(+LNet) steps from a rocprofv3 --kernel-trace database.

A step starts at its ``fill_kernel`` (the style encoder's input, first kernel of ENet.forward) and
its StyleConv tail at the first kernel launched after LNet's last FourierUnit transform and the style
encoder's last persistent conv have ended.  Per phase: wall time, busy
time (union of kernel intervals) and the summed kernel time (> busy when kernels overlap), plus the
top kernels of each phase.  Usage: timeline.py run_results.db [--steps N]"""
import sqlite3
import sys
from collections import defaultdict


def load(path):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    s = "start" if "start" in cols else "start_ns"
    e = "end" if "end" in cols else "end_ns"
    return [(n, a, b) for n, a, b in db.execute(f"select name, {s}, {e} from kernels order by {s}")]


def busy(iv):
    tot, cur_a, cur_b = 0, None, None
    for a, b in sorted(iv):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
    ks = load(path)
    starts = [i for i, (n, a, b) in enumerate(ks) if n.startswith("s2v::fill_kernel")]
    if len(starts) < 2:
        print("no step markers (fill_kernel) found")
        return
    for si in range(max(0, len(starts) - 1 - nsteps), len(starts) - 1):
        i0, i2 = starts[si], starts[si + 1]
        step = ks[i0:i2]
        t0, t2 = step[0][1], ks[i2][1]
        # the tail starts with the first kernel launched after both branches ended: LNet's last FourierUnit
        # transform and the style encoder's last persistent conv (the StyleConv weights are modulated on the
        # encoder's side stream since r06, so a modulate_weights kernel no longer marks the tail)
        ends = [b for n, a, b in step if "fft2" in n or n.startswith("void s2v::conv_igemm_x3_persist<")]
        i1 = next((i for i, (n, a, b) in enumerate(step) if ends and a >= max(ends)), None)
        if i1 is None:
            i1 = next((i for i, (n, a, b) in enumerate(step) if "modulate_weights" in n), None)
        t1 = step[i1][1] if i1 is not None else t2
        print(f"step {si}: {(t2 - t0) / 1e3:8.1f} us, {len(step)} kernels")
        for name, lo, hi in (("encoder+LNet", t0, t1), ("StyleConv tail", t1, t2)):
            iv = [(max(a, lo), min(b, hi)) for n, a, b in step if b > lo and a < hi]
            per = defaultdict(float)
            for n, a, b in step:
                if b > lo and a < hi:
                    per[n.split("(")[0][:70]] += (min(b, hi) - max(a, lo)) / 1e3
            tot = sum(b - a for a, b in iv)
            print(f"  {name:15s} wall {(hi - lo) / 1e3:8.1f} us  busy {busy(iv) / 1e3:8.1f}  kernel-sum {tot / 1e3:8.1f}  "
                  f"kernels {len(iv)}")
            for n, t in sorted(per.items(), key=lambda kv: -kv[1])[:8]:
                print(f"      {t:8.1f} us  {n}")
            if name == "encoder+LNet":
                # the two branches' ends: LNet's last FourierUnit transform, the style encoder's last
                # 256x256-tile conv (LNet has none)
                fft = [b for n, a, b in step if "fft2" in n and a < hi]
                big = [b for n, a, b in step if (n.startswith("void s2v::conv_igemm_x3<256, 256") or
                                                  n.startswith("void s2v::conv_igemm_x3_persist<")) and a < hi]
                if fft and big:
                    print(f"    LNet last FFT ends {(max(fft) - lo) / 1e3:8.1f} us, style encoder's last 256x256 conv "
                          f"(persistent or full-grid) ends {(max(big) - lo) / 1e3:8.1f} us")


if __name__ == "__main__" and not {"--lnet", "--ffc", "--seq"} & set(sys.argv):
    main()


def lnet_levels(path):
    """LNet forward: wall time per decoder level (first .. last FourierUnit transform of that size: the
    separate rfft2 / irfft2 kernels, or the fused ffc_spec_fwd / ffc_spec_inv at a fused level) of the
    last forward in the trace, with busy time and kernel count."""
    ks = load(path)
    hs = (12, 24, 48)

    def fwd(n, h):
        return n.startswith(f"void s2v::rfft2_mf<{h},") or n.startswith(f"void s2v::ffc_spec_fwd<{h},")

    def inv(n, h):
        return n.startswith(f"void s2v::irfft2_mf<{h},") or n.startswith(f"void s2v::ffc_spec_inv<{h},")
    for h in hs:
        inv_i = [i for i, (n, a, b) in enumerate(ks) if inv(n, h)]
        fwd_i = [i for i, (n, a, b) in enumerate(ks) if fwd(n, h)]
        if not inv_i or len(fwd_i) < 18:
            print(f"level {h}: {len(fwd_i)} forward transforms in the trace")
            continue
        last = inv_i[-1]
        first = [i for i in fwd_i if i <= last][-18]       # the last forward's 18 FFCs of this size
        seg = [(a, b) for n, a, b in ks[first: last + 1]]
        lo, hi = ks[first][1], max(b for a, b in seg)
        print(f"level {h:2d}x{h:<2d}: wall {(hi - lo) / 1e3:8.1f} us  busy {busy(seg) / 1e3:8.1f}  "
              f"kernels {len(seg)}  per FFC {(hi - lo) / 18e3:6.1f} us")


if __name__ == "__main__" and "--lnet" in sys.argv:
    lnet_levels(sys.argv[1])


def lnet_ffc(path, k=4):
    """Every kernel of the k-th FFC of each decoder level in the last LNet forward of the trace: the
    kernels that start between the (k-1)-th and the (k+1)-th rfft2 launch of that size, sorted by start,
    as start offset / duration / end offset / name, so the per-FFC critical path can be read off."""
    ks = load(path)
    for h in (12, 24, 48):
        rf = [i for i, (n, a, b) in enumerate(ks) if n.startswith(f"void s2v::rfft2_mf<{h},")]
        if len(rf) < 18:
            print(f"level {h}: {len(rf)} rfft2 launches in the trace")
            continue
        lo, hi = ks[rf[-18 + k - 1]][1], ks[rf[-18 + k + 1]][1]
        seg = sorted((a, b, n) for n, a, b in ks if lo <= a < hi)
        t0 = ks[rf[-18 + k]][1]
        print(f"level {h}x{h}, FFC {k}: window {(hi - lo) / 2e3:.1f} us per FFC, {len(seg)} kernels, offsets vs its rfft2")
        for a, b, n in seg:
            print(f"  {(a - t0) / 1e3:+8.1f} {(b - a) / 1e3:7.1f} us -> {(b - t0) / 1e3:+8.1f}  {n.split('(')[0][:90]}")


if __name__ == "__main__" and "--ffc" in sys.argv:
    lnet_ffc(sys.argv[1])


def step_sequence(path, marker, nth=2):
    """Every kernel of one graph-replayed step (from the ``nth``-last launch of ``marker`` to the next),
    in start order: start offset, duration, idle gap before it, grid (when the trace has it), name;
    then the step's kernel time grouped by kernel name.  Usage: timeline.py db --seq MARKER"""
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    s = "start" if "start" in cols else "start_ns"
    e = "end" if "end" in cols else "end_ns"
    gcols = [c for c in ("grid_size_x", "grid_size_y", "grid_size_z", "grid_x", "grid_y", "grid_z") if c in cols]
    sel = ", ".join(["name", s, e] + gcols)
    ks = list(db.execute(f"select {sel} from kernels order by {s}"))
    mk = [i for i, k in enumerate(ks) if k[0].startswith(marker) or marker in k[0].split("(")[0]]
    if len(mk) < nth + 1:
        print(f"{len(mk)} launches of {marker!r} in the trace")
        return
    i0, i1 = mk[-nth - 1], mk[-nth]
    seg = ks[i0:i1]
    t0, prev = seg[0][1], seg[0][1]
    per = defaultdict(lambda: [0, 0.0])
    print(f"step: {(ks[i1][1] - t0) / 1e3:.1f} us, {len(seg)} kernels (columns: offset, duration, gap, grid, name)")
    for k in seg:
        n, a, b = k[0], k[1], k[2]
        g = "x".join(str(v) for v in k[3:]) if gcols else ""
        print(f"  {(a - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f} {(a - prev) / 1e3:7.1f} {g:>16s}  {n.split('(')[0][:80]}")
        prev = max(prev, b)
        p = per[n.split("(")[0][:80]]
        p[0] += 1
        p[1] += (b - a) / 1e3
    print("by kernel:")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t:9.1f} us {c:5d}  {n}")


if __name__ == "__main__" and "--seq" in sys.argv:
    step_sequence(sys.argv[1], sys.argv[sys.argv.index("--seq") + 1])
