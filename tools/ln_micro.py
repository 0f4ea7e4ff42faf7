#!/usr/bin/env python3
"""LayerNorm2d (s2v_layernorm2d: ln_stats + ln_apply4[_pool]) graph-timed at the DNet / LNet shapes;
algorithmic bytes = fp32 read of x twice (statistics, apply) + fp32 write of y.
    python tools/ln_micro.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from kernel_floor import graph_us  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = ops.Ctx(dev)
    for (n, h, w, c, pool) in ((16, 256, 256, 64, False), (16, 256, 256, 64, True), (16, 128, 128, 128, True),
                               (16, 64, 64, 256, False), (16, 96, 96, 64, False), (16, 48, 48, 128, True),
                               (16, 12, 12, 512, False)):
        x = NHWC(torch.randn(n, h, w, c, device=dev))
        wt, b = torch.randn(c, device=dev), torch.randn(c, device=dev)
        oh, ow = (h // 2, w // 2) if pool else (h, w)
        y = NHWC.empty(n, oh, ow, c, dev)
        fn = lambda: ops.layernorm2d(ctx, x, wt, b, y, act=ops.ACT_LRELU, alpha=0.2, pool=pool)  # noqa: E731
        us = graph_us(fn, 10)
        byt = 4.0 * n * c * (2 * h * w + oh * ow)
        print(f"{n}x{h}x{w}x{c} pool={int(pool)}: {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s (stats + apply)", flush=True)


if __name__ == "__main__":
    main()
