#!/usr/bin/env python3
"""Bandwidth of the GPEN native-op drop-ins (torch.ops.s2v.fused_bias_act / upfirdn2d, the
reference's fused_act.py / upfirdn2d.py CUDA-extension call forms) at GPEN-512 activation shapes
(FullGenerator(512, 512, 8, 2): StyledConv outputs concatenated with the noise branch -> 2C
channels, gpen_model.py:340-363; ToRGB / Upsample FIR x2, :37-56).  Algorithmic bytes = fp32 read of
the input (+ bias) + fp32 write of the output.   python tools/native_ops_bw.py [--iters 50]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import torch_ops  # noqa: E402

CH = {4: 512, 8: 512, 16: 512, 32: 512, 64: 512, 128: 256, 256: 128, 512: 64}


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = "cuda"
    k = torch.tensor([1.0, 3.0, 3.0, 1.0], device=dev)
    k = (k[None, :] * k[:, None]) / 64.0
    rows = []
    for r in (64, 128, 256, 512):
        c = 2 * CH[r]
        x = torch.randn(a.batch, c, r, r, device=dev)
        b = torch.randn(c, device=dev)
        us = timed(lambda: torch_ops.fused_leaky_relu(x, b), a.iters)
        nb = 2 * x.numel() * 4 + b.numel() * 4
        rows.append({"op": "fused_bias_act", "shape": list(x.shape), "us": round(us, 2), "bytes": nb,
                     "GBps": round(nb / us / 1e3, 1), "frac_of_8TBps": round(nb / us / 8e6, 4)})
        xs = torch.randn(a.batch, 3, r // 2, r // 2, device=dev)
        for name, up, pad in (("upfirdn2d up2 (ToRGB skip)", 2, (2, 1)), ("upfirdn2d blur", 1, (1, 1))):
            src = xs if up == 2 else torch.randn(a.batch, CH[r], r, r, device=dev)
            us = timed(lambda: torch_ops.upfirdn2d(src, k * (4 if up == 2 else 1), up=up, down=1, pad=pad), a.iters)
            out_n = src.numel() * up * up
            nb = (src.numel() + out_n) * 4
            rows.append({"op": name, "shape": list(src.shape), "us": round(us, 2), "bytes": nb,
                         "GBps": round(nb / us / 1e3, 1), "frac_of_8TBps": round(nb / us / 8e6, 4)})
    for rr in rows:
        print(f"{rr['op']:28s} {str(rr['shape']):22s} {rr['us']:9.1f} us {rr['bytes'] / 1e6:9.1f} MB "
              f"{rr['GBps']:8.0f} GB/s  {rr['frac_of_8TBps']:.3f}")
    if a.out:
        json.dump({"method": "HIP events over --iters back-to-back calls of the torch custom op (includes the "
                             "op's output allocation); algorithmic fp32 bytes", "rows": rows},
                  open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
