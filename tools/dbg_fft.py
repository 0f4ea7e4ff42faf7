#!/usr/bin/env python3
"""Debug: s2v_irfft2 / s2v_rfft2 error pattern against torch.fft (max |err| by h, w, channel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC  # noqa: E402

dev = "cuda"
ctx = ops.Ctx(dev)
for (n, h, c) in ((2, 48, 48), (2, 24, 96), (2, 12, 384)):
    w = h
    wf = w // 2 + 1
    g = torch.Generator().manual_seed(3)
    tables = ops.fft_tables(h, w, dev)
    sp = torch.rand((n, h * wf, 2 * c), generator=g, dtype=torch.float64) * 2 - 1
    y = NHWC.empty(n, h, w, c, dev)
    ops.irfft2(ctx, sp.float().to(dev), tables, y)
    z = sp.reshape(n, h, wf, 2, c)
    ref = torch.fft.irfftn(torch.complex(z[..., 0, :], z[..., 1, :]), s=(h, w), dim=(1, 2), norm="ortho")
    e = (y.t.double().cpu() - ref).abs()
    print(f"irfft {h}: max {e.max():.3e} mean {e.mean():.3e}; by h {[round(float(v), 6) for v in e.amax(dim=(0, 2, 3))]}")
    print(f"   by w {[round(float(v), 6) for v in e.amax(dim=(0, 1, 3))]}")
    print(f"   by c {[round(float(v), 6) for v in e.amax(dim=(0, 1, 2))][:16]}")
    x = torch.rand((n, h, w, c), generator=g, dtype=torch.float64) * 2 - 1
    spec = torch.empty((n, h * wf, 2 * c), device=dev)
    ops.rfft2(ctx, NHWC(x.float().to(dev)), tables, spec)
    r = torch.fft.rfftn(x, dim=(1, 2), norm="ortho")
    got = spec.double().cpu().reshape(n, h, wf, 2, c)
    e2 = torch.maximum((got[..., 0, :] - r.real).abs(), (got[..., 1, :] - r.imag).abs())
    print(f"rfft {h}: max {e2.max():.3e} mean {e2.mean():.3e}; by u {[round(float(v), 6) for v in e2.amax(dim=(0, 2, 3))]}")
