#!/usr/bin/env python3
"""Every conv launch of an engine forward with the plan libs2v's planner picks for it, on the CPU.

The engine runs with torch.ops.s2v replaced by a stand-in whose conv ops fill an s2v_conv_params from
their arguments (the same fields csrc/torch_launch.cpp fills) and call the host-only
s2v_conv2d_plan of the in-tree libs2v.so (the device CU count falls back to 256 without a GPU); every
other op is a no-op.  Nothing is computed.

    python tools/plan_table.py lnet|enet|dnet [--batch 16] [--csv out.csv]
"""
import argparse
import ctypes
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import _lib, ops  # noqa: E402


def _nv(t, step=1):
    n, h, w, c = t.shape
    return n, h, w, c, t.stride(2) // step, t.stride(0)


class PlanOps:
    def __init__(self, lib):
        self.lib = lib
        self.rows = []
        from s2v_amd import torch_ops
        self.ns = torch_ops.load()

    group = None

    def group_begin_(self):
        self.group = []

    def group_abort_(self):
        self.group = None

    def group_end_(self, ws, dry):
        members, self.group = self.group, None
        arr = (_lib.ConvParams * len(members))(*[p for p, _ in members])
        out = (ctypes.c_int * 5)()
        rc = self.lib.s2v_conv2d_group_plan(arr, len(members), out)
        if rc:
            self.rows.append(("group!", tuple(e for _, e in members), [0] * 11))
        else:
            self.rows.append(("group", tuple(e[:7] for _, e in members), [out[0] + 1] + list(out)[1:1 + len(members)]))
        return [0, 0 if rc else 1]

    def _plan(self, p, what, extra):
        out = (ctypes.c_int * 11)()
        rc = self.lib.s2v_conv2d_plan(ctypes.byref(p), out)
        if rc:
            raise RuntimeError(f"{what}: {ops._lib.load().s2v_last_error().decode()}")
        plan = list(out)
        if self.group is not None:
            self.group.append((p, extra))
            return [0] + plan
        self.rows.append((what, extra, plan))
        return [0] + plan

    def conv2d_(self, x, y, wt, wt_split, wt_scale, cout, kernel, stride, padding, dilation, in_mode, pad_mode, prec,
                scale, shift, in_scale, nc_scale, pre_act, pre_alpha, pix_add, pix_w, res, res_offset, res_after,
                act, alpha, out_step, out_pool, x_split, ws, grid_cap, force_tile, force_splits, *rest):
        p = _lib.ConvParams()
        n, h, w, c, xcs, _ = _nv(x)
        yn, yh, yw, yc, ycs, _ = _nv(y, out_step)
        p.x, p.n, p.h, p.w, p.cin, p.xcs = x.data_ptr(), n, h, w, c, xcs
        p.in_mode, p.pad_mode, p.pre_act = in_mode, pad_mode, pre_act
        p.in_scale = in_scale.data_ptr() if in_scale is not None else None
        p.in_scale_ns = in_scale.stride(0) if in_scale is not None else 0
        p.kh, p.kw = kernel
        p.sh, p.sw = stride
        p.ph, p.pw = padding
        p.dh, p.dw = dilation
        p.wt, p.npad, p.kpad, p.cout = wt.data_ptr(), wt.shape[0], wt.shape[1], cout
        f = 2 if out_pool else 1
        p.y, p.oh, p.ow, p.ycs = y.data_ptr(), yh * f, yw * f, ycs
        if out_step > 1:
            p.out_step, p.out_full_h, p.out_full_w = out_step, yh * out_step, yw * out_step
        p.nc_scale = nc_scale.data_ptr() if nc_scale is not None else None
        p.pix_add = pix_add.data_ptr() if pix_add is not None else None
        if res is not None:
            _, rh, rw, _, rcs, _ = _nv(res, out_step)
            p.res, p.res_cs, p.res_h, p.res_w = res.data_ptr(), rcs, rh, rw
        p.act, p.batch, p.out_pool, p.x_split, p.prec = act, 1, int(out_pool), int(x_split), prec
        p.force_tile, p.force_splits, p.grid_cap = force_tile, force_splits, grid_cap
        p.wt_x3 = wt.data_ptr() if prec else None
        return self._plan(p, "conv", (n, h, w, c, yh * f, yw * f, cout, p.kh, p.kw, grid_cap))

    def modulated_conv2d_(self, x, y, wt, s, d, wbuf, cout, kernel, padding, in_mode, prec, x_split, scale, shift,
                          pix_add, pix_w, res, res_after, act, alpha, ws, force_splits, st0, st1, st2, x_scale, flag,
                          dry, d2s=0, force_tile=0, *rest):
        p = _lib.ConvParams()
        n, h, w, c, xcs, xns = _nv(x)
        p.x, p.n, p.h, p.w, p.cin, p.xcs = x.data_ptr(), 1, h, w, c, xcs
        p.batch, p.x_bs = n, xns
        p.in_mode = in_mode
        p.kh, p.kw = kernel
        p.sh = p.sw = p.dh = p.dw = 1
        p.ph, p.pw = padding
        p.wt, p.npad, p.kpad, p.cout = wbuf.data_ptr(), wt.shape[0], wt.shape[1], cout
        p.w_bs = wt.shape[0] * wt.shape[1]
        if d2s:
            oh, ow = y.shape[1] // 2, y.shape[2] // 2
            p.out_step, p.out_full_h, p.out_full_w, p.d2s_cout = 2, y.shape[1], y.shape[2], cout // 4
            p.ycs = y.stride(2)
        else:
            oh, ow = y.shape[1], y.shape[2]
            p.ycs = y.stride(2)
        p.y, p.oh, p.ow = y.data_ptr(), oh, ow
        p.pix_add = pix_add.data_ptr() if pix_add is not None else None
        if res is not None:
            p.res, p.res_cs, p.res_h, p.res_w = res.data_ptr(), res.stride(2), res.shape[1], res.shape[2]
        p.act, p.prec, p.x_split, p.force_splits, p.force_tile = act, prec, int(x_split), force_splits, force_tile
        p.wt_x3 = wbuf.data_ptr() if prec else None
        return self._plan(p, "modconv", (n, h, w, c, oh, ow, cout, p.kh, p.kw, 0))

    def gemm_kn_(self, a, b, out, batch, a_bs, b_bs, out_bs, res, res_bs, act, alpha, prec, ws, force_tile,
                 force_splits, dry, *rest):
        p = _lib.ConvParams()
        M, K, N = a.shape[-2], a.shape[-1], b.shape[-1]
        p.x, p.n, p.h, p.w, p.cin, p.xcs = a.data_ptr(), 1, 1, M, K, K
        p.kh = p.kw = p.sh = p.sw = p.dh = p.dw = 1
        p.wt, p.cout, p.b_kn, p.ldb, p.prec = b.data_ptr(), N, 1, N, prec
        p.y, p.oh, p.ow, p.ycs = out.data_ptr(), 1, M, N
        p.batch, p.x_bs, p.w_bs, p.y_bs = batch, a_bs, b_bs, out_bs
        p.force_tile, p.force_splits = force_tile, force_splits
        return self._plan(p, "gemm", (batch, 1, M, K, 1, M, N, 1, 1, 0))

    def __getattr__(self, name):
        schema = getattr(self.ns, name).default._schema
        ret = str(schema.returns[0].type) if schema.returns else ""

        def fn(*a):
            return [0] * 12 if ret.startswith("List") else 0 if ret == "int" else None
        return fn


def run(which, batch):
    from helpers import synth_sd
    from s2v_amd import synth
    lib = _lib.load()
    po = PlanOps(lib)
    ops.S2V = po
    ops._require_cuda = lambda t, what: None
    ctx = ops.Ctx("cpu")
    if which == "lnet":
        from s2v_amd.engine.lnet import LNetEngine
        eng = LNetEngine(synth_sd("lnet"), "cpu")
        face6 = ops.NHWC(torch.zeros(batch, 96, 96, 6))
        eng.forward(ctx, torch.zeros(batch, 1, 80, 16), face6, ops.NHWC(torch.zeros(batch, 96, 96, 4)), pad_rgb=True)
    elif which == "enet":
        from s2v_amd.engine.enet import ENetEngine
        eng = ENetEngine(synth_sd("enet"), "cpu")
        eng.forward(ctx, torch.zeros(batch, 1, 80, 16), torch.zeros(batch, 6, 256, 256), torch.zeros(batch, 3, 256, 256),
                    torch.empty(batch, 3, 384, 384), torch.empty(batch, 3, 96, 96))
    elif which == "dnet":
        from s2v_amd.engine.dnet import DNetEngine
        eng = DNetEngine(synth_sd("dnet"), "cpu")
        eng.forward(ctx, torch.zeros(batch, 3, 256, 256), torch.zeros(batch, 73, 26))
    return po.rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=("lnet", "enet", "dnet"))
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    rows = run(a.which, a.batch)
    syms = Counter()
    nsplit = 0
    for what, shp, plan in rows:
        if what.startswith("group"):
            print(f"{what:8s} members (n,h,w,cin,oh,ow,cout)={shp} x3 tile cfg (force_tile)={plan[0]} splits={plan[1:]}")
            syms[what + f" tile {plan[0]}"] += 1
            nsplit += any(v > 1 for v in plan[1:])
            continue
        sym = ops.plan_symbol(plan)
        syms[sym[10:60]] += 1
        nsplit += plan[5] > 1
        print(f"{what:8s} n,h,w,cin,oh,ow,cout,kh,kw,cap={shp} splits={plan[5]} {sym[10:70]}")
    print(f"{len(rows)} conv launches, {nsplit} with split-K (+{nsplit} reduce launches)")
    for k, v in syms.most_common():
        print(f"  {v:4d} {k}")


if __name__ == "__main__":
    main()
