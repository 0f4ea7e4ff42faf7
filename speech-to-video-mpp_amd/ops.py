"""Tensor-level wrappers over the C ABI (libs2v.so).

PyTorch is used only as the device allocator and stream provider: every op here hands raw
device pointers + sizes to a HIP kernel in libs2v.  Inputs must be CUDA (HIP) fp32 tensors; a
CPU tensor raises (there is no CPU path in the product).

Layout: activations are NHWC tensors [N, H, W, Ctot]; an ``NHWC`` view selects a channel slice
[coff, coff + c) of one, which is how the reference's torch.cat / split / narrow disappear.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from ._lib import (ACT_GELU_TANH, ACT_LRELU, ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH,  # noqa: F401
                   IN_DIRECT, IN_NEAREST_UP2, IN_TRANSPOSED, PAD_REFLECT, PAD_ZERO, PREC_BF16X3, PREC_F16X3, PREC_F32,
                   check)

F32 = 4

# Arithmetic of the implicit-GEMM convolutions (s2v_conv_params.prec):
#   "f16x3"  (default) split-fp32 on the f16 MFMA: 22 significant bits per operand, <= 3*2^-22
#            relative error per product for operands in the f16 normal range (weights are pre-scaled
#            into it by a power of two, undone exactly in the epilogue);
#   "bf16x3" split-fp32 on the bf16 MFMA: 16 significant bits per operand, <= 3*2^-16 per product,
#            any fp32 range;
#   "f32"    exact fp32 MFMA.
# All three run fp32 tensors with fp32 accumulation.  The S2V_PRECISION environment variable sets
# the process default; set_precision() changes it.
_PRECISIONS = {"f16x3": PREC_F16X3, "bf16x3": PREC_BF16X3, "f32": PREC_F32}
SPLIT_PRECISIONS = ("f16x3", "bf16x3")
PRECISION = os.environ.get("S2V_PRECISION", "f16x3")
if PRECISION not in _PRECISIONS:
    raise ValueError(f"S2V_PRECISION must be one of {sorted(_PRECISIONS)}, got {PRECISION!r}")


# in-launch split-K fold (s2v_conv_params.tile_counters), opt-in with S2V_SPLITK_FOLD=1.  It gives
# the separate reduce kernel's sums bit for bit, but its agent-scope release / acquire per split
# block (L2 writeback + invalidate on this part) measured 1.5x slower end to end on MI355X (lipsync
# 445 -> 290 frames/s, r01), so the separate reduce launch stays the default.
USE_TILE_COUNTERS = os.environ.get("S2V_SPLITK_FOLD", "0") == "1"


def set_precision(name: str) -> str:
    """Select the conv arithmetic ("f16x3", "bf16x3" or "f32") for launches issued from now on; returns the
    previous setting.  A captured HIP graph keeps the precision it was captured with."""
    global PRECISION
    if name not in _PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}, got {name!r}")
    prev, PRECISION = PRECISION, name
    return prev


def prec_code() -> int:
    return _PRECISIONS[PRECISION]

# Optional per-launch observer (bench.py's live roofline): called as hook(ctx, params, flops, launch)
# where launch() performs the conv; the hook may bracket it with events.
CONV_HOOK = None


def _require_cuda(t: torch.Tensor, what: str):
    if not (t.is_cuda and t.dtype == torch.float32):
        raise _lib.S2VError(f"{what}: expected a float32 HIP device tensor, got {t.dtype} on {t.device} "
                            "(the s2v path has no CPU fallback)")


class NHWC:
    """Channel-slice view of a contiguous [N, H, W, Ctot] fp32 device tensor.  ``split``: the
    tensor holds the split-fp32 layout of the current precision (s2v_split_act; only convolutions
    with x_split read it)."""
    __slots__ = ("t", "n", "h", "w", "cs", "coff", "c", "split")

    def __init__(self, t: torch.Tensor, coff: int = 0, c: int | None = None, split: bool = False):
        assert t.dim() == 4 and t.is_contiguous(), "NHWC view needs a contiguous 4-D tensor"
        _require_cuda(t, "NHWC")
        self.t = t
        self.n, self.h, self.w, self.cs = t.shape
        self.coff = coff
        self.c = self.cs - coff if c is None else c
        self.split = split
        assert 0 <= coff and coff + self.c <= self.cs
        assert not split or (coff % 32 == 0 and self.c % 32 == 0), "split views cover whole 32-channel blocks"

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + F32 * self.coff

    def slice(self, coff: int, c: int) -> "NHWC":
        return NHWC(self.t, self.coff + coff, c, self.split)

    @staticmethod
    def empty(n, h, w, c, device) -> "NHWC":
        return NHWC(torch.empty((n, h, w, c), device=device, dtype=torch.float32))


class Workspace:
    """Grow-only scratch buffer shared by the ops of one stream (split-K partials, norm stats).
    Grows only outside graph capture; a capture that needs more raises.  A replaced buffer is kept
    alive: HIP graphs captured earlier hold its address (an eager call of another shape — a ragged
    last batch — may grow the workspace after a capture; freeing the old one would leave those
    graphs writing into memory the allocator hands out again)."""

    def __init__(self, device):
        self.device = device
        self.buf = torch.empty(0, dtype=torch.uint8, device=device)
        self._retired = []

    def get(self, nbytes: int):
        if nbytes <= 0:
            return None, 0
        if self.buf.numel() < nbytes:
            if torch.device(self.device).type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise _lib.S2VError("workspace must be sized by an eager run before graph capture")
            if self.buf.numel() > 0:
                self._retired.append(self.buf)
            self.buf = torch.empty(int(nbytes * 1.25) + 256, dtype=torch.uint8, device=self.device)
        return self.buf.data_ptr(), self.buf.numel()


class Ctx:
    """Execution context: device, stream handle, workspace."""

    N_COUNTERS = 1 << 18

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = Workspace(self.device)
        self.lib = _lib.load()
        self._counters = None

    def counters(self):
        """Zeroed split-K tile counters (s2v_conv_params.tile_counters), made once per context
        (eagerly, before any graph capture replays the convs that use them)."""
        if self._counters is None:
            if self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
                return None
            self._counters = torch.zeros(self.N_COUNTERS, dtype=torch.int32, device=self.device)
        return self._counters

    @property
    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)


# ----------------------------------------------------------------------------- weights
def _pad2(t: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    out = torch.zeros((rows, cols), dtype=torch.float32)
    out[: t.shape[0], : t.shape[1]] = t
    return out


class ConvW:
    """Packed convolution weights [npad][kpad] with k = (ky*kw + kx)*cin + c, plus the folded
    per-output-channel epilogue scale/shift (bias, eval BatchNorm)."""

    def __init__(self, weight: torch.Tensor, bias=None, device="cuda", *, stride=1, padding=0, dilation=1,
                 transposed=False, output_padding=0, pad_mode=PAD_ZERO, in_mode=IN_DIRECT, bn=None, bn_eps=1e-5,
                 post_scale=None):
        w = weight.detach().to("cpu", torch.float32)
        if w.dim() == 2:
            w = w[:, :, None, None]
        elif w.dim() == 3:            # Conv1d [O, I, k] -> 1 x k
            w = w[:, :, None, :]
        if transposed:                # ConvTranspose2d [I, O, kh, kw] -> [O, I, kh, kw]
            w = w.transpose(0, 1)
            in_mode = IN_TRANSPOSED
        self.cout, self.cin, self.kh, self.kw = (int(s) for s in w.shape)
        self._w_oihw = w if in_mode == IN_TRANSPOSED else None
        self.poly = None
        pair = lambda v: (v, v) if isinstance(v, int) else tuple(v)  # noqa: E731
        self.sh, self.sw = pair(stride)
        self.ph, self.pw = pair(padding)
        self.dh, self.dw = pair(dilation)
        if weight.dim() == 3:
            self.sh, self.ph, self.dh = 1, 0, 1
        self.oph, self.opw = pair(output_padding)
        self.pad_mode, self.in_mode = pad_mode, in_mode
        K = self.kh * self.kw * self.cin
        self.K = K
        self.kpad = (K + 31) // 32 * 32
        # rows padded so every N tile the planner may pick (BN <= 128, or 256 when cout > 128) reads
        # inside the packed buffer: the kernels load whole BN-row slabs of B without a row guard
        self.npad = (self.cout + 127) // 128 * 128 if self.cout <= 128 else (self.cout + 255) // 256 * 256
        wk = w.permute(0, 2, 3, 1).reshape(self.cout, K)
        self.wt = _pad2(wk, self.npad, self.kpad).to(device)
        scale = shift = None
        b = None if bias is None else bias.detach().to("cpu", torch.float32)
        if bn is not None:
            g, beta, mean, var = (t.detach().to("cpu", torch.float32) for t in bn)
            s = g / torch.sqrt(var + bn_eps)
            scale = s
            shift = beta - mean * s + (b * s if b is not None else 0.0)
        elif b is not None:
            shift = b
        if post_scale is not None:
            scale = (scale if scale is not None else torch.ones(self.cout)) * post_scale
            if shift is not None:
                shift = shift * post_scale
        self.scale = None if scale is None else scale.contiguous().to(device)
        self.shift = None if shift is None else shift.contiguous().to(device)

    _split = None

    def split_scale(self, prec: int) -> float:
        """Power-of-two pre-scale of the split weights (s2v_conv_params.wt_scale): f16 halves get
        max|W| into [2^13, 2^14) so every weight and its lo half stay in the f16 normal range; bf16
        has fp32's exponent range and needs none."""
        if prec != PREC_F16X3:
            return 1.0
        if getattr(self, "_f16_scale", None) is None:
            m = float(self.wt.abs().max())
            self._f16_scale = 1.0 if m == 0.0 else float(2.0 ** math.floor(math.log2(16384.0 / m)))
        return self._f16_scale

    def wt_x3(self, ctx: "Ctx", prec: int = PREC_BF16X3) -> torch.Tensor:
        """The packed weights in the split layout of ``prec`` (built once per precision, on first use)."""
        if self._split is None:
            self._split = {}
        if prec not in self._split:
            if self.wt.is_cuda and torch.cuda.is_current_stream_capturing():
                raise _lib.S2VError("split weights must be built by an eager run before graph capture")
            out = torch.empty(self.wt.shape, dtype=torch.float32, device=self.wt.device)
            check(ctx.lib.s2v_split_weights(self.wt.data_ptr(), self.npad, self.kpad, prec, self.split_scale(prec),
                                            out.data_ptr(), ctx.stream), "s2v_split_weights")
            self._split[prec] = out
        return self._split[prec]

    def make_polyphase(self, device):
        """Polyphase plan of a stride-2 ConvTranspose2d: output parity class (ry, rx) is a stride-1
        direct conv of the input with the taps ky = ry + p (mod 2), flipped, padded by T - 1 - c0
        (c0 = (ry + p - ky_min) / 2), written with output step 2 at offset (ry, rx).  Work drops
        from kh*kw taps per output pixel (3/4 of them zero) to the algorithmic count."""
        assert self.in_mode == IN_TRANSPOSED and (self.sh, self.sw) == (2, 2) and (self.dh, self.dw) == (1, 1)
        w = self._w_oihw
        plans = []
        for ry in range(2):
            ty = [k for k in range(self.kh) if (ry + self.ph - k) % 2 == 0]
            for rx in range(2):
                tx = [k for k in range(self.kw) if (rx + self.pw - k) % 2 == 0]
                if not ty or not tx:
                    raise NotImplementedError("polyphase class without taps")
                c0y, c0x = (ry + self.ph - ty[0]) // 2, (rx + self.pw - tx[0]) // 2
                sub = w[:, :, ty[::-1]][:, :, :, tx[::-1]]
                cw = ConvW(sub, None, device, padding=(len(ty) - 1 - c0y, len(tx) - 1 - c0x))
                cw.scale, cw.shift = self.scale, self.shift
                plans.append(((ry, rx), cw, (ry, rx)))
        self.poly = plans
        return self

    def out_hw(self, h, w):
        if self.in_mode == IN_TRANSPOSED:
            return ((h - 1) * self.sh - 2 * self.ph + self.dh * (self.kh - 1) + self.oph + 1,
                    (w - 1) * self.sw - 2 * self.pw + self.dw * (self.kw - 1) + self.opw + 1)
        if self.in_mode == IN_NEAREST_UP2:
            h, w = 2 * h, 2 * w
        return ((h + 2 * self.ph - self.dh * (self.kh - 1) - 1) // self.sh + 1,
                (w + 2 * self.pw - self.dw * (self.kw - 1) - 1) // self.sw + 1)


def _ptr(t):
    return None if t is None else t.data_ptr()


def conv2d(ctx: Ctx, x: NHWC, cw: ConvW, y: NHWC, *, act=ACT_NONE, alpha=0.0, res: NHWC | None = None,
           res_after=False, res_offset=(0, 0), nc_scale=None, in_scale=None, pre_act=ACT_NONE, pre_alpha=0.0,
           pix_add=None, pix_w=0.0, scale=None, shift=None, force_tile=0, force_splits=0, pool=False):
    """Fused conv (see s2v_conv_params).  nc_scale / in_scale: [N, C] device tensors.  A transposed
    ConvW with a polyphase plan (``cw.poly``) runs as one stride-1 conv per output parity class.
    ``pool``: y is the 2x2 average pool of the activated conv output (half the conv's size)."""
    if getattr(cw, "poly", None) is not None:
        assert pix_add is None, "polyphase transposed conv: no pix_add epilogue"
        assert res is None or (res.t.data_ptr() == y.t.data_ptr() and res.coff == y.coff and not res_after), \
            "polyphase transposed conv: only an in-place residual (res is the output view)"
        oh, ow = cw.out_hw(x.h, x.w)
        assert (y.n, y.h, y.w, y.c) == (x.n, oh, ow, cw.cout), "conv_transpose: output view mismatch"
        for (ry, rx), sub, _ in cw.poly:
            ch, cwid = (oh - ry + 1) // 2, (ow - rx + 1) // 2
            if ch <= 0 or cwid <= 0:
                continue
            base = NHWC.__new__(NHWC)
            base.t, base.n, base.h, base.w, base.cs, base.c = y.t, y.n, ch, cwid, y.cs, y.c
            base.split = False
            base.coff = y.coff + (ry * y.w + rx) * y.cs
            _conv(ctx, x, sub, base, (ch, cwid), (2, y.h, y.w), act, alpha, None if res is None else base, False,
                  (0, 0), nc_scale, in_scale, pre_act, pre_alpha, None, 0.0, scale, shift, force_tile, force_splits)
        return y
    oh, ow = cw.out_hw(x.h, x.w)
    assert x.c == cw.cin, f"conv: input has {x.c} channels, weights expect {cw.cin}"
    f = 2 if pool else 1
    assert (y.n, y.h * f, y.w * f, y.c) == (x.n, oh, ow, cw.cout), \
        f"conv: output view {(y.n, y.h, y.w, y.c)} != {(x.n, oh // f, ow // f, cw.cout)}"
    return _conv(ctx, x, cw, y, (oh, ow), None, act, alpha, res, res_after, res_offset, nc_scale, in_scale, pre_act,
                 pre_alpha, pix_add, pix_w, scale, shift, force_tile, force_splits, pool=pool)


def _conv(ctx, x, cw, y, ohw, out_view, act, alpha, res, res_after, res_offset, nc_scale, in_scale, pre_act,
          pre_alpha, pix_add, pix_w, scale, shift, force_tile, force_splits, per_sample_wt=None, pool=False):
    oh, ow = ohw
    p = _lib.ConvParams()
    p.x, p.n, p.h, p.w, p.cin, p.xcs = x.ptr, x.n, x.h, x.w, x.c, x.cs
    p.in_mode, p.pad_mode, p.pre_act, p.pre_alpha = cw.in_mode, cw.pad_mode, pre_act, pre_alpha
    if in_scale is not None:
        p.in_scale, p.in_scale_ns = in_scale.data_ptr(), in_scale.stride(0)
    p.kh, p.kw, p.sh, p.sw, p.ph, p.pw, p.dh, p.dw = cw.kh, cw.kw, cw.sh, cw.sw, cw.ph, cw.pw, cw.dh, cw.dw
    p.wt, p.kpad, p.npad, p.cout = cw.wt.data_ptr(), cw.kpad, cw.npad, cw.cout
    p.prec = prec_code()
    p.y, p.oh, p.ow, p.ycs = y.ptr, oh, ow, y.cs
    sc = cw.scale if scale is None else scale
    sh = cw.shift if shift is None else shift
    p.scale, p.shift = _ptr(sc), _ptr(sh)
    if nc_scale is not None:
        p.nc_scale, p.nc_scale_ns = nc_scale.data_ptr(), nc_scale.stride(0)
    if pix_add is not None:
        p.pix_add, p.pix_w = pix_add.data_ptr(), pix_w
    if res is not None:
        p.res, p.res_cs, p.res_h, p.res_w = res.ptr, res.cs, res.h, res.w
        p.res_oy, p.res_ox = res_offset
        p.res_after_act = int(res_after)
    p.act, p.alpha = act, alpha
    p.batch = 1
    p.force_tile, p.force_splits = force_tile, force_splits
    p.out_pool = int(pool)
    p.x_split = int(getattr(x, "split", False))
    if p.x_split:
        assert p.prec != PREC_F32, "split-layout inputs need a split precision (f16x3 / bf16x3)"
    if out_view is not None:
        p.out_step, p.out_full_h, p.out_full_w = out_view
    if per_sample_wt is not None:        # batch mode: one image per batch entry, its own weights
        assert in_scale is None and nc_scale is None and out_view is None
        p.n, p.batch = 1, x.n
        p.w_bs = cw.npad * cw.kpad
        p.x_bs, p.y_bs = x.h * x.w * x.cs, y.h * y.w * y.cs
        if res is not None:
            p.res_bs = res.h * res.w * res.cs
    use_x3 = False
    if p.prec != PREC_F32:
        p.wt_x3 = p.wt                   # placeholder: the plan query only checks it is set
        use_x3 = bool(_plan(ctx, p)[6]) and not p.b_kn
        p.wt_x3 = None
    if per_sample_wt is not None:
        wb, wscale = per_sample_wt(p.prec if use_x3 else PREC_F32)   # as the kernel reads them
        if use_x3:
            p.wt, p.wt_x3, p.wt_scale = None, wb.data_ptr(), wscale
        else:
            p.wt = wb.data_ptr()
    elif use_x3:                         # implicit-GEMM path: pre-split packed weights
        p.wt_x3 = cw.wt_x3(ctx, p.prec).data_ptr()
        p.wt_scale = cw.split_scale(p.prec)
    need = ctx.lib.s2v_conv2d_ws_bytes(ctypes.byref(p))
    p.ws, p.ws_bytes = ctx.ws.get(need)
    _set_counters(ctx, p, need)
    if CONV_HOOK is not None:
        # algorithmic MACs: a transposed conv only counts real (non-inserted-zero) taps
        taps = cw.kh * cw.kw
        pix = x.n * x.h * x.w if cw.in_mode == IN_TRANSPOSED else x.n * oh * ow
        flops = 2.0 * pix * taps * cw.cin * cw.cout
        CONV_HOOK(ctx, p, flops, lambda: check(ctx.lib.s2v_conv2d(ctypes.byref(p), ctx.stream), "s2v_conv2d"))
        return y
    check(ctx.lib.s2v_conv2d(ctypes.byref(p), ctx.stream), "s2v_conv2d")
    return y


def modulated_conv2d(ctx: Ctx, x: NHWC, cw: ConvW, y: NHWC, s: torch.Tensor, d: torch.Tensor | None = None, *,
                     act=ACT_NONE, alpha=0.0, res: NHWC | None = None, res_after=False, pix_add=None, pix_w=0.0,
                     shift=None, force_splits=0):
    """StyleGAN2 modulated conv with per-sample weights W * s[b, c] (* d[b, o]) built by
    s2v_modulate_weights, then one batched conv (no prologue / epilogue scaling in the GEMM).
    s: [B, cin] (row stride s.stride(0)); d: [B, cout] demodulation or None."""
    oh, ow = cw.out_hw(x.h, x.w)
    assert cw.in_mode != IN_TRANSPOSED and cw.poly is None, "modulated_conv2d: direct / up2 convs only"
    assert x.c == cw.cin and (y.n, y.h, y.w, y.c) == (x.n, oh, ow, cw.cout)
    b = x.n

    def weights(prec):
        # the split implicit GEMM reads split weights; the VALU kernels (small K / Cout) fp32.
        # Demodulated rows have |w * s * d| <= post (ENet / GFPGAN / GPEN: sqrt 2), so f16 halves
        # take a fixed 2^11 pre-scale (room up to |w| < 32); without demodulation the range is open
        # and the weights go unscaled (f16 subnormal halves keep an absolute error <= 2^-25).
        wb = torch.empty((b, cw.npad, cw.kpad), device=cw.wt.device)
        dp, dns = (None, 0) if d is None else (d.data_ptr(), d.stride(0))
        if prec == PREC_F32:
            check(ctx.lib.s2v_modulate_weights(cw.wt.data_ptr(), cw.npad, cw.kpad, cw.K, cw.cin, cw.cout, s.data_ptr(),
                                               s.stride(0), dp, dns, b, wb.data_ptr(), ctx.stream),
                  "s2v_modulate_weights")
            return wb, 1.0
        scale = 2048.0 if (prec == PREC_F16X3 and d is not None) else 1.0
        check(ctx.lib.s2v_modulate_weights_split(cw.wt.data_ptr(), cw.npad, cw.kpad, cw.K, cw.cin, cw.cout,
                                                 s.data_ptr(), s.stride(0), dp, dns, b, prec, scale, wb.data_ptr(),
                                                 ctx.stream), "s2v_modulate_weights_split")
        return wb, scale
    return _conv(ctx, x, cw, y, (oh, ow), None, act, alpha, res, res_after, (0, 0), None, None, ACT_NONE, 0.0,
                 pix_add, pix_w, None, shift, 0, force_splits, per_sample_wt=weights)


def gemm_kn(ctx: Ctx, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, batch: int, a_bs: int, b_bs: int,
            out_bs: int, res: torch.Tensor | None = None, res_bs: int = 0, act=ACT_NONE, alpha=0.0,
            force_tile=0, force_splits=0):
    """Batched out[z] = a[z] @ b[z] (+res[z]) with a [M, K] row-major (K contiguous, lda = K),
    b [K, N] row-major (ldb = N), out [M, N] (ldc = N).  Used for the FourierUnit DFT products."""
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    p = _lib.ConvParams()
    p.x, p.n, p.h, p.w, p.cin, p.xcs = a.data_ptr(), 1, 1, M, K, K
    p.kh = p.kw = p.sh = p.sw = p.dh = p.dw = 1
    p.wt, p.cout, p.b_kn, p.ldb = b.data_ptr(), N, 1, N
    p.prec = prec_code()
    p.y, p.oh, p.ow, p.ycs = out.data_ptr(), 1, M, N
    if res is not None:
        p.res, p.res_cs, p.res_h, p.res_w = res.data_ptr(), N, 1, M
        p.res_bs = res_bs
    p.act, p.alpha = act, alpha
    p.batch, p.x_bs, p.w_bs, p.y_bs = batch, a_bs, b_bs, out_bs
    p.force_tile, p.force_splits = force_tile, force_splits
    need = ctx.lib.s2v_conv2d_ws_bytes(ctypes.byref(p))
    p.ws, p.ws_bytes = ctx.ws.get(need)
    _set_counters(ctx, p, need)
    if CONV_HOOK is not None:   # DFT products: executed work, not reference-algorithmic FLOPs
        CONV_HOOK(ctx, p, 0.0, lambda: check(ctx.lib.s2v_conv2d(ctypes.byref(p), ctx.stream), "s2v_conv2d(gemm)"))
        return out
    check(ctx.lib.s2v_conv2d(ctypes.byref(p), ctx.stream), "s2v_conv2d(gemm)")
    return out


def _set_counters(ctx: Ctx, p, ws_need):
    """Split-K launches fold their partial sums in-launch when the context has tile counters."""
    if ws_need and USE_TILE_COUNTERS:
        c = getattr(ctx, "counters", None)
        t = c() if callable(c) else None
        if t is not None:
            p.tile_counters, p.n_counters = t.data_ptr(), t.numel()


def _plan(ctx: Ctx, p):
    out = (ctypes.c_int * 10)()
    check(ctx.lib.s2v_conv2d_plan(ctypes.byref(p), out), "s2v_conv2d_plan")
    return list(out)


def conv_symbol(ctx: Ctx, p) -> str:
    """Kernel symbol (as rocprofv3 reports it, demangled) the launch of ``p`` runs."""
    bm, bn, wm, avec, bkn, splits, x3, nw, ks, pf = _plan(ctx, p)
    if avec == 5:
        return f"void s2v::conv_glds_x3<{bm}, {bn}, {wm}, {ks}, {x3 - 1}>(s2v::ConvArgs)"
    if bm == 0:
        if wm < 0:
            if bkn >= 2000:
                return f"void s2v::conv_smallk4<{-wm}, {bkn - 2000}>(s2v::ConvArgs, int, int, int, int)"
            return f"void s2v::conv_smallk<{-wm}, {avec}>(s2v::ConvArgs, int, int, int, int)"
        if bkn >= 1000:
            return f"void s2v::conv_halo_small<{bn}, {bkn - 1000}>(s2v::ConvArgs, int, int)"
        if wm:
            return f"void s2v::conv_small_cpar<{bn}, {wm}, {'true' if avec else 'false'}>(s2v::ConvArgs, int)"
        return f"void s2v::conv_direct_small<{bn}>(s2v::ConvArgs, int)"
    if x3:
        return (f"void s2v::conv_igemm_x3<{bm}, {bn}, {wm}, {nw}, {ks}, {pf}, {avec}, {bkn}, {x3 - 1}>"
                "(s2v::ConvArgs)")
    return f"void s2v::conv_igemm<{bm}, {bn}, {wm}, {avec}, {bkn}>(s2v::ConvArgs)"


def split_act(ctx: Ctx, x: NHWC, out: NHWC | None = None) -> NHWC:
    """fp32 activations -> the split layout of the current precision (s2v_split_act), the input
    form of the LDS-DMA convolutions.  ``out``: a whole contiguous tensor of x's shape."""
    prec = prec_code()
    assert prec != PREC_F32, "split_act needs a split precision (f16x3 / bf16x3)"
    if out is None:
        out = NHWC.empty(x.n, x.h, x.w, x.c, x.t.device)
    assert (out.n, out.h, out.w, out.c) == (x.n, x.h, x.w, x.c) and out.coff == 0
    check(ctx.lib.s2v_split_act(x.ptr, x.n * x.h * x.w, x.c, x.cs, prec, out.ptr, out.cs, ctx.stream), "s2v_split_act")
    out.split = True
    return out


TUNE_HALO_MIN_BLOCKS, TUNE_GLDS_TILE, TUNE_SMALLK_TILE, TUNE_X3_RATE_512, TUNE_IN_FUSED = 0, 1, 2, 3, 4


def tune(ctx: Ctx, key: int, value: int) -> int:
    """Set a planner knob (s2v_tune); returns the previous value."""
    old = ctypes.c_longlong(0)
    check(ctx.lib.s2v_tune(key, value, ctypes.byref(old)), "s2v_tune")
    return old.value


def conv_splits(ctx: Ctx, p) -> int:
    return _plan(ctx, p)[5]


def layernorm2d(ctx: Ctx, x: NHWC, weight, bias, y: NHWC, *, act=ACT_LRELU, alpha=0.1, pool=False,
                res: NHWC | None = None, eps=1e-5):
    need = ctx.lib.s2v_layernorm2d_ws_bytes(x.n, x.h, x.w, x.c)
    ws, nb = ctx.ws.get(need)
    check(ctx.lib.s2v_layernorm2d(x.ptr, x.n, x.h, x.w, x.c, x.cs, weight.data_ptr(), bias.data_ptr(), eps, act, alpha,
                                  int(pool), None if res is None else res.ptr, 0 if res is None else res.cs,
                                  y.ptr, y.cs, ws, nb, ctx.stream), "s2v_layernorm2d")
    return y


def instnorm(ctx: Ctx, x: NHWC, y: NHWC, gamma=None, beta=None, gb_ns=0, *, act=ACT_NONE, alpha=0.0,
             res: NHWC | None = None, eps=1e-5, pad_out: NHWC | None = None):
    """gamma/beta: raw device pointers (ints) or None; gb_ns = per-sample row stride.  ``pad_out``
    ([n, h+2, w+2, c] view) also receives F.pad(y, (1, 1, 1, 1), 'reflect')."""
    need = ctx.lib.s2v_instnorm_ws_bytes(x.n, x.h, x.w, x.c)
    ws, nb = ctx.ws.get(need)
    rp, rcs = (None, 0) if res is None else (res.ptr, res.cs)
    if pad_out is not None:
        assert (pad_out.n, pad_out.h, pad_out.w, pad_out.c) == (x.n, x.h + 2, x.w + 2, x.c)
        check(ctx.lib.s2v_instnorm_adain_pad(x.ptr, x.n, x.h, x.w, x.c, x.cs, gamma, beta, gb_ns, eps, act, alpha,
                                             rp, rcs, y.ptr, y.cs, pad_out.ptr, pad_out.cs, ws, nb, ctx.stream),
              "s2v_instnorm_adain_pad")
        return y
    check(ctx.lib.s2v_instnorm_adain(x.ptr, x.n, x.h, x.w, x.c, x.cs, gamma, beta, gb_ns, eps, act, alpha,
                                     rp, rcs, y.ptr, y.cs, ws, nb, ctx.stream), "s2v_instnorm_adain")
    return y


def adain_params(ctx: Ctx, hid: torch.Tensor, nhidden: int, w2t: torch.Tensor, bias: torch.Tensor, seg: torch.Tensor,
                 out: torch.Tensor):
    batch, total = out.shape
    check(ctx.lib.s2v_adain_params(hid.data_ptr(), batch, hid.stride(0), nhidden, w2t.data_ptr(), bias.data_ptr(),
                                   seg.data_ptr(), total, out.data_ptr(), out.stride(0), ctx.stream),
          "s2v_adain_params")
    return out


def modconv_demod(ctx: Ctx, s: torch.Tensor, wsq: torch.Tensor, out: torch.Tensor, *, eps=1e-8, post=1.0):
    """s: [B, cin] view (row stride s.stride(0)), wsq: [cout, cin], out: [B, cout]."""
    batch, cin = s.shape
    cout = wsq.shape[0]
    check(ctx.lib.s2v_modconv_demod(s.data_ptr(), batch, s.stride(0), cin, wsq.data_ptr(), cout, eps, post,
                                    out.data_ptr(), out.stride(0), ctx.stream), "s2v_modconv_demod")
    return out


def torch_bilinear_scale(in_size: int, out_size: int, scale_factor=None) -> float:
    """area_pixel_compute_scale (align_corners=False) as PyTorch computes it (float32)."""
    if scale_factor is not None and scale_factor > 0:
        return float(torch.tensor(1.0 / scale_factor, dtype=torch.float32))
    return float(torch.tensor(in_size, dtype=torch.float32) / out_size)


def resize(ctx: Ctx, x_ptr: int, x_shape, x_strides, y_ptr: int, y_hw, y_strides, *, scale_factor=None,
           mode=0):
    """x_shape = (n, c, ih, iw); strides (sn, sc, sy, sx) in elements, for input and output."""
    n, c, ih, iw = x_shape
    oh, ow = y_hw
    sh = torch_bilinear_scale(ih, oh, scale_factor) if mode == 0 else (
        float(torch.tensor(1.0 / scale_factor, dtype=torch.float32)) if scale_factor else ih / oh)
    sw = torch_bilinear_scale(iw, ow, scale_factor) if mode == 0 else (
        float(torch.tensor(1.0 / scale_factor, dtype=torch.float32)) if scale_factor else iw / ow)
    check(ctx.lib.s2v_resize(x_ptr, n, c, ih, iw, *x_strides, y_ptr, oh, ow, *y_strides, sh, sw, mode, ctx.stream),
          "s2v_resize")


def nhwc_strides(v: NHWC):
    return (v.h * v.w * v.cs, 1, v.w * v.cs, v.cs)


def resize_nhwc(ctx: Ctx, x: NHWC, y: NHWC, scale_factor=None, mode=0):
    resize(ctx, x.ptr, (x.n, x.c, x.h, x.w), nhwc_strides(x), y.ptr, (y.h, y.w), nhwc_strides(y),
           scale_factor=scale_factor, mode=mode)
    return y


def nchw_to_nhwc(ctx: Ctx, x: torch.Tensor, y: NHWC, size=None):
    """NCHW device tensor (any strides) -> NHWC view, optionally bilinear-resized to y's size."""
    _require_cuda(x, "nchw_to_nhwc")
    n, c, h, w = x.shape
    sn, sc, sy, sx = x.stride()
    resize(ctx, x.data_ptr(), (n, c, h, w), (sn, sc, sy, sx), y.ptr, (y.h, y.w), nhwc_strides(y))
    return y


def nhwc_to_nchw(ctx: Ctx, x: NHWC, out: torch.Tensor, crop=(0, 0)):
    """NHWC view (optionally cropped by (top, left) to out's H, W) -> contiguous NCHW tensor."""
    n, c, oh, ow = out.shape
    base = x.ptr + F32 * (crop[0] * x.w + crop[1]) * x.cs
    resize(ctx, base, (n, c, oh, ow), nhwc_strides(x), out.data_ptr(), (oh, ow), out.stride())
    return out


def pad_reflect(ctx: Ctx, x: NHWC, y: NHWC, pads):
    pt, pb, pl, pr = pads
    check(ctx.lib.s2v_pad_reflect(x.ptr, x.n, x.h, x.w, x.c, x.cs, pt, pb, pl, pr, y.ptr, y.cs, ctx.stream),
          "s2v_pad_reflect")
    return y


def row_layernorm(ctx: Ctx, x: torch.Tensor, weight, bias, y: torch.Tensor, eps=1e-5):
    rows, dim = x.shape
    check(ctx.lib.s2v_row_layernorm(x.data_ptr(), rows, dim, x.stride(0), weight.data_ptr(), bias.data_ptr(), eps,
                                    y.data_ptr(), y.stride(0), ctx.stream), "s2v_row_layernorm")
    return y


def attention(ctx: Ctx, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: torch.Tensor, *, batch, heads,
              tokens, dim_head=64, scale=None):
    """q, k, v, out: [batch*tokens, *] row views (row stride = stride(0)); head h = cols [64h, 64h+64)."""
    scale = dim_head ** -0.5 if scale is None else scale
    check(ctx.lib.s2v_attention(q.data_ptr(), k.data_ptr(), v.data_ptr(), batch, heads, tokens, dim_head,
                                q.stride(0), k.stride(0), v.stride(0), tokens * q.stride(0), tokens * k.stride(0),
                                tokens * v.stride(0), scale, out.data_ptr(), out.stride(0), tokens * out.stride(0),
                                ctx.stream), "s2v_attention")
    return out


def flow_warp(ctx: Ctx, flow: NHWC, src: torch.Tensor, y: NHWC):
    """flow: NHWC view with >= 2 channels (x, y); src: NCHW-strided device tensor."""
    n, c, h, w = src.shape
    check(ctx.lib.s2v_flow_warp(flow.ptr, flow.n, flow.h, flow.w, flow.cs, src.data_ptr(), c, h, w, *src.stride(),
                                y.ptr, y.cs, ctx.stream), "s2v_flow_warp")
    return y


def fill(ctx: Ctx, t: torch.Tensor, value: float = 0.0):
    check(ctx.lib.s2v_fill(t.data_ptr(), t.numel(), value, ctx.stream), "s2v_fill")
    return t


def pad_cin(w: torch.Tensor, cin: int) -> torch.Tensor:
    """Zero-pad a conv weight [O, I, kh, kw] along I (vectorised 4-channel image layout)."""
    if w.shape[1] >= cin:
        return w
    z = torch.zeros((w.shape[0], cin - w.shape[1]) + tuple(w.shape[2:]), dtype=w.dtype)
    return torch.cat([w, z], 1)


def gaussian_noise(ctx: Ctx, out: torch.Tensor, seed: int, offset: int = 0, ctr: torch.Tensor | None = None,
                   shift: int = 40):
    """N(0,1) into ``out``; with a device counter ``ctr`` (int64 [1]) the stream offset advances by
    ctr << shift, read when the kernel runs (fresh draws on every graph replay)."""
    if ctr is None:
        check(ctx.lib.s2v_gaussian_noise(out.data_ptr(), out.numel(), seed & (2 ** 64 - 1), offset & (2 ** 64 - 1),
                                         ctx.stream), "s2v_gaussian_noise")
    else:
        check(ctx.lib.s2v_gaussian_noise_ctr(out.data_ptr(), out.numel(), seed & (2 ** 64 - 1),
                                             offset & (2 ** 64 - 1), ctr.data_ptr(), shift, ctx.stream),
              "s2v_gaussian_noise_ctr")
    return out


class NoiseCounter:
    """Device-side draw counter of an engine's random noise (StyleConv / GFPGAN randomize_noise):
    bumped by a kernel at the start of each forward, so a captured graph draws fresh noise per
    replay.  Created on the first (eager) forward, never inside a capture."""

    def __init__(self):
        self.t = None

    def bump(self, ctx: Ctx) -> torch.Tensor:
        if self.t is None:
            if ctx.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise _lib.S2VError("noise counter must be created by an eager run before graph capture")
            self.t = torch.zeros(1, dtype=torch.int64, device=ctx.device)
        check(ctx.lib.s2v_counter_add(self.t.data_ptr(), 1, ctx.stream), "s2v_counter_add")
        return self.t


# ----------------------------------------------------------------------------- DFT matrices
_DFT_CACHE = {}


def fourier_matrices(h: int, w: int, device):
    """Real matrices of torch.fft.rfftn / irfftn(s=(h, w)) with norm='ortho' (ffc.py:99, :121).

    D2  [2F, P]: spectrum rows ordered (u*Wf + v)*2 + part (part 0 = real, 1 = imag)
    Iv  [P, 2F]: the inverse (Hermitian c2r) acting on the same row order.
    Built by applying torch.fft (float64) to basis vectors, so they are exactly the reference's
    transforms, including the c2r treatment of the imaginary DC/Nyquist bins."""
    key = (h, w, str(device))
    if key not in _DFT_CACHE:
        P, wf = h * w, w // 2 + 1
        F = h * wf
        eye = torch.eye(P, dtype=torch.float64).reshape(P, h, w)
        spec = torch.fft.rfftn(eye, dim=(-2, -1), norm="ortho").reshape(P, F)      # [P, F] complex
        d2 = torch.stack([spec.real, spec.imag], -1).reshape(P, 2 * F).t()           # [2F, P]
        basis = torch.zeros(2 * F, F, dtype=torch.complex128)
        idx = torch.arange(F)
        basis[2 * idx, idx] = 1.0
        basis[2 * idx + 1, idx] = 1.0j
        iv = torch.fft.irfftn(basis.reshape(2 * F, h, wf), s=(h, w), dim=(-2, -1), norm="ortho")
        iv = iv.reshape(2 * F, P).t()                                                # [P, 2F]
        _DFT_CACHE[key] = (d2.float().contiguous().to(device), iv.float().contiguous().to(device))
    return _DFT_CACHE[key]


# ----------------------------------------------------------------------------- FIR / elementwise
def fir2d(ctx: Ctx, x: NHWC, kernel: torch.Tensor, y: NHWC, *, up=1, down=1, pad0=(0, 0), gain=1.0, bias=None,
          act=ACT_NONE, alpha=0.0, post=1.0):
    """upfirdn2d on NHWC views (pad0 = (pad_y0, pad_x0); the far pads follow from y's size)
    with y = post * act(gain * fir + bias[c])."""
    assert x.n == y.n and x.c == y.c, "fir2d: batch / channel mismatch"
    kh, kw = kernel.shape
    check(ctx.lib.s2v_fir2d(x.ptr, x.n, x.h, x.w, x.c, x.cs, kernel.data_ptr(), kh, kw, up, down, pad0[0], pad0[1],
                            y.ptr, y.h, y.w, y.cs, gain, _ptr(bias), act, alpha, post, ctx.stream), "s2v_fir2d")
    return y


def eltwise(ctx: Ctx, x: NHWC, y: NHWC, *, a=1.0, mul: NHWC | None = None, add: NHWC | None = None, bias=None,
            act=ACT_NONE, alpha=0.0, post=1.0):
    """y = post * act(x * a * mul + add + bias[c]) over NHWC views of equal n/h/w/c (in place ok)."""
    assert (x.n, x.h, x.w, x.c) == (y.n, y.h, y.w, y.c)
    for v in (mul, add):
        assert v is None or (v.n, v.h, v.w, v.c) == (x.n, x.h, x.w, x.c)
    check(ctx.lib.s2v_eltwise(x.ptr, x.cs, None if mul is None else mul.ptr, 0 if mul is None else mul.cs,
                              None if add is None else add.ptr, 0 if add is None else add.cs, _ptr(bias),
                              x.n * x.h * x.w, x.c, a, act, alpha, post, y.ptr, y.cs, ctx.stream), "s2v_eltwise")
    return y


# ----------------------------------------------------------------------------- separable FFT
_FFT_TABLES = {}


def fft_tables(h: int, w: int, device):
    """1-D ortho transform matrices for s2v_rfft2 / s2v_irfft2 (include/s2v.h), built by applying
    torch.fft to basis vectors in float64: fw[w][2][Wf] | fh[h][2][u] | ih[u][2][h] | iw[Wf][2][w]."""
    key = (h, w, str(device))
    if key not in _FFT_TABLES:
        wf = w // 2 + 1
        rw = torch.fft.rfft(torch.eye(w, dtype=torch.float64), dim=1, norm="ortho")         # [w, Wf]
        fw = torch.stack([rw.real, rw.imag], 1)                                           # [w, 2, Wf]
        fhc = torch.fft.fft(torch.eye(h, dtype=torch.complex128), dim=1, norm="ortho")      # [h, u]
        fh = torch.stack([fhc.real, fhc.imag], 1)                                         # [h, 2, u]
        ihc = torch.fft.ifft(torch.eye(h, dtype=torch.complex128), dim=1, norm="ortho")     # [u, h]
        ih = torch.stack([ihc.real, ihc.imag], 1)                                         # [u, 2, h]
        eye = torch.eye(wf, dtype=torch.float64)
        cre = torch.fft.irfft(torch.complex(eye, torch.zeros_like(eye)), n=w, dim=1, norm="ortho")   # [v, w]
        cim = torch.fft.irfft(torch.complex(torch.zeros_like(eye), eye), n=w, dim=1, norm="ortho")
        iw = torch.stack([cre, cim], 1)                                                   # [Wf, 2, w]
        t = torch.cat([fw.reshape(-1), fh.reshape(-1), ih.reshape(-1), iw.reshape(-1)]).float().contiguous()
        assert t.numel() == 2 * wf * w + 4 * h * h + 2 * w * wf
        _FFT_TABLES[key] = t.to(device)
    return _FFT_TABLES[key]


def rfft2(ctx: Ctx, x: NHWC, tables: torch.Tensor, spec: torch.Tensor):
    """x NHWC [n,h,w,C] -> spec [n, h*(w//2+1), 2C] (channel = part*C + c), rfftn ortho."""
    check(ctx.lib.s2v_rfft2(x.ptr, x.n, x.h, x.w, x.c, x.cs, tables.data_ptr(), spec.data_ptr(), spec.shape[-1],
                            ctx.stream), "s2v_rfft2")
    return spec


def irfft2(ctx: Ctx, spec: torch.Tensor, tables: torch.Tensor, y: NHWC, res: NHWC | None = None):
    """spec [n, F, >=2C] -> y NHWC = irfftn(spec, s=(h, w), ortho) (+ res)."""
    check(ctx.lib.s2v_irfft2(spec.data_ptr(), y.n, y.h, y.w, y.c, spec.shape[-1], tables.data_ptr(),
                             None if res is None else res.ptr, 0 if res is None else res.cs, y.ptr, y.cs, ctx.stream),
          "s2v_irfft2")
    return y
