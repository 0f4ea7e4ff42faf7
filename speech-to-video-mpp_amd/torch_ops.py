"""PyTorch custom ops of libs2v (``TORCH_LIBRARY(s2v)``, csrc/torch_ops.cpp) — the PyTorch-facing
boundary of the HIP kernels.  Kernels are registered for the HIP device only; CPU tensors raise.

Drop-ins for the reference's only native FFI (GPEN's JIT-built pybind11 extensions):

    # third_part/GPEN/face_model/op/fused_act.py:11-19 and op/upfirdn2d.py:10-18
    from s2v_amd.torch_ops import fused, upfirdn2d_op      # instead of cpp_extension.load(...)

    fused.fused_bias_act(input, bias, refer, act, grad, alpha, scale)          (fused_bias_act.cpp:4-21)
    upfirdn2d_op.upfirdn2d(input, kernel, up_x, up_y, down_x, down_y,
                           pad_x0, pad_x1, pad_y0, pad_y1)                      (upfirdn2d.cpp:4-23)

plus the module-level ``fused_leaky_relu`` / ``upfirdn2d`` with the device-branch semantics of
op/fused_act.py:92-96 and op/upfirdn2d.py:149-157 (forward / inference only, like the engines),
the functional model-path ops ``torch.ops.s2v.{conv2d_nhwc, layernorm2d, instnorm_adain, attention,
rfft2, irfft2, resize_bilinear, flow_warp, mel_spectrogram}``, and the in-place launch ops
(LAUNCH_OPS) through which the engines dispatch every kernel of the model forwards.
"""
from __future__ import annotations

import os
import threading

import torch

from . import _lib

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libs2v_torch.so")
OPS = ("fused_bias_act", "upfirdn2d", "conv2d_nhwc", "layernorm2d", "instnorm_adain", "attention", "rfft2", "irfft2",
       "resize_bilinear", "flow_warp", "mel_spectrogram")
# the launch ops every kernel of the model forwards is dispatched through (csrc/torch_launch.cpp,
# called by s2v_amd.ops): in-place on caller-owned views, capturable
LAUNCH_OPS = ("conv2d_", "modulated_conv2d_", "modulate_weights_", "gemm_kn_", "split_weights_", "split_act_", "layernorm2d_", "instnorm_",
              "adain_params_", "modconv_demod_", "row_layernorm_", "attention_", "resize_", "pad_reflect_",
              "flow_warp_", "flow_warp_cat_", "fill_value_", "gaussian_noise_", "counter_add_", "rfft2_", "irfft2_", "eltwise_", "fir2d_",
              "lipsync_inputs_", "to_u8_", "mel_chunks_", "melspectrogram_")
_lock = threading.Lock()
_loaded = False


def load():
    """Register the s2v ops with the dispatcher (loads libs2v.so first); raises if not built."""
    global _loaded
    if _loaded:
        return torch.ops.s2v
    with _lock:
        if not _loaded:
            _lib.load()
            if not os.path.exists(LIB_PATH):
                raise _lib.S2VError(f"{LIB_PATH} is missing: build it with `make -C {os.path.dirname(LIB_PATH)}/csrc`")
            torch.ops.load_library(LIB_PATH)
            _loaded = True
    return torch.ops.s2v


class _Ns:
    """Attribute access forwarding to torch.ops.s2v (loaded on first use)."""

    def __getattr__(self, name):
        return getattr(load(), name)


fused = _Ns()          # fused.fused_bias_act(...)
upfirdn2d_op = _Ns()   # upfirdn2d_op.upfirdn2d(...)


def fused_leaky_relu(input, bias, negative_slope=0.2, scale=2 ** 0.5, device="cuda"):
    """op/fused_act.py:92-96 on the device: scale * leaky_relu(input + bias[c], negative_slope)."""
    return load().fused_bias_act(input, bias, input.new_empty(0), 3, 0, negative_slope, scale)


def upfirdn2d(input, kernel, up=1, down=1, pad=(0, 0), device="cuda"):
    """op/upfirdn2d.py:149-157 / UpFirDn2d.forward (:92-124) on the device: NCHW in and out, the
    planes passed to the op as [N*C, H, W, 1]."""
    n, c, h, w = input.shape
    kh, kw = kernel.shape
    out = load().upfirdn2d(input.reshape(-1, h, w, 1), kernel, up, up, down, down, pad[0], pad[1], pad[0], pad[1])
    out_h = (h * up + pad[0] + pad[1] - kh) // down + 1
    out_w = (w * up + pad[0] + pad[1] - kw) // down + 1
    return out.view(-1, c, out_h, out_w)
