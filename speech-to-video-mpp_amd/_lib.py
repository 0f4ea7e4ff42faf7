"""ctypes binding of libs2v.so (the C ABI declared in include/s2v.h).

The library is built in-tree (``make -C speech-to-video-mpp_amd/csrc`` or
``__graft_entry__.build()``) and loaded from this package directory only.  There is no CPU
fallback anywhere on the product path: if the library is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

# the package's in-tree build (libs2v_torch.so, the model path's launch ops, links this same file)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libs2v.so")

ACT_NONE, ACT_RELU, ACT_LRELU, ACT_SIGMOID, ACT_TANH, ACT_GELU_TANH = range(6)
IN_DIRECT, IN_NEAREST_UP2, IN_TRANSPOSED = range(3)
PAD_ZERO, PAD_REFLECT = range(2)
PREC_F32, PREC_BF16X3, PREC_F16X3 = range(3)

_c_int, _c_float, _c_ll, _c_size, _vp = ctypes.c_int, ctypes.c_float, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_void_p


class ConvParams(ctypes.Structure):
    """Mirror of s2v_conv_params (include/s2v.h)."""
    _fields_ = [
        ("x", _vp), ("n", _c_int), ("h", _c_int), ("w", _c_int), ("cin", _c_int), ("xcs", _c_int),
        ("in_mode", _c_int), ("pad_mode", _c_int), ("pre_act", _c_int), ("pre_alpha", _c_float),
        ("in_scale", _vp), ("in_scale_ns", _c_int),
        ("kh", _c_int), ("kw", _c_int), ("sh", _c_int), ("sw", _c_int), ("ph", _c_int), ("pw", _c_int),
        ("dh", _c_int), ("dw", _c_int),
        ("wt", _vp), ("kpad", _c_int), ("npad", _c_int), ("cout", _c_int), ("b_kn", _c_int), ("ldb", _c_int),
        ("y", _vp), ("oh", _c_int), ("ow", _c_int), ("ycs", _c_int),
        ("scale", _vp), ("shift", _vp), ("nc_scale", _vp), ("nc_scale_ns", _c_int),
        ("pix_add", _vp), ("pix_w", _c_float),
        ("res", _vp), ("res_cs", _c_int), ("res_h", _c_int), ("res_w", _c_int), ("res_oy", _c_int),
        ("res_ox", _c_int), ("res_after_act", _c_int),
        ("act", _c_int), ("alpha", _c_float),
        ("batch", _c_int), ("x_bs", _c_ll), ("w_bs", _c_ll), ("y_bs", _c_ll), ("res_bs", _c_ll),
        ("ws", _vp), ("ws_bytes", _c_size),
        ("force_tile", _c_int), ("force_splits", _c_int),
        ("out_step", _c_int), ("out_full_h", _c_int), ("out_full_w", _c_int),
        ("prec", _c_int), ("wt_x3", _vp),
        ("grid_cap", _c_int),
        ("wt_scale", _c_float),
        ("out_pool", _c_int),
        ("x_split", _c_int),
        ("stamps", _vp), ("stamp_ctr", _vp), ("stamp_slot", _c_int), ("stamp_stride", _c_int),
        ("stamp_reps", _c_int),
        ("x_scale", _c_float), ("nonfinite", _vp),
        ("d2s_cout", _c_int),
        ("post_mul", _vp), ("post_add", _vp), ("post_cs", _c_int), ("post_c0", _c_int),
        ("dup_src", _vp), ("dup_bias", _vp), ("dup_a", _c_float), ("dup_cs", _c_int), ("dup_off", _c_int),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "s2v_conv2d": (_c_int, [ctypes.POINTER(ConvParams), _vp]),
    "s2v_conv2d_ws_bytes": (_c_size, [ctypes.POINTER(ConvParams)]),
    "s2v_conv2d_plan": (_c_int, [ctypes.POINTER(ConvParams), ctypes.POINTER(_c_int)]),
    "s2v_conv2d_group": (_c_int, [ctypes.POINTER(ConvParams), _c_int, _vp]),
    "s2v_conv2d_group_ws_bytes": (_c_size, [ctypes.POINTER(ConvParams), _c_int]),
    "s2v_conv2d_group_plan": (_c_int, [ctypes.POINTER(ConvParams), _c_int, ctypes.POINTER(_c_int)]),
    "s2v_tune": (_c_int, [_c_int, _c_ll, ctypes.POINTER(_c_ll)]),
    "s2v_layernorm2d": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_float, _c_int, _c_float,
                                 _c_int, _vp, _c_int, _vp, _c_int, _vp, _c_size, _vp]),
    "s2v_layernorm2d_ws_bytes": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "s2v_instnorm_adain": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_float, _c_int,
                                    _c_float, _vp, _c_int, _vp, _c_int, _vp, _c_size, _vp]),
    "s2v_instnorm_adain_pad": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_float,
                                        _c_int, _c_float, _vp, _c_int, _vp, _c_int, _vp, _c_int, _vp, _c_size, _vp]),
    "s2v_instnorm_ws_bytes": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "s2v_adain_params": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _c_int, _vp, _c_int, _vp]),
    "s2v_modconv_demod": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_float, _c_float, _vp, _c_int, _vp]),
    "s2v_modconv_demod_rows": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _vp, _c_float, _c_float, _vp, _c_int,
                                        _vp]),
    "s2v_torgb_up2": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _c_int, _vp, _vp,
                               _c_int, _vp, _c_int, _vp]),
    "s2v_resize": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll, _c_ll, _c_ll, _vp, _c_int, _c_int,
                            _c_ll, _c_ll, _c_ll, _c_ll, _c_float, _c_float, _c_int, _vp]),
    "s2v_row_pack": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp]),
    "s2v_pad_reflect": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp,
                                 _c_int, _vp]),
    "s2v_row_layernorm": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _c_float, _vp, _c_int, _vp]),
    "s2v_attention": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll,
                               _c_ll, _c_float, _vp, _c_int, _c_ll, _vp]),
    "s2v_flow_warp": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_ll, _c_ll,
                               _c_ll, _c_ll, _vp, _c_int, _vp]),
    "s2v_flow_warp_cat": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_ll, _c_ll,
                                   _c_ll, _c_ll, _vp, _c_int, _vp]),
    "s2v_melspectrogram": (_c_int, [_vp, _c_ll, _vp, _c_int, _vp, _c_ll, _vp]),
    "s2v_mel_chunks": (_c_int, [_vp, _c_ll, _vp, _c_int, _c_int, _vp, _vp]),
    "s2v_fused_bias_act": (_c_int, [_vp, _vp, _vp, _vp, _c_ll, _c_int, _c_ll, _c_int, _c_int, _c_float, _c_float,
                                    _vp]),
    "s2v_upfirdn2d": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_int,
                               _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _vp]),
    "s2v_fused_bias_act_dt": (_c_int, [_c_int, _vp, _vp, _vp, _vp, _c_ll, _c_int, _c_ll, _c_int, _c_int,
                                       ctypes.c_double, ctypes.c_double, _vp]),
    "s2v_upfirdn2d_dt": (_c_int, [_c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int,
                                  _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _vp]),
    "s2v_fir2d": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_int,
                           _c_int, _vp, _c_int, _c_int, _c_int, _c_float, _vp, _c_int, _c_float, _c_float, _vp]),
    "s2v_fft_tables_floats": (_c_size, [_c_int, _c_int]),
    "s2v_rfft2": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _vp]),
    "s2v_irfft2": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _vp, _c_int, _vp]),
    "s2v_f16_split_check": (_c_int, [_vp, _c_ll, _vp, _vp]),
    "s2v_ffc_channels": (_c_int, [_c_int]),
    "s2v_ffc_spec_fwd": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_float, _c_float, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _c_int, _vp]),
    "s2v_ffc_spec_inv": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _c_float, _c_float, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _c_int, _vp]),
    "s2v_ffc_norm": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_float, _c_float, _vp, _vp, _c_int,
                              _c_float, _c_int, _c_float, _vp, _c_int, _vp, _c_int, _vp, _c_int, _vp, _c_int, _vp]),
    "s2v_split_weights": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_float, _vp, _vp]),
    "s2v_split_act": (_c_int, [_vp, _c_ll, _c_int, _c_int, _c_int, _vp, _c_int, _vp]),
    "s2v_amax": (_c_int, [_vp, _c_ll, _c_int, _c_int, _vp, _vp]),
    "s2v_split_weights_x3": (_c_int, [_vp, _c_int, _c_int, _vp, _vp]),
    "s2v_modulate_weights_split": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _c_int,
                                            _c_int, _c_int, _c_float, _vp, _vp]),
    "s2v_modulate_weights_x3": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _c_int,
                                         _c_int, _vp, _vp]),
    "s2v_modulate_weights": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _c_int, _c_int,
                                      _vp, _vp]),
    "s2v_gaussian_noise": (_c_int, [_vp, _c_ll, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    "s2v_gaussian_noise_ctr": (_c_int, [_vp, _c_ll, ctypes.c_uint64, ctypes.c_uint64, _vp, _c_int, _vp]),
    "s2v_counter_add": (_c_int, [_vp, ctypes.c_uint64, _vp]),
    "s2v_lipsync_inputs": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp]),
    "s2v_to_u8": (_c_int, [_vp, _c_ll, _c_float, _c_float, _c_float, _c_float, _vp, _vp]),
    "s2v_eltwise": (_c_int, [_vp, _c_int, _vp, _c_int, _vp, _c_int, _vp, _c_ll, _c_int, _c_float, _c_int, _c_float,
                             _c_float, _vp, _c_int, _vp]),
    "s2v_fill": (_c_int, [_vp, _c_ll, _c_float, _vp]),
    "s2v_resize_linear": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll, _vp, _c_int, _c_int, _c_ll,
                                   _c_ll, _c_int, _vp]),
    "s2v_resize_linear_fxfy": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll, _vp, _c_int, _c_int, _c_ll,
                                        _c_ll, _c_int, ctypes.c_double, ctypes.c_double, _vp]),
    "s2v_laplacian_blend_ws_bytes": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "s2v_laplacian_blend": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_size,
                                     _vp]),
    "s2v_parse_mask": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll, _c_ll, _vp, _vp, _vp, _vp]),
    "s2v_img_u8_to_m11": (_c_int, [_vp, _c_ll, _c_int, _vp, _c_int, _vp]),
    "s2v_sr_u8_in": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp]),
    "s2v_sr_f32_out": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp]),
    "s2v_bgr_mean_nhwc4": (_c_int, [_vp, _c_int, _c_ll, _vp, _vp]),
    "s2v_maxpool2d_nhwc": (_c_int, [_vp] + [_c_int] * 7 + [_vp, _c_int, _c_int, _vp]),
    "s2v_retina_decode": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_float, _vp, _vp, _c_int, _vp]),
    "s2v_retina_split": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp]),
    "s2v_warp_affine": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll, _c_int, _vp, _vp, _c_int, _c_int,
                                 _c_ll, _c_ll, _vp]),
    "s2v_face_paste": (_c_int, [_vp, _vp, _c_int, _vp, _vp, _vp] + [_c_int] * 6 + [_vp]),
    "s2v_gaussian_blur_ws_bytes": (_c_size, [_c_int, _c_int, _c_int]),
    "s2v_gaussian_blur": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp, _c_int, _c_int, _vp, _c_size,
                                   _vp]),
    "s2v_filter3x3_u8": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp]),
    "s2v_u8_to_gan": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "s2v_gan_to_u8": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "s2v_u8_div255_f64": (_c_int, [_vp, _c_ll, _vp, _vp]),
    "s2v_u8_div255_f64_border": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "s2v_face_blend": (_c_int, [_vp, _vp, _vp, _vp, _vp, _c_ll, _vp]),
    "s2v_warp_affine_border": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_ll, _c_ll, _c_int, _vp, _vp, _c_int,
                                        _c_int, _c_ll, _c_ll, _vp, _vp]),
    "s2v_tensor2img_u8": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "s2v_restore_mask": (_c_int, [_vp] + [_c_int] * 7 + [_vp, _vp, _vp]),
    "s2v_restore_parts": (_c_int, []),
    "s2v_erode_rect_f32": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp]),
    "s2v_restore_paste": (_c_int, [_vp, _c_int, _vp, _vp, _vp] + [_c_int] * 4 + [_vp, _c_int, _vp, _c_int, _c_int,
                                                                             _c_int, _vp]),
    "s2v_pil_resize_crop": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_ll, _vp, _c_int, _vp, _c_int, _c_int, _c_int,
                                     _vp]),
    "s2v_spatial_mean_nhwc": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "s2v_last_error": (ctypes.c_char_p, []),
    "s2v_device_cus": (_c_int, []),
    "s2v_version": (ctypes.c_char_p, []),
}

EXPORTS = tuple(_SIGS)

_lock = threading.Lock()
_lib = None


class S2VError(RuntimeError):
    pass


def load():
    """Load libs2v.so (raises if it was not built — there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise S2VError(f"{LIB_PATH} is missing: build it with `make -C {os.path.dirname(LIB_PATH)}/csrc` "
                               "(or __graft_entry__.build()); the HIP path has no CPU fallback")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().s2v_last_error().decode(errors="replace")
        raise S2VError(f"{what} failed ({rc}): {msg}")
