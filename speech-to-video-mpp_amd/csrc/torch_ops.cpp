// PyTorch custom-op boundary of libs2v: TORCH_LIBRARY(s2v) schemas with kernels for the HIP
// device only (dispatch key CUDA on ROCm builds).  There is no CPU kernel: a CPU tensor raises
// "could not run ... with arguments from the 'CPU' backend".  Every op validates its tensors,
// allocates its outputs through the PyTorch caching allocator and launches on the current HIP
// stream through the C ABI of include/s2v.h (the same kernels the model engines call).
//
//   s2v::fused_bias_act / s2v::upfirdn2d   the exact signatures of GPEN's pybind11 ops
//       (third_part/GPEN/face_model/op/fused_bias_act.cpp:4-21, upfirdn2d.cpp:4-23): with
//       `fused = torch.ops.s2v` and `upfirdn2d_op = torch.ops.s2v` the reference's
//       op/fused_act.py:60-66 / op/upfirdn2d.py:114-124 calls run unchanged.  Unlike the reference,
//       an unsupported upfirdn2d configuration raises instead of returning uninitialised memory.
//   model-path ops over whole tensors (NHWC activations, the engines' layout):
//       conv2d_nhwc, layernorm2d, instnorm_adain, attention, rfft2, irfft2, resize_bilinear,
//       flow_warp, mel_spectrogram.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include "../../include/s2v.h"

namespace {

void *stream() { return (void *)at::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char *what) {
    TORCH_CHECK(rc == 0, what, " failed (", rc, "): ", s2v_last_error());
}

void need_f32_dev(const at::Tensor &t, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, ": expected a HIP device tensor (the s2v ops have no CPU kernel)");
    TORCH_CHECK(t.scalar_type() == at::kFloat, name, ": expected float32, got ", t.scalar_type());
}

const float *fptr(const c10::optional<at::Tensor> &t) { return t && t->defined() ? t->data_ptr<float>() : nullptr; }

// ---------------------------------------------------------------- GPEN native-op signatures
// float32, float16 and float64, as the reference dispatches (AT_DISPATCH_FLOATING_TYPES_AND_HALF,
// fused_bias_act_kernel.cu:79, upfirdn2d_kernel.cu:225); every tensor argument in the input's dtype
// (the reference reads them with data_ptr<scalar_t>()).  Other dtypes raise.
int dt_code(const at::Tensor &t, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, ": expected a HIP device tensor (the s2v ops have no CPU kernel)");
    switch (t.scalar_type()) {
        case at::kFloat: return S2V_DT_F32;
        case at::kHalf: return S2V_DT_F16;
        case at::kDouble: return S2V_DT_F64;
        default: TORCH_CHECK(false, name, ": expected float32, float16 or float64, got ", t.scalar_type());
    }
    return -1;
}

void same_dtype(const at::Tensor &t, const at::Tensor &like, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, ": expected a HIP device tensor");
    TORCH_CHECK(t.scalar_type() == like.scalar_type(), name, ": expected ", like.scalar_type(), " like the input, got ",
                t.scalar_type());
}

at::Tensor fused_bias_act(const at::Tensor &input, const at::Tensor &bias, const at::Tensor &refer, int64_t act,
                          int64_t grad, double alpha, double scale) {
    const int dt = dt_code(input, "fused_bias_act input");
    const at::Tensor x = input.contiguous();
    const at::Tensor b = bias.numel() ? bias.contiguous() : bias;
    const at::Tensor r = refer.numel() ? refer.contiguous() : refer;
    if (b.numel()) same_dtype(b, x, "fused_bias_act bias");
    if (r.numel()) {
        same_dtype(r, x, "fused_bias_act refer");
        TORCH_CHECK(r.numel() == x.numel(), "fused_bias_act: refer has ", r.numel(), " elements, input ", x.numel());
    }
    auto y = at::empty_like(x);
    int c = 1;
    int64_t step_b = 1;
    if (x.dim() > 1) c = (int)x.size(1);
    for (int64_t i = 2; i < x.dim(); ++i) step_b *= x.size(i);
    TORCH_CHECK(b.numel() == 0 || b.numel() == c, "fused_bias_act: bias has ", b.numel(), " entries, input ", c,
                " channels");
    check(s2v_fused_bias_act_dt(dt, x.data_ptr(), b.numel() ? b.data_ptr() : nullptr, r.numel() ? r.data_ptr() : nullptr,
                                y.data_ptr(), x.numel(), c, step_b, (int)act, (int)grad, alpha, scale, stream()),
          "s2v_fused_bias_act");
    return y;
}

at::Tensor upfirdn2d(const at::Tensor &input, const at::Tensor &kernel, int64_t up_x, int64_t up_y, int64_t down_x,
                     int64_t down_y, int64_t pad_x0, int64_t pad_x1, int64_t pad_y0, int64_t pad_y1) {
    const int dt = dt_code(input, "upfirdn2d input");
    same_dtype(kernel, input, "upfirdn2d kernel");
    TORCH_CHECK(input.dim() == 4 && kernel.dim() == 2, "upfirdn2d: input [major, H, W, minor], kernel [kh, kw]");
    const at::Tensor x = input.contiguous(), k = kernel.contiguous();
    const int64_t major = x.size(0), in_h = x.size(1), in_w = x.size(2), minor = x.size(3);
    const int64_t kh = k.size(0), kw = k.size(1);
    const int64_t out_h = (in_h * up_y + pad_y0 + pad_y1 - kh) / down_y + 1;
    const int64_t out_w = (in_w * up_x + pad_x0 + pad_x1 - kw) / down_x + 1;
    TORCH_CHECK(out_h > 0 && out_w > 0, "upfirdn2d: empty output");
    auto y = at::empty({major, out_h, out_w, minor}, x.options());
    check(s2v_upfirdn2d_dt(dt, x.data_ptr(), (int)major, (int)in_h, (int)in_w, (int)minor, k.data_ptr(), (int)kh, (int)kw,
                           (int)up_x, (int)up_y, (int)down_x, (int)down_y, (int)pad_x0, (int)pad_x1, (int)pad_y0,
                           (int)pad_y1, y.data_ptr(), (int)out_h, (int)out_w, stream()),
          "s2v_upfirdn2d");
    return y;
}

// ---------------------------------------------------------------- model-path ops
// Implicit-GEMM conv over a whole NHWC tensor with packed weights [npad][kpad] (k = (ky*kw + kx)*cin
// + c) and, for the split precisions, the matching split copy (s2v_split_weights) and its scale.
at::Tensor conv2d_nhwc(const at::Tensor &x, const at::Tensor &w_packed, const c10::optional<at::Tensor> &w_split,
                       double wt_scale, int64_t cout, int64_t kh, int64_t kw, at::IntArrayRef stride,
                       at::IntArrayRef padding, at::IntArrayRef dilation, int64_t in_mode, int64_t pad_mode,
                       const c10::optional<at::Tensor> &scale, const c10::optional<at::Tensor> &shift, int64_t act,
                       double alpha, const c10::optional<at::Tensor> &res, bool res_after_act, int64_t prec,
                       bool pool) {
    need_f32_dev(x, "conv2d_nhwc x");
    need_f32_dev(w_packed, "conv2d_nhwc w_packed");
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "conv2d_nhwc: x must be a contiguous [N, H, W, C] tensor");
    TORCH_CHECK(w_packed.dim() == 2 && w_packed.is_contiguous(), "conv2d_nhwc: w_packed [npad, kpad]");
    TORCH_CHECK(stride.size() == 2 && padding.size() == 2 && dilation.size() == 2, "conv2d_nhwc: 2-element lists");
    s2v_conv_params p{};
    p.x = x.data_ptr<float>();
    p.n = (int)x.size(0); p.h = (int)x.size(1); p.w = (int)x.size(2); p.cin = (int)x.size(3); p.xcs = p.cin;
    p.in_mode = (int)in_mode; p.pad_mode = (int)pad_mode;
    p.kh = (int)kh; p.kw = (int)kw; p.sh = (int)stride[0]; p.sw = (int)stride[1];
    p.ph = (int)padding[0]; p.pw = (int)padding[1]; p.dh = (int)dilation[0]; p.dw = (int)dilation[1];
    p.wt = w_packed.data_ptr<float>(); p.npad = (int)w_packed.size(0); p.kpad = (int)w_packed.size(1);
    p.cout = (int)cout;
    int uh = p.h, uw = p.w;
    if (in_mode == S2V_IN_NEAREST_UP2) { uh *= 2; uw *= 2; }
    TORCH_CHECK(in_mode != S2V_IN_TRANSPOSED, "conv2d_nhwc: direct or nearest-x2 input only");
    p.oh = (uh + 2 * p.ph - p.dh * (p.kh - 1) - 1) / p.sh + 1;
    p.ow = (uw + 2 * p.pw - p.dw * (p.kw - 1) - 1) / p.sw + 1;
    TORCH_CHECK(p.oh > 0 && p.ow > 0, "conv2d_nhwc: empty output");
    const int f = pool ? 2 : 1;
    auto y = at::empty({p.n, p.oh / f, p.ow / f, cout}, x.options());
    p.y = y.data_ptr<float>(); p.ycs = (int)cout;
    p.scale = fptr(scale); p.shift = fptr(shift);
    at::Tensor r;
    if (res && res->defined()) {
        r = res->contiguous();
        need_f32_dev(r, "conv2d_nhwc res");
        TORCH_CHECK(r.sizes() == y.sizes(), "conv2d_nhwc: res must match the output shape");
        p.res = r.data_ptr<float>(); p.res_cs = (int)cout; p.res_h = p.oh; p.res_w = p.ow;
        p.res_after_act = res_after_act;
    }
    p.act = (int)act; p.alpha = (float)alpha;
    p.batch = 1;
    p.prec = (int)prec;
    p.out_pool = pool;
    if (prec != S2V_PREC_F32) {
        TORCH_CHECK(w_split && w_split->defined() && w_split->sizes() == w_packed.sizes(),
                    "conv2d_nhwc: split precisions need w_split (s2v_split_weights of w_packed)");
        p.wt_x3 = w_split->data_ptr();
        p.wt_scale = (float)wt_scale;
    }
    const size_t ws = s2v_conv2d_ws_bytes(&p);
    at::Tensor wsb;
    if (ws) {
        wsb = at::empty({(int64_t)ws}, x.options().dtype(at::kByte));
        p.ws = (float *)wsb.data_ptr(); p.ws_bytes = ws;
    }
    check(s2v_conv2d(&p, stream()), "s2v_conv2d");
    return y;
}

at::Tensor layernorm2d(const at::Tensor &x, const at::Tensor &weight, const at::Tensor &bias, double eps, int64_t act,
                       double alpha, bool pool) {
    need_f32_dev(x, "layernorm2d x");
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "layernorm2d: contiguous NHWC x");
    const int n = (int)x.size(0), h = (int)x.size(1), w = (int)x.size(2), c = (int)x.size(3);
    auto y = at::empty({n, pool ? h / 2 : h, pool ? w / 2 : w, c}, x.options());
    const size_t wsz = s2v_layernorm2d_ws_bytes(n, h, w, c);
    auto ws = at::empty({(int64_t)wsz}, x.options().dtype(at::kByte));
    const at::Tensor wg = weight.contiguous(), bs = bias.contiguous();
    check(s2v_layernorm2d(x.data_ptr<float>(), n, h, w, c, c, wg.data_ptr<float>(), bs.data_ptr<float>(), (float)eps,
                          (int)act, (float)alpha, pool, nullptr, 0, y.data_ptr<float>(), c, ws.data_ptr(), wsz,
                          stream()),
          "s2v_layernorm2d");
    return y;
}

at::Tensor instnorm_adain(const at::Tensor &x, const c10::optional<at::Tensor> &gamma,
                          const c10::optional<at::Tensor> &beta, double eps, int64_t act, double alpha) {
    need_f32_dev(x, "instnorm_adain x");
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "instnorm_adain: contiguous NHWC x");
    const int n = (int)x.size(0), h = (int)x.size(1), w = (int)x.size(2), c = (int)x.size(3);
    at::Tensor g, b;
    if (gamma && gamma->defined()) g = gamma->contiguous();
    if (beta && beta->defined()) b = beta->contiguous();
    TORCH_CHECK(!g.defined() || (g.dim() == 2 && g.size(0) == n && g.size(1) == c), "instnorm_adain: gamma [N, C]");
    TORCH_CHECK(!b.defined() || (b.dim() == 2 && b.size(0) == n && b.size(1) == c), "instnorm_adain: beta [N, C]");
    auto y = at::empty_like(x);
    const size_t wsz = s2v_instnorm_ws_bytes(n, h, w, c);
    auto ws = at::empty({(int64_t)wsz}, x.options().dtype(at::kByte));
    check(s2v_instnorm_adain(x.data_ptr<float>(), n, h, w, c, c, g.defined() ? g.data_ptr<float>() : nullptr,
                             b.defined() ? b.data_ptr<float>() : nullptr, c, (float)eps, (int)act, (float)alpha, nullptr,
                             0, y.data_ptr<float>(), c, ws.data_ptr(), wsz, stream()),
          "s2v_instnorm_adain");
    return y;
}

// q, k, v [B, T, heads * 64] -> softmax(q k^T * scale) v per head (transformer.py:73-80)
at::Tensor attention(const at::Tensor &q, const at::Tensor &k, const at::Tensor &v, int64_t heads, double scale) {
    need_f32_dev(q, "attention q");
    need_f32_dev(k, "attention k");
    need_f32_dev(v, "attention v");
    const at::Tensor qc = q.contiguous(), kc = k.contiguous(), vc = v.contiguous();
    TORCH_CHECK(qc.dim() == 3 && kc.sizes() == qc.sizes() && vc.size(0) == qc.size(0) && vc.size(1) == qc.size(1) &&
                    qc.size(2) == heads * 64 && vc.size(2) == heads * 64,
                "attention: q, k, v [B, T, heads*64]");
    const int b = (int)qc.size(0), t = (int)qc.size(1), d = (int)qc.size(2);
    auto o = at::empty_like(vc);
    check(s2v_attention(qc.data_ptr<float>(), kc.data_ptr<float>(), vc.data_ptr<float>(), b, (int)heads, t, 64, d, d,
                        d, (long long)t * d, (long long)t * d, (long long)t * d, (float)scale, o.data_ptr<float>(), d,
                        (long long)t * d, stream()),
          "s2v_attention");
    return o;
}

at::Tensor rfft2(const at::Tensor &x, const at::Tensor &tables) {
    need_f32_dev(x, "rfft2 x");
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "rfft2: contiguous NHWC x");
    const int n = (int)x.size(0), h = (int)x.size(1), w = (int)x.size(2), c = (int)x.size(3);
    auto spec = at::empty({n, (int64_t)h * (w / 2 + 1), 2 * (int64_t)c}, x.options());
    check(s2v_rfft2(x.data_ptr<float>(), n, h, w, c, c, tables.data_ptr<float>(), spec.data_ptr<float>(), 2 * c,
                    stream()),
          "s2v_rfft2");
    return spec;
}

at::Tensor irfft2(const at::Tensor &spec, const at::Tensor &tables, int64_t h, int64_t w,
                  const c10::optional<at::Tensor> &res) {
    need_f32_dev(spec, "irfft2 spec");
    TORCH_CHECK(spec.dim() == 3 && spec.is_contiguous() && spec.size(1) == h * (w / 2 + 1) && spec.size(2) % 2 == 0,
                "irfft2: spec [N, h*(w/2+1), 2C]");
    const int n = (int)spec.size(0), c = (int)spec.size(2) / 2;
    auto y = at::empty({n, h, w, c}, spec.options());
    at::Tensor r;
    if (res && res->defined()) {
        r = res->contiguous();
        TORCH_CHECK(r.sizes() == y.sizes(), "irfft2: res must be [N, h, w, C]");
    }
    check(s2v_irfft2(spec.data_ptr<float>(), n, (int)h, (int)w, c, 2 * c, tables.data_ptr<float>(),
                     r.defined() ? r.data_ptr<float>() : nullptr, c, y.data_ptr<float>(), c, stream()),
          "s2v_irfft2");
    return y;
}

// F.interpolate(x, (oh, ow), mode='bilinear' | 'nearest', align_corners=False) on NCHW input -> NCHW
at::Tensor resize_bilinear(const at::Tensor &x, int64_t oh, int64_t ow, double scale_h, double scale_w, int64_t mode) {
    need_f32_dev(x, "resize x");
    TORCH_CHECK(x.dim() == 4, "resize: NCHW x");
    auto y = at::empty({x.size(0), x.size(1), oh, ow}, x.options());
    check(s2v_resize(x.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), x.stride(0),
                     x.stride(1), x.stride(2), x.stride(3), y.data_ptr<float>(), (int)oh, (int)ow, y.stride(0),
                     y.stride(1), y.stride(2), y.stride(3), (float)scale_h, (float)scale_w, (int)mode, stream()),
          "s2v_resize");
    return y;
}

// flow_util.convert_flow_to_deformation + warp_image (flow_util.py:3-56): flow [N, 2, fh, fw],
// src [N, C, H, W] -> [N, C, H, W]
at::Tensor flow_warp(const at::Tensor &flow, const at::Tensor &src) {
    need_f32_dev(flow, "flow_warp flow");
    need_f32_dev(src, "flow_warp src");
    TORCH_CHECK(flow.dim() == 4 && flow.size(1) == 2 && src.dim() == 4 && src.size(0) == flow.size(0),
                "flow_warp: flow [N, 2, fh, fw], src [N, C, H, W]");
    const at::Tensor fl = flow.permute({0, 2, 3, 1}).contiguous();     // NHWC (x, y) pairs
    const int n = (int)src.size(0), c = (int)src.size(1), h = (int)src.size(2), w = (int)src.size(3);
    auto y = at::empty({n, h, w, c}, src.options());
    check(s2v_flow_warp(fl.data_ptr<float>(), n, (int)flow.size(2), (int)flow.size(3), 2, src.data_ptr<float>(), c, h,
                        w, src.stride(0), src.stride(1), src.stride(2), src.stride(3), y.data_ptr<float>(), c,
                        stream()),
          "s2v_flow_warp");
    return y.permute({0, 3, 1, 2});
}

// futils/audio.py melspectrogram: wav [S] -> [80, 1 + S / 200]; tables from s2v_amd.audio.tables()
at::Tensor mel_spectrogram(const at::Tensor &wav, const at::Tensor &tables, bool pad_reflect) {
    need_f32_dev(wav, "mel_spectrogram wav");
    need_f32_dev(tables, "mel_spectrogram tables");
    const at::Tensor x = wav.contiguous();
    TORCH_CHECK(x.dim() == 1, "mel_spectrogram: wav [S]");
    const int64_t frames = 1 + x.size(0) / 200;
    auto y = at::empty({80, frames}, x.options());
    check(s2v_melspectrogram(x.data_ptr<float>(), x.size(0), tables.data_ptr<float>(), pad_reflect, y.data_ptr<float>(),
                             frames, stream()),
          "s2v_melspectrogram");
    return y;
}

}  // namespace

TORCH_LIBRARY(s2v, m) {
    m.def("fused_bias_act(Tensor input, Tensor bias, Tensor refer, int act, int grad, float alpha, float scale) -> Tensor");
    m.def("upfirdn2d(Tensor input, Tensor kernel, int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1, "
          "int pad_y0, int pad_y1) -> Tensor");
    m.def("conv2d_nhwc(Tensor x, Tensor w_packed, Tensor? w_split, float wt_scale, int cout, int kh, int kw, "
          "int[2] stride, int[2] padding, int[2] dilation, int in_mode, int pad_mode, Tensor? scale, Tensor? shift, "
          "int act, float alpha, Tensor? res, bool res_after_act, int prec, bool pool) -> Tensor");
    m.def("layernorm2d(Tensor x, Tensor weight, Tensor bias, float eps, int act, float alpha, bool pool) -> Tensor");
    m.def("instnorm_adain(Tensor x, Tensor? gamma, Tensor? beta, float eps, int act, float alpha) -> Tensor");
    m.def("attention(Tensor q, Tensor k, Tensor v, int heads, float scale) -> Tensor");
    m.def("rfft2(Tensor x, Tensor tables) -> Tensor");
    m.def("irfft2(Tensor spec, Tensor tables, int h, int w, Tensor? res) -> Tensor");
    m.def("resize_bilinear(Tensor x, int oh, int ow, float scale_h, float scale_w, int mode) -> Tensor");
    m.def("flow_warp(Tensor flow, Tensor src) -> Tensor");
    m.def("mel_spectrogram(Tensor wav, Tensor tables, bool pad_reflect) -> Tensor");
}

TORCH_LIBRARY_IMPL(s2v, CUDA, m) {
    m.impl("fused_bias_act", &fused_bias_act);
    m.impl("upfirdn2d", &upfirdn2d);
    m.impl("conv2d_nhwc", &conv2d_nhwc);
    m.impl("layernorm2d", &layernorm2d);
    m.impl("instnorm_adain", &instnorm_adain);
    m.impl("attention", &attention);
    m.impl("rfft2", &rfft2);
    m.impl("irfft2", &irfft2);
    m.impl("resize_bilinear", &resize_bilinear);
    m.impl("flow_warp", &flow_warp);
    m.impl("mel_spectrogram", &mel_spectrogram);
}
