// Model-path launch ops of libs2v: TORCH_LIBRARY_FRAGMENT(s2v) ops that the engines (s2v_amd.ops,
// engine/*.py) dispatch for every kernel of the LNet / ENet / DNet / GFPGAN / GPEN forwards.  The
// reference's forwards are aten ops dispatched under torch.no_grad() (inference.py:266,
// models/ENet.py:82-139); these are their replacement at the same level: torch.profiler attributes
// the model path to ``s2v::*`` ops, and a hipGraph capture of a forward records just the kernels.
//
// Conventions (every op):
//   * the outputs are written in place into caller-owned tensors (schema ``Tensor(a!)``) — the
//     engines lay activations out once per forward, NHWC, with torch.cat / split as channel-slice
//     views; nothing here allocates, so every op is capturable;
//   * an NHWC view is a 4-D torch view [N, H, W, C] with unit channel stride and pixels of pitch
//     ``stride(2)`` (a channel slice of a contiguous NHWC tensor); the shapes and strides are
//     validated here (TORCH_CHECK -> RuntimeError), so a bad view is an error, not an out-of-bounds
//     device access;
//   * a device guard selects the inputs' device, and the kernels run on its current HIP stream;
//   * ops that need a split-K / norm workspace take ``Tensor? ws`` (uint8) and return the bytes they
//     need: when ``ws`` is missing or too small they launch nothing and return that size (> 0), the
//     caller grows its workspace (outside graph capture) and calls again; 0 means launched.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <vector>

#include "../../include/s2v.h"

namespace {

using at::Tensor;
using OptT = c10::optional<Tensor>;

void *stream() { return (void *)at::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char *what) { TORCH_CHECK(rc == 0, what, " failed (", rc, "): ", s2v_last_error()); }

bool has(const OptT &t) { return t && t->defined(); }

void same_dev(const Tensor &t, const at::Device &dev, const char *what) {
    TORCH_CHECK(t.is_cuda(), what, ": expected a HIP device tensor (the s2v ops have no CPU kernel)");
    TORCH_CHECK(t.device() == dev, what, ": on ", t.device(), ", the op's inputs are on ", dev);
}

void f32(const Tensor &t, const at::Device &dev, const char *what) {
    same_dev(t, dev, what);
    TORCH_CHECK(t.scalar_type() == at::kFloat, what, ": expected float32, got ", t.scalar_type());
}

// contiguous float32 device vector of at least ``n`` elements
const float *vec(const OptT &t, const at::Device &dev, int64_t n, const char *what) {
    if (!has(t)) return nullptr;
    f32(*t, dev, what);
    TORCH_CHECK(t->is_contiguous() && t->numel() >= n, what, ": contiguous, >= ", n, " elements (got ", t->numel(),
                ")");
    return t->data_ptr<float>();
}

// NHWC channel-slice view.  ``step`` > 1: every step-th pixel of a wider tensor in both directions
// (one output parity class of a polyphase transposed conv); full_h / full_w are that tensor's size.
struct NV {
    float *p;
    int n, h, w, c, cs;
    long long ns;
    int full_h, full_w;
};

NV nhwc(const Tensor &t, const at::Device &dev, const char *what, int step = 1, bool batch_any = false) {
    f32(t, dev, what);
    TORCH_CHECK(t.dim() == 4, what, ": NHWC view [N, H, W, C] expected, got ", t.dim(), "-D");
    TORCH_CHECK(t.size(3) > 0 && (t.stride(3) == 1 || t.size(3) == 1), what, ": channels must be contiguous (stride 1)");
    NV v{t.data_ptr<float>(), (int)t.size(0), (int)t.size(1), (int)t.size(2), (int)t.size(3), 0, t.stride(0), 0, 0};
    TORCH_CHECK(t.stride(2) % step == 0, what, ": pixel stride ", t.stride(2), " is not a multiple of step ", step);
    v.cs = (int)(t.stride(2) / step);
    TORCH_CHECK(v.cs >= v.c, what, ": pixel pitch ", v.cs, " < channels ", v.c);
    if (step == 1) {
        TORCH_CHECK(v.h == 1 || t.stride(1) == (int64_t)v.w * v.cs, what, ": rows must be contiguous pixel runs");
        TORCH_CHECK(batch_any || v.n == 1 || t.stride(0) == (int64_t)v.h * v.w * v.cs, what,
                    ": images must be contiguous [H, W] planes");
        v.full_h = v.h;
        v.full_w = v.w;
    } else {
        TORCH_CHECK(t.stride(1) % ((int64_t)step * v.cs) == 0, what, ": strided view rows");
        v.full_w = (int)(t.stride(1) / ((int64_t)step * v.cs));
        TORCH_CHECK(v.n == 1 || t.stride(0) % ((int64_t)v.full_w * v.cs) == 0, what, ": strided view planes");
        v.full_h = v.n == 1 ? step * v.h : (int)(t.stride(0) / ((int64_t)v.full_w * v.cs));
        TORCH_CHECK(v.full_w >= step * (v.w - 1) + 1 && v.full_h >= step * (v.h - 1) + 1, what, ": strided view extent");
    }
    return v;
}

// [rows, >= cols] row view (unit column stride); returns the row stride
int64_t rows_view(const Tensor &t, const at::Device &dev, int64_t rows, int64_t cols, const char *what) {
    f32(t, dev, what);
    TORCH_CHECK(t.dim() == 2 && t.size(0) == rows && t.size(1) >= cols && (cols <= 1 || t.stride(1) == 1), what,
                ": [", rows, ", ", cols, "] row view expected, got ", t.sizes(), " strides ", t.strides());
    return t.stride(0);
}

struct Ws {
    void *p = nullptr;
    size_t bytes = 0;
};

Ws workspace(const OptT &ws, const at::Device &dev) {
    Ws w;
    if (has(ws)) {
        same_dev(*ws, dev, "ws");
        TORCH_CHECK(ws->scalar_type() == at::kByte && ws->is_contiguous(), "ws: contiguous uint8 workspace");
        w.p = ws->data_ptr();
        w.bytes = (size_t)ws->numel();
    }
    return w;
}

// optional launch timer (s2v_conv_params.stamps): stamps uint64 pairs, stamp_ctr uint64 [1] replay
// counter, pos = (slot, stride, reps)
void set_stamps(s2v_conv_params &p, const OptT &stamps, const OptT &ctr, at::IntArrayRef pos, const at::Device &dev) {
    if (!has(stamps)) return;
    TORCH_CHECK(has(ctr) && pos.size() == 3, "conv stamps: stamp_ctr and (slot, stride, reps)");
    same_dev(*stamps, dev, "conv stamps");
    same_dev(*ctr, dev, "conv stamp_ctr");
    TORCH_CHECK(stamps->scalar_type() == at::kLong && stamps->is_contiguous() && ctr->scalar_type() == at::kLong &&
                    ctr->numel() >= 1,
                "conv stamps: int64 tensors");
    TORCH_CHECK(pos[0] >= 0 && pos[0] < pos[1] && pos[2] > 0 && stamps->numel() >= 2 * pos[1] * pos[2],
                "conv stamps: slot / stride / reps outside the stamp buffer");
    p.stamps = (unsigned long long *)stamps->data_ptr();
    p.stamp_ctr = (const unsigned long long *)ctr->data_ptr();
    p.stamp_slot = (int)pos[0]; p.stamp_stride = (int)pos[1]; p.stamp_reps = (int)pos[2];
}

// split-precision activation range (s2v_conv_params.x_scale / nonfinite): int32 [1] flag
void set_range(s2v_conv_params &p, double x_scale, const OptT &nonfinite, const at::Device &dev) {
    p.x_scale = (float)x_scale;
    if (!has(nonfinite)) return;
    same_dev(*nonfinite, dev, "conv nonfinite");
    TORCH_CHECK(nonfinite->scalar_type() == at::kInt && nonfinite->numel() >= 1, "conv nonfinite: int32 [1]");
    p.nonfinite = nonfinite->data_ptr<int>();
}

std::vector<int64_t> plan_list(const s2v_conv_params &p, int64_t need) {
    int pl[11] = {0};
    check(s2v_conv2d_plan(&p, pl), "s2v_conv2d_plan");
    std::vector<int64_t> out{need};
    for (int i = 0; i < 11; ++i) out.push_back(pl[i]);
    return out;
}

// ------------------------------------------------------------------------------------------ conv
// Shared parameter fill of conv2d_ / modulated_conv2d_.
void conv_common(s2v_conv_params &p, const Tensor &x, const Tensor &y, int64_t cout, at::IntArrayRef kernel,
                 at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t in_mode,
                 int64_t pad_mode, const OptT &scale, const OptT &shift, const OptT &pix_add, double pix_w,
                 const OptT &res, at::IntArrayRef res_offset, bool res_after_act, int64_t act, double alpha,
                 int64_t out_step, bool out_pool, bool x_split, bool batch_mode, int64_t prec, int64_t force_tile,
                 int64_t force_splits) {
    const at::Device dev = x.device();
    TORCH_CHECK(kernel.size() == 2 && stride.size() == 2 && padding.size() == 2 && dilation.size() == 2 &&
                    res_offset.size() == 2, "conv: kernel / stride / padding / dilation / res_offset are pairs");
    TORCH_CHECK(out_step >= 1 && (out_step == 1 || !out_pool), "conv: out_step >= 1 (no pooled strided output)");
    const NV xv = nhwc(x, dev, "conv x", 1, batch_mode);
    const NV yv = nhwc(y, dev, "conv y", (int)out_step, batch_mode);
    TORCH_CHECK(yv.n == xv.n, "conv: x has ", xv.n, " images, y ", yv.n);
    TORCH_CHECK(yv.c == cout, "conv: y has ", yv.c, " channels, cout is ", cout);
    p.x = xv.p; p.n = xv.n; p.h = xv.h; p.w = xv.w; p.cin = xv.c; p.xcs = xv.cs;
    p.in_mode = (int)in_mode; p.pad_mode = (int)pad_mode;
    p.kh = (int)kernel[0]; p.kw = (int)kernel[1]; p.sh = (int)stride[0]; p.sw = (int)stride[1];
    p.ph = (int)padding[0]; p.pw = (int)padding[1]; p.dh = (int)dilation[0]; p.dw = (int)dilation[1];
    // (negative padding: the polyphase sub-convolutions of a transposed conv, whose parity classes start
    // inside the input)
    TORCH_CHECK(p.kh > 0 && p.kw > 0 && p.sh > 0 && p.sw > 0 && p.dh > 0 && p.dw > 0 &&
                    (out_step > 1 || (p.ph >= 0 && p.pw >= 0)),
                "conv: bad kernel geometry");
    p.cout = (int)cout;
    p.y = yv.p; p.ycs = yv.cs;
    const int f = out_pool ? 2 : 1;
    p.oh = yv.h * f; p.ow = yv.w * f;
    if (out_step == 1 && in_mode != S2V_IN_TRANSPOSED) {
        int uh = p.h, uw = p.w;
        if (in_mode == S2V_IN_NEAREST_UP2) { uh *= 2; uw *= 2; }
        const int oh = (uh + 2 * p.ph - p.dh * (p.kh - 1) - 1) / p.sh + 1;
        const int ow = (uw + 2 * p.pw - p.dw * (p.kw - 1) - 1) / p.sw + 1;
        TORCH_CHECK(oh / f == yv.h && ow / f == yv.w, "conv: y is ", yv.h, "x", yv.w, ", the conv gives ", oh / f,
                    "x", ow / f);
        p.oh = oh; p.ow = ow;
    }
    if (out_step > 1) { p.out_step = (int)out_step; p.out_full_h = yv.full_h; p.out_full_w = yv.full_w; }
    p.scale = vec(scale, dev, cout, "conv scale");
    p.shift = vec(shift, dev, cout, "conv shift");
    if (has(pix_add)) {
        f32(*pix_add, dev, "conv pix_add");
        TORCH_CHECK(pix_add->is_contiguous() && pix_add->numel() == (int64_t)xv.n * p.oh * p.ow,
                    "conv pix_add: contiguous [N, OH, OW]");
        TORCH_CHECK(out_step == 1, "conv: no pix_add with a strided output");
        p.pix_add = pix_add->data_ptr<float>();
        p.pix_w = (float)pix_w;
    }
    if (has(res)) {
        const NV rv = nhwc(*res, dev, "conv res", (int)out_step, batch_mode);
        TORCH_CHECK(rv.n == xv.n && rv.c == cout, "conv res: [N, h, w, cout] expected");
        p.res = rv.p; p.res_cs = rv.cs; p.res_h = rv.h; p.res_w = rv.w;
        p.res_oy = (int)res_offset[0]; p.res_ox = (int)res_offset[1];
        TORCH_CHECK(out_step > 1 || (p.res_oy >= 0 && p.res_ox >= 0 && p.res_oy + p.oh <= rv.h &&
                                     p.res_ox + p.ow <= rv.w),
                    "conv res: the output window at (", p.res_oy, ", ", p.res_ox, ") leaves the ", rv.h, "x", rv.w,
                    " residual");
        TORCH_CHECK(out_step == 1 || rv.p == yv.p, "conv: a strided output takes only an in-place residual");
        p.res_after_act = res_after_act;
    }
    p.act = (int)act; p.alpha = (float)alpha;
    p.batch = 1;
    if (batch_mode) {   // one image per batch entry, each with its own weights
        p.batch = xv.n; p.n = 1;
        p.x_bs = xv.ns; p.y_bs = yv.n > 1 ? y.stride(0) : 0;
        if (p.res) p.res_bs = res->stride(0);
    }
    p.force_tile = (int)force_tile; p.force_splits = (int)force_splits;
    p.out_pool = out_pool;
    p.x_split = x_split;
    p.prec = (int)prec;
}

// Conv groups (s2v_conv2d_group): between group_begin_() and group_end_() every conv2d_ call is
// validated and recorded instead of launched; group_end_ launches the recorded convs as one group
// (or, when they cannot form one, one after the other).  Per thread: the recording belongs to the
// Python thread issuing the forward.
thread_local std::vector<s2v_conv_params> g_group;
thread_local bool g_recording = false;
thread_local int g_group_dev = 0;             // device index of the members (the launch goes to its stream)

void group_begin_() {
    TORCH_CHECK(!g_recording, "conv group: group_begin_ inside an open group");
    g_group.clear();
    g_recording = true;
}

void group_abort_() {
    g_group.clear();
    g_recording = false;
}

// Returns [ws_need] while the workspace is short (nothing launched, the group stays open), else
// [0, grouped] after the launch (grouped 1: one group launch; 0: the members launched one by one).
std::vector<int64_t> group_end_(const OptT &ws, bool dry) {
    TORCH_CHECK(g_recording, "conv group: group_end_ without group_begin_");
    const int n = (int)g_group.size();
    if (n == 0) {
        group_abort_();
        return {0, 0};
    }
    const at::Device dev(at::kCUDA, (c10::DeviceIndex)g_group_dev);
    const c10::DeviceGuard guard(dev);
    const Ws w = workspace(ws, dev);
    int gp[1 + S2V_CONV_GROUP_MAX] = {0};
    const bool grouped = n <= S2V_CONV_GROUP_MAX && s2v_conv2d_group_plan(g_group.data(), n, gp) == 0;
    size_t need = 0;
    if (grouped) {
        need = s2v_conv2d_group_ws_bytes(g_group.data(), n);
    } else {
        for (const auto &p : g_group) need = std::max(need, s2v_conv2d_ws_bytes(&p));
    }
    if (dry || w.bytes < need) return {(int64_t)need};
    if (grouped) {
        g_group[0].ws = (float *)w.p; g_group[0].ws_bytes = w.bytes;
        check(s2v_conv2d_group(g_group.data(), n, stream()), "s2v_conv2d_group");
    } else {
        for (auto &p : g_group) {
            p.ws = (float *)w.p; p.ws_bytes = w.bytes;
            check(s2v_conv2d(&p, stream()), "s2v_conv2d");
        }
    }
    group_abort_();
    return {0, grouped ? 1 : 0};
}

// Implicit-GEMM convolution (s2v_conv_params, include/s2v.h) with packed weights [npad][kpad]
// (and, for the split precisions, their s2v_split_weights copy).  Returns [ws_need, plan...]:
// ws_need 0 = launched (or dry run of a launch that needs no workspace); > 0 = bytes of workspace
// the launch needs (nothing launched when ``ws`` is smaller, or ``dry``); plan = s2v_conv2d_plan's
// eleven ints (the kernel instance the launch runs).
std::vector<int64_t> conv2d_(const Tensor &x, const Tensor &y, const Tensor &wt, const OptT &wt_split,
                             double wt_scale, int64_t cout, at::IntArrayRef kernel, at::IntArrayRef stride,
                             at::IntArrayRef padding, at::IntArrayRef dilation, int64_t in_mode, int64_t pad_mode,
                             int64_t prec, const OptT &scale, const OptT &shift, const OptT &in_scale,
                             const OptT &nc_scale, int64_t pre_act, double pre_alpha, const OptT &pix_add,
                             double pix_w, const OptT &res, at::IntArrayRef res_offset, bool res_after_act,
                             int64_t act, double alpha, int64_t out_step, bool out_pool, bool x_split, const OptT &ws,
                             int64_t grid_cap, int64_t force_tile, int64_t force_splits, const OptT &stamps,
                             const OptT &stamp_ctr, at::IntArrayRef stamp_pos, double x_scale, const OptT &nonfinite,
                             bool dry, const OptT &post_mul, const OptT &post_add, int64_t post_c0, const OptT &dup_src,
                             const OptT &dup_bias, double dup_a, int64_t dup_off) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    s2v_conv_params p{};
    conv_common(p, x, y, cout, kernel, stride, padding, dilation, in_mode, pad_mode, scale, shift, pix_add, pix_w, res,
                res_offset, res_after_act, act, alpha, out_step, out_pool, x_split, false, prec, force_tile,
                force_splits);
    if (has(post_mul) || has(post_add)) {      // SFT fold: NHWC views of the output's pixels, cout - post_c0 channels
        TORCH_CHECK(has(post_mul) && has(post_add), "conv: post_mul and post_add go together");
        const NV mv = nhwc(*post_mul, dev, "conv post_mul"), av = nhwc(*post_add, dev, "conv post_add");
        TORCH_CHECK(mv.n == p.n && mv.h == p.oh && mv.w == p.ow && mv.c == cout - post_c0 && av.n == mv.n &&
                        av.h == mv.h && av.w == mv.w && av.c == mv.c && av.cs == mv.cs,
                    "conv post_mul / post_add: [N, OH, OW, cout - post_c0] views of one pitch");
        p.post_mul = mv.p; p.post_add = av.p; p.post_cs = mv.cs; p.post_c0 = (int)post_c0;
    }
    if (has(dup_src)) {                         // second output: act(dup_a * dup_src + dup_bias) at channel dup_off
        const NV dv = nhwc(*dup_src, dev, "conv dup_src");
        TORCH_CHECK(dv.n == p.n && dv.h == p.oh && dv.w == p.ow && dv.c == cout, "conv dup_src: [N, OH, OW, cout]");
        p.dup_src = dv.p; p.dup_cs = dv.cs; p.dup_a = (float)dup_a; p.dup_off = (int)dup_off;
        p.dup_bias = vec(dup_bias, dev, cout, "conv dup_bias");
    }
    f32(wt, dev, "conv wt");
    TORCH_CHECK(wt.dim() == 2 && wt.is_contiguous() && wt.size(0) >= cout, "conv wt: packed [npad, kpad]");
    p.wt = wt.data_ptr<float>(); p.npad = (int)wt.size(0); p.kpad = (int)wt.size(1);
    TORCH_CHECK((int64_t)p.kpad >= (int64_t)p.kh * p.kw * p.cin, "conv wt: kpad ", p.kpad, " < K ",
                p.kh * p.kw * p.cin);
    p.pre_act = (int)pre_act; p.pre_alpha = (float)pre_alpha;
    if (has(in_scale)) {
        p.in_scale = in_scale->data_ptr<float>();
        p.in_scale_ns = (int)rows_view(*in_scale, dev, p.n, p.cin, "conv in_scale");
    }
    if (has(nc_scale)) {
        p.nc_scale = nc_scale->data_ptr<float>();
        p.nc_scale_ns = (int)rows_view(*nc_scale, dev, p.n, cout, "conv nc_scale");
    }
    if (prec != S2V_PREC_F32) {
        // the plan only checks that split weights are present before choosing an x3 kernel
        p.wt_x3 = p.wt;
        int pl[11] = {0};
        check(s2v_conv2d_plan(&p, pl), "s2v_conv2d_plan");
        p.wt_x3 = nullptr;
        if (pl[6]) {
            TORCH_CHECK(has(wt_split) && wt_split->sizes() == wt.sizes() && wt_split->device() == dev &&
                            wt_split->is_contiguous(),
                        "conv: the split precisions need wt_split (s2v_split_weights of wt, same shape)");
            p.wt_x3 = wt_split->data_ptr();
            p.wt_scale = (float)wt_scale;
        }
    }
    TORCH_CHECK(grid_cap >= 0 && grid_cap % 8 == 0, "conv grid_cap: 0 or a positive multiple of 8");
    p.grid_cap = (int)grid_cap;
    set_stamps(p, stamps, stamp_ctr, stamp_pos, dev);
    set_range(p, x_scale, nonfinite, dev);
    if (g_recording && !dry) {            // conv group: record (validated by the plan) instead of launching
        TORCH_CHECK(!p.stamps, "conv group: no launch stamps on group members");
        TORCH_CHECK(g_group.empty() || g_group_dev == dev.index(), "conv group: members on one device");
        auto out = plan_list(p, 0);
        g_group_dev = dev.index();
        g_group.push_back(p);
        return out;
    }
    const size_t need = s2v_conv2d_ws_bytes(&p);
    const Ws w = workspace(ws, dev);
    if (dry || w.bytes < need) return plan_list(p, (int64_t)need);
    p.ws = (float *)w.p; p.ws_bytes = w.bytes;
    auto out = plan_list(p, 0);
    check(s2v_conv2d(&p, stream()), "s2v_conv2d");
    return out;
}

// StyleGAN2 modulated conv (base_blocks.py:487-533, stylegan2_clean_arch.py:66-99, gpen_model.py:
// 225-262) with per-sample weights: W * s[b, i] (* d[b, o]) written into ``wbuf`` ([B, npad, kpad]
// fp32-sized) in the form the planned kernel reads (the split layout of ``prec`` with a 2^11 f16
// pre-scale when demodulated, or fp32), then one batched conv.  Returns as conv2d_.
std::vector<int64_t> modulated_conv2d_(const Tensor &x, const Tensor &y, const Tensor &wt, const Tensor &s,
                                       const OptT &d, const Tensor &wbuf, int64_t cout, at::IntArrayRef kernel,
                                       at::IntArrayRef padding, int64_t in_mode, int64_t prec, bool x_split,
                                       const OptT &scale,
                                       const OptT &shift, const OptT &pix_add,
                                       double pix_w, const OptT &res, bool res_after_act, int64_t act, double alpha,
                                       const OptT &ws, int64_t force_splits, const OptT &stamps, const OptT &stamp_ctr,
                                       at::IntArrayRef stamp_pos, double x_scale, const OptT &nonfinite, bool dry,
                                       int64_t d2s, int64_t force_tile, double premod) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    TORCH_CHECK(!g_recording, "conv group: modulated convs cannot be group members");
    s2v_conv_params p{};
    const int64_t one[2] = {1, 1}, zero[2] = {0, 0};
    TORCH_CHECK(in_mode == S2V_IN_DIRECT || in_mode == S2V_IN_NEAREST_UP2, "modconv: direct or nearest-x2 input");
    if (d2s) {
        // depth-to-space (polyphase x2 upsample): y is the full [N, 2H, 2W, cout / 4] output; the conv
        // runs on x's grid with its 4 parity classes as 4 blocks of cout / 4 output columns
        TORCH_CHECK(cout % 4 == 0 && in_mode == S2V_IN_DIRECT && !has(res) && y.dim() == 4 &&
                        y.size(3) == cout / 4 && y.size(1) % 2 == 0 && y.size(2) % 2 == 0,
                    "modconv d2s: y [N, 2H, 2W, cout / 4], direct input, no res");
        const Tensor yc = y.slice(1, 0, y.size(1), 2).slice(2, 0, y.size(2), 2);   // parity class (0, 0)
        conv_common(p, x, yc, cout / 4, kernel, at::IntArrayRef(one, 2), padding, at::IntArrayRef(one, 2), in_mode,
                    S2V_PAD_ZERO, scale, shift, c10::nullopt, 0.0, res, at::IntArrayRef(zero, 2), false, act, alpha, 2,
                    false, x_split, true, prec, force_tile, force_splits);
        p.cout = (int)cout;
        p.d2s_cout = (int)(cout / 4);
        TORCH_CHECK(!p.scale || (scale->numel() >= cout), "modconv d2s: scale needs cout entries");
        TORCH_CHECK(!p.shift || (shift->numel() >= cout), "modconv d2s: shift needs cout entries");
        if (has(pix_add)) {
            f32(*pix_add, dev, "modconv pix_add");
            TORCH_CHECK(pix_add->is_contiguous() && pix_add->numel() == y.size(0) * y.size(1) * y.size(2),
                        "modconv d2s pix_add: contiguous [N, 2H, 2W]");
            p.pix_add = pix_add->data_ptr<float>();
            p.pix_w = (float)pix_w;
        }
    } else {
        conv_common(p, x, y, cout, kernel, at::IntArrayRef(one, 2), padding, at::IntArrayRef(one, 2), in_mode,
                    S2V_PAD_ZERO, scale, shift, pix_add, pix_w, res, at::IntArrayRef(zero, 2), res_after_act, act, alpha,
                    1, false, x_split, true, prec, force_tile, force_splits);
    }
    f32(wt, dev, "modconv wt");
    TORCH_CHECK(wt.dim() == 2 && wt.is_contiguous() && wt.size(0) >= cout, "modconv wt: packed [npad, kpad]");
    const int npad = (int)wt.size(0), kpad = (int)wt.size(1), K = p.kh * p.kw * p.cin, B = p.batch;
    TORCH_CHECK(kpad >= K, "modconv wt: kpad < K");
    const int s_ns = (int)rows_view(s, dev, B, p.cin, "modconv s");
    int d_ns = 0;
    if (has(d)) d_ns = (int)rows_view(*d, dev, B, cout, "modconv d");
    f32(wbuf, dev, "modconv wbuf");
    TORCH_CHECK(wbuf.is_contiguous() && wbuf.numel() >= (int64_t)B * npad * kpad, "modconv wbuf: [B, npad, kpad]");
    p.wt = wbuf.data_ptr<float>(); p.npad = npad; p.kpad = kpad;
    p.w_bs = (long long)npad * kpad;
    bool x3 = false;
    if (prec != S2V_PREC_F32) {
        p.wt_x3 = p.wt;
        int pl[11] = {0};
        check(s2v_conv2d_plan(&p, pl), "s2v_conv2d_plan");
        x3 = pl[6] != 0;
        p.wt_x3 = nullptr;
    }
    float wscale = 1.f;
    if (x3) {
        // demodulated rows have |w * s * d| <= post (sqrt 2 on these paths): f16 halves take a fixed 2^11
        // pre-scale; without demodulation the range is open and the weights go unscaled
        wscale = (prec == S2V_PREC_F16X3 && has(d)) ? 2048.f : 1.f;
        p.wt = nullptr; p.wt_x3 = wbuf.data_ptr(); p.wt_scale = wscale;
    }
    set_stamps(p, stamps, stamp_ctr, stamp_pos, dev);
    set_range(p, x_scale, nonfinite, dev);
    const size_t need = s2v_conv2d_ws_bytes(&p);
    const Ws w = workspace(ws, dev);
    if (dry || w.bytes < need) return plan_list(p, (int64_t)need);
    p.ws = (float *)w.p; p.ws_bytes = w.bytes;
    auto out = plan_list(p, 0);
    const float *dp = has(d) ? d->data_ptr<float>() : nullptr;
    // premod != 0: wbuf already holds the modulated weights (modulate_weights_, e.g. written on a side stream
    // ahead of the conv): > 0 the split layout at that pre-scale, < 0 fp32; they must be the layout this plan reads
    TORCH_CHECK(premod == 0.0 || (x3 ? premod == (double)wscale : premod < 0.0),
                "modconv: the pre-modulated weights (premod ", premod, ") are not the layout this conv reads (",
                x3 ? "split, pre-scale " : "fp32", x3 ? wscale : 0.f, ")");
    if (premod == 0.0 && x3)
        check(s2v_modulate_weights_split(wt.data_ptr<float>(), npad, kpad, K, p.cin, (int)cout, s.data_ptr<float>(),
                                         s_ns, dp, d_ns, B, (int)prec, wscale, wbuf.data_ptr(), stream()),
              "s2v_modulate_weights_split");
    else if (premod == 0.0)
        check(s2v_modulate_weights(wt.data_ptr<float>(), npad, kpad, K, p.cin, (int)cout, s.data_ptr<float>(), s_ns, dp,
                                   d_ns, B, wbuf.data_ptr<float>(), stream()),
              "s2v_modulate_weights");
    check(s2v_conv2d(&p, stream()), "s2v_conv2d");
    return out;
}

// The per-sample modulation alone (W * s[b, c] (* d[b, o]) into wbuf [B, npad, kpad]): prec != f32 writes the
// split layout at pre-scale wscale (what modulated_conv2d_ plans for a split-precision conv), f32 plain fp32.  A
// later modulated_conv2d_(..., premod) reads it instead of modulating again.
void modulate_weights_(const Tensor &wt, const Tensor &s, const OptT &d, const Tensor &wbuf, int64_t cout, int64_t cin,
                       int64_t taps, int64_t prec, double wscale) {
    const c10::DeviceGuard guard(wt.device());
    const at::Device dev = wt.device();
    f32(wt, dev, "modulate wt");
    TORCH_CHECK(wt.dim() == 2 && wt.is_contiguous() && wt.size(0) >= cout, "modulate wt: packed [npad, kpad]");
    const int npad = (int)wt.size(0), kpad = (int)wt.size(1), K = (int)(taps * cin);
    TORCH_CHECK(kpad >= K && cin > 0 && cout > 0, "modulate: kpad < taps * cin");
    f32(wbuf, dev, "modulate wbuf");
    TORCH_CHECK(wbuf.dim() == 3 && wbuf.is_contiguous() && wbuf.size(1) == npad && wbuf.size(2) == kpad,
                "modulate wbuf: [B, npad, kpad]");
    const int B = (int)wbuf.size(0);
    const int s_ns = (int)rows_view(s, dev, B, cin, "modulate s");
    int d_ns = 0;
    if (has(d)) d_ns = (int)rows_view(*d, dev, B, cout, "modulate d");
    const float *dp = has(d) ? d->data_ptr<float>() : nullptr;
    if (prec != S2V_PREC_F32)
        check(s2v_modulate_weights_split(wt.data_ptr<float>(), npad, kpad, K, (int)cin, (int)cout, s.data_ptr<float>(),
                                         s_ns, dp, d_ns, B, (int)prec, (float)wscale, wbuf.data_ptr(), stream()),
              "s2v_modulate_weights_split");
    else
        check(s2v_modulate_weights(wt.data_ptr<float>(), npad, kpad, K, (int)cin, (int)cout, s.data_ptr<float>(), s_ns,
                                   dp, d_ns, B, wbuf.data_ptr<float>(), stream()),
              "s2v_modulate_weights");
}

// batched activation GEMM out[z] = a[z] @ b[z] (+ res[z]): a [.., M, K], b [.., K, N], out [.., M, N]
// row-major with unit column stride (the FourierUnit DFT products).  Returns as conv2d_.
std::vector<int64_t> gemm_kn_(const Tensor &a, const Tensor &b, const Tensor &out, int64_t batch, int64_t a_bs,
                              int64_t b_bs, int64_t out_bs, const OptT &res, int64_t res_bs, int64_t act, double alpha,
                              int64_t prec, const OptT &ws, int64_t force_tile, int64_t force_splits, bool dry) {
    const c10::DeviceGuard guard(a.device());
    const at::Device dev = a.device();
    f32(a, dev, "gemm a"); f32(b, dev, "gemm b"); f32(out, dev, "gemm out");
    TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && out.is_contiguous(), "gemm: contiguous operands");
    const int64_t M = a.size(-2), K = a.size(-1), N = b.size(-1);
    TORCH_CHECK(b.size(-2) == K && out.size(-2) == M && out.size(-1) == N, "gemm: [M, K] @ [K, N] -> [M, N]");
    TORCH_CHECK(batch >= 1 && (batch - 1) * a_bs + M * K <= a.numel() && (batch - 1) * b_bs + K * N <= b.numel() &&
                    (batch - 1) * out_bs + M * N <= out.numel(),
                "gemm: batch strides leave the operands");
    s2v_conv_params p{};
    p.x = a.data_ptr<float>(); p.n = 1; p.h = 1; p.w = (int)M; p.cin = (int)K; p.xcs = (int)K;
    p.kh = p.kw = p.sh = p.sw = p.dh = p.dw = 1;
    p.wt = b.data_ptr<float>(); p.cout = (int)N; p.b_kn = 1; p.ldb = (int)N;
    p.prec = (int)prec;
    p.y = out.data_ptr<float>(); p.oh = 1; p.ow = (int)M; p.ycs = (int)N;
    if (has(res)) {
        f32(*res, dev, "gemm res");
        TORCH_CHECK(res->is_contiguous() && (batch - 1) * res_bs + M * N <= res->numel(), "gemm res");
        p.res = res->data_ptr<float>(); p.res_cs = (int)N; p.res_h = 1; p.res_w = (int)M; p.res_bs = res_bs;
    }
    p.act = (int)act; p.alpha = (float)alpha;
    p.batch = (int)batch; p.x_bs = a_bs; p.w_bs = b_bs; p.y_bs = out_bs;
    p.force_tile = (int)force_tile; p.force_splits = (int)force_splits;
    const size_t need = s2v_conv2d_ws_bytes(&p);
    const Ws w = workspace(ws, dev);
    if (dry || w.bytes < need) return plan_list(p, (int64_t)need);
    p.ws = (float *)w.p; p.ws_bytes = w.bytes;
    auto o = plan_list(p, 0);
    check(s2v_conv2d(&p, stream()), "s2v_conv2d(gemm)");
    return o;
}

// max |x| of an NHWC view into out (float32 [1], zeroed here first)
void amax_(const Tensor &x, const Tensor &out) {
    const c10::DeviceGuard guard(x.device());
    const NV xv = nhwc(x, x.device(), "amax x");
    f32(out, x.device(), "amax out");
    TORCH_CHECK(out.numel() >= 1 && out.is_contiguous(), "amax out: float32 [1]");
    check(s2v_fill(out.data_ptr<float>(), 1, 0.f, stream()), "s2v_fill");
    check(s2v_amax(xv.p, (long long)xv.n * xv.h * xv.w, xv.c, xv.cs, out.data_ptr<float>(), stream()), "s2v_amax");
}

void split_weights_(const Tensor &w, const Tensor &out, int64_t prec, double scale) {
    const c10::DeviceGuard guard(w.device());
    f32(w, w.device(), "split_weights w");
    f32(out, w.device(), "split_weights out");
    TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && out.sizes() == w.sizes() && out.is_contiguous() &&
                    w.size(1) % 32 == 0,
                "split_weights: packed [rows, kpad], kpad % 32 == 0, out of the same shape");
    check(s2v_split_weights(w.data_ptr<float>(), (int)w.size(0), (int)w.size(1), (int)prec, (float)scale,
                            out.data_ptr(), stream()),
          "s2v_split_weights");
}

void split_act_(const Tensor &x, const Tensor &out, int64_t prec) {
    const c10::DeviceGuard guard(x.device());
    const NV xv = nhwc(x, x.device(), "split_act x"), ov = nhwc(out, x.device(), "split_act out");
    TORCH_CHECK(xv.n == ov.n && xv.h == ov.h && xv.w == ov.w && xv.c == ov.c, "split_act: out must match x");
    check(s2v_split_act(xv.p, (long long)xv.n * xv.h * xv.w, xv.c, xv.cs, (int)prec, ov.p, ov.cs, stream()),
          "s2v_split_act");
}

// ------------------------------------------------------------------------------------------ norms
int64_t layernorm2d_(const Tensor &x, const Tensor &weight, const Tensor &bias, double eps, int64_t act,
                     double alpha, bool pool, const OptT &res, const Tensor &y, const OptT &ws) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "layernorm2d x"), yv = nhwc(y, dev, "layernorm2d y");
    const int f = pool ? 2 : 1;
    TORCH_CHECK(yv.n == xv.n && yv.h * f == xv.h && yv.w * f == xv.w && yv.c == xv.c, "layernorm2d: y shape");
    const float *wp = vec(weight, dev, xv.c, "layernorm2d weight"), *bp = vec(bias, dev, xv.c, "layernorm2d bias");
    const float *rp = nullptr;
    int rcs = 0;
    if (has(res)) {
        const NV rv = nhwc(*res, dev, "layernorm2d res");
        TORCH_CHECK(rv.n == yv.n && rv.h == yv.h && rv.w == yv.w && rv.c == yv.c, "layernorm2d: res shape");
        rp = rv.p; rcs = rv.cs;
    }
    const size_t need = s2v_layernorm2d_ws_bytes(xv.n, xv.h, xv.w, xv.c);
    const Ws w = workspace(ws, dev);
    if (w.bytes < need) return (int64_t)need;
    check(s2v_layernorm2d(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, wp, bp, (float)eps, (int)act, (float)alpha, pool, rp,
                          rcs, yv.p, yv.cs, w.p, w.bytes, stream()),
          "s2v_layernorm2d");
    return 0;
}

// gamma / beta: [N, C] row views (ADAIN parameters, base_blocks.py:143-157) or absent
int64_t instnorm_(const Tensor &x, const OptT &gamma, const OptT &beta, double eps, int64_t act, double alpha,
                  const OptT &res, const Tensor &y, const OptT &pad_out, const OptT &ws) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "instnorm x"), yv = nhwc(y, dev, "instnorm y");
    TORCH_CHECK(yv.n == xv.n && yv.h == xv.h && yv.w == xv.w && yv.c == xv.c, "instnorm: y shape");
    TORCH_CHECK(has(gamma) == has(beta), "instnorm: gamma and beta together");
    const float *gp = nullptr, *bp = nullptr;
    int ns = 0;
    if (has(gamma)) {
        ns = (int)rows_view(*gamma, dev, xv.n, xv.c, "instnorm gamma");
        TORCH_CHECK(rows_view(*beta, dev, xv.n, xv.c, "instnorm beta") == ns, "instnorm: gamma / beta row strides");
        gp = gamma->data_ptr<float>(); bp = beta->data_ptr<float>();
    }
    const float *rp = nullptr;
    int rcs = 0;
    if (has(res)) {
        const NV rv = nhwc(*res, dev, "instnorm res");
        TORCH_CHECK(rv.n == xv.n && rv.h == xv.h && rv.w == xv.w && rv.c == xv.c, "instnorm: res shape");
        rp = rv.p; rcs = rv.cs;
    }
    const size_t need = s2v_instnorm_ws_bytes(xv.n, xv.h, xv.w, xv.c);
    const Ws w = workspace(ws, dev);
    if (w.bytes < need) return (int64_t)need;
    if (has(pad_out)) {
        const NV pv = nhwc(*pad_out, dev, "instnorm pad_out");
        TORCH_CHECK(pv.n == xv.n && pv.h == xv.h + 2 && pv.w == xv.w + 2 && pv.c == xv.c,
                    "instnorm pad_out: [N, H + 2, W + 2, C]");
        check(s2v_instnorm_adain_pad(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, gp, bp, ns, (float)eps, (int)act,
                                     (float)alpha, rp, rcs, yv.p, yv.cs, pv.p, pv.cs, w.p, w.bytes, stream()),
              "s2v_instnorm_adain_pad");
    } else {
        check(s2v_instnorm_adain(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, gp, bp, ns, (float)eps, (int)act, (float)alpha, rp,
                                 rcs, yv.p, yv.cs, w.p, w.bytes, stream()),
              "s2v_instnorm_adain");
    }
    return 0;
}

void adain_params_(const Tensor &hid, int64_t nhidden, const Tensor &w2t, const Tensor &bias, const Tensor &seg,
                   const Tensor &out) {
    const c10::DeviceGuard guard(hid.device());
    const at::Device dev = hid.device();
    const int64_t batch = out.size(0), total = out.size(1);
    const int64_t hns = rows_view(hid, dev, batch, 1, "adain hid");
    const int64_t ons = rows_view(out, dev, batch, total, "adain out");
    f32(w2t, dev, "adain w2t");
    TORCH_CHECK(w2t.is_contiguous() && w2t.dim() == 2 && w2t.size(0) == nhidden && w2t.size(1) == total,
                "adain w2t: [nhidden, total]");
    vec(bias, dev, total, "adain bias");
    same_dev(seg, dev, "adain seg");
    TORCH_CHECK(seg.scalar_type() == at::kInt && seg.is_contiguous() && seg.numel() >= total, "adain seg: int32 [total]");
    check(s2v_adain_params(hid.data_ptr<float>(), (int)batch, (int)hns, (int)nhidden, w2t.data_ptr<float>(),
                           bias.data_ptr<float>(), seg.data_ptr<int>(), (int)total, out.data_ptr<float>(), (int)ons,
                           stream()),
          "s2v_adain_params");
}

void modconv_demod_(const Tensor &s, const Tensor &wsq, const Tensor &d, double eps, double post) {
    const c10::DeviceGuard guard(s.device());
    const at::Device dev = s.device();
    const int64_t batch = d.size(0), cout = wsq.size(0), cin = wsq.size(1);
    const int64_t sns = rows_view(s, dev, batch, cin, "demod s"), dns = rows_view(d, dev, batch, cout, "demod d");
    vec(wsq, dev, cout * cin, "demod wsq");
    check(s2v_modconv_demod(s.data_ptr<float>(), (int)batch, (int)sns, (int)cin, wsq.data_ptr<float>(), (int)cout,
                            (float)eps, (float)post, d.data_ptr<float>(), (int)dns, stream()),
          "s2v_modconv_demod");
}

void modconv_demod_rows_(const Tensor &s, const Tensor &rows, const Tensor &wsq, const Tensor &d, double eps,
                         double post, int64_t s_reach) {
    const c10::DeviceGuard guard(s.device());
    const at::Device dev = s.device();
    const int64_t batch = d.size(0), nrows = rows.size(0);
    same_dev(rows, dev, "demod rows");
    TORCH_CHECK(rows.scalar_type() == at::kInt && rows.is_contiguous() && rows.dim() == 2 && rows.size(1) == 4,
                "demod rows: int32 [nrows, 4]");
    // s_reach: the table's largest s_off + cin (ops.DemodRows checks the table against wsq on the host)
    const int64_t sns = rows_view(s, dev, batch, std::max<int64_t>(s_reach, 2), "demod s");
    vec(wsq, dev, wsq.numel(), "demod wsq");
    const int64_t dns = rows_view(d, dev, batch, nrows, "demod d");
    check(s2v_modconv_demod_rows(s.data_ptr<float>(), (int)batch, (int)sns, rows.data_ptr<int>(), (int)nrows,
                                 wsq.data_ptr<float>(), (float)eps, (float)post, d.data_ptr<float>(), (int)dns,
                                 stream()),
          "s2v_modconv_demod_rows");
}

void row_layernorm_(const Tensor &x, const Tensor &weight, const Tensor &bias, double eps, const Tensor &y) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const int64_t rows = x.size(0), dim = x.size(1);
    const int64_t xld = rows_view(x, dev, rows, dim, "row_layernorm x");
    const int64_t yld = rows_view(y, dev, rows, dim, "row_layernorm y");
    check(s2v_row_layernorm(x.data_ptr<float>(), (int)rows, (int)dim, (int)xld, vec(weight, dev, dim, "ln weight"),
                            vec(bias, dev, dim, "ln bias"), (float)eps, y.data_ptr<float>(), (int)yld, stream()),
          "s2v_row_layernorm");
}

// q, k, v, out: [batch * tokens, >= heads * dim_head] row views (transformer.py:73-80)
void attention_(const Tensor &q, const Tensor &k, const Tensor &v, const Tensor &out, int64_t batch, int64_t heads,
                int64_t tokens, int64_t dim_head, double scale) {
    const c10::DeviceGuard guard(q.device());
    const at::Device dev = q.device();
    const int64_t rows = batch * tokens, cols = heads * dim_head;
    const int64_t lq = rows_view(q, dev, rows, cols, "attention q"), lk = rows_view(k, dev, rows, cols, "attention k");
    const int64_t lv = rows_view(v, dev, rows, cols, "attention v"), lo = rows_view(out, dev, rows, cols, "attention out");
    check(s2v_attention(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), (int)batch, (int)heads,
                        (int)tokens, (int)dim_head, (int)lq, (int)lk, (int)lv, tokens * lq, tokens * lk, tokens * lv,
                        (float)scale, out.data_ptr<float>(), (int)lo, tokens * lo, stream()),
          "s2v_attention");
}

// ------------------------------------------------------------------------------------------ data movement
// A strided 4-D view given as (base tensor, element offset, sizes (n, c, h, w), strides in elements,
// any sign): every element it addresses must lie inside ``base``.
const float *strided(const Tensor &base, int64_t off, at::IntArrayRef size, at::IntArrayRef st, const at::Device &dev,
                     const char *what) {
    f32(base, dev, what);
    TORCH_CHECK(size.size() == 4 && st.size() == 4, what, ": 4 sizes and 4 strides");
    int64_t lo = off, hi = off;
    for (int i = 0; i < 4; ++i) {
        TORCH_CHECK(size[i] > 0, what, ": empty view");
        const int64_t span = (size[i] - 1) * st[i];
        if (span < 0) lo += span; else hi += span;
    }
    const int64_t avail = base.storage().nbytes() / 4 - base.storage_offset();
    TORCH_CHECK(lo >= 0 && hi < avail, what, ": view [", lo, ", ", hi, "] leaves its tensor (", avail, " elements)");
    return base.data_ptr<float>() + off;
}

// bilinear (mode 0) / nearest (mode 1) resize between strided views in (n, c, y, x) index order
void resize_(const Tensor &x, int64_t x_off, at::IntArrayRef x_size, at::IntArrayRef x_stride, const Tensor &y,
             int64_t y_off, at::IntArrayRef y_size, at::IntArrayRef y_stride, double scale_h, double scale_w,
             int64_t mode) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const float *xp = strided(x, x_off, x_size, x_stride, dev, "resize x");
    float *yp = const_cast<float *>(strided(y, y_off, y_size, y_stride, dev, "resize y"));
    TORCH_CHECK(x_size[0] == y_size[0] && x_size[1] == y_size[1], "resize: n / c of x and y differ");
    check(s2v_resize(xp, (int)x_size[0], (int)x_size[1], (int)x_size[2], (int)x_size[3], x_stride[0], x_stride[1],
                     x_stride[2], x_stride[3], yp, (int)y_size[2], (int)y_size[3], y_stride[0], y_stride[1],
                     y_stride[2], y_stride[3], (float)scale_h, (float)scale_w, (int)mode, stream()),
          "s2v_resize");
}

void row_pack_(const Tensor &x, const Tensor &y, int64_t kw, int64_t pw) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "row_pack x"), yv = nhwc(y, dev, "row_pack y");
    TORCH_CHECK(yv.n == xv.n && yv.h == xv.h && yv.w == xv.w && yv.c == yv.cs && yv.c >= kw * xv.c,
                "row_pack: y must be a dense [n, h, w, >= kw * c] tensor");
    check(s2v_row_pack(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, (int)kw, (int)pw, yv.p, yv.cs, stream()), "s2v_row_pack");
}

void pad_reflect_(const Tensor &x, const Tensor &y, at::IntArrayRef pads) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    TORCH_CHECK(pads.size() == 4, "pad_reflect: pads (top, bottom, left, right)");
    const NV xv = nhwc(x, dev, "pad_reflect x"), yv = nhwc(y, dev, "pad_reflect y");
    TORCH_CHECK(yv.n == xv.n && yv.c == xv.c && yv.h == xv.h + pads[0] + pads[1] && yv.w == xv.w + pads[2] + pads[3],
                "pad_reflect: y shape");
    check(s2v_pad_reflect(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, (int)pads[0], (int)pads[1], (int)pads[2], (int)pads[3],
                          yv.p, yv.cs, stream()),
          "s2v_pad_reflect");
}

// ToRGB + x2 bilinear skip upsample (s2v_torgb_up2): x NHWC view [N, H, W, C], wt packed 1x1 rows
// [>= 3, kpad], s [N, >= C] row view, bias [3] or None, skip NHWC [N, H/2, W/2, >= 4], y NHWC [N, H, W, >= 4]
void torgb_up2_(const Tensor &x, const Tensor &wt, const Tensor &s, const OptT &bias, const Tensor &skip,
                const Tensor &y) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "torgb x"), kv = nhwc(skip, dev, "torgb skip"), yv = nhwc(y, dev, "torgb y");
    f32(wt, dev, "torgb wt");
    TORCH_CHECK(wt.dim() == 2 && wt.is_contiguous() && wt.size(0) >= 3 && wt.size(1) >= xv.c,
                "torgb wt: packed 1x1 rows [>= 3, kpad >= C]");
    const int s_ns = (int)rows_view(s, dev, xv.n, xv.c, "torgb s");
    const float *bp = vec(bias, dev, 3, "torgb bias");
    TORCH_CHECK(kv.n == xv.n && yv.n == xv.n && yv.h == xv.h && yv.w == xv.w && 2 * kv.h == xv.h && 2 * kv.w == xv.w &&
                    kv.c == 4 && yv.c == 4,
                "torgb: skip [N, H/2, W/2, 4] and y [N, H, W, 4] views expected");
    check(s2v_torgb_up2(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, wt.data_ptr<float>(), (int)wt.size(1), s.data_ptr<float>(),
                        s_ns, bp, kv.p, kv.cs, yv.p, yv.cs, stream()),
          "s2v_torgb_up2");
}

// flow NHWC view (>= 2 channels: x, y), src [N, C, H, W] (any strides), y NHWC view [N, H, W, C]
void flow_warp_(const Tensor &flow, const Tensor &src, const Tensor &y) {
    const c10::DeviceGuard guard(flow.device());
    const at::Device dev = flow.device();
    const NV fv = nhwc(flow, dev, "flow_warp flow"), yv = nhwc(y, dev, "flow_warp y");
    f32(src, dev, "flow_warp src");
    TORCH_CHECK(src.dim() == 4 && src.size(0) == fv.n && fv.c >= 2, "flow_warp: src [N, C, H, W], flow >= 2 channels");
    TORCH_CHECK(yv.n == fv.n && yv.h == src.size(2) && yv.w == src.size(3) && yv.c == src.size(1), "flow_warp: y shape");
    check(s2v_flow_warp(fv.p, fv.n, fv.h, fv.w, fv.cs, src.data_ptr<float>(), (int)src.size(1), (int)src.size(2),
                        (int)src.size(3), src.stride(0), src.stride(1), src.stride(2), src.stride(3), yv.p, yv.cs,
                        stream()),
          "s2v_flow_warp");
}

// y NHWC view [N, H, W, 2C] <- [src | warp(src)] (s2v_flow_warp_cat)
void flow_warp_cat_(const Tensor &flow, const Tensor &src, const Tensor &y) {
    const c10::DeviceGuard guard(flow.device());
    const at::Device dev = flow.device();
    const NV fv = nhwc(flow, dev, "flow_warp_cat flow"), yv = nhwc(y, dev, "flow_warp_cat y");
    f32(src, dev, "flow_warp_cat src");
    TORCH_CHECK(src.dim() == 4 && src.size(0) == fv.n && fv.c >= 2, "flow_warp_cat: src [N, C, H, W], flow >= 2 channels");
    TORCH_CHECK(yv.n == fv.n && yv.h == src.size(2) && yv.w == src.size(3) && yv.c == 2 * src.size(1),
                "flow_warp_cat: y [N, H, W, 2C]");
    check(s2v_flow_warp_cat(fv.p, fv.n, fv.h, fv.w, fv.cs, src.data_ptr<float>(), (int)src.size(1), (int)src.size(2),
                            (int)src.size(3), src.stride(0), src.stride(1), src.stride(2), src.stride(3), yv.p, yv.cs,
                            stream()),
          "s2v_flow_warp_cat");
}

void fill_value_(const Tensor &y, double value) {
    const c10::DeviceGuard guard(y.device());
    f32(y, y.device(), "fill y");
    TORCH_CHECK(y.is_contiguous(), "fill: contiguous y");
    check(s2v_fill(y.data_ptr<float>(), y.numel(), (float)value, stream()), "s2v_fill");
}

// N(0, 1) noise (base_blocks.py:528-531); seed / offset are the 64-bit patterns of the counter-based
// generator; with ``ctr`` (int64 [1]) the offset advances by ctr << shift, read when the kernel runs
void gaussian_noise_(const Tensor &y, int64_t seed, int64_t offset, const OptT &ctr, int64_t shift) {
    const c10::DeviceGuard guard(y.device());
    f32(y, y.device(), "noise y");
    TORCH_CHECK(y.is_contiguous(), "noise: contiguous y");
    if (has(ctr)) {
        same_dev(*ctr, y.device(), "noise ctr");
        TORCH_CHECK(ctr->scalar_type() == at::kLong && ctr->numel() >= 1, "noise ctr: int64 [1]");
        check(s2v_gaussian_noise_ctr(y.data_ptr<float>(), y.numel(), (unsigned long long)seed,
                                     (unsigned long long)offset, (const unsigned long long *)ctr->data_ptr(), (int)shift,
                                     stream()),
              "s2v_gaussian_noise_ctr");
    } else {
        check(s2v_gaussian_noise(y.data_ptr<float>(), y.numel(), (unsigned long long)seed, (unsigned long long)offset,
                                 stream()),
              "s2v_gaussian_noise");
    }
}

void counter_add_(const Tensor &ctr, int64_t inc) {
    const c10::DeviceGuard guard(ctr.device());
    same_dev(ctr, ctr.device(), "counter");
    TORCH_CHECK(ctr.scalar_type() == at::kLong && ctr.numel() >= 1, "counter: int64 [1]");
    check(s2v_counter_add((unsigned long long *)ctr.data_ptr(), (unsigned long long)inc, stream()), "s2v_counter_add");
}

void rfft2_(const Tensor &x, const Tensor &tables, const Tensor &spec) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "rfft2 x");
    vec(tables, dev, (int64_t)s2v_fft_tables_floats(xv.h, xv.w), "rfft2 tables");
    f32(spec, dev, "rfft2 spec");
    TORCH_CHECK(spec.dim() == 3 && spec.is_contiguous() && spec.size(0) == xv.n &&
                    spec.size(1) == (int64_t)xv.h * (xv.w / 2 + 1) && spec.size(2) >= 2 * xv.c,
                "rfft2 spec: [N, h * (w/2 + 1), >= 2C]");
    check(s2v_rfft2(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, tables.data_ptr<float>(), spec.data_ptr<float>(),
                    (int)spec.size(2), stream()),
          "s2v_rfft2");
}

// ------------------------------------------------------------------------------------------ LNet FFC
// split packed weights [npad, kpad] (s2v_split_weights output, float32 storage of the 16-bit halves)
const void *split_rows(const Tensor &w, const at::Device &dev, int64_t rows, int64_t k, const char *what) {
    f32(w, dev, what);
    TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(0) >= rows && w.size(1) >= k && w.size(1) % 32 == 0, what,
                ": split packed weights [npad >= ", rows, ", kpad >= ", k, "] expected, got ", w.sizes());
    return w.data_ptr();
}

int *range_flag(const OptT &flag, const at::Device &dev) {
    if (!has(flag)) return nullptr;
    same_dev(*flag, dev, "ffc flag");
    TORCH_CHECK(flag->scalar_type() == at::kInt && flag->numel() >= 1, "ffc flag: int32 [1]");
    return flag->data_ptr<int>();
}

// x_g: NHWC [N, h, h, cg] channel view of the FFC input; t1 [N, h, h, cc], spec [N, F, 2cc] dense
void ffc_spec_fwd_(const Tensor &xg, const Tensor &w1, double wt_scale, double x_scale, const OptT &scale,
                   const OptT &shift, const Tensor &tables, const Tensor &t1, const Tensor &spec, const OptT &flag,
                   int64_t prec) {
    const c10::DeviceGuard guard(xg.device());
    const at::Device dev = xg.device();
    const NV xv = nhwc(xg, dev, "ffc x_g");
    const int c = s2v_ffc_channels(xv.h), cg = c - c / 4, cc = cg / 2;
    TORCH_CHECK(c > 0 && xv.w == xv.h && xv.c == cg, "ffc_spec_fwd: x_g [N, h, h, 3C/4] with h in {12, 24, 48}");
    const NV tv = nhwc(t1, dev, "ffc t1");
    TORCH_CHECK(tv.n == xv.n && tv.h == xv.h && tv.w == xv.w && tv.c == cc && tv.cs == cc, "ffc t1: dense [N, h, h, cc]");
    f32(spec, dev, "ffc spec");
    TORCH_CHECK(spec.dim() == 3 && spec.is_contiguous() && spec.size(0) == xv.n &&
                    spec.size(1) == (int64_t)xv.h * (xv.h / 2 + 1) && spec.size(2) == 2 * cc,
                "ffc spec: dense [N, F, 2cc]");
    vec(tables, dev, (int64_t)s2v_fft_tables_floats(xv.h, xv.h), "ffc tables");
    check(s2v_ffc_spec_fwd(xv.p, xv.cs, xv.n, xv.h, split_rows(w1, dev, cc, cg, "ffc w1"), (int)w1.size(1),
                           (float)wt_scale, (float)x_scale, vec(scale, dev, cc, "ffc scale1"), vec(shift, dev, cc, "ffc shift1"),
                           tables.data_ptr<float>(), tv.p, spec.data_ptr<float>(), range_flag(flag, dev), (int)prec,
                           stream()),
          "s2v_ffc_spec_fwd");
}

void ffc_spec_inv_(const Tensor &spec, const Tensor &wfu, double wt_scale, double x_scale, const OptT &scale,
                   const OptT &shift, const Tensor &tables, const Tensor &t1, const Tensor &u, const OptT &flag,
                   int64_t prec) {
    const c10::DeviceGuard guard(spec.device());
    const at::Device dev = spec.device();
    const NV tv = nhwc(t1, dev, "ffc t1"), uv = nhwc(u, dev, "ffc u");
    const int c = s2v_ffc_channels(tv.h), cg = c - c / 4, cc = cg / 2;
    TORCH_CHECK(c > 0 && tv.w == tv.h && tv.c == cc && tv.cs == cc, "ffc t1: dense [N, h, h, cc]");
    TORCH_CHECK(uv.n == tv.n && uv.h == tv.h && uv.w == tv.w && uv.c == cc && uv.cs == cc, "ffc u: dense [N, h, h, cc]");
    f32(spec, dev, "ffc spec");
    TORCH_CHECK(spec.dim() == 3 && spec.is_contiguous() && spec.size(0) == tv.n &&
                    spec.size(1) == (int64_t)tv.h * (tv.h / 2 + 1) && spec.size(2) == 2 * cc,
                "ffc spec: dense [N, F, 2cc]");
    vec(tables, dev, (int64_t)s2v_fft_tables_floats(tv.h, tv.h), "ffc tables");
    check(s2v_ffc_spec_inv(spec.data_ptr<float>(), tv.n, tv.h, split_rows(wfu, dev, 2 * cc, cg, "ffc wfu"),
                           (int)wfu.size(1), (float)wt_scale, (float)x_scale, vec(scale, dev, 2 * cc, "ffc scale_fu"),
                           vec(shift, dev, 2 * cc, "ffc shift_fu"), tables.data_ptr<float>(), tv.p, uv.p,
                           range_flag(flag, dev), (int)prec, stream()),
          "s2v_ffc_spec_inv");
}

// y: [N, h, h, C] (conv_to_l | conv_l2g outputs), u dense [N, h, h, cc]; gamma / beta [N, C] row views
void ffc_norm_(const Tensor &y, const Tensor &u, const Tensor &w2, double wt_scale, double x_scale, const OptT &gamma,
               const OptT &beta, double eps, int64_t act, double alpha, const OptT &res, const Tensor &out,
               const OptT &pad_out, const OptT &flag, int64_t prec) {
    const c10::DeviceGuard guard(y.device());
    const at::Device dev = y.device();
    const NV yv = nhwc(y, dev, "ffc_norm y"), uv = nhwc(u, dev, "ffc_norm u"), ov = nhwc(out, dev, "ffc_norm out");
    const int c = s2v_ffc_channels(yv.h), cg = c - c / 4, cc = cg / 2;
    TORCH_CHECK(c > 0 && yv.w == yv.h && yv.c == c, "ffc_norm: y [N, h, h, C] with h in {12, 24, 48}");
    TORCH_CHECK(uv.n == yv.n && uv.h == yv.h && uv.w == yv.w && uv.c == cc && uv.cs == cc, "ffc_norm u: dense [N, h, h, cc]");
    TORCH_CHECK(ov.n == yv.n && ov.h == yv.h && ov.w == yv.w && ov.c == c, "ffc_norm: out shape");
    TORCH_CHECK(has(gamma) == has(beta), "ffc_norm: gamma and beta together");
    const float *gp = nullptr, *bp = nullptr;
    int ns = 0;
    if (has(gamma)) {
        ns = (int)rows_view(*gamma, dev, yv.n, c, "ffc_norm gamma");
        TORCH_CHECK(rows_view(*beta, dev, yv.n, c, "ffc_norm beta") == ns, "ffc_norm: gamma / beta row strides");
        gp = gamma->data_ptr<float>(); bp = beta->data_ptr<float>();
    }
    const float *rp = nullptr;
    int rcs = 0;
    if (has(res)) {
        const NV rv = nhwc(*res, dev, "ffc_norm res");
        TORCH_CHECK(rv.n == yv.n && rv.h == yv.h && rv.w == yv.w && rv.c == c, "ffc_norm: res shape");
        rp = rv.p; rcs = rv.cs;
    }
    float *pp = nullptr;
    int pcs = 0;
    if (has(pad_out)) {
        const NV pv = nhwc(*pad_out, dev, "ffc_norm pad_out");
        TORCH_CHECK(pv.n == yv.n && pv.h == yv.h + 2 && pv.w == yv.w + 2 && pv.c == c, "ffc_norm pad_out: [N, h+2, h+2, C]");
        pp = pv.p; pcs = pv.cs;
    }
    check(s2v_ffc_norm(yv.p, yv.cs, yv.n, yv.h, uv.p, split_rows(w2, dev, cg, cc, "ffc w2"), (int)w2.size(1),
                       (float)wt_scale, (float)x_scale, gp, bp, ns, (float)eps, (int)act, (float)alpha, rp, rcs, ov.p,
                       ov.cs, pp, pcs, range_flag(flag, dev), (int)prec, stream()),
          "s2v_ffc_norm");
}

void irfft2_(const Tensor &spec, const Tensor &tables, const OptT &res, const Tensor &y) {
    const c10::DeviceGuard guard(spec.device());
    const at::Device dev = spec.device();
    const NV yv = nhwc(y, dev, "irfft2 y");
    vec(tables, dev, (int64_t)s2v_fft_tables_floats(yv.h, yv.w), "irfft2 tables");
    f32(spec, dev, "irfft2 spec");
    TORCH_CHECK(spec.dim() == 3 && spec.is_contiguous() && spec.size(0) == yv.n &&
                    spec.size(1) == (int64_t)yv.h * (yv.w / 2 + 1) && spec.size(2) >= 2 * yv.c,
                "irfft2 spec: [N, h * (w/2 + 1), >= 2C]");
    const float *rp = nullptr;
    int rcs = 0;
    if (has(res)) {
        const NV rv = nhwc(*res, dev, "irfft2 res");
        TORCH_CHECK(rv.n == yv.n && rv.h == yv.h && rv.w == yv.w && rv.c == yv.c, "irfft2: res shape");
        rp = rv.p; rcs = rv.cs;
    }
    check(s2v_irfft2(spec.data_ptr<float>(), yv.n, yv.h, yv.w, yv.c, (int)spec.size(2), tables.data_ptr<float>(), rp,
                     rcs, yv.p, yv.cs, stream()),
          "s2v_irfft2");
}

void eltwise_(const Tensor &x, const OptT &mul, const OptT &add, const OptT &bias, double a, int64_t act,
              double alpha, double post, const Tensor &y) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "eltwise x"), yv = nhwc(y, dev, "eltwise y");
    TORCH_CHECK(yv.n == xv.n && yv.h == xv.h && yv.w == xv.w && yv.c == xv.c, "eltwise: y shape");
    const float *mp = nullptr, *ap = nullptr;
    int mcs = 0, acs = 0;
    if (has(mul)) {
        const NV v = nhwc(*mul, dev, "eltwise mul");
        TORCH_CHECK(v.n == xv.n && v.h == xv.h && v.w == xv.w && v.c == xv.c, "eltwise: mul shape");
        mp = v.p; mcs = v.cs;
    }
    if (has(add)) {
        const NV v = nhwc(*add, dev, "eltwise add");
        TORCH_CHECK(v.n == xv.n && v.h == xv.h && v.w == xv.w && v.c == xv.c, "eltwise: add shape");
        ap = v.p; acs = v.cs;
    }
    check(s2v_eltwise(xv.p, xv.cs, mp, mcs, ap, acs, vec(bias, dev, xv.c, "eltwise bias"),
                      (long long)xv.n * xv.h * xv.w, xv.c, (float)a, (int)act, (float)alpha, (float)post, yv.p, yv.cs,
                      stream()),
          "s2v_eltwise");
}

void fir2d_(const Tensor &x, const Tensor &kernel, const Tensor &y, int64_t up, int64_t down, int64_t pad_y0,
            int64_t pad_x0, double gain, const OptT &bias, int64_t act, double alpha, double post) {
    const c10::DeviceGuard guard(x.device());
    const at::Device dev = x.device();
    const NV xv = nhwc(x, dev, "fir2d x"), yv = nhwc(y, dev, "fir2d y");
    TORCH_CHECK(xv.n == yv.n && xv.c == yv.c, "fir2d: batch / channel mismatch");
    f32(kernel, dev, "fir2d kernel");
    TORCH_CHECK(kernel.dim() == 2 && kernel.is_contiguous(), "fir2d kernel: [kh, kw]");
    check(s2v_fir2d(xv.p, xv.n, xv.h, xv.w, xv.c, xv.cs, kernel.data_ptr<float>(), (int)kernel.size(0),
                    (int)kernel.size(1), (int)up, (int)down, (int)pad_y0, (int)pad_x0, yv.p, yv.h, yv.w, yv.cs,
                    (float)gain, vec(bias, dev, xv.c, "fir2d bias"), (int)act, (float)alpha, (float)post, stream()),
          "s2v_fir2d");
}

// ------------------------------------------------------------------------------------------ pipeline glue
// fake None: ref_u8 holds the references (an enhancer replaced them) and only face6 / gt are built
void lipsync_inputs_(const Tensor &src, const OptT &fake, const Tensor &ref_u8, const Tensor &face6,
                     const Tensor &gt) {
    const c10::DeviceGuard guard(src.device());
    const at::Device dev = src.device();
    f32(src, dev, "lipsync src"); f32(face6, dev, "lipsync face6");
    f32(gt, dev, "lipsync gt");
    same_dev(ref_u8, dev, "lipsync ref_u8");
    TORCH_CHECK(src.dim() == 4 && src.size(1) == 3 && src.is_contiguous(), "lipsync: src [N, 3, H, W] contiguous");
    const int64_t n = src.size(0), h = src.size(2), w = src.size(3);
    if (has(fake)) {
        f32(*fake, dev, "lipsync fake");
        TORCH_CHECK(fake->is_contiguous() && fake->sizes() == src.sizes(), "lipsync: fake like src");
    }
    TORCH_CHECK(ref_u8.scalar_type() == at::kByte && ref_u8.is_contiguous() && ref_u8.sizes() == src.sizes(),
                "lipsync: ref_u8 uint8 like src");
    TORCH_CHECK(face6.is_contiguous() && face6.dim() == 4 && face6.size(0) == n && face6.size(1) == 6 &&
                    face6.size(2) == h && face6.size(3) == w,
                "lipsync: face6 [N, 6, H, W]");
    TORCH_CHECK(gt.is_contiguous() && gt.sizes() == src.sizes(), "lipsync: gt like src");
    check(s2v_lipsync_inputs(src.data_ptr<float>(), has(fake) ? fake->data_ptr<float>() : nullptr, (int)n, (int)h, (int)w,
                             ref_u8.data_ptr<uint8_t>(), face6.data_ptr<float>(), gt.data_ptr<float>(), stream()),
          "s2v_lipsync_inputs");
}

void to_u8_(const Tensor &x, const Tensor &y, double lo, double hi, double scale, double offset) {
    const c10::DeviceGuard guard(x.device());
    f32(x, x.device(), "to_u8 x");
    same_dev(y, x.device(), "to_u8 y");
    TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && y.scalar_type() == at::kByte && y.numel() == x.numel(),
                "to_u8: contiguous x and uint8 y of the same size");
    check(s2v_to_u8(x.data_ptr<float>(), x.numel(), (float)lo, (float)hi, (float)scale, (float)offset,
                    y.data_ptr<uint8_t>(), stream()),
          "s2v_to_u8");
}

void mel_chunks_(const Tensor &mel, const Tensor &starts, int64_t step, const Tensor &out) {
    const c10::DeviceGuard guard(mel.device());
    const at::Device dev = mel.device();
    f32(mel, dev, "mel_chunks mel");
    f32(out, dev, "mel_chunks out");
    same_dev(starts, dev, "mel_chunks starts");
    TORCH_CHECK(mel.dim() == 2 && mel.size(0) == 80 && mel.is_contiguous(), "mel_chunks: mel [80, frames]");
    TORCH_CHECK(starts.scalar_type() == at::kInt && starts.is_contiguous(), "mel_chunks: int32 starts");
    const int64_t nch = starts.numel();
    TORCH_CHECK(out.is_contiguous() && out.numel() == nch * 80 * step, "mel_chunks: out [n, 80, step]");
    check(s2v_mel_chunks(mel.data_ptr<float>(), mel.size(1), starts.data_ptr<int>(), (int)nch, (int)step,
                         out.data_ptr<float>(), stream()),
          "s2v_mel_chunks");
}

void melspectrogram_(const Tensor &wav, const Tensor &tables, bool pad_reflect, const Tensor &out) {
    const c10::DeviceGuard guard(wav.device());
    const at::Device dev = wav.device();
    f32(wav, dev, "mel wav");
    f32(out, dev, "mel out");
    TORCH_CHECK(wav.dim() == 1 && wav.is_contiguous(), "mel: wav [S]");
    const int64_t frames = 1 + wav.size(0) / 200;
    TORCH_CHECK(out.is_contiguous() && out.dim() == 2 && out.size(0) == 80 && out.size(1) == frames,
                "mel: out [80, 1 + S / 200]");
    vec(tables, dev, 80 * 401 + 3 * 800, "mel tables");
    check(s2v_melspectrogram(wav.data_ptr<float>(), wav.size(0), tables.data_ptr<float>(), pad_reflect,
                             out.data_ptr<float>(), frames, stream()),
          "s2v_melspectrogram");
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(s2v, m) {
    m.def("conv2d_(Tensor x, Tensor(a!) y, Tensor wt, Tensor? wt_split, float wt_scale, int cout, int[2] kernel, "
          "int[2] stride, int[2] padding, int[2] dilation, int in_mode, int pad_mode, int prec, Tensor? scale, "
          "Tensor? shift, Tensor? in_scale, Tensor? nc_scale, int pre_act, float pre_alpha, Tensor? pix_add, "
          "float pix_w, Tensor? res, int[2] res_offset, bool res_after_act, int act, float alpha, int out_step, "
          "bool out_pool, bool x_split, Tensor? ws, int grid_cap, int force_tile, int force_splits, "
          "Tensor(s!)? stamps, Tensor? stamp_ctr, int[3] stamp_pos, float x_scale, Tensor(f!)? nonfinite, "
          "bool dry, Tensor? post_mul=None, Tensor? post_add=None, int post_c0=0, Tensor? dup_src=None, "
          "Tensor? dup_bias=None, float dup_a=0., int dup_off=0) -> int[]");
    m.def("modulated_conv2d_(Tensor x, Tensor(a!) y, Tensor wt, Tensor s, Tensor? d, Tensor(b!) wbuf, int cout, "
          "int[2] kernel, int[2] padding, int in_mode, int prec, bool x_split, Tensor? scale, Tensor? shift, "
          "Tensor? pix_add, "
          "float pix_w, Tensor? res, "
          "bool res_after_act, int act, float alpha, Tensor? ws, int force_splits, Tensor(s!)? stamps, Tensor? stamp_ctr, "
          "int[3] stamp_pos, float x_scale, Tensor(f!)? nonfinite, bool dry, int d2s=0, int force_tile=0, "
          "float premod=0.) -> int[]");
    m.def("modulate_weights_(Tensor wt, Tensor s, Tensor? d, Tensor(a!) wbuf, int cout, int cin, int taps, int prec, "
          "float wscale) -> ()");
    m.def("amax_(Tensor x, Tensor(a!) out) -> ()");
    // conv groups: host-side recording, no tensor to dispatch on (catch-all kernels)
    m.def("group_begin_() -> ()", &group_begin_);
    m.def("group_abort_() -> ()", &group_abort_);
    m.def("group_end_(Tensor? ws, bool dry) -> int[]", &group_end_);
    m.def("gemm_kn_(Tensor a, Tensor b, Tensor(a!) out, int batch, int a_bs, int b_bs, int out_bs, Tensor? res, "
          "int res_bs, int act, float alpha, int prec, Tensor? ws, int force_tile, int force_splits, bool dry) -> int[]");
    m.def("split_weights_(Tensor w, Tensor(a!) out, int prec, float scale) -> ()");
    m.def("split_act_(Tensor x, Tensor(a!) out, int prec) -> ()");
    m.def("layernorm2d_(Tensor x, Tensor weight, Tensor bias, float eps, int act, float alpha, bool pool, "
          "Tensor? res, Tensor(a!) y, Tensor? ws) -> int");
    m.def("instnorm_(Tensor x, Tensor? gamma, Tensor? beta, float eps, int act, float alpha, Tensor? res, "
          "Tensor(a!) y, Tensor(b!)? pad_out, Tensor? ws) -> int");
    m.def("adain_params_(Tensor hid, int nhidden, Tensor w2t, Tensor bias, Tensor seg, Tensor(a!) out) -> ()");
    m.def("modconv_demod_(Tensor s, Tensor wsq, Tensor(a!) d, float eps, float post) -> ()");
    m.def("modconv_demod_rows_(Tensor s, Tensor rows, Tensor wsq, Tensor(a!) d, float eps, float post, "
          "int s_reach) -> ()");
    m.def("row_layernorm_(Tensor x, Tensor weight, Tensor bias, float eps, Tensor(a!) y) -> ()");
    m.def("attention_(Tensor q, Tensor k, Tensor v, Tensor(a!) out, int batch, int heads, int tokens, int dim_head, "
          "float scale) -> ()");
    m.def("resize_(Tensor x, int x_off, int[4] x_size, int[4] x_stride, Tensor(a!) y, int y_off, int[4] y_size, "
          "int[4] y_stride, float scale_h, float scale_w, int mode) -> ()");
    m.def("pad_reflect_(Tensor x, Tensor(a!) y, int[4] pads) -> ()");
    m.def("row_pack_(Tensor x, Tensor(a!) y, int kw, int pw) -> ()");
    m.def("torgb_up2_(Tensor x, Tensor wt, Tensor s, Tensor? bias, Tensor skip, Tensor(a!) y) -> ()");
    m.def("flow_warp_(Tensor flow, Tensor src, Tensor(a!) y) -> ()");
    m.def("flow_warp_cat_(Tensor flow, Tensor src, Tensor(a!) y) -> ()");
    m.def("fill_value_(Tensor(a!) y, float value) -> ()");
    m.def("gaussian_noise_(Tensor(a!) y, int seed, int offset, Tensor? ctr, int shift) -> ()");
    m.def("counter_add_(Tensor(a!) ctr, int inc) -> ()");
    m.def("rfft2_(Tensor x, Tensor tables, Tensor(a!) spec) -> ()");
    m.def("irfft2_(Tensor spec, Tensor tables, Tensor? res, Tensor(a!) y) -> ()");
    m.def("ffc_spec_fwd_(Tensor x_g, Tensor w1, float wt_scale, float x_scale, Tensor? scale, Tensor? shift, "
          "Tensor tables, Tensor(a!) t1, Tensor(b!) spec, Tensor? flag, int prec) -> ()");
    m.def("ffc_spec_inv_(Tensor spec, Tensor wfu, float wt_scale, float x_scale, Tensor? scale, Tensor? shift, "
          "Tensor tables, Tensor t1, Tensor(a!) u, Tensor? flag, int prec) -> ()");
    // y may be the same tensor as out (LNet normalises in place), hence mutable
    m.def("ffc_norm_(Tensor(c!) y, Tensor u, Tensor w2, float wt_scale, float x_scale, Tensor? gamma, Tensor? beta, "
          "float eps, int act, float alpha, Tensor? res, Tensor(a!) out, Tensor(b!)? pad_out, Tensor? flag, int prec) -> ()");
    m.def("eltwise_(Tensor x, Tensor? mul, Tensor? add, Tensor? bias, float a, int act, float alpha, float post, "
          "Tensor(a!) y) -> ()");
    m.def("fir2d_(Tensor x, Tensor kernel, Tensor(a!) y, int up, int down, int pad_y0, int pad_x0, float gain, "
          "Tensor? bias, int act, float alpha, float post) -> ()");
    m.def("lipsync_inputs_(Tensor src, Tensor? fake, Tensor(a!) ref_u8, Tensor(b!) face6, Tensor(c!) gt) -> ()");
    m.def("to_u8_(Tensor x, Tensor(a!) y, float lo, float hi, float scale, float offset) -> ()");
    m.def("mel_chunks_(Tensor mel, Tensor starts, int step, Tensor(a!) out) -> ()");
    m.def("melspectrogram_(Tensor wav, Tensor tables, bool pad_reflect, Tensor(a!) out) -> ()");
}

TORCH_LIBRARY_IMPL(s2v, CUDA, m) {
    m.impl("conv2d_", &conv2d_);
    m.impl("modulated_conv2d_", &modulated_conv2d_);
    m.impl("modulate_weights_", &modulate_weights_);
    m.impl("gemm_kn_", &gemm_kn_);
    m.impl("split_weights_", &split_weights_);
    m.impl("amax_", &amax_);
    m.impl("split_act_", &split_act_);
    m.impl("layernorm2d_", &layernorm2d_);
    m.impl("instnorm_", &instnorm_);
    m.impl("adain_params_", &adain_params_);
    m.impl("modconv_demod_", &modconv_demod_);
    m.impl("modconv_demod_rows_", &modconv_demod_rows_);
    m.impl("row_layernorm_", &row_layernorm_);
    m.impl("attention_", &attention_);
    m.impl("resize_", &resize_);
    m.impl("pad_reflect_", &pad_reflect_);
    m.impl("row_pack_", &row_pack_);
    m.impl("torgb_up2_", &torgb_up2_);
    m.impl("flow_warp_", &flow_warp_);
    m.impl("flow_warp_cat_", &flow_warp_cat_);
    m.impl("fill_value_", &fill_value_);
    m.impl("gaussian_noise_", &gaussian_noise_);
    m.impl("counter_add_", &counter_add_);
    m.impl("rfft2_", &rfft2_);
    m.impl("irfft2_", &irfft2_);
    m.impl("ffc_spec_fwd_", &ffc_spec_fwd_);
    m.impl("ffc_spec_inv_", &ffc_spec_inv_);
    m.impl("ffc_norm_", &ffc_norm_);
    m.impl("eltwise_", &eltwise_);
    m.impl("fir2d_", &fir2d_);
    m.impl("lipsync_inputs_", &lipsync_inputs_);
    m.impl("to_u8_", &to_u8_);
    m.impl("mel_chunks_", &mel_chunks_);
    m.impl("melspectrogram_", &melspectrogram_);
}
