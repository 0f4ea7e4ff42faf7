/*
 * s2v.h — C ABI of libs2v.so, the MI355X (gfx950) compute path for the per-frame lip-sync
 * inference path of Ryukhaan/speech-to-video-mpp (VideoReTalking fork).
 *
 * Conventions (all entry points):
 *   - every pointer is a device pointer (HBM) unless documented otherwise; fp32 data;
 *   - activations are NHWC: element (n, y, x, c) of a view lives at
 *     data[((n*H + y)*W + x)*cs + c]; ``cs`` (channel stride / pixel pitch) lets a view be a
 *     channel slice of a wider tensor (this is how concat/split of the reference are fused away);
 *   - work is enqueued on ``stream`` (a hipStream_t); nothing synchronises, nothing allocates,
 *     so every call is hipGraph-capturable;
 *   - return 0 on success, a negative S2V_E* code on invalid arguments (nothing launched) or a
 *     launch failure; s2v_last_error() returns a message for the last failure on this thread.
 *
 * The reference's only native FFI on this path is GPEN's pybind11 ops (fused_bias_act,
 * upfirdn2d); every other entry point replaces a PyTorch aten call sequence the reference's
 * Python makes (file:line cited per function).
 */
#ifndef S2V_H_
#define S2V_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *s2v_stream_t; /* hipStream_t */

enum {
    S2V_OK = 0,
    S2V_E_INVALID = -1, /* bad shape / stride / alignment / unsupported mode */
    S2V_E_LAUNCH = -2,  /* hipGetLastError() after launch was not hipSuccess */
    S2V_E_WORKSPACE = -3 /* workspace missing or too small */
};

/* activation codes (epilogues / prologues) */
enum {
    S2V_ACT_NONE = 0,
    S2V_ACT_RELU = 1,
    S2V_ACT_LRELU = 2,     /* x >= 0 ? x : alpha * x */
    S2V_ACT_SIGMOID = 3,
    S2V_ACT_TANH = 4,
    S2V_ACT_GELU_TANH = 5  /* models/transformer.py:11-15 */
};

/* input addressing modes of the implicit-GEMM convolution */
enum {
    S2V_IN_DIRECT = 0,     /* ordinary (dilated, strided) conv                                */
    S2V_IN_NEAREST_UP2 = 1,/* conv over nearest-x2-upsampled input (UpBlock2d, base_blocks.py:123) */
    S2V_IN_TRANSPOSED = 2  /* ConvTranspose2d: out[o] += in[(o + pad - k*dil)/stride] (DNet decoder) */
};

enum { S2V_PAD_ZERO = 0, S2V_PAD_REFLECT = 1 };

/*
 * Fused convolution / GEMM: implicit GEMM on the MFMA, in the arithmetic ``prec`` selects (below;
 * default S2V_PREC_F16X3: split-fp32 operands on v_mfma_f32_16x16x32_f16, fp32 accumulate).
 *   out[n, oy, ox, o] = epilogue( sum_{ky,kx,c} A(n, oy, ox, ky, kx, c) * W[o][(ky*kw + kx)*cin + c] )
 * A = prologue(x) addressed per ``in_mode`` / ``pad_mode``; prologue = act(x * in_scale[n, c]).
 * Epilogue order:  v = acc * scale[o] * nc_scale[n, o] + shift[o] + pix_w * pix_add[n, oy, ox]
 *                  (+ res if !res_after_act);  v = act(v);  (+ res if res_after_act).
 * Weights are pre-packed [npad][kpad] (k = (ky*kw + kx)*cin + c, zero padded; npad % 128 == 0,
 * kpad % 32 == 0) — or, with ``b_kn`` = 1, an unpacked row-major [K][N] matrix (ldb) for
 * activation x activation GEMMs (the FourierUnit DFT products).
 * ``batch`` > 1 repeats the problem with per-batch pointer offsets (elements).
 */
typedef struct s2v_conv_params {
    /* input */
    const float *x; int n, h, w, cin, xcs;
    int in_mode; int pad_mode;                  /* PAD_REFLECT: direct or nearest-x2 input (reflected in the upsampled frame) */
    int pre_act; float pre_alpha;
    const float *in_scale; int in_scale_ns;     /* [n][in_scale_ns], may be NULL */
    /* filter */
    int kh, kw, sh, sw, ph, pw, dh, dw;
    const float *wt; int kpad, npad; int cout;  /* packed weights */
    int b_kn; int ldb;                          /* b_kn: wt is [K][ldb] row-major, N = cout */
    /* output */
    float *y; int oh, ow, ycs;
    /* epilogue */
    const float *scale, *shift;                 /* [cout], may be NULL */
    const float *nc_scale; int nc_scale_ns;     /* [n][nc_scale_ns], may be NULL */
    const float *pix_add; float pix_w;          /* [n][oh][ow], may be NULL */
    const float *res; int res_cs, res_h, res_w, res_oy, res_ox; int res_after_act; /* may be NULL */
    int act; float alpha;
    /* batching (GEMM mode) */
    int batch; long long x_bs, w_bs, y_bs, res_bs;
    /* split-K workspace (see s2v_conv2d_ws_bytes) */
    float *ws; size_t ws_bytes;
    int force_tile; int force_splits;           /* 0 = heuristic (tests use these) */
    /* strided output (0 = contiguous [n][oh][ow] rows of pitch ycs): output pixel (n, oy, ox)
     * is written at y + ((n*out_full_h + oy*out_step)*out_full_w + ox*out_step)*ycs — one parity
     * class of a polyphase transposed conv.  No pix_add; res only in place (res == y). */
    int out_step; int out_full_h, out_full_w;
    /* arithmetic of the implicit-GEMM kernels and of the Cout <= 4 heads with a 5x5 / 7x7 stride-1 filter over
     * 32 / 64 channels (conv_head_x3: the filter column in N, the row in K; S2V_HEAD_X3=0 turns it off); the
     * other Cout <= 4 VALU kernels and the K <= 64 kernels are always fp32:
     *   S2V_PREC_F32     v_mfma_f32_32x32x2_f32, exact fp32 products (reads ``wt``);
     *   S2V_PREC_BF16X3  split-fp32 on v_mfma_f32_32x32x16_bf16: a*b ~ ah*bh + ah*bl + al*bh with
     *                    ah = bf16(a), al = bf16(a - ah); <= 3*2^-16 relative error per product, any range;
     *   S2V_PREC_F16X3   the same split on v_mfma_f32_32x32x16_f16 (ah = f16(a), al = f16(a - ah)):
     *                    <= 3*2^-22 relative per product for operands in the f16 normal range
     *                    (|a| < 65504; smaller values keep an absolute error <= 2^-25).
     * Packed weights are read from ``wt_x3`` (s2v_split_weights layout of the same precision, the
     * weights multiplied by ``wt_scale`` before the split — a power of two, 0 means 1 — which the
     * kernel divides out of the accumulators exactly); a b_kn matrix is split on the fly. */
    int prec;
    const void *wt_x3;
    /* persistent launch of the 256x256 buffer-load split-precision tile: when > 0 (a multiple of 8) and the
     * launch has more tiles than this, it runs ``grid_cap`` blocks that each loop over the tiles of their
     * XCD (conv_igemm_x3_persist); the CUs left free serve a concurrent latency-bound graph branch (the
     * ENet style encoder beside LNet takes half the device's CUs).  0: one block per tile.  Other tiles
     * ignore it; s2v_conv2d_plan reports the persistent blocks in out11[10]. */
    int grid_cap;
    float wt_scale;
    /* 2x2 average-pooled output (ResBlock 'down': lrelu(conv1) then F.interpolate(x0.5, bilinear) ==
     * the mean of each 2x2 quad, base_blocks.py:40-49): y is [n][oh/2][ow/2] (pitch ycs) and holds
     * 0.25 * sum of the four epilogue values (act included) of each quad.  oh, ow even; implicit-GEMM
     * path only; no res / nc_scale / pix_add / strided output; one K split. */
    int out_pool;
    /* x holds the split layout of ``prec`` (s2v_split_act: per pixel and 32-channel block, 32 hi
     * halves then 32 lo halves — the fp32 tensor's bytes and pitch): both operands are staged by
     * LDS-DMA (conv_glds_x3).  Needs prec BF16X3 / F16X3, a direct zero-padded conv with cin % 32 == 0,
     * <= 32 taps, packed weights, no in_scale / pre_act, xcs % 4 == 0 and a 16-byte aligned x. */
    int x_split;
    /* optional launch timer of the implicit-GEMM kernels (bench.py's roofline of graph-replayed,
     * overlapped launches): with ``stamps`` set, the launch records the device real-time clock
     * (s_memrealtime, 100 MHz) of its first block's start (atomic min) and its last block's end
     * (atomic max) into stamps[2 s], stamps[2 s + 1] with slot s = (*stamp_ctr % stamp_reps) *
     * stamp_stride + stamp_slot — stamp_ctr a device replay counter read when the kernel runs, so a
     * captured graph records every replay in its own slot.  The caller initialises the pairs to
     * (UINT64_MAX, 0). */
    unsigned long long *stamps;
    const unsigned long long *stamp_ctr;
    int stamp_slot, stamp_stride, stamp_reps;
    /* activation range of the split precisions (f16x3: f16 halves cover |v| < 65504, lo halves lose
     * precision below 2^-3): the implicit-GEMM x3 kernels multiply the A operand by ``x_scale`` (a
     * power of two, 0 means 1; the epilogue divides it out exactly) before splitting it, and when
     * ``nonfinite`` is set, a launch whose accumulators hold a non-finite value sets *nonfinite = 1
     * (a range overflow is never silent).  The host picks x_scale per layer from the input's max |v|
     * (s2v_amax). */
    float x_scale;
    int *nonfinite;
    /* Depth-to-space output (the polyphase x2-bilinear-upsample StyleConv, ENet.py:119-129 via
     * base_blocks.py:487-533): with d2s_cout > 0 (requires out_step == 2, cout == 4 * d2s_cout, no
     * res / pool) output column n = cls * d2s_cout + o of conv pixel (n_, oy, ox) goes to
     * y + ((n_*out_full_h + 2*oy + cls/2)*out_full_w + 2*ox + cls%2)*ycs + o, and pix_add is read
     * at that full-resolution pixel ([N, out_full_h, out_full_w]). */
    int d2s_cout;
    /* enhancer epilogue folds (dense outputs only: out_step <= 1, no pool, no d2s), after act and res:
     *  SFT (gfpganv1_clean_arch.py:98-106):   out[m][n] = v * post_mul[m][n - post_c0] + post_add[m][n - post_c0]
     *      for n >= post_c0 (rows of pitch post_cs; post_mul and post_add share it);
     *  second output (GPEN NoiseInjection concat half, gpen_model.py:292-302):
     *      y[m][dup_off + n] = act(dup_a * dup_src[m][n] + dup_bias[n]) for n < cout (rows of pitch dup_cs;
     *      dup_bias may be NULL); dup_off >= cout and dup_off + cout <= ycs. */
    const float *post_mul, *post_add; int post_cs, post_c0;
    const float *dup_src, *dup_bias; float dup_a; int dup_cs, dup_off;
} s2v_conv_params;

enum { S2V_PREC_F32 = 0, S2V_PREC_BF16X3 = 1, S2V_PREC_F16X3 = 2 };

/* Replaces the nn.Conv2d / ConvTranspose2d / Conv1d / Linear calls of models/LNet.py,
 * ENet.py, DNet.py, base_blocks.py, ffc.py, transformer.py (inventory: SURVEY.md App. A). */
int s2v_conv2d(const s2v_conv_params *p, s2v_stream_t stream);
size_t s2v_conv2d_ws_bytes(const s2v_conv_params *p);
/* The launch plan s2v_conv2d would use: out11 = {BM, BN, WAVES_M, AVEC, B_KN, splits, prec, NW, KS, PF,
 * PERSIST} of the conv_igemm<BM,BN,WAVES_M,AVEC,B_KN> (prec 0) or
 * conv_igemm_x3<BM,BN,WAVES_M,NW,KS,PF,AVEC,B_KN,prec-1> (prec 1 / 2) instance — conv_igemm_x3_persist<...>
 * with PERSIST (> 0) blocks under ``grid_cap``, conv_glds_x3<BM,BN,WAVES_M,KS,prec-1> when AVEC == 5 —
 * or {0, CO, TPP, LW, 0, 1, 0, ...} for conv_small_cpar<CO,TPP,LW> (conv_direct_small<CO> when TPP == 0),
 * or {0, cout, -QPT, PX, 0, 1, ...} for conv_smallk<QPT,PX>.  force_tile: 0 = planner, 1..6 (f32) / 1..12
 * (split precisions) a fixed tile of the selected precision's table (tests / tuning). */
int s2v_conv2d_plan(const s2v_conv_params *p, int *out11);
/* Up to S2V_CONV_GROUP_MAX independent convolutions as ONE kernel launch (a tile table over the members'
 * tile grids on one tile configuration, each member with its own split-K factor), plus one launch
 * folding every member's split-K partials with that member's epilogue.  Replaces a fork of independent
 * convs that read the same block input (LNet's FFC: convl2l + convg2l, convl2g and the spectral
 * branch's first 1x1, ffc.py:176-233) — one launch filling the chip instead of three under-filled ones.
 * Members: split precision (one prec for all), packed split weights, a direct zero-padded conv with
 * cin % 32 == 0 and <= 32 taps, batch 1, no in_scale / pre_act / out_pool / grid_cap / x_split /
 * force_tile.  The workspace is member 0's (ws, ws_bytes >= s2v_conv2d_group_ws_bytes); plan: out[0] =
 * the x3 tile configuration (force_tile - 1 numbering), out[1 + i] = member i's split-K factor. */
#define S2V_CONV_GROUP_MAX 4
int s2v_conv2d_group(const s2v_conv_params *ps, int n, s2v_stream_t stream);
size_t s2v_conv2d_group_ws_bytes(const s2v_conv_params *ps, int n);
int s2v_conv2d_group_plan(const s2v_conv_params *ps, int n, int *out);
/* Planner knobs (tests / tuning; process-wide, not thread-safe against concurrent planning):
 *   S2V_TUNE_HALO_MIN_BLOCKS  the halo-tiled small-Cout kernel needs at least this many 8x128 tiles
 *                             (default 0, env S2V_HALO_MIN_BLOCKS; fewer go channel-parallel).  Below
 *                             ~3 tiles per CU it splits the channels (split-K workspace, see
 *                             s2v_conv2d_ws_bytes) and folds them with the epilogue;
 *   S2V_TUNE_GLDS_TILE        force an LDS-DMA tile config (-1 = planner, env S2V_GLDS_TILE);
 *   S2V_TUNE_SMALLK_TILE      1: split-precision convs with K <= 128 on large M take one N tile over
 *                             cout (default, env S2V_SMALLK_TILE); 0: the throughput model;
 *   S2V_TUNE_X3_RATE_512      the planner's sustained rate (TFLOP/s) of the 512x128 split-precision
 *                             tile (0 = the built-in table, env S2V_X3_RATE_512; A/B tuning);
 *   S2V_TUNE_IN_FUSED         max plane pixels (env S2V_IN_FUSED, default 576) of the one-launch InstanceNorm /
 *                             ADAIN (moments + apply per plane and 16-32-channel group, >= 512 blocks where
 *                             possible); 0: always stats + apply launches.  576 (LNet 12^2 and 24^2): LNet
 *                             B=16 11.65 -> 11.43 ms, lipsync 28.5 -> 28.0 ms on MI355X (r03).
 *   S2V_TUNE_RESIZE_UP2       1 (env S2V_RESIZE_UP2, default): exact x2 bilinear resizes take the 2x2-quad
 *                             kernel; 0: the generic float4 resize kernel.
 * Sets ``value``, returns the previous one in *old_value (may be NULL). */
enum { S2V_TUNE_HALO_MIN_BLOCKS = 0, S2V_TUNE_GLDS_TILE = 1, S2V_TUNE_SMALLK_TILE = 2, S2V_TUNE_X3_RATE_512 = 3,
       S2V_TUNE_IN_FUSED = 4, S2V_TUNE_RESIZE_UP2 = 5, S2V_TUNE_COUNT = 6 };
int s2v_tune(int key, long long value, long long *old_value);

/* max |x| over an NHWC view (pixels x c at pitch xcs) -> *out (fp32 bits; NaN propagates as the
 * largest value).  *out must be 0 before the launch (the kernel folds with an atomic max). */
int s2v_amax(const float *x, long long pixels, int c, int xcs, float *out, s2v_stream_t stream);

/* Split packed fp32 weights [rows][kpad] (kpad % 32 == 0) into the layout of ``prec``
 * (S2V_PREC_BF16X3 / S2V_PREC_F16X3): [rows][kpad/32][hi 32 | lo 32] 16-bit (same byte size),
 * v = w * scale (a power of two), hi = T_rne(v), lo = T_rne(v - hi).  Pass ``scale`` as the conv's
 * wt_scale.  s2v_split_weights_x3 = the bf16 form with scale 1. */
int s2v_split_weights(const float *w, int rows, int kpad, int prec, float scale, void *out, s2v_stream_t stream);
int s2v_split_weights_x3(const float *w, int rows, int kpad, void *out, s2v_stream_t stream);
/* fp32 NHWC activations [pixels][xcs] -> the split layout of ``prec`` at pitch ocs (floats; the
 * conv input of s2v_conv_params.x_split): per pixel and 32-channel block [hi 32 | lo 32] 16-bit,
 * hi = T_rne(v), lo = T_rne(v - hi).  c % 32 == 0, ocs % 32 == 0, out 128-byte aligned. */
int s2v_split_act(const float *x, long long pixels, int c, int xcs, int prec, float *out, int ocs,
                  s2v_stream_t stream);

/* LayerNorm2d (base_blocks.py:52-69) over (H,W,C) per sample, fused affine + act
 * (+ 2x2 average pool: DownBlock2d base_blocks.py:95-109) (+ residual after act: Jump + out,
 * LNet.py:75).  ws: >= s2v_layernorm2d_ws_bytes(n, h, w, c) bytes. */
int s2v_layernorm2d(const float *x, int n, int h, int w, int c, int xcs,
                    const float *weight, const float *bias, float eps, int act, float alpha, int pool,
                    const float *res, int res_cs, float *y, int ycs, void *ws, size_t ws_bytes,
                    s2v_stream_t stream);
size_t s2v_layernorm2d_ws_bytes(int n, int h, int w, int c);

/* ADAIN apply (base_blocks.py:143-157): InstanceNorm2d(eps) * (1 + gamma[n,c]) + beta[n,c],
 * then act, then + res.  gamma/beta rows have stride gb_ns per sample. */
int s2v_instnorm_adain(const float *x, int n, int h, int w, int c, int xcs,
                       const float *gamma, const float *beta, int gb_ns, float eps, int act, float alpha,
                       const float *res, int res_cs, float *y, int ycs, void *ws, size_t ws_bytes,
                       s2v_stream_t stream);
/* s2v_instnorm_adain that also writes F.pad(y, (1, 1, 1, 1), 'reflect') to yp ([n][h+2][w+2],
 * pitch ypcs): the FFC's reflect-padded 3x3 convs read the next block's input without a separate
 * pad pass.  Vector path only (c % 4 == 0, 4-aligned pitches, 16-byte aligned x / y / yp / res). */
int s2v_instnorm_adain_pad(const float *x, int n, int h, int w, int c, int xcs, const float *gamma,
                           const float *beta, int gb_ns, float eps, int act, float alpha, const float *res, int res_cs,
                           float *y, int ycs, float *yp, int ypcs, void *ws, size_t ws_bytes, s2v_stream_t stream);
size_t s2v_instnorm_ws_bytes(int n, int h, int w, int c);

/* Segmented GEMV for all ADAIN gamma/beta heads at once (base_blocks.py:148-155):
 *   out[b][o] = bias[o] + sum_j W2t[j][o] * hid[b][seg[o]*nhidden + j]
 * W2t is [nhidden][total] (transposed so consecutive o are contiguous). */
int s2v_adain_params(const float *hid, int batch, int hid_ns, int nhidden, const float *w2t,
                     const float *bias, const int *seg, int total, float *out, int out_ns,
                     s2v_stream_t stream);

/* StyleGAN2 demodulation (base_blocks.py:492-494) without per-sample weights:
 *   d[b][o] = rsqrt(sum_i s[b][i]^2 * wsq[o][i] + eps) * post */
int s2v_modconv_demod(const float *s, int batch, int s_ns, int cin, const float *wsq, int cout,
                      float eps, float post, float *d, int d_ns, s2v_stream_t stream);

/* Every demodulated layer of a StyleGAN2 decoder in one launch (stylegan2_clean_arch.py:81-83,
 * gpen_model.py:225-247): for r < nrows, with (s_off, cin, w_off, -) = rows[4r..4r+3] (16-byte
 * aligned int32 table),
 *   d[b][r] = rsqrt(sum_{i<cin} s[b][s_off + i]^2 * wsq[w_off + (r - r0) * cin + i] + eps) * post
 * i.e. w_off already points at row r's squared-weight row. */
int s2v_modconv_demod_rows(const float *s, int batch, int s_ns, const int *rows, int nrows,
                           const float *wsq, float eps, float post, float *d, int d_ns,
                           s2v_stream_t stream);

/* Bilinear resize (F.interpolate mode='bilinear', align_corners=False, no antialias) between
 * arbitrary strided 4-D views; scale_h/scale_w as torch's area_pixel_compute_scale.
 * Element (n,c,y,x) at base + n*sn + c*sc + y*sy + x*sx (strides in elements).
 * mode 0 bilinear, 1 nearest (floor(dst*scale)). Output index order is (n, y, x, c). */
int s2v_resize(const float *x, int n, int c, int ih, int iw, long long xsn, long long xsc, long long xsy,
               long long xsx, float *y, int oh, int ow, long long ysn, long long ysc, long long ysy,
               long long ysx, float scale_h, float scale_w, int mode, s2v_stream_t stream);

/* ENet / StyleGAN2 ToRGB and its skip upsample in one pass (base_blocks.py:536-554, ENet.py:119-129;
 * replaces s2v_modulate_weights + the small-Cout conv with ``res`` + the x2 s2v_resize of the skip):
 *   y[b,p,o] = (sum_c wt[o][c] * s[b][c] * x[b,p,c] + bias[o]) + up2(skip)[b,p,o]   (o < 3)
 *   y[b,p,3] = up2(skip)[b,p,3]
 * x NHWC [n][h][w] (pixel pitch xcs, c % 32 == 0), wt packed 1x1 rows [3+][kpad], s [n][s_ns], bias [3]
 * or NULL, skip NHWC [n][h/2][w/2] (pitch skcs >= 4), y NHWC [n][h][w] (pitch ycs >= 4); up2 is
 * F.interpolate(scale_factor=2, mode='bilinear', align_corners=False).  h*w % 32 == 0. */
int s2v_torgb_up2(const float *x, int n, int h, int w, int c, int xcs, const float *wt, int kpad, const float *s,
                  int s_ns, const float *bias, const float *skip, int skcs, float *y, int ycs, s2v_stream_t stream);

/* Row-tap packing of a small-channel input for a kh x kw conv (r04): y[n][h][w][dx * c + ci] =
 * x[n][h][w + dx - pw][ci] (zero outside the row), channels [kw * c, ycs) zero; the conv then runs as
 * a kh x 1 conv over ycs channels with the taps' weights at the same channel positions.  No
 * reference counterpart (a layout step of this framework's 7x7 first-layer convs: LNet.py:33-34
 * first_inp / first_ref, DNet.py:93 input_layer, base_blocks.py:267 EditingNet first). */
int s2v_row_pack(const float *x, int n, int h, int w, int c, int xcs, int kw, int pw, float *y, int ycs,
                 s2v_stream_t stream);

/* F.pad(mode='reflect') on NHWC (ENet.py:119). */
int s2v_pad_reflect(const float *x, int n, int h, int w, int c, int xcs, int pt, int pb, int pl, int pr,
                    float *y, int ycs, s2v_stream_t stream);

/* Row LayerNorm over the last dim (transformer.py:24-35 nn.LayerNorm). */
int s2v_row_layernorm(const float *x, int rows, int dim, int xld, const float *weight, const float *bias,
                      float eps, float *y, int yld, s2v_stream_t stream);

/* Multi-head attention core (transformer.py:73-80): per (b, head):
 *   O = softmax(Q K^T * scale) V; tokens <= 256, dim_head == 64. Q/K/V/O rows are tokens with
 *   leading dims q_ld.. and per-batch strides; head h uses columns [h*64, h*64+64). */
int s2v_attention(const float *q, const float *k, const float *v, int batch, int heads, int tokens,
                  int dim_head, int ld_q, int ld_k, int ld_v, long long bs_q, long long bs_k, long long bs_v,
                  float scale, float *o, int ld_o, long long bs_o, s2v_stream_t stream);

/* DNet warp (flow_util.py:3-56) fused: flow [n][fh][fw][2] NHWC -> deformation grid
 * (align_corners=True convention) -> bilinear resize to (h, w) -> grid_sample(bilinear, zeros,
 * align_corners=False) of src (NCHW-strided view, c channels). Output NHWC slice. */
int s2v_flow_warp(const float *flow, int n, int fh, int fw, int flow_cs, const float *src, int c, int h,
                  int w, long long ssn, long long ssc, long long ssy, long long ssx, float *y, int ycs,
                  s2v_stream_t stream);
/* The same warp written beside a copy of its source: y[p, 0:c) = src[p], y[p, c:2c) = warp(src)[p]
 * (EditingNet's torch.cat([input_image, warp_image], 1), DNet.py:114-115) in one pass; ycs >= 2c. */
int s2v_flow_warp_cat(const float *flow, int n, int fh, int fw, int flow_cs, const float *src, int c, int h,
                      int w, long long ssn, long long ssc, long long ssy, long long ssx, float *y, int ycs,
                      s2v_stream_t stream);

/* Mel spectrogram (futils/audio.py:45-51, :20-23, :57-61, :92-123 + hparams.py:21-61):
 * preemphasis(0.97) -> STFT(n_fft 800, hop 200, periodic Hann, center=True, zero or reflect
 * pad) -> |.| -> mel (80 x 401, Slaney) -> 20 log10(max(1e-5, .)) - 20 -> clip(8 (S+100)/100 - 4,
 * -4, 4).  ``tables`` = mel basis [80][401] | cos(2 pi k/800) [800] | sin [800] | window [800]
 * (the sin table carries the -i of the forward DFT only through |.|).  Output [80][frames],
 * frames = 1 + n_samples / 200. */
int s2v_melspectrogram(const float *wav, long long n_samples, const float *tables, int pad_reflect,
                       float *out, long long frames, s2v_stream_t stream);

/* Per-video-frame 16-column mel windows (inference.py:209-216): out[i][80][step] =
 * mel[:, starts[i] : starts[i] + step]; starts (device int32) computed by the host. */
int s2v_mel_chunks(const float *mel, long long frames, const int *starts, int nchunks, int step, float *out,
                   s2v_stream_t stream);

/* GPEN native ops, same signatures/semantics as third_part/GPEN/face_model/op/:
 *   fused_bias_act (fused_bias_act.cpp:4-21, fused_bias_act_kernel.cu:18-99)
 *   y = scale * act(x + b[(i / step_b) % C]) with act 1 = linear, 3 = leaky relu(alpha);
 *   grad = 1 is the backward form using ref > 0.  size = numel, step_b = prod of dims after C. */
int s2v_fused_bias_act(const float *x, const float *b, const float *ref, float *y, long long size, int c,
                       long long step_b, int act, int grad, float alpha, float scale, s2v_stream_t stream);
/* upfirdn2d (upfirdn2d.cpp:4-23, upfirdn2d_kernel.cu:140-271) on [major][H][W][minor]; any
 * up/down/pad combination (the reference silently returns garbage for unsupported ones). */
int s2v_upfirdn2d(const float *x, int major, int in_h, int in_w, int minor, const float *k, int kh, int kw,
                  int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1,
                  float *y, int out_h, int out_w, s2v_stream_t stream);
/* The same two ops over the element types of the reference's AT_DISPATCH_FLOATING_TYPES_AND_HALF
 * (fused_bias_act_kernel.cu:79, upfirdn2d_kernel.cu:225).  Every pointer (bias, refer, kernel
 * included) holds `dtype` elements.  Arithmetic: S2V_DT_F64 in double throughout (alpha / scale
 * taken as double); S2V_DT_F16 loads halves, computes in fp32 and rounds once on the store (the
 * reference's CUDA path rounds after every operation; its CPU fallback computes each op in fp32);
 * S2V_DT_F32 is s2v_fused_bias_act / s2v_upfirdn2d. */
enum { S2V_DT_F32 = 0, S2V_DT_F16 = 1, S2V_DT_F64 = 2 };
int s2v_fused_bias_act_dt(int dtype, const void *x, const void *b, const void *ref, void *y, long long size, int c,
                          long long step_b, int act, int grad, double alpha, double scale, s2v_stream_t stream);
int s2v_upfirdn2d_dt(int dtype, const void *x, int major, int in_h, int in_w, int minor, const void *k, int kh,
                     int kw, int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0,
                     int pad_y1, void *y, int out_h, int out_w, s2v_stream_t stream);

/* FourierUnit transforms (models/ffc.py:93-126): torch.fft.rfftn / irfftn over (H, W),
 * norm='ortho', as separable 1-D passes staged in LDS (one block per sample x 4 channels).
 *   s2v_rfft2:  x NHWC [n][h][w] (pitch xcs)  ->  spec[n][u*Wf + v][part*C + c] (pitch scs >= 2C),
 *               Wf = w/2 + 1, part 0 = real, 1 = imaginary (the FourierUnit's [B, F, 2C] layout)
 *   s2v_irfft2: spec (same layout)  ->  y NHWC = irfftn(spec, s=(h, w)) (+ res NHWC, may be NULL)
 * tables: s2v_fft_tables_floats(h, w) floats = fw[w][2][Wf] | fh[h][2][h(u)] | ih[h(u)][2][h] |
 * iw[Wf][2][w], the 1-D ortho transform matrices (host-built from torch.fft on basis vectors),
 * [.][0][.] real and [.][1][.] imaginary parts.
 * C % 4 == 0, 16-byte aligned x / spec, h*w small enough for LDS (<= 48x48 fits). */
size_t s2v_fft_tables_floats(int h, int w);
int s2v_rfft2(const float *x, int n, int h, int w, int c, int xcs, const float *tables, float *spec, int scs,
              s2v_stream_t stream);
int s2v_irfft2(const float *spec, int n, int h, int w, int c, int scs, const float *tables, const float *res,
               int rcs, float *y, int ycs, s2v_stream_t stream);

/* LNet's FFC (FineADAINLama, models/base_blocks.py:368-386; FFC models/ffc.py:176-233 with ratio 0.75) as
 * three fused kernels per FFC at the decoder levels h in {12, 24, 48} (C = s2v_ffc_channels(h) = 1024 /
 * 256 / 128; cl = C/4, cg = 3C/4, cc = cg/2; F = h (h/2 + 1)), n images.  Replaces the launch chain
 * st1 -> rfft2 -> fu -> irfft2 -> st2 -> instnorm (the reference's SpectralTransform / FourierUnit
 * forward, ffc.py:60-173, and ADAIN, base_blocks.py:127-157):
 *   s2v_ffc_spec_fwd: t1 = relu(bn1(x_g conv1)) -> t1 [n][h*h][cc] dense, spec = rfftn(t1, ortho) ->
 *                     spec [n][F][2cc] dense ((part, c) channel order, as s2v_rfft2); x_g: the block input's
 *                     global channels (pitch xcs)
 *   s2v_ffc_spec_inv: u = irfftn(relu(bn_fu(spec conv_fu))) + t1 -> u [n][h*h][cc] dense
 *   s2v_ffc_norm:     z = [y_l | y_g + u conv2] (y [n][h*h][C] with conv_to_l's and conv_l2g's outputs, pitch
 *                     ycs), out = act((z - mean) rstd (1 + gamma) + beta) (+ res); pad (optional, [n][h+2][h+2]
 *                     pitch pad_cs) also receives F.pad(out, 1, 'reflect').  out may be y itself.
 * w1 / wfu / w2: packed weights in the split layout of prec (s2v_split_weights with weight pre-scale
 * wt_scale; kpad >= the K of the conv, npad >= 128); scale / shift: folded BatchNorm per output channel (may
 * be NULL); x_scale: the f16x3 activation pre-scale of the conv's input (power of two, 1 = none); tables:
 * s2v_fft_tables for (h, h); flag (may be NULL): set to 1 when an accumulator is not finite (the f16x3 range
 * guard).  prec: S2V_PREC_F16X3 or S2V_PREC_BF16X3 (the exact-f32 arithmetic uses the separate kernels). */
/* Self-check of the split-fp32 f16 operand split (conv_x3_impl.hpp split4): both variants (X3_F16_MIX 1 / 0)
 * on x (n % 4 == 0 floats); *mismatch (device int, zeroed by the caller) += the float4s whose halves differ. */
int s2v_f16_split_check(const float *x, long long n, int *mismatch, s2v_stream_t stream);

int s2v_ffc_channels(int h);
int s2v_ffc_spec_fwd(const float *x_g, int xcs, int n, int h, const void *w1, int w1_kpad, float wt_scale, float x_scale,
                     const float *scale, const float *shift, const float *tables, float *t1, float *spec, int *flag,
                     int prec, s2v_stream_t stream);
int s2v_ffc_spec_inv(const float *spec, int n, int h, const void *wfu, int wfu_kpad, float wt_scale, float x_scale,
                     const float *scale, const float *shift, const float *tables, const float *t1, float *u, int *flag,
                     int prec, s2v_stream_t stream);
int s2v_ffc_norm(const float *y, int ycs, int n, int h, const float *u, const void *w2, int w2_kpad, float wt_scale,
                 float x_scale, const float *gamma, const float *beta, int gb_ns, float eps, int act, float alpha,
                 const float *res, int res_cs, float *out, int out_cs, float *pad, int pad_cs, int *flag, int prec,
                 s2v_stream_t stream);

/* Per-sample modulated conv weights (StyleGAN2 ModulatedConv2d, base_blocks.py:487-495,
 * stylegan2_clean_arch.py:66-80, gpen_model.py:245-256) from packed [npad][kpad] weights:
 *   out[b][o][k] = wt[o][k] * s[b][k % cin] * (d ? d[b][o] : 1)   (k < K; padding stays 0)
 * out is [batch][npad][kpad]; run the conv with batch = B, n = 1 and w_bs = npad * kpad. */
int s2v_modulate_weights(const float *wt, int npad, int kpad, int K, int cin, int cout, const float *s, int s_ns,
                         const float *d, int d_ns, int batch, float *out, s2v_stream_t stream);
/* Same, times ``scale`` (a power of two: the conv's wt_scale), written in the split layout of ``prec``
 * (kpad % 32 == 0): pass ``out`` as wt_x3.  s2v_modulate_weights_x3 = bf16, scale 1. */
int s2v_modulate_weights_split(const float *wt, int npad, int kpad, int K, int cin, int cout, const float *s,
                               int s_ns, const float *d, int d_ns, int batch, int prec, float scale, void *out,
                               s2v_stream_t stream);
int s2v_modulate_weights_x3(const float *wt, int npad, int kpad, int K, int cin, int cout, const float *s, int s_ns,
                            const float *d, int d_ns, int batch, void *out, s2v_stream_t stream);

/* NHWC FIR resampling with fused epilogue (the engines' form of upfirdn2d, GPEN gpen_model.py:37-91
 * Upsample / Blur and the blur after the transposed modulated conv, :270-276):
 *   y[n,oy,ox,c] = post * act(gain * sum_{i,j} kflip[i][j] * xu[n, oy*down + i - pad_y0, ox*down + j - pad_x0, c]
 *                             + bias[c])
 * xu = x zero-inserted by `up`; positions outside it are zero (pad_y1 / pad_x1 are implied by oh / ow).
 * x / y are channel-slice views (pitch xcs / ycs); kernel [kh][kw] (<= 64 taps) in device memory. */
int s2v_fir2d(const float *x, int n, int ih, int iw, int c, int xcs, const float *k, int kh, int kw, int up,
              int down, int pad_y0, int pad_x0, float *y, int oh, int ow, int ycs, float gain, const float *bias,
              int act, float alpha, float post, s2v_stream_t stream);

/* N(0,1) noise from a counter-based generator (StyleConv noise injection,
 * base_blocks.py:528-531): y[i] = BoxMuller(splitmix64(seed ^ splitmix64(offset + i))). */
int s2v_gaussian_noise(float *y, long long n, unsigned long long seed, unsigned long long offset,
                       s2v_stream_t stream);
/* Same with the offset advanced by (*ctr << shift), ctr a device counter read when the kernel runs,
 * and the counter bump that goes with it (ctr[0] += inc): a captured HIP graph that bumps the counter
 * and then draws draws fresh noise on every replay, like the reference's per-call normal_(). */
int s2v_gaussian_noise_ctr(float *y, long long n, unsigned long long seed, unsigned long long offset,
                           const unsigned long long *ctr, int shift, s2v_stream_t stream);
int s2v_counter_add(unsigned long long *ctr, unsigned long long inc, s2v_stream_t stream);

/* Full-clip pipeline glue.  DNet fake [n,3,h,w] in [-1,1] -> uint8 reference frames
 * (preprocessing/facing.py:190-191) and the ENet inputs built from them and the original crops src
 * (inference.py:393-399): face6 = [masked original | ref] / 255 (rows >= h/2 of the original zeroed),
 * gt = ref / 255.  All NCHW.  fake NULL: ref_u8 is an input (the references a Step-5 enhancer replaced,
 * inference.py:234-238) and only face6 / gt are written. */
int s2v_lipsync_inputs(const float *src, const float *fake, int n, int h, int w, unsigned char *ref_u8,
                       float *face6, float *gt, s2v_stream_t stream);
/* y = uint8((clamp(x, lo, hi) + offset) * scale) with truncation (inference.py:267, :288). */
int s2v_to_u8(const float *x, long long n, float lo, float hi, float scale, float offset, unsigned char *y,
              s2v_stream_t stream);
/* Elementwise over NHWC views: y = post * act(a * x [* mul] [+ add] [+ bias[c]]) — GFPGAN SFT
 * (gfpganv1_clean_arch.py:98-106), U-Net skip adds, GPEN NoiseInjection halves (gpen_model.py:287-302). */
int s2v_eltwise(const float *x, int xcs, const float *mul, int mcs, const float *add, int acs, const float *bias,
                long long pixels, int c, float a, int act, float alpha, float post, float *y, int ycs,
                s2v_stream_t stream);

/* y[0:n) = value (channel padding of 3-channel images to the vectorised 4-channel layout). */
int s2v_fill(float *y, long long n, float value, s2v_stream_t stream);

/* ---- Mouth-region post-process (inference.py:302-313) ----------------------- */

/* cv2.resize(src, (ow, oh)) with INTER_LINEAR (OpenCV imgproc resize.cpp) on HWC images:
 * element (b, y, x, ch) at x + b*xis + y*xrs + x*c + ch (pitches in elements; ROIs of larger frames
 * are plain pointer offsets).  mode 0: uint8 -> uint8 (11-bit fixed-point weights), 1: fp32 -> fp32,
 * 2: fp32 -> uint8 truncated (np.uint8 of the float result, inference.py:313), 3: uint8 -> fp32
 * (v == 255 ? 1 : 0: the mask paste of inference.py:305-308, resized / 255. stored into uint8),
 * 4: fp64 -> fp64 (double sums, float coefficients: FaceEnhancement's mask_sharp). */
int s2v_resize_linear(const void *x, int n, int h, int w, int c, long long xrs, long long xis, void *y, int oh,
                      int ow, long long yrs, long long yis, int mode, s2v_stream_t stream);
/* The same for cv2.resize(src, (0, 0), fx=fx, fy=fy): (ow, oh) = (round(w fx), round(h fy)) chosen by
 * the caller, source coordinates scaled by 1 / fx, 1 / fy (OpenCV keeps the given factors). */
int s2v_resize_linear_fxfy(const void *x, int n, int h, int w, int c, long long xrs, long long xis, void *y, int oh,
                           int ow, long long yrs, long long yis, int mode, double fx, double fy, s2v_stream_t stream);

/* Laplacian_Pyramid_Blending_with_mask (futils/inference_utils.py:181-222): A, B uint8 [n][h][w][c],
 * m fp32 [n][h][w] -> out fp32 [n][h][w][c]; cv2.pyrDown / pyrUp semantics (reflect-101 borders,
 * uint8 Gaussian pyramids of A and B, fp32 of m); ``clip`` applies np.clip(out, 0, 255) (:313).
 * h and w must be divisible by 2^(levels-1) (the reference's np.subtract fails otherwise).
 * ws: >= s2v_laplacian_blend_ws_bytes(n, h, w, c, levels) bytes (0 for levels == 1). */
size_t s2v_laplacian_blend_ws_bytes(int n, int h, int w, int c, int levels);
int s2v_laplacian_blend(const unsigned char *a, const unsigned char *b, const float *m, int n, int h, int w, int c,
                        int levels, int clip, float *out, void *ws, size_t ws_bytes, s2v_stream_t stream);

/* FaceParse mask (face_parsing.py:47-57, :65-81): per pixel the first argmax over c parsing logits
 * at x + b*xbs + p*ps + k*cs (NCHW: ps = 1, cs = h*w; NHWC: ps = c, cs = 1) -> out[b*h*w + p] =
 * cmap[argmax] (uint8, may be NULL) and / or cls[...] = argmax (may be NULL). */
int s2v_parse_mask(const float *x, int n, int h, int w, int c, long long xbs, long long ps, long long cs,
                   const unsigned char *cmap, unsigned char *out, int *cls, s2v_stream_t stream);

/* FaceParse.img2tensor (face_parsing.py:59-63): uint8 HWC pixels (3 bytes, BGR if ``flip``) ->
 * fp32 RGB (img / 255. * 2 - 1, in float64 then rounded) at pixel pitch ycs (>= 3; channel 3 = 0). */
int s2v_img_u8_to_m11(const unsigned char *x, long long pixels, int flip, float *y, int ycs, s2v_stream_t stream);

/* ---- Super-resolution front / back end (real_esrnet.py:99-137) ---------------- */

/* RealESRNet.process input (real_esrnet.py:100-115): uint8 HWC frames [n,h,w,3] (BGR if ``flip``)
 * -> fp32 RGB x / 255 at pixel pitch ycs (>= 3; channel 3 = 0) of [n, h+pad_b, w+pad_r],
 * F.pad 'reflect' on the bottom / right (pad < dimension, as F.pad requires). */
int s2v_sr_u8_in(const unsigned char *x, int n, int h, int w, int flip, int pad_b, int pad_r, float *y, int ycs,
                 s2v_stream_t stream);
/* RealESRNet.process output (:126-131): the top-left h x w crop of an NHWC fp32 image [n,xh,xw,xcs]
 * -> uint8 [n,h,w,3] = round_half_even(clamp(x, 0, 1) * 255) (channels reversed if ``flip``). */
int s2v_sr_f32_out(const float *x, int n, int h, int w, int xh, int xw, int xcs, int flip, unsigned char *y,
                   s2v_stream_t stream);

/* ---- Face detection / alignment / paste-back (face_enhancement.py:91-193) ----- */

/* RetinaFaceDetection.detect input (retinaface_detection.py:59-73): BGR pixels (xtype 0 uint8,
 * 1 fp32) -> fp32 NHWC4 (b - 104, g - 117, r - 123, 0); y 16-byte aligned. */
int s2v_bgr_mean_nhwc4(const void *x, int xtype, long long pixels, float *y, s2v_stream_t stream);
/* F.max_pool2d(x, k, s, p) on NHWC fp32 (c % 4 == 0; the ResNet-50 stem pool: 3, 2, 1). */
int s2v_maxpool2d_nhwc(const float *x, int n, int h, int w, int c, int k, int s, int p, float *y, int oh, int ow,
                       s2v_stream_t stream);
/* RetinaFace priors + decode + threshold (prior_box.py:20-34, box_utils.py:209-247,
 * retinaface_detection.py:81-104) for cfg_re50 (steps 8/16/32, min sizes 16,32 / 64,128 / 256,512,
 * variances 0.1 / 0.2).  heads[l]: level l fused head output, NHWC [hs[l]][ws[l]][cs] with channels
 * [box anchor0 (4) | box anchor1 (4) | class logits a0 (2) | a1 (2) | landmarks a0 (10) | a1 (10)]
 * (cs >= 32); hs / ws must be ceil(im / step).  Every prior whose softmax score > thresh is written
 * to cand as 16 floats [prior index (int bits), x1, y1, x2, y2 (pixels), score, 5 x (x, y)] at
 * slot atomicAdd(count): the order of the slots is arbitrary (the host sorts by prior index).
 * max_cand must be >= the number of priors. */
int s2v_retina_decode(const float *const *heads, const int *hs, const int *ws, int cs, int im_h, int im_w,
                      float thresh, float *cand, int *count, int max_cand, s2v_stream_t stream);
/* RetinaFace.forward's outputs in phase 'test' (retinaface.py:115-124) from the same head maps for n
 * images (image b of level l at heads[l] + b*hs[l]*ws[l]*cs): loc [n][P][4], conf = softmax [n][P][2],
 * landms [n][P][10], priors in PriorBox order. */
int s2v_retina_split(const float *const *heads, const int *hs, const int *ws, int cs, int im_h, int im_w, int n,
                     float *loc, float *conf, float *landms, s2v_stream_t stream);
/* cv2.warpAffine(src, M, (ow, oh), flags=INTER_LINEAR or INTER_AREA, BORDER_CONSTANT 0) on n HWC
 * images (dtype 0 uint8, 1 fp32, 2 fp64; pitches in elements): M = n device 2x3 fp64 forward
 * matrices, inverted on the device (invertAffineTransform); OpenCV's fixed-point source coordinates
 * (AB_BITS 10, INTER_BITS 5), uint8 through 15-bit weights, float in tap order. */
int s2v_warp_affine(const void *x, int n, int h, int w, int c, long long xrs, long long xis, int dtype,
                    const double *M, void *y, int oh, int ow, long long yrs, long long yis, s2v_stream_t stream);
/* FaceEnhancement paste-back (face_enhancement.py:143-157) with both warps fused: for frame pixels
 * in [y0, y0+wh) x [x0, x0+ww): t = warpAffine(mask fp32 [S][S], M); where t > full_mask:
 * full_mask = t and full_img (uint8 [H][W][3]) = warpAffine(face uint8 [S][S][3], M).  Pixels
 * outside the window must be ones where the warped mask is 0 (the window bounds the warped crop). */
int s2v_face_paste(const float *mask, const unsigned char *face, int S, const double *M, float *full_mask,
                   unsigned char *full_img, int H, int W, int y0, int x0, int wh, int ww, s2v_stream_t stream);
/* cv2.GaussianBlur on one [h][w] channel, BORDER_REFLECT_101, separable with the ksize taps of
 * ``kern`` (work type dtype: 1 fp32, 2 fp64; kern in that type, device memory): row pass in tap
 * order, column pass as SymmColumnFilter.  xtype 0: uint8 input read as v / 255. (mask_postprocess's
 * mask_sharp), else the work type; zero_border > 0 zeroes the input outside [zb, h-zb) x [zb, w-zb)
 * first (face_enhancement.py:84-85).  ytype 1 fp32 / 2 fp64 (fp64 -> fp32 is one rounding).
 * ws >= s2v_gaussian_blur_ws_bytes(h, w, dtype). */
size_t s2v_gaussian_blur_ws_bytes(int h, int w, int dtype);
int s2v_gaussian_blur(const void *x, int xtype, int h, int w, int zero_border, const void *kern, int ksize, void *y,
                      int ytype, int dtype, void *ws, size_t ws_bytes, s2v_stream_t stream);
/* cv2.filter2D(img, -1, kern 3x3 fp32) on uint8 HWC, BORDER_REFLECT_101, cvRound + saturate. */
int s2v_filter3x3_u8(const unsigned char *x, int h, int w, int c, const float *kern, unsigned char *y,
                     s2v_stream_t stream);
/* FaceGAN.img2tensor / tensor2img (face_gan.py:44-59): uint8 HWC BGR [n][h][w][3] <-> fp32 NCHW
 * RGB [n][3][h][w] in [-1, 1]; the way back is np.clip(x * 0.5 + 0.5, 0, 1) * 255 truncated. */
int s2v_u8_to_gan(const unsigned char *x, int n, int h, int w, float *y, s2v_stream_t stream);
int s2v_gan_to_u8(const float *x, int n, int h, int w, unsigned char *y, s2v_stream_t stream);
/* y = x / 255. as float64 (mask_sharp, face_enhancement.py:137). */
int s2v_u8_div255_f64(const unsigned char *x, long long n, double *y, s2v_stream_t stream);
/* mask_sharp of FaceEnhancement.process after mask_postprocess mutated it: parse / 255. with the
 * ``border``-pixel frame zeroed (face_enhancement.py:84-85 on the array of :144).  x: uint8 [h, w],
 * y: fp64 [h, w]. */
int s2v_u8_div255_f64_border(const unsigned char *x, int h, int w, int border, double *y, s2v_stream_t stream);
/* Final blend of FaceEnhancement.process on uint8 HWC frames (3 channels): mask_sharp == NULL:
 * convertScaleAbs(base * (1 - full_mask) + full_img * full_mask) (use_sr, :175-176); else
 * img = that (base = ori_img), then convertScaleAbs(ori * (1 - mask_sharp) + img * mask_sharp) with
 * the fp64 mask_sharp (:189-191). */
int s2v_face_blend(const unsigned char *base, const float *full_mask, const unsigned char *full_img,
                   const double *mask_sharp, unsigned char *out, long long pixels, s2v_stream_t stream);

/* ---- GFPGANer.enhance restore composition (third_part/GFPGAN/gfpgan/utils.py:97-143, inference.py:300-301;
 * facexlib 0.2.5 FaceRestoreHelper, requirements.txt:5, not vendored) ------------------------------- */

/* s2v_warp_affine with BORDER_CONSTANT value border[ch] (host array of c values, saturated to the
 * image type; NULL = 0): align_warp_face's cv2.warpAffine(img, affine, (512, 512),
 * borderValue=(135, 133, 132)).  xis == 0 warps one source image with each of the n matrices. */
int s2v_warp_affine_border(const void *x, int n, int h, int w, int c, long long xrs, long long xis, int dtype,
                           const double *M, void *y, int oh, int ow, long long yrs, long long yis,
                           const double *border, s2v_stream_t stream);
/* basicsr tensor2img(x, rgb2bgr=True, min_max=(-1, 1)) (gfpgan/utils.py:121): fp32 NCHW RGB
 * [n][3][h][w] -> uint8 HWC BGR, round((clamp(x, -1, 1) + 1) / 2 * 255) half to even. */
int s2v_tensor2img_u8(const float *x, int n, int h, int w, unsigned char *y, s2v_stream_t stream);
/* paste_faces_to_input_image's square mask (upscale 1) on the frame window [y0, y0+wh) x [x0, x0+ww)
 * of an H x W frame: erosion [wh][ww] fp32 = cv2.erode(warpAffine(ones(S, S) fp32, M), ones((2, 2)))
 * (frame coordinates) with M the device fp64 2x3 inverse affine (warpAffine inverts it again, as OpenCV
 * does); area[0] (device fp64) = the sum of the erosion over the window, in a fixed order; area holds
 * 1 + s2v_restore_parts() doubles (area[1..] are the per-block partials).  A window holding the warped crop's whole
 * footprint gives the frame's sum. */
int s2v_restore_mask(const double *M, int S, int H, int W, int y0, int x0, int wh, int ww, float *erosion,
                     double *area, s2v_stream_t stream);
/* The per-block partial count of s2v_restore_mask: its area buffer holds 1 + s2v_restore_parts() doubles. */
int s2v_restore_parts(void);
/* cv2.erode(x, ones((k, k), uint8)) on an fp32 [h][w] image (anchor k / 2, border never wins);
 * ws: h * w floats, distinct from x and y. */
int s2v_erode_rect_f32(const float *x, int h, int w, int k, float *y, float *ws, s2v_stream_t stream);
/* out = soft * (erosion * warpAffine(face uint8 [S][S][3], M)) + (1 - soft) * base in fp32 on HWC
 * [H][W][3] frames, soft / erosion [wh][ww] covering the frame window [y0, +wh) x [x0, +ww) (0 outside);
 * base / out uint8 (0) or the fp32 accumulator of several faces (1; in place allowed), uint8 out
 * truncates (astype(uint8)). */
int s2v_restore_paste(const unsigned char *face, int S, const double *M, const float *soft, const float *erosion,
                      int y0, int x0, int wh, int ww, const void *base, int base_f32, void *out, int out_f32, int H,
                      int W, s2v_stream_t stream);

/* ---- 3DMM coefficient regression front end (facing.py:100-130) ---------------- */

/* face3d util/preprocess.py resize_n_crop_img (:147-167) as align_img (:186-216) calls it, then the
 * network input of facing.py:120: PIL img.resize((w, h), resample = filter: 2 BILINEAR, 3 BICUBIC)
 * and img.crop((left, up, left + ow, up + oh)) on n uint8 RGB frames [n][h0][w0][3] (frame stride
 * xis bytes) with Pillow's Resample.c arithmetic (double taps, 22-bit fixed point, uint8 rows
 * between the horizontal and vertical pass; crop pixels outside the resized image are 0) ->
 * fp32 float32(pixel / 255.) NHWC [n][oh][ow][ycs] (channels >= 3 zero).  params: DEVICE int32
 * [n][4] = (w, h, left, up) per frame; a resample that needs more than 48 taps per output
 * coordinate (more than an 11.75x bicubic downscale) writes NaN.  Replaces facing.py:118-121
 * (align_img + np.array(im) / 255. + torch.tensor) for every frame of the clip at once. */
int s2v_pil_resize_crop(const unsigned char *x, int n, int h0, int w0, long long xis, const int *params, int filter,
                        float *y, int oh, int ow, int ycs, s2v_stream_t stream);
/* nn.AdaptiveAvgPool2d((1, 1)) on NHWC fp32: y[b][c] = mean of x[b][0..hw)[c] (fp64 sum)
 * (face3d models/networks.py ResNet._forward_impl avgpool). */
int s2v_spatial_mean_nhwc(const float *x, int n, int hw, int c, float *y, s2v_stream_t stream);

const char *s2v_last_error(void);
/* number of compute units of the current device (0 if no device) */
int s2v_device_cus(void);
const char *s2v_version(void);

#ifdef __cplusplus
}
#endif
#endif /* S2V_H_ */
