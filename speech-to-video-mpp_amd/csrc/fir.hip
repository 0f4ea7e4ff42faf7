// NHWC FIR resampling with a fused bias/activation epilogue (the StyleGAN2 / GPEN blur path).
//
// Semantics are upfirdn2d's (third_part/GPEN/face_model/op/upfirdn2d.py:160-193): zero-insert
// `up`, pad, correlate with the flipped kernel, keep every `down`-th sample; here on NHWC views
// with channel pitches so the result lands directly in a channel slice of a concat buffer, and
// with y = post * act(gain * fir + bias[c]) fused (FusedLeakyReLU, op/fused_act.py:92-96).
// HBM-bound: each thread produces 4 channels of one output pixel with 16-byte loads/stores.
#include "common.hpp"

namespace s2v {

constexpr int FIR_MAX_TAPS = 64;
#ifndef FIR_BLUR_ROWS
#define FIR_BLUR_ROWS 1     // the 4x4 blur as FIR_ROWS-row strips per thread (fir2d_blur4_rows)
#endif

// UP / DOWN / KS > 0: compile-time resampling factors and square filter size (the StyleGAN2 /
// GPEN cases up2 / down2 / blur with the 4x4 [1 3 3 1] kernel): the zero-insertion test and the
// index division become shifts and the tap loops unroll; 0 = runtime values (any combination).
template <bool VEC, int UP = 0, int DOWN = 0, int KS = 0>
__global__ __launch_bounds__(256) void fir2d_kernel(const float *__restrict__ x, int ih, int iw, int c, int xcs,
                                                    const float *__restrict__ k, int kh_, int kw_, int up_, int down_,
                                                    int py0, int px0, float *__restrict__ y, int oh, int ow, int ycs,
                                                    float gain, const float *__restrict__ bias, int act, float alpha,
                                                    float post, long long total) {
    const int up = UP ? UP : up_, down = DOWN ? DOWN : down_;
    const int kh = KS ? KS : kh_, kw = KS ? KS : kw_;
    __shared__ float ks[FIR_MAX_TAPS];
    for (int i = threadIdx.x; i < kh * kw; i += 256) ks[i] = k[kh * kw - 1 - i];   // flipped
    __syncthreads();
    const int cv = VEC ? c / 4 : c;
    // XCD-aware order: the 4x4 FIR's neighbouring rows are read by blocks of the same L2
    const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
    for (long long e = blk * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int cc = (int)(e % cv);
        long long t = e / cv;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int n = (int)(t / oh);
        const float *xb = x + (long long)n * ih * iw * xcs + (VEC ? 4 * cc : cc);
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
        for (int i = 0; i < (KS ? KS : 1); ++i) {
            for (int ii = 0; ii < (KS ? 1 : kh); ++ii) {
                const int ti = KS ? i : ii;
                const int uy = oy * down + ti - py0;
                if (uy < 0 || uy % up) continue;
                const int iy = uy / up;
                if (iy >= ih) continue;
#pragma unroll
                for (int j = 0; j < (KS ? KS : 1); ++j) {
                    for (int jj = 0; jj < (KS ? 1 : kw); ++jj) {
                        const int tj = KS ? j : jj;
                        const int ux = ox * down + tj - px0;
                        if (ux < 0 || ux % up) continue;
                        const int ix = ux / up;
                        if (ix >= iw) continue;
                        const float kv = ks[ti * kw + tj];
                        const float *src = xb + ((long long)iy * iw + ix) * xcs;
                        if (VEC) {
                            const float4 v = *(const float4 *)src;
                            a0 = fmaf(v.x, kv, a0); a1 = fmaf(v.y, kv, a1); a2 = fmaf(v.z, kv, a2); a3 = fmaf(v.w, kv, a3);
                        } else {
                            a0 = fmaf(*src, kv, a0);
                        }
                    }
                }
            }
        }
        float *dst = y + (((long long)n * oh + oy) * ow + ox) * ycs + (VEC ? 4 * cc : cc);
        if (VEC) {
            float4 b = bias ? *(const float4 *)(bias + 4 * cc) : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 o;
            o.x = post * apply_act(fmaf(gain, a0, b.x), act, alpha);
            o.y = post * apply_act(fmaf(gain, a1, b.y), act, alpha);
            o.z = post * apply_act(fmaf(gain, a2, b.z), act, alpha);
            o.w = post * apply_act(fmaf(gain, a3, b.w), act, alpha);
            *(float4 *)dst = o;
        } else {
            *dst = post * apply_act(fmaf(gain, a0, bias ? bias[cc] : 0.f), act, alpha);
        }
    }
}

// The 4x4 blur (up = down = 1, GPEN / StyleGAN2 Blur) on float4 channel quads, FIR_ROWS vertically
// consecutive outputs per thread: the FIR_ROWS + 3 input rows of the strip are each loaded once (4
// float4 taps) and feed every output row they touch, 7 loads per output instead of 16 (the one-output
// form ran the 8 x 512 x 64^2 blur at 3.2 TB/s, bound by its L1 / L2 tap re-reads).  Each output sums its
// taps in the one-output order (filter row, then column), so the results are the same bits.
constexpr int FIR_ROWS = 4;

__global__ __launch_bounds__(256) void fir2d_blur4_rows(const float *__restrict__ x, int ih, int iw, int c, int xcs,
                                                        const float *__restrict__ k, int py0, int px0,
                                                        float *__restrict__ y, int oh, int ow, int ycs, float gain,
                                                        const float *__restrict__ bias, int act, float alpha, float post,
                                                        long long total) {
    __shared__ float ks[16];
    if (threadIdx.x < 16) ks[threadIdx.x] = k[15 - threadIdx.x];   // flipped
    __syncthreads();
    const int cv = c / 4, ohs = (oh + FIR_ROWS - 1) / FIR_ROWS;
    const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
    for (long long e = blk * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int cc = (int)(e % cv);
        long long t = e / cv;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy0 = (int)(t % ohs) * FIR_ROWS;
        const int n = (int)(t / ohs);
        const float *xb = x + (long long)n * ih * iw * xcs + 4 * cc;
        float4 acc[FIR_ROWS];
#pragma unroll
        for (int r = 0; r < FIR_ROWS; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < FIR_ROWS + 3; ++i) {
            const int iy = oy0 + i - py0;
            if (iy < 0 || iy >= ih) continue;
            float4 v[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ix = ox + j - px0;
                ok[j] = ix >= 0 && ix < iw;
                v[j] = ok[j] ? *(const float4 *)(xb + ((long long)iy * iw + ix) * xcs) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int r = 0; r < FIR_ROWS; ++r) {
                const int ti = i - r;
                if (ti < 0 || ti > 3) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!ok[j]) continue;
                    const float kv = ks[ti * 4 + j];
                    acc[r].x = fmaf(v[j].x, kv, acc[r].x);
                    acc[r].y = fmaf(v[j].y, kv, acc[r].y);
                    acc[r].z = fmaf(v[j].z, kv, acc[r].z);
                    acc[r].w = fmaf(v[j].w, kv, acc[r].w);
                }
            }
        }
        const float4 b = bias ? *(const float4 *)(bias + 4 * cc) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < FIR_ROWS; ++r) {
            if (oy0 + r >= oh) break;
            float4 o;
            o.x = post * apply_act(fmaf(gain, acc[r].x, b.x), act, alpha);
            o.y = post * apply_act(fmaf(gain, acc[r].y, b.y), act, alpha);
            o.z = post * apply_act(fmaf(gain, acc[r].z, b.z), act, alpha);
            o.w = post * apply_act(fmaf(gain, acc[r].w, b.w), act, alpha);
            *(float4 *)(y + (((long long)n * oh + oy0 + r) * ow + ox) * ycs + 4 * cc) = o;
        }
    }
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_fir2d(const float *x, int n, int ih, int iw, int c, int xcs, const float *k, int kh, int kw,
                         int up, int down, int pad_y0, int pad_x0, float *y, int oh, int ow, int ycs, float gain,
                         const float *bias, int act, float alpha, float post, s2v_stream_t stream) {
    S2V_REQUIRE(x && k && y && n > 0 && ih > 0 && iw > 0 && c > 0 && oh > 0 && ow > 0, "fir2d: bad args");
    S2V_REQUIRE(xcs >= c && ycs >= c, "fir2d: channel pitch smaller than channel count");
    S2V_REQUIRE(kh > 0 && kw > 0 && kh * kw <= FIR_MAX_TAPS, "fir2d: kernel must have 1..64 taps");
    S2V_REQUIRE(up >= 1 && down >= 1, "fir2d: up/down must be >= 1");
    const bool vec = (c % 4 == 0) && (xcs % 4 == 0) && (ycs % 4 == 0) && ((uintptr_t)x % 16 == 0) &&
                     ((uintptr_t)y % 16 == 0) && (!bias || (uintptr_t)bias % 16 == 0);
    const long long total = (long long)n * oh * ow * (vec ? c / 4 : c);
    long long blocks = (total + 255) / 256;
    if (blocks > 65535LL * 16) blocks = 65535LL * 16;
    hipStream_t st = (hipStream_t)stream;
#define S2V_FIR_ARGS x, ih, iw, c, xcs, k, kh, kw, up, down, pad_y0, pad_x0, y, oh, ow, ycs, gain, bias, act, alpha, post, total
    if (vec && kh == 4 && kw == 4 && up == 1 && down == 1 && FIR_BLUR_ROWS) {
        const long long tot = (long long)n * ((oh + FIR_ROWS - 1) / FIR_ROWS) * ow * (c / 4);
        long long b = (tot + 255) / 256;
        if (b > 65535LL * 16) b = 65535LL * 16;
        fir2d_blur4_rows<<<(unsigned)b, 256, 0, st>>>(x, ih, iw, c, xcs, k, pad_y0, pad_x0, y, oh, ow, ycs, gain, bias,
                                                      act, alpha, post, tot);
    } else if (vec && kh == 4 && kw == 4 && up == 1 && down == 1)
        fir2d_kernel<true, 1, 1, 4><<<(unsigned)blocks, 256, 0, st>>>(S2V_FIR_ARGS);
    else if (vec && kh == 4 && kw == 4 && up == 2 && down == 1)
        fir2d_kernel<true, 2, 1, 4><<<(unsigned)blocks, 256, 0, st>>>(S2V_FIR_ARGS);
    else if (vec && kh == 4 && kw == 4 && up == 1 && down == 2)
        fir2d_kernel<true, 1, 2, 4><<<(unsigned)blocks, 256, 0, st>>>(S2V_FIR_ARGS);
    else if (vec)
        fir2d_kernel<true><<<(unsigned)blocks, 256, 0, st>>>(S2V_FIR_ARGS);
    else
        fir2d_kernel<false><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
            x, ih, iw, c, xcs, k, kh, kw, up, down, pad_y0, pad_x0, y, oh, ow, ycs, gain, bias, act, alpha, post, total);
#undef S2V_FIR_ARGS
    return check_launch("fir2d");
}
