// Resampling, padding, attention, flow warp, mel front end and the GPEN native ops.
// All HBM/latency-bound; one thread per output element with the channel index fastest so that
// NHWC reads/writes coalesce.
#include "common.hpp"

namespace s2v {

// torch upsample_bilinear2d (align_corners=False): src = scale*(dst+0.5)-0.5, clamped at 0
__device__ __forceinline__ void bilin_index(float scale, int dst, int in, int &i0, int &i1, float &l0, float &l1) {
    float src = scale * ((float)dst + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    i0 = (int)src;
    i1 = i0 + ((i0 < in - 1) ? 1 : 0);
    l1 = src - (float)i0;
    l0 = 1.f - l1;
}

__global__ __launch_bounds__(256) void resize_kernel(const float *__restrict__ x, int n, int c, int ih, int iw,
                                                     long long xsn, long long xsc, long long xsy, long long xsx,
                                                     float *__restrict__ y, int oh, int ow, long long ysn,
                                                     long long ysc, long long ysy, long long ysx, float sh, float sw,
                                                     int mode) {
    const long long total = (long long)n * oh * ow * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int cc = (int)(e % c);
        long long t = e / c;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int nn = (int)(t / oh);
        const float *xb = x + nn * xsn + cc * xsc;
        float v;
        if (mode == 0) {
            int y0, y1, x0, x1;
            float ly0, ly1, lx0, lx1;
            bilin_index(sh, oy, ih, y0, y1, ly0, ly1);
            bilin_index(sw, ox, iw, x0, x1, lx0, lx1);
            v = ly0 * (lx0 * xb[y0 * xsy + x0 * xsx] + lx1 * xb[y0 * xsy + x1 * xsx]) +
                ly1 * (lx0 * xb[y1 * xsy + x0 * xsx] + lx1 * xb[y1 * xsy + x1 * xsx]);
        } else {
            const int sy = min((int)floorf((float)oy * sh), ih - 1);
            const int sx = min((int)floorf((float)ox * sw), iw - 1);
            v = xb[sy * xsy + sx * xsx];
        }
        y[nn * ysn + cc * ysc + oy * ysy + ox * ysx] = v;
    }
}

// NHWC fast path: channel-contiguous views (xsc == ysc == 1), c % 4 == 0, 16-byte aligned:
// one float4 of channels per thread; one output row per blockIdx.y (grid-stride), 32-bit index
// math only (the per-element 64-bit divisions of a flat index dominated this HBM-bound kernel).
__global__ __launch_bounds__(256) void resize_nhwc4_kernel(const float *__restrict__ x, int n, int c4, int ih,
                                                           int iw, long long xsn, int xsy, int xsx,
                                                           float *__restrict__ y, int oh, int ow, long long ysn,
                                                           int ysy, int ysx, float sh, float sw, int mode) {
    const int row_elems = ow * c4;
    for (int r = blockIdx.y; r < n * oh; r += gridDim.y) {
        const int nn = r / oh, oy = r - nn * oh;
        const float *xb = x + nn * xsn;
        float *yr = y + nn * ysn + (long long)oy * ysy;
        int y0 = 0, y1 = 0, sy = 0;
        float ly0 = 1.f, ly1 = 0.f;
        if (mode == 0) bilin_index(sh, oy, ih, y0, y1, ly0, ly1);
        else sy = min((int)floorf((float)oy * sh), ih - 1);
        for (int e = blockIdx.x * 256 + threadIdx.x; e < row_elems; e += gridDim.x * 256) {
            const int ox = e / c4, cq = e - ox * c4;
            float4 v;
            if (mode == 0) {
                int x0, x1;
                float lx0, lx1;
                bilin_index(sw, ox, iw, x0, x1, lx0, lx1);
                const float *b0 = xb + (long long)y0 * xsy + 4 * cq, *b1 = xb + (long long)y1 * xsy + 4 * cq;
                const float4 a = *(const float4 *)(b0 + x0 * xsx), b = *(const float4 *)(b0 + x1 * xsx);
                const float4 cc = *(const float4 *)(b1 + x0 * xsx), d = *(const float4 *)(b1 + x1 * xsx);
                v.x = ly0 * (lx0 * a.x + lx1 * b.x) + ly1 * (lx0 * cc.x + lx1 * d.x);
                v.y = ly0 * (lx0 * a.y + lx1 * b.y) + ly1 * (lx0 * cc.y + lx1 * d.y);
                v.z = ly0 * (lx0 * a.z + lx1 * b.z) + ly1 * (lx0 * cc.z + lx1 * d.z);
                v.w = ly0 * (lx0 * a.w + lx1 * b.w) + ly1 * (lx0 * cc.w + lx1 * d.w);
            } else {
                const int sx = min((int)floorf((float)ox * sw), iw - 1);
                v = *(const float4 *)(xb + (long long)sy * xsy + sx * xsx + 4 * cq);
            }
            *(float4 *)(yr + ox * ysx + 4 * cq) = v;
        }
    }
}

// Exact x2 bilinear upsample (align_corners=False, source scale 0.5) of a float4-channel NHWC
// view: one thread = one channel quad of one source pixel -> the 2x2 output quad it centres.  The
// 3x3 source neighbourhood (rows / columns clamped to the image) is loaded once, 9 float4 loads for
// 4 outputs, and each output takes its 4 taps from those registers by the same index / weight rule
// (bilin_index) and expression as resize_nhwc4_kernel, so the result is the generic kernel's bit for
// bit.  (Loading each output's 4 taps separately, 16 loads with the centre pixel requested 4 times,
// returned wrong data in the upper quarter-wave under two concurrently replayed graphs on MI355X:
// tools/dbg_lanes4.py)
__device__ __forceinline__ float4 sel3(int k, const float4 &a, const float4 &b, const float4 &c) {
    return k == 0 ? a : (k == 1 ? b : c);
}

__global__ __launch_bounds__(256) void up2_bilinear_nhwc4_kernel(const float *__restrict__ x, int n, int c4, int ih,
                                                                 int iw, long long xsn, int xsy, int xsx,
                                                                 float *__restrict__ y, long long ysn, int ysy,
                                                                 int ysx) {
    const int per_row = iw * c4;
    for (int r = blockIdx.y; r < n * ih; r += gridDim.y) {
        const int nn = r / ih, iy = r - nn * ih;
        const float *xb = x + nn * xsn;
        int ya0, ya1, yb0, yb1;
        float la0, la1, lb0, lb1;
        bilin_index(0.5f, 2 * iy, ih, ya0, ya1, la0, la1);
        bilin_index(0.5f, 2 * iy + 1, ih, yb0, yb1, lb0, lb1);
        const int rm = iy > 0 ? iy - 1 : 0, rp = iy < ih - 1 ? iy + 1 : iy;
        float *y0r = y + nn * ysn + (long long)(2 * iy) * ysy;
        float *y1r = y0r + ysy;
        for (int e = blockIdx.x * 256 + threadIdx.x; e < per_row; e += gridDim.x * 256) {
            const int ix = e / c4, cq = e - ix * c4;
            int xa0, xa1, xb0, xb1;
            float ma0, ma1, mb0, mb1;
            bilin_index(0.5f, 2 * ix, iw, xa0, xa1, ma0, ma1);
            bilin_index(0.5f, 2 * ix + 1, iw, xb0, xb1, mb0, mb1);
            const int cm = ix > 0 ? ix - 1 : 0, cp = ix < iw - 1 ? ix + 1 : ix;
            const float *q0 = xb + (long long)rm * xsy + 4 * cq, *q1 = xb + (long long)iy * xsy + 4 * cq,
                        *q2 = xb + (long long)rp * xsy + 4 * cq;
            const float4 n00 = *(const float4 *)(q0 + cm * xsx), n01 = *(const float4 *)(q0 + ix * xsx),
                         n02 = *(const float4 *)(q0 + cp * xsx);
            const float4 n10 = *(const float4 *)(q1 + cm * xsx), n11 = *(const float4 *)(q1 + ix * xsx),
                         n12 = *(const float4 *)(q1 + cp * xsx);
            const float4 n20 = *(const float4 *)(q2 + cm * xsx), n21 = *(const float4 *)(q2 + ix * xsx),
                         n22 = *(const float4 *)(q2 + cp * xsx);
            // neighbourhood value of a source (row, column) index pair (every tap lies in [i - 1, i + 1])
            auto tap = [&](int yy, int xx) {
                const int a = yy - iy + 1, b = xx - ix + 1;
                return sel3(a, sel3(b, n00, n01, n02), sel3(b, n10, n11, n12), sel3(b, n20, n21, n22));
            };
            auto lerp4 = [&](int y0, int y1, int x0, int x1, float ly0, float ly1, float lx0, float lx1) {
                const float4 a = tap(y0, x0), b = tap(y0, x1), c = tap(y1, x0), d = tap(y1, x1);
                float4 v;
                v.x = ly0 * (lx0 * a.x + lx1 * b.x) + ly1 * (lx0 * c.x + lx1 * d.x);
                v.y = ly0 * (lx0 * a.y + lx1 * b.y) + ly1 * (lx0 * c.y + lx1 * d.y);
                v.z = ly0 * (lx0 * a.z + lx1 * b.z) + ly1 * (lx0 * c.z + lx1 * d.z);
                v.w = ly0 * (lx0 * a.w + lx1 * b.w) + ly1 * (lx0 * c.w + lx1 * d.w);
                return v;
            };
            *(float4 *)(y0r + (2 * ix) * ysx + 4 * cq) = lerp4(ya0, ya1, xa0, xa1, la0, la1, ma0, ma1);
            *(float4 *)(y0r + (2 * ix + 1) * ysx + 4 * cq) = lerp4(ya0, ya1, xb0, xb1, la0, la1, mb0, mb1);
            *(float4 *)(y1r + (2 * ix) * ysx + 4 * cq) = lerp4(yb0, yb1, xa0, xa1, lb0, lb1, ma0, ma1);
            *(float4 *)(y1r + (2 * ix + 1) * ysx + 4 * cq) = lerp4(yb0, yb1, xb0, xb1, lb0, lb1, mb0, mb1);
        }
    }
}

__global__ __launch_bounds__(256) void pad_reflect_kernel(const float *__restrict__ x, int n, int h, int w, int c,
                                                          int xcs, int pt, int pl, int oh, int ow,
                                                          float *__restrict__ y, int ycs) {
    const long long total = (long long)n * oh * ow * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int cc = (int)(e % c);
        long long t = e / c;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int nn = (int)(t / oh);
        const int iy = reflect_idx(oy - pt, h), ix = reflect_idx(ox - pl, w);
        y[(((long long)nn * oh + oy) * ow + ox) * ycs + cc] = x[(((long long)nn * h + iy) * w + ix) * xcs + cc];
    }
}

// Row-tap packing for small-channel wide-kernel convs (s2v_row_pack): y[n, h, w, dx * c + ci] =
// x[n, h, w + dx - pw, ci] (zero outside the row), channels [kw * c, ycs) zero.  A kh x kw conv over
// c <= 8 channels then runs as a kh x 1 conv over ycs (a multiple of 32) channels on the buffer-load
// tiles instead of the per-element gather (LNet first_inp / first_ref, DNet input_layer / e_first: 7x7
// over 3 or 6 channels).  One output channel quad per thread, one float4 store.
__global__ __launch_bounds__(256) void row_pack_kernel(const float *__restrict__ x, int n, int h, int w, int c,
                                                       int xcs, int kw, int pw, float *__restrict__ y, int ycs) {
    const int q4 = ycs >> 2;
    const long long total = (long long)n * h * w * q4;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int q = (int)(e % q4);
        const long long pix = e / q4;
        const int ox = (int)(pix % w);
        const float *xr = x + (pix - ox) * xcs;            // pixel (n, h, 0) of this row
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ch = 4 * q + i, dx = ch / c, ci = ch - dx * c;
            const int ix = ox + dx - pw;
            v[i] = (dx < kw && (unsigned)ix < (unsigned)w) ? xr[(long long)ix * xcs + ci] : 0.f;
        }
        *(float4 *)(y + pix * ycs + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// float4 form (c, pitches % 4 == 0, 16-byte aligned): one channel quad per thread
__global__ __launch_bounds__(256) void pad_reflect4_kernel(const float *__restrict__ x, int n, int h, int w, int c4,
                                                           int xcs, int pt, int pl, int oh, int ow,
                                                           float *__restrict__ y, int ycs) {
    const long long total = (long long)n * oh * ow * c4;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int cq = (int)(e % c4);
        long long t = e / c4;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int nn = (int)(t / oh);
        const int iy = reflect_idx(oy - pt, h), ix = reflect_idx(ox - pl, w);
        *(float4 *)(y + (((long long)nn * oh + oy) * ow + ox) * ycs + 4 * cq) =
            *(const float4 *)(x + (((long long)nn * h + iy) * w + ix) * xcs + 4 * cq);
    }
}

// ------------------------------------------------------------------ attention
// one block per (b, head); K padded to 65 floats per row (conflict-free column reads)
__global__ __launch_bounds__(256) void attention_kernel(const float *__restrict__ q, const float *__restrict__ k,
                                                        const float *__restrict__ v, int heads, int T, int ldq, int ldk,
                                                        int ldv, long long bsq, long long bsk, long long bsv,
                                                        float scale, float *__restrict__ o, int ldo, long long bso) {
    extern __shared__ float sm[];
    float *Ks = sm;                    // [T][65]
    float *Vs = Ks + T * 65;           // [T][64]
    float *scr = Vs + T * 64;          // per wave: q[64] + p[T]
    const int b = blockIdx.x / heads, hd = blockIdx.x - (blockIdx.x / heads) * heads;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float *kb = k + b * bsk + hd * 64;
    const float *vb = v + b * bsv + hd * 64;
    for (int e = threadIdx.x; e < T * 64; e += 256) {
        const int j = e >> 6, d = e & 63;
        Ks[j * 65 + d] = kb[(long long)j * ldk + d];
        Vs[j * 64 + d] = vb[(long long)j * ldv + d];
    }
    __syncthreads();
    float *qs = scr + wv * (64 + T);
    float *ps = qs + 64;
    const float *qb = q + b * bsq + hd * 64;
    float *ob = o + b * bso + hd * 64;
    // query rows interleave over the blocks of blockIdx.y (row groups) and the 4 waves
    for (int i = blockIdx.y * 4 + wv; i < T; i += 4 * gridDim.y) {
        qs[lane] = qb[(long long)i * ldq + lane];
        __builtin_amdgcn_wave_barrier();
        float sv[4];
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = lane + 64 * t;
            float s = -INFINITY;
            if (j < T) {
                float acc = 0.f;
                const float *kr = Ks + j * 65;
#pragma unroll 16
                for (int d = 0; d < 64; ++d) acc = fmaf(qs[d], kr[d], acc);
                s = acc * scale;
            }
            sv[t] = s;
            mx = fmaxf(mx, s);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = lane + 64 * t;
            const float pe = (j < T) ? expf(sv[t] - mx) : 0.f;
            sv[t] = pe;
            sum += pe;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
        const float inv = 1.f / sum;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = lane + 64 * t;
            if (j < T) ps[j] = sv[t] * inv;
        }
        __builtin_amdgcn_wave_barrier();
        float acc = 0.f;
        for (int j = 0; j < T; ++j) acc = fmaf(ps[j], Vs[j * 64 + lane], acc);
        ob[(long long)i * ldo + lane] = acc;
        __builtin_amdgcn_wave_barrier();
    }
}

// ------------------------------------------------------------------ flow warp
// flow_util.py: grid (align_corners=True convention) + 2*flow/(W-1, H-1) -> bilinear resize
// (align_corners=False) -> grid_sample(bilinear, zeros, align_corners=False)
__device__ __forceinline__ void deform_at(const float *flow, int fh, int fw, int fcs, int fy, int fx, float &gx,
                                          float &gy) {
    const float *f = flow + ((long long)fy * fw + fx) * fcs;
    gx = (2.f * ((float)fx / (float)(fw - 1)) - 1.f) + 2.f * (f[0] / (float)(fw - 1));
    gy = (2.f * ((float)fy / (float)(fh - 1)) - 1.f) + 2.f * (f[1] / (float)(fh - 1));
}

// Blocks walk the pixels XCD-contiguously: block b runs on XCD b % 8, so logical block L is chosen
// such that each XCD takes one contiguous eighth of the (image, row) range.  The bilinear taps of
// neighbouring output rows share source lines; with the plain order every XCD's L2 fetched those
// lines for its own interleaved rows (r05: 4.5-5.9x the algorithmic bytes in FETCH_SIZE).
// CAT: y[p, 0:c) = src[p] and y[p, c:2c) = the warp (EditingNet's torch.cat([input_image, warp_image], 1), DNet.py:114-115, in
// one pass: whole 2c-float pixels written, no separate NCHW -> NHWC copy).
template <bool CAT>
__global__ __launch_bounds__(256) void flow_warp_kernel(const float *__restrict__ flow, int n, int fh, int fw,
                                                        int fcs, const float *__restrict__ src, int c, int h, int w,
                                                        long long ssn, long long ssc, long long ssy, long long ssx,
                                                        float *__restrict__ y, int ycs) {
    const long long total = (long long)n * h * w;
    const int nb = (int)gridDim.x, per = nb >> 3, rem = nb & 7, xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
    const int L = xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
    const long long e = L * 256LL + threadIdx.x;
    if (e >= total) return;
    const int ox = (int)(e % w);
    const int oy = (int)((e / w) % h);
    const int nn = (int)(e / ((long long)w * h));
    const float *fb = flow + (long long)nn * fh * fw * fcs;
    float gx, gy;
    if (fh == h && fw == w) {
        deform_at(fb, fh, fw, fcs, oy, ox, gx, gy);
    } else {
        int y0, y1, x0, x1;
        float ly0, ly1, lx0, lx1;
        bilin_index((float)fh / (float)h, oy, fh, y0, y1, ly0, ly1);
        bilin_index((float)fw / (float)w, ox, fw, x0, x1, lx0, lx1);
        float ax, ay, bx, by, cx, cy, dx, dy;
        deform_at(fb, fh, fw, fcs, y0, x0, ax, ay);
        deform_at(fb, fh, fw, fcs, y0, x1, bx, by);
        deform_at(fb, fh, fw, fcs, y1, x0, cx, cy);
        deform_at(fb, fh, fw, fcs, y1, x1, dx, dy);
        gx = ly0 * (lx0 * ax + lx1 * bx) + ly1 * (lx0 * cx + lx1 * dx);
        gy = ly0 * (lx0 * ay + lx1 * by) + ly1 * (lx0 * cy + lx1 * dy);
    }
    const float ix = ((gx + 1.f) * (float)w - 1.f) * 0.5f;
    const float iy = ((gy + 1.f) * (float)h - 1.f) * 0.5f;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int ix0 = (int)fx0, iy0 = (int)fy0, ix1 = ix0 + 1, iy1 = iy0 + 1;
    const float wnw = ((float)ix1 - ix) * ((float)iy1 - iy);
    const float wne = (ix - (float)ix0) * ((float)iy1 - iy);
    const float wsw = ((float)ix1 - ix) * (iy - (float)iy0);
    const float wse = (ix - (float)ix0) * (iy - (float)iy0);
    const bool vnw = ix0 >= 0 && ix0 < w && iy0 >= 0 && iy0 < h;
    const bool vne = ix1 >= 0 && ix1 < w && iy0 >= 0 && iy0 < h;
    const bool vsw = ix0 >= 0 && ix0 < w && iy1 >= 0 && iy1 < h;
    const bool vse = ix1 >= 0 && ix1 < w && iy1 >= 0 && iy1 < h;
    const float *sb = src + nn * ssn;
    float *yo = y + e * ycs;
    if (CAT) {
        for (int cc = 0; cc < c; ++cc) yo[cc] = sb[cc * ssc + oy * ssy + ox * ssx];
        yo += c;
    }
    for (int cc = 0; cc < c; ++cc) {
        const float *sc = sb + cc * ssc;
        float acc = 0.f;
        if (vnw) acc += sc[iy0 * ssy + ix0 * ssx] * wnw;
        if (vne) acc += sc[iy0 * ssy + ix1 * ssx] * wne;
        if (vsw) acc += sc[iy1 * ssy + ix0 * ssx] * wsw;
        if (vse) acc += sc[iy1 * ssy + ix1 * ssx] * wse;
        yo[cc] = acc;
    }
}

// ------------------------------------------------------------------ mel spectrogram
// tables: mel basis [80][401] | cos[800] | sin[800] | periodic Hann window[800]
constexpr int kNfft = 800, kHop = 200, kBins = 401, kMels = 80;

__global__ __launch_bounds__(256) void mel_kernel(const float *__restrict__ wav, long long ns,
                                                  const float *__restrict__ tables, int pad_reflect,
                                                  float *__restrict__ out, long long frames) {
    __shared__ float xs[kNfft];
    __shared__ float cs[kNfft], sn[kNfft];
    __shared__ float mag[kBins];
    const long long t = blockIdx.x;
    const float *basis = tables;
    const float *ct = tables + kMels * kBins;
    const float *st = ct + kNfft;
    const float *win = st + kNfft;
    for (int i = threadIdx.x; i < kNfft; i += 256) {
        cs[i] = ct[i];
        sn[i] = st[i];
        // padded index -> sample index (center=True: pad n_fft/2 both sides)
        long long j = t * kHop + i - kNfft / 2;
        float v = 0.f;
        if (pad_reflect) {
            if (j < 0) j = -j;
            if (j >= ns) j = 2 * ns - 2 - j;
        }
        if (j >= 0 && j < ns) {
            // preemphasis y[j] = x[j] - 0.97 x[j-1]  (lfilter([1,-k],[1]), zero initial state)
            v = wav[j] - (j > 0 ? 0.97f * wav[j - 1] : 0.f);
        }
        xs[i] = v * win[i];
    }
    __syncthreads();
    for (int f = threadIdx.x; f < kBins; f += 256) {
        float re = 0.f, im = 0.f;
        int idx = 0;
        for (int i = 0; i < kNfft; ++i) {
            re = fmaf(xs[i], cs[idx], re);
            im = fmaf(xs[i], sn[idx], im);
            idx += f;
            if (idx >= kNfft) idx -= kNfft;
        }
        mag[f] = sqrtf(re * re + im * im);
    }
    __syncthreads();
    if (threadIdx.x < kMels) {
        const float *br = basis + threadIdx.x * kBins;
        float acc = 0.f;
        for (int f = 0; f < kBins; ++f) acc = fmaf(br[f], mag[f], acc);
        float db = 20.f * log10f(fmaxf(1e-5f, acc)) - 20.f;
        float v = 8.f * ((db + 100.f) / 100.f) - 4.f;
        v = fminf(fmaxf(v, -4.f), 4.f);
        out[threadIdx.x * frames + t] = v;
    }
}

__global__ __launch_bounds__(256) void mel_chunks_kernel(const float *__restrict__ mel, long long frames,
                                                         const int *__restrict__ starts, int nchunks, int step,
                                                         float *__restrict__ out) {
    const long long total = (long long)nchunks * kMels * step;
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= total) return;
    const int tt = (int)(e % step);
    const int m = (int)((e / step) % kMels);
    const int i = (int)(e / ((long long)step * kMels));
    out[e] = mel[(long long)m * frames + starts[i] + tt];
}

// ------------------------------------------------------------------ GPEN ops
// Element type T of the reference's AT_DISPATCH_FLOATING_TYPES_AND_HALF (fused_bias_act_kernel.cu:79,
// upfirdn2d_kernel.cu:225): float, double, half (_Float16).  Arithmetic runs in OpT: double for
// double, fp32 for float and half (the half result is rounded once, on the store).
template <typename T> struct OpT { using type = float; };
template <> struct OpT<double> { using type = double; };
template <typename T> struct alignas(4 * sizeof(T)) Vec4 { T v[4]; };

template <typename T, typename A>
__device__ __forceinline__ A bias_act(A v, A r, int mode, A alpha) {
    switch (mode) {
        case 30: return v > A(0) ? v : v * alpha;
        case 31: return r > A(0) ? v : v * alpha;
        case 12:
        case 32: return A(0);
        default: return v;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void fused_bias_act_kernel(const T *__restrict__ x, const T *__restrict__ b,
                                                             const T *__restrict__ ref, T *__restrict__ y,
                                                             long long size, int c, long long step_b, int act, int grad,
                                                             typename OpT<T>::type alpha, typename OpT<T>::type scale) {
    using A = typename OpT<T>::type;
    const int mode = act * 10 + grad;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < size; i += (long long)gridDim.x * 256) {
        A v = (A)x[i];
        if (b) v += (A)b[(i / step_b) % c];
        const A r = ref ? (A)ref[i] : A(0);
        y[i] = (T)(bias_act<T, A>(v, r, mode, alpha) * scale);
    }
}

// Row form (step_b % 4 == 0, 4-element aligned; the GPEN call on [N, C, H, W] has step_b = H*W): a
// block row walks one (n, c) plane with 4-element vector loads / stores (16 B for float, 8 B for
// half, 32 B for double), the bias channel fixed per row — no per-element 64-bit index division.
template <typename T>
__global__ __launch_bounds__(256) void fused_bias_act_rows(const T *__restrict__ x, const T *__restrict__ b,
                                                           const T *__restrict__ ref, T *__restrict__ y,
                                                           long long rows, int c, long long step4, int act, int grad,
                                                           typename OpT<T>::type alpha, typename OpT<T>::type scale) {
    using A = typename OpT<T>::type;
    const int mode = act * 10 + grad;
    for (long long r = blockIdx.y; r < rows; r += gridDim.y) {
        const A bv = b ? (A)b[r % c] : A(0);
        const Vec4<T> *xr = (const Vec4<T> *)x + r * step4;
        const Vec4<T> *rr = ref ? (const Vec4<T> *)ref + r * step4 : nullptr;
        Vec4<T> *yr = (Vec4<T> *)y + r * step4;
        for (long long i = blockIdx.x * 256LL + threadIdx.x; i < step4; i += (long long)gridDim.x * 256) {
            const Vec4<T> v = xr[i];
            Vec4<T> q{};
            if (mode == 31) q = rr[i];
            Vec4<T> o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o.v[j] = (T)(bias_act<T, A>((A)v.v[j] + bv, (A)q.v[j], mode, alpha) * scale);
            yr[i] = o;
        }
    }
}

// out = down( FIR( zero-pad( zero-insert-up(x) ), flip(k) ) ) per plane, [major][H][W][minor].
// UP / DN / KS > 0 fix the factors and the square filter at compile time (the GPEN Upsample /
// Downsample / Blur forms with the 4x4 kernel): shifts instead of divisions, unrolled taps.
template <typename T, int UP = 0, int DN = 0, int KS = 0>
__global__ __launch_bounds__(256) void upfirdn2d_kernel(const T *__restrict__ x, int major, int ih, int iw,
                                                        int minor, const T *__restrict__ k, int kh_, int kw_,
                                                        int upx_, int upy_, int dnx_, int dny_, int px0, int py0,
                                                        T *__restrict__ y, int oh, int ow) {
    using A = typename OpT<T>::type;
    const int upx = UP ? UP : upx_, upy = UP ? UP : upy_, dnx = DN ? DN : dnx_, dny = DN ? DN : dny_;
    const int kh = KS ? KS : kh_, kw = KS ? KS : kw_;
    const long long total = (long long)major * oh * ow * minor;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int mi = (int)(e % minor);
        long long t = e / minor;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int mj = (int)(t / oh);
        const T *xb = x + (long long)mj * ih * iw * minor + mi;
        A acc = A(0);
#pragma unroll
        for (int i = 0; i < (KS ? KS : 1); ++i) {
            for (int ii = 0; ii < (KS ? 1 : kh); ++ii) {
                const int ti = KS ? i : ii;
                const int uy = oy * dny + ti - py0;   // row in the zero-inserted image
                if (uy < 0 || uy % upy) continue;
                const int iy = uy / upy;
                if (iy >= ih) continue;
#pragma unroll
                for (int j = 0; j < (KS ? KS : 1); ++j) {
                    for (int jj = 0; jj < (KS ? 1 : kw); ++jj) {
                        const int tj = KS ? j : jj;
                        const int ux = ox * dnx + tj - px0;
                        if (ux < 0 || ux % upx) continue;
                        const int ix = ux / upx;
                        if (ix >= iw) continue;
                        acc = fma((A)xb[((long long)iy * iw + ix) * minor], (A)k[(kh - 1 - ti) * kw + (kw - 1 - tj)], acc);
                    }
                }
            }
        }
        y[e] = (T)acc;
    }
}

// Plane form (minor == 1, the NCHW tensors GPEN passes as [N*C, H, W, 1]) with the 4x4 filter:
// a block owns a 16 x 64 output tile of one plane, stages the input rows it touches in LDS with
// coalesced row loads (zeros outside the image), and each thread computes 4 adjacent outputs.
template <typename T, int UP, int DN>
__global__ __launch_bounds__(256) void upfirdn2d_plane4(const T *__restrict__ x, int ih, int iw,
                                                        const T *__restrict__ k, int px0, int py0,
                                                        T *__restrict__ y, int oh, int ow, int tiles_x,
                                                        int tiles_y) {
    using A = typename OpT<T>::type;
    constexpr int TY = 16, TX = 64;
    // input rows / cols a tile touches: zero-inserted coordinates u = o*DN + t - p, t in [0, 4)
    constexpr int RH = ((TY - 1) * DN + 3) / UP + 2, RW = ((TX - 1) * DN + 3) / UP + 2;
    __shared__ A tile[RH][RW + 1];
    __shared__ A ks[16];
    if (threadIdx.x < 16) ks[threadIdx.x] = (A)k[15 - threadIdx.x];          // flipped
    int t = blockIdx.x;
    const int txi = t % tiles_x;
    t /= tiles_x;
    const int tyi = t % tiles_y;
    const long long plane = t / tiles_y;
    const int oy0 = tyi * TY, ox0 = txi * TX;
    // first input row / col of the tile (floor division of the first zero-inserted coordinate)
    const int uy0 = oy0 * DN - py0, ux0 = ox0 * DN - px0;
    const int iy0 = uy0 >= 0 ? uy0 / UP : -((-uy0 + UP - 1) / UP);
    const int ix0 = ux0 >= 0 ? ux0 / UP : -((-ux0 + UP - 1) / UP);
    const T *xp = x + plane * ih * iw;
    for (int e = threadIdx.x; e < RH * RW; e += 256) {
        const int r = e / RW, cidx = e - r * RW;
        const int gy = iy0 + r, gx = ix0 + cidx;
        tile[r][cidx] = ((unsigned)gy < (unsigned)ih && (unsigned)gx < (unsigned)iw) ? (A)xp[(long long)gy * iw + gx] : A(0);
    }
    __syncthreads();
    const int ry = threadIdx.x >> 4, rx = (threadIdx.x & 15) * 4;
    const int oy = oy0 + ry;
    if (oy >= oh) return;
    A acc[4] = {A(0), A(0), A(0), A(0)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int uy = oy * DN + i - py0;
        if (UP > 1 && (uy % UP + UP) % UP) continue;
        const int ly = (uy >= 0 ? uy / UP : -((-uy + UP - 1) / UP)) - iy0;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ux = (ox0 + rx + p) * DN + j - px0;
                if (UP > 1 && (ux % UP + UP) % UP) continue;
                const int lx = (ux >= 0 ? ux / UP : -((-ux + UP - 1) / UP)) - ix0;
                acc[p] = fma(tile[ly][lx], ks[i * 4 + j], acc[p]);
            }
        }
    }
    T *yp = y + plane * oh * ow + (long long)oy * ow;
#pragma unroll
    for (int p = 0; p < 4; ++p)
        if (ox0 + rx + p < ow) yp[ox0 + rx + p] = (T)acc[p];
}

// ------------------------------------------------------------------ noise
// Counter-based N(0,1) (splitmix64 + Box-Muller): StyleConv noise injection
// (base_blocks.py:528-531 draws normal_() per call; only its distribution is reproducible).
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void gaussian_kernel(float *__restrict__ y, long long n, unsigned long long seed,
                                                       unsigned long long offset, const unsigned long long *ctr,
                                                       int shift) {
    if (ctr) offset += *ctr << shift;          // device-side draw counter: fresh noise per graph replay
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const unsigned long long z = splitmix64(seed ^ splitmix64(offset + (unsigned long long)i));
        const float u1 = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
        const float u2 = (float)((z >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
        y[i] = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
    }
}

// ------------------------------------------------------------------ pipeline glue
// DNet fake image -> uint8 reference frame (facing.py:190-191: uint8((clamp(x,-1,1)+1)/2*255),
// truncation like numpy's float->uint8 cast) and the ENet inputs built from it (inference.py:
// 393-399: lower half of the original crop zeroed, [masked | ref] / 255; gt = ref).
__global__ __launch_bounds__(256) void lipsync_inputs_kernel(const float *__restrict__ src, const float *__restrict__ fake,
                                                            int n, int h, int w, unsigned char *ref_u8,
                                                            float *__restrict__ face6, float *__restrict__ gt) {
    const long long plane = (long long)h * w;
    const long long total = (long long)n * 3 * plane;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long p = e % plane;
        const int c = (int)((e / plane) % 3);
        const int b = (int)(e / (3 * plane));
        const int y = (int)(p / w);
        unsigned char q;
        if (fake) {
            const float f = fminf(fmaxf(fake[e], -1.f), 1.f);
            q = (unsigned char)((f + 1.f) * 0.5f * 255.f);
            ref_u8[e] = q;
        } else {
            q = ref_u8[e];                     // references given (enhanced by a Step-5 hook)
        }
        const float r = (float)q / 255.f;
        // original crop as uint8 then /255 (the reference reads frames as uint8)
        float s = fminf(fmaxf(src[e], -1.f), 1.f);
        const float o = (float)(unsigned char)((s + 1.f) * 0.5f * 255.f) / 255.f;
        const long long base6 = (long long)b * 6 * plane;
        face6[base6 + (long long)c * plane + p] = (y >= h / 2) ? 0.f : o;
        face6[base6 + (long long)(c + 3) * plane + p] = r;
        gt[e] = r;
    }
}

// ENet output -> uint8 frames (inference.py:267 clamp(0,1), :288 * 255, uint8 cast truncates)
__global__ __launch_bounds__(256) void to_u8_kernel(const float *__restrict__ x, long long n, float lo, float hi,
                                                    float scale, float offset, unsigned char *__restrict__ y) {
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
        y[e] = (unsigned char)((fminf(fmaxf(x[e], lo), hi) + offset) * scale);
}

// y = post * act(x * a + mul * + add + bias[c]) over NHWC views (SFT, skip adds, noise halves)
__global__ __launch_bounds__(256) void eltwise_kernel(const float *__restrict__ x, int xcs, const float *__restrict__ mul,
                                                      int mcs, const float *__restrict__ add, int acs,
                                                      const float *__restrict__ bias, long long pixels, int c, float a,
                                                      int act, float alpha, float post, float *__restrict__ y, int ycs) {
    const long long total = pixels * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long p = e / c;
        const int cc = (int)(e - p * c);
        float v = x[p * xcs + cc] * a;
        if (mul) v *= mul[p * mcs + cc];
        if (add) v += add[p * acs + cc];
        if (bias) v += bias[cc];
        y[p * ycs + cc] = apply_act(v, act, alpha) * post;
    }
}

// float4 form (c, pitches % 4 == 0, 16-byte aligned views, < 2^31 quads): one channel quad per
// thread, 32-bit index math
__global__ __launch_bounds__(256) void eltwise4_kernel(const float *__restrict__ x, int xcs, const float *__restrict__ mul,
                                                       int mcs, const float *__restrict__ add, int acs,
                                                       const float *__restrict__ bias, unsigned quads, unsigned c4,
                                                       float a, int act, float alpha, float post,
                                                       float *__restrict__ y, int ycs) {
    for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < quads; e += gridDim.x * 256u) {
        const unsigned p = e / c4, q = e - p * c4;
        const long long pp = (long long)p;
        float4 v = *(const float4 *)(x + pp * xcs + 4 * q);
        v.x *= a; v.y *= a; v.z *= a; v.w *= a;
        if (mul) {
            const float4 m = *(const float4 *)(mul + pp * mcs + 4 * q);
            v.x *= m.x; v.y *= m.y; v.z *= m.z; v.w *= m.w;
        }
        if (add) {
            const float4 d = *(const float4 *)(add + pp * acs + 4 * q);
            v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
        }
        if (bias) {
            const float4 b = *(const float4 *)(bias + 4 * q);
            v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
        }
        v.x = apply_act(v.x, act, alpha) * post; v.y = apply_act(v.y, act, alpha) * post;
        v.z = apply_act(v.z, act, alpha) * post; v.w = apply_act(v.w, act, alpha) * post;
        *(float4 *)(y + pp * ycs + 4 * q) = v;
    }
}

__global__ __launch_bounds__(256) void fill_kernel(float *__restrict__ y, long long n, float v) {
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) y[e] = v;
}

// max |x| of an NHWC view (the split precisions' per-layer activation range, conv x_scale).  A block
// walks pixel rows (TPR = 2^tpr_shift threads per row, 16-byte channel quads when VEC), keeps a
// running max of the fp32 bits (non-negative floats order as unsigned ints; a NaN has the largest
// bits, so it propagates), reduces it over the wave and the block, and folds it with one atomic max.
// No per-element division: the row walk is a grid-stride loop over pixels.
template <bool VEC>
__global__ __launch_bounds__(256) void amax_kernel(const float *__restrict__ x, long long pixels, int c, int xcs,
                                                   int tpr_shift, unsigned *__restrict__ out) {
    __shared__ unsigned red[4];
    const int tid = threadIdx.x;
    const int tpr = 1 << tpr_shift, lane_r = tid & (tpr - 1);
    const int rpb = 256 >> tpr_shift;
    unsigned mb = 0;
    for (long long p = (long long)blockIdx.x * rpb + (tid >> tpr_shift); p < pixels; p += (long long)gridDim.x * rpb) {
        const float *row = x + p * xcs;
        if (VEC) {
            for (int q = lane_r; q < (c >> 2); q += tpr) {
                const float4 v = *(const float4 *)(row + 4 * q);
                const unsigned a = max(__float_as_uint(fabsf(v.x)), __float_as_uint(fabsf(v.y)));
                const unsigned b = max(__float_as_uint(fabsf(v.z)), __float_as_uint(fabsf(v.w)));
                mb = max(mb, max(a, b));
            }
        } else {
            for (int j = lane_r; j < c; j += tpr) mb = max(mb, __float_as_uint(fabsf(row[j])));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
    if ((tid & 63) == 0) red[tid >> 6] = mb;
    __syncthreads();
    if (tid == 0) {
        mb = max(max(red[0], red[1]), max(red[2], red[3]));
        if (mb) atomicMax(out, mb);
    }
}

// Per-sample StyleGAN2 weights (base_blocks.py:487-495 / stylegan2_clean_arch.py:66-80 /
// gpen_model.py:245-256): out[b][o][k] = wt[o][k] * s[b][k % cin] * d[b][o] for packed
// [npad][kpad] weights (k = tap * cin + c); padding rows / columns stay zero.  The conv then runs
// in batch mode with these weights, free of prologue / epilogue scaling.
__global__ __launch_bounds__(256) void modulate_weights_kernel(const float *__restrict__ wt, int npad, int kpad,
                                                               int K, int cin, int cout, const float *__restrict__ s,
                                                               int s_ns, const float *__restrict__ d, int d_ns,
                                                               int batch, float *__restrict__ out) {
    const long long per = (long long)npad * kpad;
    const long long total = per * batch;
    for (long long e = (blockIdx.x * 256LL + threadIdx.x) * 4; e < total; e += (long long)gridDim.x * 256 * 4) {
        const int b = (int)(e / per);
        const long long r = e - b * per;
        const int o = (int)(r / kpad), k = (int)(r - (long long)o * kpad);
        float4 w = *(const float4 *)(wt + r);
        const float dd = (d && o < cout) ? d[(long long)b * d_ns + o] : 1.f;
        float f[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = (k + j < K) ? s[(long long)b * s_ns + (k + j) % cin] * dd : 0.f;
        w.x *= f[0]; w.y *= f[1]; w.z *= f[2]; w.w *= f[3];
        *(float4 *)(out + e) = w;
    }
}

static unsigned grid_for(long long total) {
    long long b = (total + 255) / 256;
    if (b > 65535LL * 16) b = 65535LL * 16;
    return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_resize(const float *x, int n, int c, int ih, int iw, long long xsn, long long xsc, long long xsy,
                          long long xsx, float *y, int oh, int ow, long long ysn, long long ysc, long long ysy,
                          long long ysx, float scale_h, float scale_w, int mode, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && c > 0 && ih > 0 && iw > 0 && oh > 0 && ow > 0, "resize: bad args");
    S2V_REQUIRE(mode == 0 || mode == 1, "resize: bad mode");
    const bool v4 = xsc == 1 && ysc == 1 && c % 4 == 0 && xsx % 4 == 0 && ysx % 4 == 0 && xsy % 4 == 0 &&
                    ysy % 4 == 0 && xsn % 4 == 0 && ysn % 4 == 0 && ((uintptr_t)x % 16) == 0 &&
                    ((uintptr_t)y % 16) == 0 && xsy < (1LL << 31) && ysy < (1LL << 31);
    if (v4 && mode == 0 && oh == 2 * ih && ow == 2 * iw && scale_h == 0.5f && scale_w == 0.5f &&
        (long long)ysy * 2 < (1LL << 31) && tune_get(S2V_TUNE_RESIZE_UP2)) {
        // exact x2 (StyleConv / ToRGB upsamples): 2x2 output quads per thread
        const long long row = (long long)iw * (c / 4);
        const unsigned gx = (unsigned)((row + 255) / 256);
        const long long rows = (long long)n * ih;
        dim3 grid(gx, (unsigned)(rows < 65535 ? rows : 65535));
        up2_bilinear_nhwc4_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, n, c / 4, ih, iw, xsn, (int)xsy, (int)xsx,
                                                                        y, ysn, (int)ysy, (int)ysx);
        return check_launch("resize");
    }
    if (v4) {
        // ~4 float4 per thread along a row, a few rows per block (grid-stride over rows)
        const long long row = (long long)ow * (c / 4);
        const unsigned gx = (unsigned)((row + 1023) / 1024);
        const long long rows = (long long)n * oh;
        const long long gy = (rows + 3) / 4;
        dim3 grid(gx, (unsigned)(gy < 65535 ? gy : 65535));
        resize_nhwc4_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, n, c / 4, ih, iw, xsn, (int)xsy, (int)xsx, y, oh,
                                                                  ow, ysn, (int)ysy, (int)ysx, scale_h, scale_w, mode);
        return check_launch("resize");
    }
    resize_kernel<<<grid_for((long long)n * oh * ow * c), 256, 0, (hipStream_t)stream>>>(
        x, n, c, ih, iw, xsn, xsc, xsy, xsx, y, oh, ow, ysn, ysc, ysy, ysx, scale_h, scale_w, mode);
    return check_launch("resize");
}

extern "C" int s2v_row_pack(const float *x, int n, int h, int w, int c, int xcs, int kw, int pw, float *y, int ycs,
                            s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && c > 0 && xcs >= c && kw > 0 && pw >= 0,
                "row_pack: bad args");
    S2V_REQUIRE(ycs % 4 == 0 && ycs >= kw * c && ((uintptr_t)y & 15) == 0,
                "row_pack: output pitch must be a multiple of 4 floats holding kw * c channels, 16-byte aligned");
    row_pack_kernel<<<grid_for((long long)n * h * w * (ycs / 4)), 256, 0, (hipStream_t)stream>>>(
        x, n, h, w, c, xcs, kw, pw, y, ycs);
    return check_launch("row_pack");
}

extern "C" int s2v_pad_reflect(const float *x, int n, int h, int w, int c, int xcs, int pt, int pb, int pl, int pr,
                               float *y, int ycs, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && c > 0 && xcs >= c && ycs >= c, "pad_reflect: bad args");
    S2V_REQUIRE(pt >= 0 && pb >= 0 && pl >= 0 && pr >= 0 && pt < h && pb < h && pl < w && pr < w,
                "pad_reflect: padding must be < input size");
    const int oh = h + pt + pb, ow = w + pl + pr;
    if (c % 4 == 0 && xcs % 4 == 0 && ycs % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0)
        pad_reflect4_kernel<<<grid_for((long long)n * oh * ow * (c / 4)), 256, 0, (hipStream_t)stream>>>(
            x, n, h, w, c / 4, xcs, pt, pl, oh, ow, y, ycs);
    else
        pad_reflect_kernel<<<grid_for((long long)n * oh * ow * c), 256, 0, (hipStream_t)stream>>>(
            x, n, h, w, c, xcs, pt, pl, oh, ow, y, ycs);
    return check_launch("pad_reflect");
}

extern "C" int s2v_attention(const float *q, const float *k, const float *v, int batch, int heads, int tokens,
                             int dim_head, int ld_q, int ld_k, int ld_v, long long bs_q, long long bs_k,
                             long long bs_v, float scale, float *o, int ld_o, long long bs_o, s2v_stream_t stream) {
    S2V_REQUIRE(q && k && v && o && batch > 0 && heads > 0, "attention: bad args");
    S2V_REQUIRE(dim_head == 64 && tokens > 0 && tokens <= 256, "attention: needs dim_head 64, tokens <= 256");
    const size_t smem = ((size_t)tokens * 65 + (size_t)tokens * 64 + 4 * (64 + (size_t)tokens)) * sizeof(float);
    S2V_REQUIRE(smem <= 160 * 1024, "attention: too many tokens for LDS");
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)attention_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    // enough row groups per (sample, head) to cover the CUs (LNet: 16 x 4 heads -> 64 x 4 blocks)
    int rg = 1;
    while (batch * heads * rg < 2 * device_cus() && 4 * rg * 2 <= tokens && rg < 16) rg *= 2;
    attention_kernel<<<dim3(batch * heads, rg), 256, smem, (hipStream_t)stream>>>(q, k, v, heads, tokens, ld_q, ld_k,
                                                                                 ld_v, bs_q, bs_k, bs_v, scale, o, ld_o,
                                                                                 bs_o);
    return check_launch("attention");
}

extern "C" int s2v_flow_warp(const float *flow, int n, int fh, int fw, int flow_cs, const float *src, int c, int h,
                             int w, long long ssn, long long ssc, long long ssy, long long ssx, float *y, int ycs,
                             s2v_stream_t stream) {
    S2V_REQUIRE(flow && src && y && n > 0 && fh > 1 && fw > 1 && c > 0 && h > 0 && w > 0 && flow_cs >= 2 && ycs >= c,
                "flow_warp: bad args");
    flow_warp_kernel<false><<<cdiv((long long)n * h * w, 256), 256, 0, (hipStream_t)stream>>>(
        flow, n, fh, fw, flow_cs, src, c, h, w, ssn, ssc, ssy, ssx, y, ycs);
    return check_launch("flow_warp");
}

extern "C" int s2v_flow_warp_cat(const float *flow, int n, int fh, int fw, int flow_cs, const float *src, int c, int h,
                                 int w, long long ssn, long long ssc, long long ssy, long long ssx, float *y, int ycs,
                                 s2v_stream_t stream) {
    S2V_REQUIRE(flow && src && y && n > 0 && fh > 1 && fw > 1 && c > 0 && h > 0 && w > 0 && flow_cs >= 2 &&
                    ycs >= 2 * c,
                "flow_warp_cat: bad args");
    flow_warp_kernel<true><<<cdiv((long long)n * h * w, 256), 256, 0, (hipStream_t)stream>>>(
        flow, n, fh, fw, flow_cs, src, c, h, w, ssn, ssc, ssy, ssx, y, ycs);
    return check_launch("flow_warp_cat");
}

extern "C" int s2v_melspectrogram(const float *wav, long long n_samples, const float *tables, int pad_reflect,
                                  float *out, long long frames, s2v_stream_t stream) {
    S2V_REQUIRE(wav && tables && out && n_samples > 0, "melspectrogram: bad args");
    S2V_REQUIRE(frames == 1 + n_samples / kHop, "melspectrogram: frames must be 1 + n_samples/200");
    S2V_REQUIRE(!pad_reflect || n_samples > kNfft / 2, "melspectrogram: reflect padding needs > 400 samples");
    S2V_REQUIRE(frames < 2147483647LL, "melspectrogram: too long");
    mel_kernel<<<(unsigned)frames, 256, 0, (hipStream_t)stream>>>(wav, n_samples, tables, pad_reflect, out, frames);
    return check_launch("mel");
}

extern "C" int s2v_mel_chunks(const float *mel, long long frames, const int *starts, int nchunks, int step,
                              float *out, s2v_stream_t stream) {
    S2V_REQUIRE(mel && starts && out && nchunks > 0 && step > 0 && frames >= step, "mel_chunks: bad args");
    mel_chunks_kernel<<<cdiv((long long)nchunks * kMels * step, 256), 256, 0, (hipStream_t)stream>>>(
        mel, frames, starts, nchunks, step, out);
    return check_launch("mel_chunks");
}

template <typename T>
static int fused_bias_act_t(const T *x, const T *b, const T *ref, T *y, long long size, int c, long long step_b, int act,
                            int grad, double alpha, double scale, s2v_stream_t stream) {
    using A = typename OpT<T>::type;
    S2V_REQUIRE(x && y && size >= 0, "fused_bias_act: bad args");
    S2V_REQUIRE(!b || (c > 0 && step_b > 0), "fused_bias_act: bias needs c > 0 and step_b > 0");
    if (size == 0) return 0;
    const uintptr_t al = 4 * sizeof(T) - 1;
    const bool rows_ok = step_b > 0 && step_b % 4 == 0 && size % step_b == 0 && ((uintptr_t)x & al) == 0 &&
                         ((uintptr_t)y & al) == 0 && (!ref || ((uintptr_t)ref & al) == 0);
    if (rows_ok) {
        const long long rows = size / step_b, step4 = step_b / 4;
        const unsigned gx = (unsigned)((step4 + 255) / 256 < 64 ? (step4 + 255) / 256 : 64);
        const unsigned gy = (unsigned)(rows < 65535 ? rows : 65535);
        fused_bias_act_rows<T><<<dim3(gx, gy), 256, 0, (hipStream_t)stream>>>(x, b, ref, y, rows, b ? c : 1, step4, act,
                                                                              grad, (A)alpha, (A)scale);
    } else {
        fused_bias_act_kernel<T><<<grid_for(size), 256, 0, (hipStream_t)stream>>>(x, b, ref, y, size, c, step_b, act,
                                                                                    grad, (A)alpha, (A)scale);
    }
    return check_launch("fused_bias_act");
}

template <typename T>
static int upfirdn2d_t(const T *x, int major, int in_h, int in_w, int minor, const T *k, int kh, int kw, int up_x,
                       int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1, T *y, int out_h,
                       int out_w, s2v_stream_t stream) {
    S2V_REQUIRE(x && k && y && major > 0 && in_h > 0 && in_w > 0 && minor > 0 && kh > 0 && kw > 0,
                "upfirdn2d: bad args");
    S2V_REQUIRE(up_x >= 1 && up_y >= 1 && down_x >= 1 && down_y >= 1, "upfirdn2d: up/down must be >= 1");
    const int eh = (in_h * up_y + pad_y0 + pad_y1 - kh) / down_y + 1;
    const int ew = (in_w * up_x + pad_x0 + pad_x1 - kw) / down_x + 1;
    S2V_REQUIRE(eh == out_h && ew == out_w && out_h > 0 && out_w > 0,
                "upfirdn2d: output must be %dx%d (got %dx%d)", eh, ew, out_h, out_w);
    const unsigned g = grid_for((long long)major * out_h * out_w * minor);
    hipStream_t st = (hipStream_t)stream;
    const bool k4 = kh == 4 && kw == 4 && up_x == up_y && down_x == down_y;
#define S2V_UFD_ARGS x, major, in_h, in_w, minor, k, kh, kw, up_x, up_y, down_x, down_y, pad_x0, pad_y0, y, out_h, out_w
    if (k4 && minor == 1 && pad_x0 >= 0 && pad_y0 >= 0 && ((up_x == 1 && down_x <= 2) || (up_x == 2 && down_x == 1))) {
        const int tx = (out_w + 63) / 64, ty = (out_h + 15) / 16;
        const unsigned gp = (unsigned)((long long)major * tx * ty);
        if (up_x == 2) upfirdn2d_plane4<T, 2, 1><<<gp, 256, 0, st>>>(x, in_h, in_w, k, pad_x0, pad_y0, y, out_h, out_w, tx, ty);
        else if (down_x == 2) upfirdn2d_plane4<T, 1, 2><<<gp, 256, 0, st>>>(x, in_h, in_w, k, pad_x0, pad_y0, y, out_h, out_w, tx, ty);
        else upfirdn2d_plane4<T, 1, 1><<<gp, 256, 0, st>>>(x, in_h, in_w, k, pad_x0, pad_y0, y, out_h, out_w, tx, ty);
    } else if (k4 && up_x == 1 && down_x == 1) upfirdn2d_kernel<T, 1, 1, 4><<<g, 256, 0, st>>>(S2V_UFD_ARGS);
    else if (k4 && up_x == 2 && down_x == 1) upfirdn2d_kernel<T, 2, 1, 4><<<g, 256, 0, st>>>(S2V_UFD_ARGS);
    else if (k4 && up_x == 1 && down_x == 2) upfirdn2d_kernel<T, 1, 2, 4><<<g, 256, 0, st>>>(S2V_UFD_ARGS);
    else upfirdn2d_kernel<T><<<g, 256, 0, st>>>(S2V_UFD_ARGS);
#undef S2V_UFD_ARGS
    return check_launch("upfirdn2d");
}

extern "C" int s2v_fused_bias_act(const float *x, const float *b, const float *ref, float *y, long long size, int c,
                                  long long step_b, int act, int grad, float alpha, float scale,
                                  s2v_stream_t stream) {
    return fused_bias_act_t<float>(x, b, ref, y, size, c, step_b, act, grad, alpha, scale, stream);
}

extern "C" int s2v_upfirdn2d(const float *x, int major, int in_h, int in_w, int minor, const float *k, int kh, int kw,
                             int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0,
                             int pad_y1, float *y, int out_h, int out_w, s2v_stream_t stream) {
    return upfirdn2d_t<float>(x, major, in_h, in_w, minor, k, kh, kw, up_x, up_y, down_x, down_y, pad_x0, pad_x1,
                              pad_y0, pad_y1, y, out_h, out_w, stream);
}

extern "C" int s2v_fused_bias_act_dt(int dtype, const void *x, const void *b, const void *ref, void *y, long long size,
                                     int c, long long step_b, int act, int grad, double alpha, double scale,
                                     s2v_stream_t stream) {
    switch (dtype) {
        case S2V_DT_F32:
            return fused_bias_act_t<float>((const float *)x, (const float *)b, (const float *)ref, (float *)y, size, c,
                                           step_b, act, grad, alpha, scale, stream);
        case S2V_DT_F16:
            return fused_bias_act_t<_Float16>((const _Float16 *)x, (const _Float16 *)b, (const _Float16 *)ref,
                                              (_Float16 *)y, size, c, step_b, act, grad, alpha, scale, stream);
        case S2V_DT_F64:
            return fused_bias_act_t<double>((const double *)x, (const double *)b, (const double *)ref, (double *)y, size,
                                            c, step_b, act, grad, alpha, scale, stream);
    }
    S2V_REQUIRE(false, "fused_bias_act: dtype %d is not one of S2V_DT_F32 / F16 / F64", dtype);
    return S2V_E_INVALID;
}

extern "C" int s2v_upfirdn2d_dt(int dtype, const void *x, int major, int in_h, int in_w, int minor, const void *k,
                                int kh, int kw, int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1,
                                int pad_y0, int pad_y1, void *y, int out_h, int out_w, s2v_stream_t stream) {
#define S2V_UFD_DT(T) upfirdn2d_t<T>((const T *)x, major, in_h, in_w, minor, (const T *)k, kh, kw, up_x, up_y, down_x, \
                                     down_y, pad_x0, pad_x1, pad_y0, pad_y1, (T *)y, out_h, out_w, stream)
    switch (dtype) {
        case S2V_DT_F32: return S2V_UFD_DT(float);
        case S2V_DT_F16: return S2V_UFD_DT(_Float16);
        case S2V_DT_F64: return S2V_UFD_DT(double);
    }
#undef S2V_UFD_DT
    S2V_REQUIRE(false, "upfirdn2d: dtype %d is not one of S2V_DT_F32 / F16 / F64", dtype);
    return S2V_E_INVALID;
}

extern "C" int s2v_gaussian_noise(float *y, long long n, unsigned long long seed, unsigned long long offset,
                                  s2v_stream_t stream) {
    S2V_REQUIRE(y && n >= 0, "gaussian_noise: bad args");
    if (n == 0) return 0;
    gaussian_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(y, n, seed, offset, nullptr, 0);
    return check_launch("gaussian_noise");
}

extern "C" int s2v_gaussian_noise_ctr(float *y, long long n, unsigned long long seed, unsigned long long offset,
                                      const unsigned long long *ctr, int shift, s2v_stream_t stream) {
    S2V_REQUIRE(y && ctr && n >= 0 && shift >= 0 && shift < 64, "gaussian_noise_ctr: bad args");
    if (n == 0) return 0;
    gaussian_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(y, n, seed, offset, ctr, shift);
    return check_launch("gaussian_noise_ctr");
}

__global__ void counter_add_kernel(unsigned long long *ctr, unsigned long long inc) {
    if (threadIdx.x == 0) ctr[0] += inc;
}

extern "C" int s2v_counter_add(unsigned long long *ctr, unsigned long long inc, s2v_stream_t stream) {
    S2V_REQUIRE(ctr && ((uintptr_t)ctr % 8) == 0, "counter_add: bad args");
    counter_add_kernel<<<1, 64, 0, (hipStream_t)stream>>>(ctr, inc);
    return check_launch("counter_add");
}

extern "C" int s2v_lipsync_inputs(const float *src, const float *fake, int n, int h, int w, unsigned char *ref_u8,
                                  float *face6, float *gt, s2v_stream_t stream) {
    S2V_REQUIRE(src && ref_u8 && face6 && gt && n > 0 && h > 1 && w > 0, "lipsync_inputs: bad args");
    lipsync_inputs_kernel<<<grid_for((long long)n * 3 * h * w), 256, 0, (hipStream_t)stream>>>(src, fake, n, h, w,
                                                                                               ref_u8, face6, gt);
    return check_launch("lipsync_inputs");
}

extern "C" int s2v_to_u8(const float *x, long long n, float lo, float hi, float scale, float offset, unsigned char *y,
                         s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n >= 0, "to_u8: bad args");
    if (n == 0) return 0;
    to_u8_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(x, n, lo, hi, scale, offset, y);
    return check_launch("to_u8");
}

extern "C" int s2v_eltwise(const float *x, int xcs, const float *mul, int mcs, const float *add, int acs,
                           const float *bias, long long pixels, int c, float a, int act, float alpha, float post,
                           float *y, int ycs, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && pixels >= 0 && c > 0 && xcs >= c && ycs >= c && (!mul || mcs >= c) && (!add || acs >= c),
                "eltwise: bad args");
    if (pixels == 0) return 0;
    const auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
    const bool v4 = c % 4 == 0 && xcs % 4 == 0 && ycs % 4 == 0 && al(x) && al(y) && (!mul || (mcs % 4 == 0 && al(mul))) &&
                    (!add || (acs % 4 == 0 && al(add))) && (!bias || al(bias)) && pixels * (c / 4) < (1LL << 31);
    if (v4) {
        const unsigned quads = (unsigned)(pixels * (c / 4));
        eltwise4_kernel<<<grid_for(quads), 256, 0, (hipStream_t)stream>>>(x, xcs, mul, mcs, add, acs, bias, quads,
                                                                          (unsigned)(c / 4), a, act, alpha, post, y, ycs);
    } else {
        eltwise_kernel<<<grid_for(pixels * c), 256, 0, (hipStream_t)stream>>>(x, xcs, mul, mcs, add, acs, bias, pixels,
                                                                               c, a, act, alpha, post, y, ycs);
    }
    return check_launch("eltwise");
}

extern "C" int s2v_fill(float *y, long long n, float value, s2v_stream_t stream) {
    S2V_REQUIRE(y && n >= 0, "fill: bad args");
    if (n == 0) return 0;
    fill_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(y, n, value);
    return check_launch("fill");
}

extern "C" int s2v_amax(const float *x, long long pixels, int c, int xcs, float *out, s2v_stream_t stream) {
    S2V_REQUIRE(x && out && pixels >= 0 && c > 0 && xcs >= c, "amax: bad args");
    if (pixels == 0) return 0;
    const bool vec = c % 4 == 0 && xcs % 4 == 0 && ((uintptr_t)x % 16) == 0;
    const int units = vec ? c / 4 : c;                  // per-row work items
    int sh = 0;
    while ((1 << sh) < units && sh < 6) ++sh;           // threads per row: units rounded up, at most 64
    const long long rows_per_block = 256 >> sh;
    long long blocks = (pixels + rows_per_block - 1) / rows_per_block;
    if (blocks > 2048) blocks = 2048;                   // 8 blocks per CU, grid-stride beyond
    if (vec)
        amax_kernel<true><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(x, pixels, c, xcs, sh, (unsigned *)out);
    else
        amax_kernel<false><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(x, pixels, c, xcs, sh, (unsigned *)out);
    return check_launch("amax");
}

extern "C" int s2v_modulate_weights(const float *wt, int npad, int kpad, int K, int cin, int cout, const float *s,
                                    int s_ns, const float *d, int d_ns, int batch, float *out, s2v_stream_t stream) {
    S2V_REQUIRE(wt && s && out && npad > 0 && kpad > 0 && K > 0 && K <= kpad && cin > 0 && cout > 0 && cout <= npad &&
                batch > 0 && s_ns >= cin && (!d || d_ns >= cout), "modulate_weights: bad args");
    S2V_REQUIRE(kpad % 4 == 0 && ((uintptr_t)wt % 16) == 0 && ((uintptr_t)out % 16) == 0,
                "modulate_weights: kpad %% 4 and 16-byte aligned weights required");
    modulate_weights_kernel<<<grid_for((long long)npad * kpad * batch / 4), 256, 0, (hipStream_t)stream>>>(
        wt, npad, kpad, K, cin, cout, s, s_ns, d, d_ns, batch, out);
    return check_launch("modulate_weights");
}
