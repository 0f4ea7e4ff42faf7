// Normalisation kernels: LayerNorm2d (+act, +pool, +residual), InstanceNorm/ADAIN (+act,
// +residual), token LayerNorm, ADAIN gamma/beta heads, StyleGAN2 demodulation.
//
// All are HBM-bound.  Statistics are accumulated in fp64 per thread (no cancellation in
// E[x^2] - E[x]^2 at 1e6-element reductions) and combined deterministically through a
// workspace of per-block partials (no float atomics), so results are run-to-run identical.
#include "common.hpp"

namespace s2v {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// block (256 threads) sum of two doubles; result valid in all threads
__device__ __forceinline__ void block_sum2(double &a, double &b) {
    __shared__ double red[2][4];
    a = wave_sum(a);
    b = wave_sum(b);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wv] = a;
        red[1][wv] = b;
    }
    __syncthreads();
    a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    __syncthreads();
}

// ------------------------------------------------------------------ LayerNorm2d
static int ln_blocks(long long elems) {
    long long b = (elems + 8191) / 8192;
    if (b < 1) b = 1;
    if (b > 256) b = 256;
    return (int)b;
}

// apply blocks per image: a grid-stride loop of LN_EPT quads per step, so the per-block statistics
// prologue (nblk partials, a block reduction) is paid by at most this many blocks per image
static unsigned ln_apply_blocks(long long quads, int n, int ept) {
    long long b = (quads + 256LL * ept - 1) / (256LL * ept);
    const long long cap = n >= 16 ? 64 : 1024 / n;
    return (unsigned)(b < cap ? b : cap);
}

__global__ __launch_bounds__(256) void ln_stats(const float *__restrict__ x, int hw, int c, int xcs, int nblk,
                                                double *__restrict__ part) {
    const int n = blockIdx.y, blk = blockIdx.x;
    const long long pix_per = ((long long)hw + nblk - 1) / nblk;
    const long long p0 = blk * pix_per;
    const long long p1 = min((long long)hw, p0 + pix_per);
    const float *xb = x + (long long)n * hw * xcs;
    double s = 0.0, q = 0.0;
    if (xcs == c && (c & 3) == 0 && ((uintptr_t)x & 15) == 0) {
        // dense rows: the block's pixel range is one contiguous span, read with four 16-byte loads in
        // flight per thread (one load per iteration left the 67 MB DNet LayerNorms at 1.7 TB/s)
        const float4 *b4 = (const float4 *)(xb + p0 * c);
        const int tot = (int)(p1 - p0) * (c >> 2);
        int e = threadIdx.x;
        for (; e + 768 < tot; e += 1024) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = b4[e + 256 * u];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s += (double)v[u].x + (double)v[u].y + (double)v[u].z + (double)v[u].w;
                q += (double)v[u].x * v[u].x + (double)v[u].y * v[u].y + (double)v[u].z * v[u].z +
                     (double)v[u].w * v[u].w;
            }
        }
        for (; e < tot; e += 256) {
            const float4 v = b4[e];
            s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
            q += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        }
    } else if ((c & 3) == 0 && (xcs & 3) == 0 && ((uintptr_t)x & 15) == 0) {
        const int c4 = c >> 2;
        const int tot = (int)(p1 - p0) * c4;
        for (int e = threadIdx.x; e < tot; e += 256) {
            const long long p = p0 + e / c4;
            const int cc = (e - (e / c4) * c4) * 4;
            const float4 v = *(const float4 *)(xb + p * xcs + cc);
            s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
            q += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        }
    } else {
        const int tot = (int)(p1 - p0) * c;
        for (int e = threadIdx.x; e < tot; e += 256) {
            const long long p = p0 + e / c;
            const int cc = e - (e / c) * c;
            const double v = xb[p * xcs + cc];
            s += v;
            q += v * v;
        }
    }
    block_sum2(s, q);
    if (threadIdx.x == 0) {
        part[((long long)n * nblk + blk) * 2 + 0] = s;
        part[((long long)n * nblk + blk) * 2 + 1] = q;
    }
}

__global__ __launch_bounds__(256) void ln_apply(const float *__restrict__ x, int h, int w, int c, int xcs,
                                                const float *__restrict__ weight, const float *__restrict__ bias,
                                                float eps, int act, float alpha, int pool, const float *res, int res_cs,
                                                float *y, int ycs, const double *__restrict__ part, int nblk) {
    const int n = blockIdx.y;
    __shared__ float st[2];
    {
        double s = 0.0, q = 0.0;
        for (int i = threadIdx.x; i < nblk; i += 256) {
            s += part[((long long)n * nblk + i) * 2 + 0];
            q += part[((long long)n * nblk + i) * 2 + 1];
        }
        block_sum2(s, q);
        if (threadIdx.x == 0) {
            const double cnt = (double)h * w * c;
            const double mean = s / cnt;
            double var = q / cnt - mean * mean;
            if (var < 0.0) var = 0.0;
            st[0] = (float)mean;
            st[1] = (float)(1.0 / sqrt(var + (double)eps));
        }
        __syncthreads();
    }
    const float mean = st[0], rstd = st[1];
    const int oh = pool ? h / 2 : h, ow = pool ? w / 2 : w;
    const int tot = oh * ow * c;
    const float *xb = x + (long long)n * h * w * xcs;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < tot; e += gridDim.x * 256) {
        const int p = e / c;
        const int cc = e - p * c;
        const int oy = p / ow, ox = p - (p / ow) * ow;
        const float g = weight[cc] * rstd, b = bias[cc];
        float v;
        if (pool) {
            const float *px = xb + ((long long)(2 * oy) * w + 2 * ox) * xcs + cc;
            float a0 = apply_act((px[0] - mean) * g + b, act, alpha);
            float a1 = apply_act((px[xcs] - mean) * g + b, act, alpha);
            float a2 = apply_act((px[(long long)w * xcs] - mean) * g + b, act, alpha);
            float a3 = apply_act((px[(long long)w * xcs + xcs] - mean) * g + b, act, alpha);
            v = (a0 + a1 + a2 + a3) * 0.25f;
        } else {
            v = apply_act((xb[p * xcs + cc] - mean) * g + b, act, alpha);
        }
        const long long op = (long long)n * oh * ow + p;
        if (res) v += res[op * res_cs + cc];
        y[op * ycs + cc] = v;
    }
}

// float4 form of the pooled apply (ConvNormAct pool=True: LNet / DNet DownBlock2d): one output pixel
// channel quad per thread, its 2x2 source quads loaded as four float4s (the scalar ln_apply ran the
// DNet 256^2 x 64 pooled LayerNorm at 2 TB/s)
__global__ __launch_bounds__(256) void ln_apply4_pool(const float *__restrict__ x, int h, int w, int c4, int xcs,
                                                      const float *__restrict__ weight, const float *__restrict__ bias,
                                                      float eps, int act, float alpha, const float *res, int res_cs,
                                                      float *y, int ycs, const double *__restrict__ part, int nblk) {
    const int n = blockIdx.y;
    __shared__ float st[2];
    {
        double s = 0.0, q = 0.0;
        for (int i = threadIdx.x; i < nblk; i += 256) {
            s += part[((long long)n * nblk + i) * 2 + 0];
            q += part[((long long)n * nblk + i) * 2 + 1];
        }
        block_sum2(s, q);
        if (threadIdx.x == 0) {
            const double cnt = (double)h * w * c4 * 4;
            const double mean = s / cnt;
            double var = q / cnt - mean * mean;
            if (var < 0.0) var = 0.0;
            st[0] = (float)mean;
            st[1] = (float)(1.0 / sqrt(var + (double)eps));
        }
        __syncthreads();
    }
    const int oh = h / 2, ow = w / 2;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= oh * ow * c4) return;
    const float mean = st[0], rstd = st[1];
    const int p = e / c4, cq = e - p * c4, cc = 4 * cq;
    const int oy = p / ow, ox = p - oy * ow;
    const float4 wv = *(const float4 *)(weight + cc), bv = *(const float4 *)(bias + cc);
    const float *px = x + (((long long)n * h + 2 * oy) * w + 2 * ox) * xcs + cc;
    const float4 a0 = *(const float4 *)px, a1 = *(const float4 *)(px + xcs);
    const float4 a2 = *(const float4 *)(px + (long long)w * xcs), a3 = *(const float4 *)(px + (long long)w * xcs + xcs);
    const float slope = act == S2V_ACT_LRELU ? alpha : 0.f;
    auto f = [&](float v, float g, float b) { return apply_act((v - mean) * (g * rstd) + b, act, slope); };
    float4 o;
    o.x = 0.25f * (f(a0.x, wv.x, bv.x) + f(a1.x, wv.x, bv.x) + f(a2.x, wv.x, bv.x) + f(a3.x, wv.x, bv.x));
    o.y = 0.25f * (f(a0.y, wv.y, bv.y) + f(a1.y, wv.y, bv.y) + f(a2.y, wv.y, bv.y) + f(a3.y, wv.y, bv.y));
    o.z = 0.25f * (f(a0.z, wv.z, bv.z) + f(a1.z, wv.z, bv.z) + f(a2.z, wv.z, bv.z) + f(a3.z, wv.z, bv.z));
    o.w = 0.25f * (f(a0.w, wv.w, bv.w) + f(a1.w, wv.w, bv.w) + f(a2.w, wv.w, bv.w) + f(a3.w, wv.w, bv.w));
    const long long op = (long long)n * oh * ow + p;
    if (res) {
        const float4 r = *(const float4 *)(res + op * res_cs + cc);
        o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
    }
    *(float4 *)(y + op * ycs + cc) = o;
}

// LN_EPT channel quads per thread step in the non-pooled apply
constexpr int LN_EPT = 4;

// float4 form without pooling (c, pitches % 4 == 0, 16-byte aligned): LN_EPT channel quads 256 apart
// per thread, all loads issued before the first store (no load waits behind a store of the same wave)
__global__ __launch_bounds__(256) void ln_apply4(const float *__restrict__ x, int hw, int c4, int xcs,
                                                 const float *__restrict__ weight, const float *__restrict__ bias,
                                                 float eps, int act, float alpha, const float *res, int res_cs,
                                                 float *y, int ycs, const double *__restrict__ part, int nblk) {
    const int n = blockIdx.y;
    __shared__ float st[2];
    {
        double s = 0.0, q = 0.0;
        for (int i = threadIdx.x; i < nblk; i += 256) {
            s += part[((long long)n * nblk + i) * 2 + 0];
            q += part[((long long)n * nblk + i) * 2 + 1];
        }
        block_sum2(s, q);
        if (threadIdx.x == 0) {
            const double cnt = (double)hw * c4 * 4;
            const double mean = s / cnt;
            double var = q / cnt - mean * mean;
            if (var < 0.0) var = 0.0;
            st[0] = (float)mean;
            st[1] = (float)(1.0 / sqrt(var + (double)eps));
        }
        __syncthreads();
    }
    const int tot = hw * c4;
    const float mean = st[0], rstd = st[1];
    for (int e0 = blockIdx.x * 256 * LN_EPT + threadIdx.x; e0 < tot; e0 += gridDim.x * 256 * LN_EPT) {
    float4 v[LN_EPT], r[LN_EPT];
#pragma unroll
    for (int k = 0; k < LN_EPT; ++k) {
        const int e = e0 + 256 * k;
        if (e >= tot) break;
        const int p = e / c4, cc = (e - p * c4) * 4;
        v[k] = *(const float4 *)(x + ((long long)n * hw + p) * xcs + cc);
        if (res) r[k] = *(const float4 *)(res + ((long long)n * hw + p) * res_cs + cc);
    }
#pragma unroll
    for (int k = 0; k < LN_EPT; ++k) {
        const int e = e0 + 256 * k;
        if (e >= tot) break;
        const int p = e / c4, cc = (e - p * c4) * 4;
        const float4 w = *(const float4 *)(weight + cc), b = *(const float4 *)(bias + cc);
        float4 o;
        o.x = apply_act((v[k].x - mean) * (w.x * rstd) + b.x, act, alpha);
        o.y = apply_act((v[k].y - mean) * (w.y * rstd) + b.y, act, alpha);
        o.z = apply_act((v[k].z - mean) * (w.z * rstd) + b.z, act, alpha);
        o.w = apply_act((v[k].w - mean) * (w.w * rstd) + b.w, act, alpha);
        if (res) {
            o.x += r[k].x; o.y += r[k].y; o.z += r[k].z; o.w += r[k].w;
        }
        *(float4 *)(y + ((long long)n * hw + p) * ycs + cc) = o;
    }
    }
}

// ------------------------------------------------------------------ InstanceNorm / ADAIN
static int in_chunks(long long hw) {
    long long k = (hw + 1023) / 1024;
    if (k > 64) k = 64;
    return (int)(k < 1 ? 1 : k);
}

// grid (chunks, ceil(c/64), n); lane -> channel, wave -> pixel phase
__global__ __launch_bounds__(256) void in_stats(const float *__restrict__ x, int hw, int c, int xcs, int chunks,
                                                double *__restrict__ part) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int cc = blockIdx.y * 64 + lane;
    const int n = blockIdx.z, ch = blockIdx.x;
    const int per = (hw + chunks - 1) / chunks;
    const int p0 = ch * per, p1 = min(hw, p0 + per);
    double s = 0.0, q = 0.0;
    if (cc < c) {
        const float *xb = x + (long long)n * hw * xcs + cc;
        for (int p = p0 + wv; p < p1; p += 4) {
            const double v = xb[(long long)p * xcs];
            s += v;
            q += v * v;
        }
    }
    __shared__ double red[2][4][64];
    red[0][wv][lane] = s;
    red[1][wv][lane] = q;
    __syncthreads();
    if (wv == 0 && cc < c) {
        s = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
        q = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
        const long long o = (((long long)n * c + cc) * chunks + ch) * 2;
        part[o] = s;
        part[o + 1] = q;
    }
}

__global__ __launch_bounds__(256) void in_apply(const float *__restrict__ x, int hw, int c, int xcs,
                                                const float *__restrict__ gamma, const float *__restrict__ beta,
                                                int gb_ns, float eps, int act, float alpha, const float *res,
                                                int res_cs, float *y, int ycs, const double *__restrict__ part,
                                                int chunks, int achunks) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int cc = blockIdx.y * 64 + lane;
    const int n = blockIdx.z;
    if (cc >= c) return;
    double s = 0.0, q = 0.0;
    const long long o = ((long long)n * c + cc) * chunks * 2;
    for (int i = 0; i < chunks; ++i) {
        s += part[o + 2 * i];
        q += part[o + 2 * i + 1];
    }
    const double mean = s / hw;
    double var = q / hw - mean * mean;
    if (var < 0.0) var = 0.0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? 1.f + gamma[(long long)n * gb_ns + cc] : 1.f;
    const float b = beta ? beta[(long long)n * gb_ns + cc] : 0.f;
    const float meanf = (float)mean;
    const int per = (hw + achunks - 1) / achunks;
    const int p0 = blockIdx.x * per, p1 = min(hw, p0 + per);
    const float *xb = x + (long long)n * hw * xcs + cc;
    float *yb = y + (long long)n * hw * ycs + cc;
    const float *rb = res ? res + (long long)n * hw * res_cs + cc : nullptr;
    for (int p = p0 + wv; p < p1; p += 4) {
        float v = apply_act((xb[(long long)p * xcs] - meanf) * rstd * g + b, act, alpha);
        if (rb) v += rb[(long long)p * res_cs];
        yb[(long long)p * ycs] = v;
    }
}

// Vectorised InstanceNorm/ADAIN (c % 4 == 0, 16-byte aligned views): a thread owns 4 channels
// (one float4) and a pixel phase; a block covers QB = min(64, c / 4) channel quads with
// 256 / QB pixel phases (so a 128-channel layer keeps every lane busy); 4 independent loads in
// flight per thread; fp64 partial sums.   grid (chunks, ceil(c / (4 QB)), n)
__device__ __forceinline__ int in_quads(int c) { return c / 4 < 64 ? c / 4 : 64; }

__global__ __launch_bounds__(256) void in_stats_v(const float *__restrict__ x, int hw, int c, int xcs, int chunks,
                                                  double *__restrict__ part) {
    const int qb = in_quads(c), nph = 256 / qb;
    const int q4 = threadIdx.x % qb, ph = threadIdx.x / qb;
    const int cc = (blockIdx.y * qb + q4) * 4;
    const int n = blockIdx.z, ch = blockIdx.x;
    const int per = (hw + chunks - 1) / chunks;
    const int p0 = ch * per, p1 = min(hw, p0 + per);
    const bool live = ph < nph && cc < c;
    double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
    if (live) {
        const float *xb = x + (long long)n * hw * xcs + cc;
        int p = p0 + ph;
        for (; p + 3 * nph < p1; p += 4 * nph) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *(const float4 *)(xb + (long long)(p + nph * u) * xcs);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double a = v[u].x, b = v[u].y, d = v[u].z, e = v[u].w;
                s[0] += a; s[1] += b; s[2] += d; s[3] += e;
                q[0] += a * a; q[1] += b * b; q[2] += d * d; q[3] += e * e;
            }
        }
        for (; p < p1; p += nph) {
            const float4 v = *(const float4 *)(xb + (long long)p * xcs);
            const double a = v.x, b = v.y, d = v.z, e = v.w;
            s[0] += a; s[1] += b; s[2] += d; s[3] += e;
            q[0] += a * a; q[1] += b * b; q[2] += d * d; q[3] += e * e;
        }
    }
    __shared__ double red[256][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        red[threadIdx.x][j] = s[j];
        red[threadIdx.x][4 + j] = q[j];
    }
    __syncthreads();
    if (ph == 0 && cc < c) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double ss = 0.0, qq = 0.0;
            for (int k = 0; k < nph; ++k) {
                ss += red[k * qb + q4][j];
                qq += red[k * qb + q4][4 + j];
            }
            const long long o = (((long long)n * c + cc + j) * chunks + ch) * 2;
            part[o] = ss;
            part[o + 1] = qq;
        }
    }
}

// The block first folds the chunk partials of its channels cooperatively (each pixel phase sums a
// stride of the chunks, LDS combine), computes (mul, add) per channel once, then applies.
__global__ __launch_bounds__(256) void in_apply_v(const float *__restrict__ x, int hw, int c, int xcs,
                                                  const float *__restrict__ gamma, const float *__restrict__ beta,
                                                  int gb_ns, float eps, int act, float alpha, const float *res,
                                                  int res_cs, float *y, int ycs, const double *__restrict__ part,
                                                  int chunks, int achunks, int w = 0, float *yp = nullptr,
                                                  int ypcs = 0, int qbo = 0) {
    const int qb = qbo > 0 ? qbo : in_quads(c), nph = 256 / qb;
    const int q4 = threadIdx.x % qb, ph = threadIdx.x / qb;
    const int cc = (blockIdx.y * qb + q4) * 4;
    const int n = blockIdx.z;
    const bool live = ph < nph && cc < c;
    __shared__ double red[256][8];
    __shared__ float coef[64][8];
    {
        double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
        if (live && part) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const long long o = ((long long)n * c + cc + j) * chunks * 2;
                for (int i = ph; i < chunks; i += nph) {
                    s[j] += part[o + 2 * i];
                    q[j] += part[o + 2 * i + 1];
                }
            }
        } else if (live) {
            // fused form (part == NULL, one block per plane and channel group): the moments of
            // the whole plane straight from x, then the apply below re-reads it (from L2)
            const float *xs = x + (long long)n * hw * xcs + cc;
#pragma unroll 4
            for (int p = ph; p < hw; p += nph) {
                const float4 v = *(const float4 *)(xs + (long long)p * xcs);
                const double a = v.x, b = v.y, d = v.z, e = v.w;
                s[0] += a; s[1] += b; s[2] += d; s[3] += e;
                q[0] += a * a; q[1] += b * b; q[2] += d * d; q[3] += e * e;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            red[threadIdx.x][j] = s[j];
            red[threadIdx.x][4 + j] = q[j];
        }
    }
    __syncthreads();
    if (ph == 0 && cc < c) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double sm = 0.0, sq = 0.0;
            for (int k = 0; k < nph; ++k) {
                sm += red[k * qb + q4][j];
                sq += red[k * qb + q4][4 + j];
            }
            const double mean = sm / hw;
            double var = sq / hw - mean * mean;
            if (var < 0.0) var = 0.0;
            const float rstd = 1.f / sqrtf((float)(var + (double)eps));   // fp64 moments, fp32 root
            const float g = gamma ? 1.f + gamma[(long long)n * gb_ns + cc + j] : 1.f;
            const float b = beta ? beta[(long long)n * gb_ns + cc + j] : 0.f;
            coef[q4][j] = rstd * g;                                  // (x - mean) * rstd * g + b
            coef[q4][4 + j] = b - (float)mean * rstd * g;
        }
    }
    __syncthreads();
    if (!live) return;
    float mul[4], add[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mul[j] = coef[q4][j];
        add[j] = coef[q4][4 + j];
    }
    const int per = (hw + achunks - 1) / achunks;
    const int p0 = blockIdx.x * per, p1 = min(hw, p0 + per);
    const float *xb = x + (long long)n * hw * xcs + cc;
    float *yb = y + (long long)n * hw * ycs + cc;
    const float *rb = res ? res + (long long)n * hw * res_cs + cc : nullptr;
    // software-pipelined: pixel p + nph is loaded before pixel p is stored (vmcnt counts loads and
    // stores in issue order: a load issued after a store would wait for that store to complete)
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f), r = v;
    if (p0 + ph < p1) {
        v = *(const float4 *)(xb + (long long)(p0 + ph) * xcs);
        if (rb) r = *(const float4 *)(rb + (long long)(p0 + ph) * res_cs);
    }
    for (int p = p0 + ph; p < p1; p += nph) {
        float4 o;
        o.x = apply_act(fmaf(v.x, mul[0], add[0]), act, alpha);
        o.y = apply_act(fmaf(v.y, mul[1], add[1]), act, alpha);
        o.z = apply_act(fmaf(v.z, mul[2], add[2]), act, alpha);
        o.w = apply_act(fmaf(v.w, mul[3], add[3]), act, alpha);
        if (rb) {
            o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
        }
        if (p + nph < p1) {
            v = *(const float4 *)(xb + (long long)(p + nph) * xcs);
            if (rb) r = *(const float4 *)(rb + (long long)(p + nph) * res_cs);
        }
        *(float4 *)(yb + (long long)p * ycs) = o;
        if (yp) {
            // reflect pad 1 (F.pad 'reflect'): pixel (r, q) lands at (r + 1, q + 1) and, on the second /
            // second-to-last row or column, also on the mirrored border row / column
            const int h = hw / w, r = p / w, q = p - r * w, W2 = w + 2;
            const int rows[2] = {r + 1, r == 1 ? 0 : (r == h - 2 ? h + 1 : -1)};
            const int cols[2] = {q + 1, q == 1 ? 0 : (q == w - 2 ? w + 1 : -1)};
            float *pb = yp + (long long)n * (h + 2) * W2 * ypcs + cc;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    if (rows[i] >= 0 && cols[j] >= 0)
                        *(float4 *)(pb + ((long long)rows[i] * W2 + cols[j]) * ypcs) = o;
        }
    }
}

static int in_chunks_v(int n, long long hw, int c) {
    const long long cq = (c + 255) / 256;
    long long k = 1;
    while ((long long)n * cq * k < 512 && k * 64 < hw && k < 64) k *= 2;
    return (int)k;
}

// pixel chunks of the apply pass: at least the stats chunks, up to >= 1024 blocks with >= 16 pixels
// each (the apply pass has no partials to keep small, and one block per CU left it latency-bound)
static int in_apply_chunks(int n, long long hw, int c, int kv) {
    const long long cq = (c + 255) / 256;
    long long k = kv;
    while ((long long)n * cq * k < 1024 && k * 2 * 16 <= hw && k < 256) k *= 2;
    return (int)k;
}

// One launch (moments + apply in one block per plane and channel group) for planes of at most
// S2V_TUNE_IN_FUSED pixels (0: never), the channel group narrowed to 16 - 32 channels so the launch
// has >= 512 blocks where it can (LNet 12^2: 16 x 1024 channels -> 512 blocks of 32 channels; 24^2:
// 256 blocks of 16): the stats pass, its launch and the dependency gap before the apply go away.
// (r02's form, one block per 256 channels — 64 blocks at 12^2 — measured slower than two launches.)
static int in_fused_qb(int n, int hw, int c) {
    if (hw > tune_get(S2V_TUNE_IN_FUSED)) return 0;
    int qb = c / 4 < 64 ? c / 4 : 64;
    while (qb > 4 && (long long)n * cdiv(c, 4 * qb) < 512) qb /= 2;
    return qb;
}

// ------------------------------------------------------------------ token LayerNorm
__global__ __launch_bounds__(256) void row_ln(const float *__restrict__ x, int rows, int dim, int xld,
                                              const float *__restrict__ w, const float *__restrict__ b, float eps,
                                              float *__restrict__ y, int yld) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float *xr = x + (long long)row * xld;
    float s = 0.f;
    for (int i = lane; i < dim; i += 64) s += xr[i];
    const float mean = wave_sumf(s) / dim;
    float q = 0.f;
    for (int i = lane; i < dim; i += 64) {
        const float d = xr[i] - mean;
        q += d * d;
    }
    const float rstd = rsqrtf(wave_sumf(q) / dim + eps);
    float *yr = y + (long long)row * yld;
    for (int i = lane; i < dim; i += 64) yr[i] = (xr[i] - mean) * rstd * w[i] + b[i];
}

// ------------------------------------------------------------------ ADAIN heads / demod
__global__ __launch_bounds__(256) void adain_heads(const float *__restrict__ hid, int batch, int hid_ns, int nh,
                                                   const float *__restrict__ w2t, const float *__restrict__ bias,
                                                   const int *__restrict__ seg, int total, float *__restrict__ out,
                                                   int out_ns) {
    constexpr int BB = 8;
    const int o = blockIdx.x * 256 + threadIdx.x;
    const int b0 = blockIdx.y * BB;
    if (o >= total) return;
    const int sg = seg[o];
    float acc[BB];
#pragma unroll
    for (int i = 0; i < BB; ++i) acc[i] = 0.f;
    // unrolled so the loads of several hidden units are in flight together (one dependent L2 round
    // trip per unit made this GEMV latency-bound: 222 us for 26 MB of weights)
#pragma unroll 8
    for (int j = 0; j < nh; ++j) {
        const float wv = w2t[(long long)j * total + o];
#pragma unroll
        for (int i = 0; i < BB; ++i)
            if (b0 + i < batch) acc[i] = fmaf(wv, hid[(long long)(b0 + i) * hid_ns + (long long)sg * nh + j], acc[i]);
    }
    const float bb = bias ? bias[o] : 0.f;
#pragma unroll
    for (int i = 0; i < BB; ++i)
        if (b0 + i < batch) out[(long long)(b0 + i) * out_ns + o] = acc[i] + bb;
}

// ADAIN heads v2: a block owns 64 consecutive outputs and a chunk of <= 16 samples; its 4 waves split
// the hidden units (wave q: units [q nh / 4, (q + 1) nh / 4)), lane = output, so every weight row
// piece is one coalesced 256-byte load and the weights are read once per 16 samples.  The hidden
// vectors of the (few) segments the block's outputs use are staged in LDS as [segment][unit][sample],
// read as float4 broadcasts; the four partial sums meet in LDS.  (v1 read 8 samples' hidden values
// from global memory per weight load: 264 us for 26 MB of weights, r03.)
// SEGW x NHMAX: the staged window (4 segments of <= 128 units: LNet's ADAIN heads; 1 segment of <= 512
// units: GFPGAN's per-layer style modulations, one 512-d latent per decoder layer)
constexpr int ADAIN_BO = 64, ADAIN_NB = 16, ADAIN_NHMAX = 128, ADAIN_NHMAX_WIDE = 512;
template <int ADAIN_SEGW, int NHMAX>
__global__ __launch_bounds__(256) void adain_heads2(const float *__restrict__ hid, int batch, int hid_ns, int nh,
                                                    const float *__restrict__ w2t, const float *__restrict__ bias,
                                                    const int *__restrict__ seg, int total, float *__restrict__ out,
                                                    int out_ns) {
    __shared__ __attribute__((aligned(16))) float hs[ADAIN_SEGW][NHMAX][ADAIN_NB];
    __shared__ float part[4][ADAIN_NB][ADAIN_BO + 1];
    __shared__ int srange[2];
    const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
    const int o0 = blockIdx.x * ADAIN_BO, b0 = blockIdx.y * ADAIN_NB;
    const int nb = min(ADAIN_NB, batch - b0);
    const int o = o0 + lane;
    const bool ok = o < total;
    const int sg = ok ? seg[o] : 0x7fffffff;
    if (q == 0) {
        int lo = sg, hi = ok ? sg : -1;
        for (int d = 32; d > 0; d >>= 1) {
            lo = min(lo, __shfl_xor(lo, d));
            hi = max(hi, __shfl_xor(hi, d));
        }
        if (lane == 0) { srange[0] = lo; srange[1] = hi; }
    }
    __syncthreads();
    const int smin = srange[0], smax = srange[1];
    const int j0 = q * nh / 4, j1 = (q + 1) * nh / 4;
    float acc[ADAIN_NB];
#pragma unroll
    for (int i = 0; i < ADAIN_NB; ++i) acc[i] = 0.f;
    for (int w0 = smin; w0 <= smax; w0 += ADAIN_SEGW) {
        if (w0 > smin) __syncthreads();                 // previous window's reads done
        const int ns = min(ADAIN_SEGW, smax - w0 + 1);
        for (int e = tid; e < ns * nh * ADAIN_NB; e += 256) {
            const int b = e % ADAIN_NB, j = (e / ADAIN_NB) % nh, s = e / (ADAIN_NB * nh);
            hs[s][j][b] = b < nb ? hid[(long long)(b0 + b) * hid_ns + (long long)(w0 + s) * nh + j] : 0.f;
        }
        __syncthreads();
        if (ok && sg >= w0 && sg < w0 + ns) {
            const float *hr = &hs[sg - w0][0][0];
            const float *wp = w2t + o;
#pragma unroll 8
            for (int j = j0; j < j1; ++j) {
                const float wv = wp[(long long)j * total];
                const float4 h0 = *(const float4 *)(hr + j * ADAIN_NB), h1 = *(const float4 *)(hr + j * ADAIN_NB + 4);
                const float4 h2 = *(const float4 *)(hr + j * ADAIN_NB + 8), h3 = *(const float4 *)(hr + j * ADAIN_NB + 12);
                acc[0] = fmaf(wv, h0.x, acc[0]); acc[1] = fmaf(wv, h0.y, acc[1]);
                acc[2] = fmaf(wv, h0.z, acc[2]); acc[3] = fmaf(wv, h0.w, acc[3]);
                acc[4] = fmaf(wv, h1.x, acc[4]); acc[5] = fmaf(wv, h1.y, acc[5]);
                acc[6] = fmaf(wv, h1.z, acc[6]); acc[7] = fmaf(wv, h1.w, acc[7]);
                acc[8] = fmaf(wv, h2.x, acc[8]); acc[9] = fmaf(wv, h2.y, acc[9]);
                acc[10] = fmaf(wv, h2.z, acc[10]); acc[11] = fmaf(wv, h2.w, acc[11]);
                acc[12] = fmaf(wv, h3.x, acc[12]); acc[13] = fmaf(wv, h3.y, acc[13]);
                acc[14] = fmaf(wv, h3.z, acc[14]); acc[15] = fmaf(wv, h3.w, acc[15]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < ADAIN_NB; ++i) part[q][i][lane] = acc[i];
    __syncthreads();
    // 64 outputs x nb samples: thread t sums the four partials of (sample t / 64 + 4 k, output t % 64)
    const float bb = ok && bias ? bias[o] : 0.f;
    for (int i = q; i < nb; i += 4) {
        const float v = part[0][i][lane] + part[1][i][lane] + part[2][i][lane] + part[3][i][lane];
        if (ok) out[(long long)(b0 + i) * out_ns + o] = v + bb;
    }
}

// One wave per output channel o; lanes stride over cin (coalesced rows of wsq), each lane keeps
// the partial sums of up to 16 samples so a wsq row is read once for the whole batch chunk.  The
// loads of a 256-wide chunk of the row (4 per lane) are issued together: the first version walked
// the row 64 values at a time with every load behind the previous FMA (18 us for a 512 x 512 layer,
// all latency, profiles/r05_hbm_enhance.json).
constexpr int DEMOD_NB = 16;
__device__ __forceinline__ void demod_row(const float *__restrict__ s, int batch, int s_ns, int cin,
                                          const float *__restrict__ wr, float eps, float post,
                                          float *__restrict__ d, int d_ns, int o, int lane) {
    for (int b0 = 0; b0 < batch; b0 += DEMOD_NB) {
        const int nb = min(DEMOD_NB, batch - b0);
        float acc[DEMOD_NB];
#pragma unroll
        for (int j = 0; j < DEMOD_NB; ++j) acc[j] = 0.f;
        for (int i0 = 0; i0 < cin; i0 += 256) {
            float w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u * 64 + lane;
                w[u] = i < cin ? wr[i] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < DEMOD_NB; ++j) {
                if (j < nb) {
                    const float *sr = s + (long long)(b0 + j) * s_ns;
                    float v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = i0 + u * 64 + lane;
                        v[u] = i < cin ? sr[i] : 0.f;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc[j] = fmaf(v[u] * v[u], w[u], acc[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < DEMOD_NB; ++j) {
            float v = acc[j];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0 && j < nb) d[(long long)(b0 + j) * d_ns + o] = rsqrtf(v + eps) * post;
        }
    }
}

__global__ __launch_bounds__(256) void demod_kernel(const float *__restrict__ s, int batch, int s_ns, int cin,
                                                    const float *__restrict__ wsq, int cout, float eps, float post,
                                                    float *__restrict__ d, int d_ns) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= cout) return;
    demod_row(s, batch, s_ns, cin, wsq + (long long)o * cin, eps, post, d, d_ns, o, threadIdx.x & 63);
}

// Every demodulated layer of a StyleGAN2 decoder in one launch: output row r of the concatenated
// demodulation vector (row r of layer l is channel r - r0_l of l) reads its modulation s at column
// rows[r].x of the style bank, rows[r].y input channels, and its squared-weight row at wsq + rows[r].z.
__global__ __launch_bounds__(256) void demod_rows_kernel(const float *__restrict__ s, int batch, int s_ns,
                                                         const int4 *__restrict__ rows, int nrows,
                                                         const float *__restrict__ wsq, float eps, float post,
                                                         float *__restrict__ d, int d_ns) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= nrows) return;
    const int4 t = rows[r];
    demod_row(s + t.x, batch, s_ns, t.y, wsq + (unsigned)t.z, eps, post, d, d_ns, r, threadIdx.x & 63);
}

}  // namespace s2v

using namespace s2v;

extern "C" size_t s2v_layernorm2d_ws_bytes(int n, int h, int w, int c) {
    return (size_t)n * ln_blocks((long long)h * w * c) * 2 * sizeof(double);
}

extern "C" int s2v_layernorm2d(const float *x, int n, int h, int w, int c, int xcs, const float *weight,
                               const float *bias, float eps, int act, float alpha, int pool, const float *res,
                               int res_cs, float *y, int ycs, void *ws, size_t ws_bytes, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && weight && bias && n > 0 && h > 0 && w > 0 && c > 0, "layernorm2d: bad args");
    S2V_REQUIRE(xcs >= c && ycs >= c && (!res || res_cs >= c), "layernorm2d: bad strides");
    S2V_REQUIRE(!pool || (h >= 2 && w >= 2), "layernorm2d: pool needs h,w >= 2");
    const int nblk = ln_blocks((long long)h * w * c);
    const size_t need = (size_t)n * nblk * 2 * sizeof(double);
    if (!ws || ws_bytes < need) {
        set_error("layernorm2d: workspace of %zu bytes required", need);
        return S2V_E_WORKSPACE;
    }
    hipStream_t s = (hipStream_t)stream;
    ln_stats<<<dim3(nblk, n), 256, 0, s>>>(x, h * w, c, xcs, nblk, (double *)ws);
    int rc = check_launch("ln_stats");
    if (rc) return rc;
    const bool vec = c % 4 == 0 && xcs % 4 == 0 && ycs % 4 == 0 && (!res || res_cs % 4 == 0) &&
                     ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)weight % 16) == 0 &&
                     ((uintptr_t)bias % 16) == 0 && (!res || ((uintptr_t)res % 16) == 0) &&
                     (long long)h * w * (c / 4) < (1LL << 31);
    if (vec && pool) {
        ln_apply4_pool<<<dim3(cdiv((long long)(h / 2) * (w / 2) * (c / 4), 256), n), 256, 0, s>>>(
            x, h, w, c / 4, xcs, weight, bias, eps, act, alpha, res, res_cs, y, ycs, (const double *)ws, nblk);
        return check_launch("ln_apply");
    }
    if (vec) {
        ln_apply4<<<dim3(ln_apply_blocks((long long)h * w * (c / 4), n, LN_EPT), n), 256, 0, s>>>(
            x, h * w, c / 4, xcs, weight, bias, eps, act, alpha, res, res_cs, y, ycs, (const double *)ws, nblk);
        return check_launch("ln_apply");
    }
    const long long out = (long long)(pool ? (h / 2) * (w / 2) : h * w) * c;
    unsigned gx = cdiv(out, 256 * 4);
    if (gx > 1024) gx = 1024;
    ln_apply<<<dim3(gx, n), 256, 0, s>>>(x, h, w, c, xcs, weight, bias, eps, act, alpha, pool, res, res_cs, y, ycs,
                                         (const double *)ws, nblk);
    return check_launch("ln_apply");
}

extern "C" size_t s2v_instnorm_ws_bytes(int n, int h, int w, int c) {
    const long long hw = (long long)h * w;
    const int k = in_chunks(hw) > in_chunks_v(n, hw, c) ? in_chunks(hw) : in_chunks_v(n, hw, c);
    return (size_t)n * c * k * 2 * sizeof(double);
}

extern "C" int s2v_instnorm_adain(const float *x, int n, int h, int w, int c, int xcs, const float *gamma,
                                  const float *beta, int gb_ns, float eps, int act, float alpha, const float *res,
                                  int res_cs, float *y, int ycs, void *ws, size_t ws_bytes, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && c > 0, "instnorm: bad args");
    S2V_REQUIRE(xcs >= c && ycs >= c && (!res || res_cs >= c), "instnorm: bad strides");
    const int hw = h * w;
    const int chunks = in_chunks(hw);
    const size_t need = (size_t)n * c * chunks * 2 * sizeof(double);
    if (!ws || ws_bytes < need) {
        set_error("instnorm: workspace of %zu bytes required", need);
        return S2V_E_WORKSPACE;
    }
    hipStream_t s = (hipStream_t)stream;
    const bool vec = c % 4 == 0 && xcs % 4 == 0 && ycs % 4 == 0 && (!res || res_cs % 4 == 0) &&
                     ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 && (!res || ((uintptr_t)res % 16) == 0);
    if (vec) {
        const int kv = in_chunks_v(n, hw, c);
        const size_t needv = (size_t)n * c * kv * 2 * sizeof(double);
        if (ws_bytes < needv) {
            set_error("instnorm: workspace of %zu bytes required", needv);
            return S2V_E_WORKSPACE;
        }
        const int qb = c / 4 < 64 ? c / 4 : 64;
        const unsigned cq = cdiv(c, 4 * qb);
        if (const int qf = in_fused_qb(n, hw, c)) {
            in_apply_v<<<dim3(1, cdiv(c, 4 * qf), n), 256, 0, s>>>(x, hw, c, xcs, gamma, beta, gb_ns, eps, act, alpha,
                                                                   res, res_cs, y, ycs, nullptr, 1, 1, 0, nullptr, 0,
                                                                   qf);
            return check_launch("in_apply");
        }
        in_stats_v<<<dim3(kv, cq, n), 256, 0, s>>>(x, hw, c, xcs, kv, (double *)ws);
        int rc = check_launch("in_stats");
        if (rc) return rc;
        const int ka = in_apply_chunks(n, hw, c, kv);
        in_apply_v<<<dim3(ka, cq, n), 256, 0, s>>>(x, hw, c, xcs, gamma, beta, gb_ns, eps, act, alpha, res, res_cs,
                                                    y, ycs, (const double *)ws, kv, ka);
        return check_launch("in_apply");
    }
    const unsigned cg = cdiv(c, 64);
    in_stats<<<dim3(chunks, cg, n), 256, 0, s>>>(x, hw, c, xcs, chunks, (double *)ws);
    int rc = check_launch("in_stats");
    if (rc) return rc;
    in_apply<<<dim3(chunks, cg, n), 256, 0, s>>>(x, hw, c, xcs, gamma, beta, gb_ns, eps, act, alpha, res, res_cs, y,
                                                 ycs, (const double *)ws, chunks, chunks);
    return check_launch("in_apply");
}

extern "C" int s2v_instnorm_adain_pad(const float *x, int n, int h, int w, int c, int xcs, const float *gamma,
                                      const float *beta, int gb_ns, float eps, int act, float alpha, const float *res,
                                      int res_cs, float *y, int ycs, float *yp, int ypcs, void *ws, size_t ws_bytes,
                                      s2v_stream_t stream) {
    S2V_REQUIRE(x && y && yp && n > 0 && h >= 2 && w >= 2 && c > 0, "instnorm_pad: bad args");
    S2V_REQUIRE(xcs >= c && ycs >= c && ypcs >= c && (!res || res_cs >= c), "instnorm_pad: bad strides");
    const bool vec = c % 4 == 0 && xcs % 4 == 0 && ycs % 4 == 0 && ypcs % 4 == 0 && (!res || res_cs % 4 == 0) &&
                     ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)yp % 16) == 0 &&
                     (!res || ((uintptr_t)res % 16) == 0);
    S2V_REQUIRE(vec, "instnorm_pad: needs c %% 4 == 0, 4-aligned pitches and 16-byte aligned tensors");
    const int hw = h * w;
    const int kv = in_chunks_v(n, hw, c);
    const size_t need = (size_t)n * c * kv * 2 * sizeof(double);
    if (!ws || ws_bytes < need) {
        set_error("instnorm_pad: workspace of %zu bytes required", need);
        return S2V_E_WORKSPACE;
    }
    hipStream_t s = (hipStream_t)stream;
    const int qb = c / 4 < 64 ? c / 4 : 64;
    const unsigned cq = cdiv(c, 4 * qb);
    if (const int qf = in_fused_qb(n, hw, c)) {
        in_apply_v<<<dim3(1, cdiv(c, 4 * qf), n), 256, 0, s>>>(x, hw, c, xcs, gamma, beta, gb_ns, eps, act, alpha, res,
                                                               res_cs, y, ycs, nullptr, 1, 1, w, yp, ypcs, qf);
        return check_launch("in_apply");
    }
    in_stats_v<<<dim3(kv, cq, n), 256, 0, s>>>(x, hw, c, xcs, kv, (double *)ws);
    int rc = check_launch("in_stats");
    if (rc) return rc;
    const int ka = in_apply_chunks(n, hw, c, kv);
    in_apply_v<<<dim3(ka, cq, n), 256, 0, s>>>(x, hw, c, xcs, gamma, beta, gb_ns, eps, act, alpha, res, res_cs, y, ycs,
                                                (const double *)ws, kv, ka, w, yp, ypcs);
    return check_launch("in_apply");
}

extern "C" int s2v_row_layernorm(const float *x, int rows, int dim, int xld, const float *weight, const float *bias,
                                 float eps, float *y, int yld, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && weight && bias && rows > 0 && dim > 0 && xld >= dim && yld >= dim, "row_layernorm: bad args");
    row_ln<<<cdiv(rows, 4), 256, 0, (hipStream_t)stream>>>(x, rows, dim, xld, weight, bias, eps, y, yld);
    return check_launch("row_ln");
}

extern "C" int s2v_adain_params(const float *hid, int batch, int hid_ns, int nhidden, const float *w2t,
                                const float *bias, const int *seg, int total, float *out, int out_ns,
                                s2v_stream_t stream) {
    S2V_REQUIRE(hid && w2t && seg && out && batch > 0 && nhidden > 0 && total > 0 && out_ns >= total,
                "adain_params: bad args");
    if (nhidden <= ADAIN_NHMAX) {
        adain_heads2<4, ADAIN_NHMAX><<<dim3(cdiv(total, ADAIN_BO), cdiv(batch, ADAIN_NB)), 256, 0, (hipStream_t)stream>>>(
            hid, batch, hid_ns, nhidden, w2t, bias, seg, total, out, out_ns);
        return check_launch("adain_heads2");
    }
    if (nhidden <= ADAIN_NHMAX_WIDE) {
        adain_heads2<1, ADAIN_NHMAX_WIDE><<<dim3(cdiv(total, ADAIN_BO), cdiv(batch, ADAIN_NB)), 256, 0,
                                            (hipStream_t)stream>>>(hid, batch, hid_ns, nhidden, w2t, bias, seg, total,
                                                                   out, out_ns);
        return check_launch("adain_heads2");
    }
    adain_heads<<<dim3(cdiv(total, 256), cdiv(batch, 8)), 256, 0, (hipStream_t)stream>>>(
        hid, batch, hid_ns, nhidden, w2t, bias, seg, total, out, out_ns);
    return check_launch("adain_heads");
}

extern "C" int s2v_modconv_demod(const float *s, int batch, int s_ns, int cin, const float *wsq, int cout, float eps,
                                 float post, float *d, int d_ns, s2v_stream_t stream) {
    S2V_REQUIRE(s && wsq && d && batch > 0 && cin > 0 && cout > 0 && s_ns >= cin && d_ns >= cout,
                "modconv_demod: bad args");
    demod_kernel<<<cdiv(cout, 4), 256, 0, (hipStream_t)stream>>>(s, batch, s_ns, cin, wsq, cout, eps, post, d,
                                                                 d_ns);
    return check_launch("demod");
}

extern "C" int s2v_modconv_demod_rows(const float *s, int batch, int s_ns, const int *rows, int nrows,
                                      const float *wsq, float eps, float post, float *d, int d_ns,
                                      s2v_stream_t stream) {
    S2V_REQUIRE(s && rows && wsq && d && batch > 0 && nrows > 0 && d_ns >= nrows && ((uintptr_t)rows % 16) == 0,
                "modconv_demod_rows: bad args");
    demod_rows_kernel<<<cdiv(nrows, 4), 256, 0, (hipStream_t)stream>>>(s, batch, s_ns, (const int4 *)rows, nrows,
                                                                       wsq, eps, post, d, d_ns);
    return check_launch("demod_rows");
}
