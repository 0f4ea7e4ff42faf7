// ENet / StyleGAN2 ToRGB with its skip upsample in one HBM pass (models/base_blocks.py:536-554:
// ToRGB = ModulatedConv2d(C, 3, 1, demodulate=False) + bias, then + F.interpolate(skip, x2,
// bilinear); ENet.py:119-129 calls it once per decoder stage).
//
//   y[b, p, o] = (sum_c W[o][c] * s[b][c] * x[b, p, c] + bias[o]) + up2(skip)[b, p, o]   o < 3
//   y[b, p, 3] = up2(skip)[b, p, 3]                 (the engine's 4th, float4-padding channel)
//
// The separate path wrote the upsampled skip (16 B / px), then the small-Cout conv read it back as
// its residual and wrote 3 scattered floats per pixel.  Here TPP lanes share a pixel and each owns
// C / TPP channels as float4s (a wave reads 64 / TPP pixel rows, 128-byte pieces), every thread
// carries PPT pixels so ~16 float4 loads are in flight, the modulated 3 x C filter (W * s[b], the
// reference's weight-then-conv order) is built once per block in LDS, partial sums meet by xor
// shuffles, and one lane per pixel reads the 2 x 2 skip taps and writes the pixel as one float4.
// Bound: HBM (C * 4 bytes read + 16 written per output pixel).
#include "common.hpp"

namespace s2v {

// torch upsample_bilinear2d (align_corners=False) source index / weights: the resize kernels' rule
__device__ __forceinline__ void up2_index(int dst, int in, int &i0, int &i1, float &l0, float &l1) {
    float src = 0.5f * ((float)dst + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    i0 = (int)src;
    i1 = i0 + ((i0 < in - 1) ? 1 : 0);
    l1 = src - (float)i0;
    l0 = 1.f - l1;
}

template <int TPP, int PPT>
__global__ __launch_bounds__(256) void torgb_up2_kernel(const float *__restrict__ x, int C, int H, int W, int xcs,
                                                        const float *__restrict__ wt, int kpad,
                                                        const float *__restrict__ s, int s_ns,
                                                        const float *__restrict__ bias,
                                                        const float *__restrict__ skip, int skcs,
                                                        float *__restrict__ y, int ycs) {
    extern __shared__ __attribute__((aligned(16))) float wm[];      // [3][C]
    constexpr int SLOTS = 256 / TPP, PB = SLOTS * PPT;             // pixels per block
    const int hw = H * W;
    const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
    const long long q0 = (long long)blk * PB;                       // first (b, p) of the block
    const int b = (int)(q0 / hw);                                   // the host keeps a block in one sample
    for (int e = threadIdx.x; e < 3 * C; e += 256) {
        const int o = e / C, c = e - o * C;
        wm[e] = wt[(long long)o * kpad + c] * s[(long long)b * s_ns + c];
    }
    __syncthreads();
    const int sub = threadIdx.x % TPP, slot = threadIdx.x / TPP;
    const float *xb = x + (long long)b * hw * xcs;
    const int p0 = (int)(q0 - (long long)b * hw) + slot;
    float acc[PPT][3];
#pragma unroll
    for (int i = 0; i < PPT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = 0.f;
    for (int c = sub * 4; c < C; c += 4 * TPP) {
        const float4 w0 = *(const float4 *)&wm[c], w1 = *(const float4 *)&wm[C + c], w2 = *(const float4 *)&wm[2 * C + c];
        float4 v[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) v[i] = *(const float4 *)(xb + (long long)(p0 + i * SLOTS) * xcs + c);
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            acc[i][0] = fmaf(v[i].x, w0.x, fmaf(v[i].y, w0.y, fmaf(v[i].z, w0.z, fmaf(v[i].w, w0.w, acc[i][0]))));
            acc[i][1] = fmaf(v[i].x, w1.x, fmaf(v[i].y, w1.y, fmaf(v[i].z, w1.z, fmaf(v[i].w, w1.w, acc[i][1]))));
            acc[i][2] = fmaf(v[i].x, w2.x, fmaf(v[i].y, w2.y, fmaf(v[i].z, w2.z, fmaf(v[i].w, w2.w, acc[i][2]))));
        }
    }
#pragma unroll
    for (int i = 0; i < PPT; ++i)
#pragma unroll
        for (int o = 0; o < 3; ++o)
#pragma unroll
            for (int off = TPP / 2; off > 0; off >>= 1) acc[i][o] += __shfl_xor(acc[i][o], off, 64);
    // lane sub == i of the pixel's group finishes pixel i (every lane holds every sum after the butterfly)
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        if (sub != i % TPP) continue;
        const int p = p0 + i * SLOTS;
        const int oy = p / W, ox = p - (p / W) * W;
        const int sh = H / 2, sw = W / 2;
        int y0, y1, x0, x1;
        float ly0, ly1, lx0, lx1;
        up2_index(oy, sh, y0, y1, ly0, ly1);
        up2_index(ox, sw, x0, x1, lx0, lx1);
        const float *sb = skip + (long long)b * sh * sw * skcs;
        const float4 ta = *(const float4 *)(sb + ((long long)y0 * sw + x0) * skcs);
        const float4 tb = *(const float4 *)(sb + ((long long)y0 * sw + x1) * skcs);
        const float4 tc = *(const float4 *)(sb + ((long long)y1 * sw + x0) * skcs);
        const float4 td = *(const float4 *)(sb + ((long long)y1 * sw + x1) * skcs);
        float4 u;
        u.x = ly0 * (lx0 * ta.x + lx1 * tb.x) + ly1 * (lx0 * tc.x + lx1 * td.x);
        u.y = ly0 * (lx0 * ta.y + lx1 * tb.y) + ly1 * (lx0 * tc.y + lx1 * td.y);
        u.z = ly0 * (lx0 * ta.z + lx1 * tb.z) + ly1 * (lx0 * tc.z + lx1 * td.z);
        u.w = ly0 * (lx0 * ta.w + lx1 * tb.w) + ly1 * (lx0 * tc.w + lx1 * td.w);
        float4 r;
        r.x = (acc[i][0] + (bias ? bias[0] : 0.f)) + u.x;
        r.y = (acc[i][1] + (bias ? bias[1] : 0.f)) + u.y;
        r.z = (acc[i][2] + (bias ? bias[2] : 0.f)) + u.z;
        r.w = u.w;
        *(float4 *)(y + ((long long)b * hw + p) * ycs) = r;
    }
}

template <int PPT>
static void launch_torgb(unsigned grid, size_t smem, const float *x, int c, int h, int w, int xcs, const float *wt,
                         int kpad, const float *s, int s_ns, const float *bias, const float *skip, int skcs, float *y,
                         int ycs, hipStream_t st) {
    torgb_up2_kernel<8, PPT><<<grid, 256, smem, st>>>(x, c, h, w, xcs, wt, kpad, s, s_ns, bias, skip, skcs, y, ycs);
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_torgb_up2(const float *x, int n, int h, int w, int c, int xcs, const float *wt, int kpad,
                             const float *s, int s_ns, const float *bias, const float *skip, int skcs, float *y,
                             int ycs, s2v_stream_t stream) {
    S2V_REQUIRE(x && wt && s && skip && y && n > 0 && h > 1 && w > 1 && c > 0, "torgb_up2: bad args");
    S2V_REQUIRE(h % 2 == 0 && w % 2 == 0, "torgb_up2: output %dx%d must be twice the skip size", h, w);
    S2V_REQUIRE(c % 32 == 0 && xcs % 4 == 0 && xcs >= c && kpad >= c && s_ns >= c && skcs % 4 == 0 && skcs >= 4 &&
                    ycs % 4 == 0 && ycs >= 4,
                "torgb_up2: C %% 32 == 0, 4-channel skip / output, float4 pitches required");
    S2V_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)skip % 16) == 0 && ((uintptr_t)y % 16) == 0,
                "torgb_up2: 16-byte aligned x / skip / y");
    const long long hw = (long long)h * w, total = (long long)n * hw;
    // ~16 float4 loads in flight per thread: C / 32 per pixel per lane
    int ppt = 16 / (c / 32);
    if (ppt < 1) ppt = 1;
    if (ppt > 4) ppt = 4;
    while (ppt > 1 && hw % (32LL * ppt) != 0) ppt >>= 1;
    S2V_REQUIRE(hw % (32LL * ppt) == 0, "torgb_up2: h * w must be a multiple of 32 (blocks stay in one sample)");
    const unsigned grid = (unsigned)(total / (32LL * ppt));
    const size_t smem = (size_t)3 * c * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    switch (ppt) {
        case 4: launch_torgb<4>(grid, smem, x, c, h, w, xcs, wt, kpad, s, s_ns, bias, skip, skcs, y, ycs, st); break;
        case 2: launch_torgb<2>(grid, smem, x, c, h, w, xcs, wt, kpad, s, s_ns, bias, skip, skcs, y, ycs, st); break;
        default: launch_torgb<1>(grid, smem, x, c, h, w, xcs, wt, kpad, s, s_ns, bias, skip, skcs, y, ycs, st); break;
    }
    return check_launch("torgb_up2");
}
