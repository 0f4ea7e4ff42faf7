// Mouth-region post-process: the kernels of inference.py:302-313 that follow
// ENet + GFPGAN — FaceParse's input conversion and mask (face_parsing.py:39-81), every cv2.resize
// of that block, and Laplacian_Pyramid_Blending_with_mask (futils/inference_utils.py:181-222).
//
// OpenCV (imgproc pyramids.cpp / resize.cpp, BORDER_DEFAULT = reflect-101) is restated here from its
// documented integer / float formulas; oracle/post.py is the NumPy restatement the tests compare
// against bit for bit.  Every float operation is rounded on its own (no FMA contraction) in the
// order the restatement uses.
//
// Laplacian blend:
//   gA[0] = A (uint8), gA[k+1] = pyrDown(gA[k]) kept in uint8 (5x5 [1 4 6 4 1]^2 integer sum,
//   (s + 128) >> 8), gM likewise in fp32 (row pass, column pass, x 1/256);
//   LS[L-1] = gA[L-1] * gM[L-1] + gB[L-1] * (1 - gM[L-1]);
//   LS[i-1] = (gA[i-1] - pyrUp(gA[i])) * gM[i-1] + (gB[i-1] - pyrUp(gB[i])) * (1 - gM[i-1]);
//   out = pyrUp(... pyrUp(LS[L-1]) + LS[L-2] ...) + LS[0]
// One kernel per level computes the Laplacian terms and the reconstruction step of that level
// (each output pixel evaluates pyrUp(ls_i) + LS[i-1] directly), so no Laplacian level is stored.
#include "common.hpp"

// HIP device code contracts a*b + c into FMAs by default: every float expression in this file is
// evaluated unfused, as NumPy / OpenCV's scalar path evaluate it
#pragma clang fp contract(off)

namespace s2v {

// cv::borderInterpolate(BORDER_REFLECT_101) for any offset (tiny pyramid levels reflect twice)
__device__ __forceinline__ int bi101(int p, int n) {
    if (n == 1) return 0;
    while ((unsigned)p >= (unsigned)n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}
// plain operators under contract(off): the __fmul_rn family is defined in the HIP headers, outside
// this pragma, and its bodies stay contractable after inlining
__device__ __forceinline__ float fm(float a, float b) { return a * b; }
__device__ __forceinline__ float fa(float a, float b) { return a + b; }
__device__ __forceinline__ float fs(float a, float b) { return a - b; }

__device__ __forceinline__ float ldf(const unsigned char *p) { return (float)*p; }
__device__ __forceinline__ float ldf(const float *p) { return *p; }

// ------------------------------------------------------------------------------- pyramids
// pyrDown of uint8 HWC images: exact integer arithmetic
__global__ __launch_bounds__(256) void pyr_down_u8_kernel(const unsigned char *__restrict__ x, int n, int h, int w,
                                                          int c, unsigned char *__restrict__ y, int oh, int ow) {
    const long long total = (long long)n * oh * ow * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int ch = (int)(e % c);
        long long t = e / c;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int b = (int)(t / oh);
        const unsigned char *xb = x + (long long)b * h * w * c + ch;
        int cx[5];
#pragma unroll
        for (int d = 0; d < 5; ++d) cx[d] = bi101(2 * ox + d - 2, w) * c;
        int acc = 0;
#pragma unroll
        for (int dy = 0; dy < 5; ++dy) {
            const unsigned char *r = xb + (long long)bi101(2 * oy + dy - 2, h) * w * c;
            const int s = r[cx[2]] * 6 + (r[cx[1]] + r[cx[3]]) * 4 + r[cx[0]] + r[cx[4]];
            acc += (dy == 2 ? 6 : (dy == 1 || dy == 3) ? 4 : 1) * s;
        }
        y[e] = (unsigned char)min((acc + 128) >> 8, 255);
    }
}

// pyrDown of fp32 single-channel masks: per source row r = s2*6 + (s1+s3)*4 + s0 + s4, the same
// over the five row results, then x 1/256
__global__ __launch_bounds__(256) void pyr_down_f32_kernel(const float *__restrict__ x, int n, int h, int w,
                                                           float *__restrict__ y, int oh, int ow) {
    const long long total = (long long)n * oh * ow;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int ox = (int)(e % ow);
        long long t = e / ow;
        const int oy = (int)(t % oh);
        const int b = (int)(t / oh);
        const float *xb = x + (long long)b * h * w;
        int cx[5];
#pragma unroll
        for (int d = 0; d < 5; ++d) cx[d] = bi101(2 * ox + d - 2, w);
        float rv[5];
#pragma unroll
        for (int dy = 0; dy < 5; ++dy) {
            const float *r = xb + (long long)bi101(2 * oy + dy - 2, h) * w;
            rv[dy] = fa(fa(fa(fm(r[cx[2]], 6.f), fm(fa(r[cx[1]], r[cx[3]]), 4.f)), r[cx[0]]), r[cx[4]]);
        }
        const float v = fa(fa(fa(fm(rv[2], 6.f), fm(fa(rv[1], rv[3]), 4.f)), rv[0]), rv[4]);
        y[e] = fm(v, 1.f / 256.f);
    }
}

// Horizontal pyrUp value for destination column X of one source row (w pixels, pitch c):
// OpenCV's edge forms (left even s0*6 + s1*2, right even s[w-2] + s[w-1]*7, right odd s[w-1]*8),
// interior s[x-1] + s[x]*6 + s[x+1] | (s[x] + s[x+1])*4; a one-pixel row is s*8
template <typename T>
__device__ __forceinline__ float up_row(const T *row, int w, int c, int X) {
    if (w == 1) return fm(ldf(row), 8.f);
    const int x = X >> 1;
    const float s0 = ldf(row + (long long)x * c);
    if ((X & 1) == 0) {
        if (x == 0) return fa(fm(s0, 6.f), fm(ldf(row + c), 2.f));
        const float sm = ldf(row + (long long)(x - 1) * c);
        if (x == w - 1) return fa(sm, fm(s0, 7.f));
        return fa(fa(sm, fm(s0, 6.f)), ldf(row + (long long)(x + 1) * c));
    }
    if (x == w - 1) return fm(s0, 8.f);
    return fm(fa(s0, ldf(row + (long long)(x + 1) * c)), 4.f);
}

// pyrUp(src)(Y, X) of one channel (src points at channel ch of image b): the vertical pass reads
// source rows borderInterpolate(2 sy, 2 h) / 2 for sy = y-1, y, y+1;
// even t0 = (R0 + R1*6) + R2, odd t1 = (R1 + R2)*4, then x 1/64
template <typename T>
__device__ __forceinline__ float pyr_up_at(const T *src, int h, int w, int c, int Y, int X) {
    const int y = Y >> 1;
    const long long pitch = (long long)w * c;
    const float r1 = up_row(src + (long long)(bi101(2 * y, 2 * h) >> 1) * pitch, w, c, X);
    const float r2 = up_row(src + (long long)(bi101(2 * y + 2, 2 * h) >> 1) * pitch, w, c, X);
    if ((Y & 1) == 0) {
        const float r0 = up_row(src + (long long)(bi101(2 * y - 2, 2 * h) >> 1) * pitch, w, c, X);
        return fm(fa(fa(r0, fm(r1, 6.f)), r2), 1.f / 64.f);
    }
    return fm(fm(fa(r1, r2), 4.f), 1.f / 64.f);
}

// One level of blend + reconstruction: level i-1 (h x w) from level i (ph x pw).
//   out = (prev ? pyrUp(prev) : 0) + (la * gm + lb * (1 - gm)),
//   la = ga - pyrUp(ga1) (top level: la = ga), lb likewise; the mask broadcasts over channels.
//   clip: np.clip(., 0, 255) of the final image (inference.py:313, face_enhancement.py:188).
__global__ __launch_bounds__(256) void lap_level_kernel(const float *__restrict__ prev,
                                                        const unsigned char *__restrict__ ga,
                                                        const unsigned char *__restrict__ gb,
                                                        const unsigned char *__restrict__ ga1,
                                                        const unsigned char *__restrict__ gb1,
                                                        const float *__restrict__ gm, int n, int h, int w, int c,
                                                        int ph, int pw, int clip, float *__restrict__ out) {
    const long long total = (long long)n * h * w * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int ch = (int)(e % c);
        long long t = e / c;
        const int X = (int)(t % w);
        t /= w;
        const int Y = (int)(t % h);
        const int b = (int)(t / h);
        float la = (float)ga[e], lb = (float)gb[e];
        const long long pofs = (long long)b * ph * pw * c + ch;
        if (ga1) {
            la = fs(la, pyr_up_at(ga1 + pofs, ph, pw, c, Y, X));
            lb = fs(lb, pyr_up_at(gb1 + pofs, ph, pw, c, Y, X));
        }
        const float m = gm[((long long)b * h + Y) * w + X];
        const float ls = fa(fm(la, m), fm(lb, fs(1.f, m)));
        float v = prev ? fa(pyr_up_at(prev + pofs, ph, pw, c, Y, X), ls) : ls;
        if (clip) v = fminf(fmaxf(v, 0.f), 255.f);
        out[e] = v;
    }
}

// ------------------------------------------------------------------------------- resize
// cv2.resize(INTER_LINEAR) on HWC images (resize.cpp resizeGeneric_ + HResizeLinear / VResizeLinear):
//   f = float((d + 0.5) * scale - 0.5), s = floor(f), f -= s; the horizontal pass clamps
//   (s < 0: s = 0, f = 0; s >= w-1: s = w-1, f = 0), the vertical pass only clamps the row index.
//   uint8: weights round((1 - f) * 2048), round(f * 2048); row pass S0*a0 + S1*a1 (int); column
//   pass as OpenCV's vector path: (((D0 >> 4) * b0) >> 16) + (((D1 >> 4) * b1) >> 16), then
//   (v + 2) >> 2 saturated.  fp32: float weights, S0*a0 + S1*a1 and D0*b0 + D1*b1.
// mode 0: u8 -> u8, 1: f32 -> f32, 2: f32 -> u8 truncated (np.uint8 of the float result,
// inference.py:313), 3: u8 -> f32 (v == 255 ? 1 : 0): the mask paste at inference.py:305-308,
// which assigns resized/255. into a uint8 array (so only 255 survives, as 1); 4: f64 -> f64.
template <int MODE>
__global__ __launch_bounds__(256) void resize_linear_kernel(const void *__restrict__ xv, int n, int h, int w, int c,
                                                            long long xrs, long long xis, void *__restrict__ yv,
                                                            int oh, int ow, long long yrs, long long yis,
                                                            double sy, double sx) {
    const long long total = (long long)n * oh * ow * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int ch = (int)(e % c);
        long long t = e / c;
        const int X = (int)(t % ow);
        t /= ow;
        const int Y = (int)(t % oh);
        const int b = (int)(t / oh);
        float fx = (float)((X + 0.5) * sx - 0.5);
        int x0 = (int)floorf(fx);
        fx -= (float)x0;
        if (x0 < 0) { x0 = 0; fx = 0.f; }
        if (x0 >= w - 1) { x0 = w - 1; fx = 0.f; }
        const int x1 = min(x0 + 1, w - 1);
        float fy = (float)((Y + 0.5) * sy - 0.5);
        const int yy = (int)floorf(fy);
        fy -= (float)yy;
        const int y0 = min(max(yy, 0), h - 1), y1 = min(max(yy + 1, 0), h - 1);
        const long long yo = (long long)b * yis + (long long)Y * yrs + (long long)X * c + ch;
        if (MODE == 0 || MODE == 3) {
            const unsigned char *xb = (const unsigned char *)xv + (long long)b * xis + ch;
            const int a0 = __float2int_rn((1.f - fx) * 2048.f), a1 = __float2int_rn(fx * 2048.f);
            const int b0 = __float2int_rn((1.f - fy) * 2048.f), b1 = __float2int_rn(fy * 2048.f);
            const unsigned char *r0 = xb + (long long)y0 * xrs, *r1 = xb + (long long)y1 * xrs;
            const int d0 = r0[x0 * c] * a0 + r0[x1 * c] * a1;
            const int d1 = r1[x0 * c] * a0 + r1[x1 * c] * a1;
            const int v = min(max(((((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16) + 2) >> 2, 0), 255);
            if (MODE == 0) ((unsigned char *)yv)[yo] = (unsigned char)v;
            else ((float *)yv)[yo] = v == 255 ? 1.f : 0.f;
        } else if (MODE == 4) {
            // CV_64F: double sums with the float coefficients (HResizeLinear / VResizeLinear<double, .., float>)
            const double *xb = (const double *)xv + (long long)b * xis + ch;
            const double a0 = (double)(1.f - fx), b0 = (double)(1.f - fy), a1 = (double)fx, b1 = (double)fy;
            const double *r0 = xb + (long long)y0 * xrs, *r1 = xb + (long long)y1 * xrs;
            const double d0 = r0[x0 * c] * a0 + r0[x1 * c] * a1;
            const double d1 = r1[x0 * c] * a0 + r1[x1 * c] * a1;
            ((double *)yv)[yo] = d0 * b0 + d1 * b1;
        } else {
            const float *xb = (const float *)xv + (long long)b * xis + ch;
            const float a0 = 1.f - fx, b0 = 1.f - fy;
            const float *r0 = xb + (long long)y0 * xrs, *r1 = xb + (long long)y1 * xrs;
            const float d0 = fa(fm(r0[x0 * c], a0), fm(r0[x1 * c], fx));
            const float d1 = fa(fm(r1[x0 * c], a0), fm(r1[x1 * c], fx));
            const float v = fa(fm(d0, b0), fm(d1, fy));
            if (MODE == 1) ((float *)yv)[yo] = v;
            else ((unsigned char *)yv)[yo] = (unsigned char)(int)v;
        }
    }
}

// ------------------------------------------------------------------------------- FaceParse
// argmax over the parsing channels (the first maximum wins, like torch.argmax; NaN counts as the
// maximum) -> colormap[class] as uint8 (face_parsing.py:51-55, :65-81) and / or the class index
__global__ __launch_bounds__(256) void parse_mask_kernel(const float *__restrict__ x, int n, long long hw, int c,
                                                         long long xbs, long long ps, long long cs,
                                                         const unsigned char *__restrict__ cmap,
                                                         unsigned char *__restrict__ out, int *__restrict__ cls) {
    const long long total = (long long)n * hw;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long b = e / hw, p = e - b * hw;
        const float *px = x + b * xbs + p * ps;
        float best = px[0];
        int bi = 0;
        for (int k = 1; k < c && best == best; ++k) {
            const float v = px[k * cs];
            if (v > best || v != v) {
                best = v;
                bi = k;
            }
        }
        if (out) out[e] = cmap[bi];
        if (cls) cls[e] = bi;
    }
}

// img2tensor (face_parsing.py:59-63): uint8 HWC BGR -> fp32 RGB in [-1, 1], computed in float64
// like NumPy (img / 255. * 2 - 1) and rounded once to fp32; 4-channel output pixels get 0 in
// channel 3 (the vectorised conv gather's layout)
__global__ __launch_bounds__(256) void img_u8_to_m11_kernel(const unsigned char *__restrict__ x, long long pixels,
                                                            int flip, float *__restrict__ y, int ycs) {
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < pixels; e += (long long)gridDim.x * 256) {
        const unsigned char *px = x + e * 3;
        float *py = y + e * ycs;
#pragma unroll
        for (int j = 0; j < 3; ++j) py[j] = (float)((double)px[flip ? 2 - j : j] / 255.0 * 2.0 - 1.0);
        if (ycs >= 4) py[3] = 0.f;
    }
}

static unsigned grid_for(long long total) {
    long long b = (total + 255) / 256;
    if (b > 65535LL * 16) b = 65535LL * 16;
    return (unsigned)(b < 1 ? 1 : b);
}

static long long align256(long long v) { return (v + 255) / 256 * 256; }

constexpr int kMaxLevels = 30;

// workspace: per level k = 1 .. L-1: gA_k | gB_k (uint8) | gM_k (fp32); then two ping-pong fp32
// buffers of level-1 size for the reconstruction (level 0 is written to ``out``)
static size_t blend_layout(int n, int h, int w, int c, int levels, long long *offs, int *hs, int *wsz) {
    long long off = 0;
    hs[0] = h;
    wsz[0] = w;
    for (int k = 1; k < levels; ++k) {
        hs[k] = (hs[k - 1] + 1) / 2;
        wsz[k] = (wsz[k - 1] + 1) / 2;
        const long long px = (long long)n * hs[k] * wsz[k];
        offs[3 * k] = off;
        off += align256(px * c);
        offs[3 * k + 1] = off;
        off += align256(px * c);
        offs[3 * k + 2] = off;
        off += align256(px * 4);
    }
    const long long l1 = levels > 1 ? (long long)n * hs[1] * wsz[1] * c * 4 : 0;
    offs[0] = off;
    offs[1] = off + align256(l1);
    off += 2 * align256(l1);
    return (size_t)off;
}

}  // namespace s2v

using namespace s2v;

extern "C" size_t s2v_laplacian_blend_ws_bytes(int n, int h, int w, int c, int levels) {
    if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || levels < 1 || levels > kMaxLevels) return 0;
    long long offs[3 * kMaxLevels];
    int hs[kMaxLevels], wsz[kMaxLevels];
    return blend_layout(n, h, w, c, levels, offs, hs, wsz);
}

extern "C" int s2v_laplacian_blend(const unsigned char *a, const unsigned char *b, const float *m, int n, int h, int w,
                                   int c, int levels, int clip, float *out, void *ws, size_t ws_bytes,
                                   s2v_stream_t stream) {
    S2V_REQUIRE(a && b && m && out && n > 0 && h > 0 && w > 0 && c > 0, "laplacian_blend: bad args");
    S2V_REQUIRE(levels >= 1 && levels <= kMaxLevels, "laplacian_blend: levels must be in [1, %d]", kMaxLevels);
    // the reference subtracts pyrUp(level i) (2x its size) from level i-1: sizes must halve exactly
    S2V_REQUIRE(h % (1 << (levels - 1)) == 0 && w % (1 << (levels - 1)) == 0,
                "laplacian_blend: %dx%d is not divisible by 2^(levels-1) = %d (the reference fails there too)", h,
                w, 1 << (levels - 1));
    long long offs[3 * kMaxLevels];
    int hs[kMaxLevels], wsz[kMaxLevels];
    const size_t need = blend_layout(n, h, w, c, levels, offs, hs, wsz);
    S2V_REQUIRE(need == 0 || (ws && ws_bytes >= need), "laplacian_blend: workspace needs %zu bytes", need);
    hipStream_t s = (hipStream_t)stream;
    char *base = (char *)ws;
    auto ga = [&](int k) { return k == 0 ? a : (const unsigned char *)(base + offs[3 * k]); };
    auto gb = [&](int k) { return k == 0 ? b : (const unsigned char *)(base + offs[3 * k + 1]); };
    auto gm = [&](int k) { return k == 0 ? m : (const float *)(base + offs[3 * k + 2]); };
    // Gaussian pyramids, levels 1 .. L-1 (the reference also builds level L, which it never reads)
    for (int k = 1; k < levels; ++k) {
        const long long px = (long long)n * hs[k] * wsz[k];
        pyr_down_u8_kernel<<<grid_for(px * c), 256, 0, s>>>(ga(k - 1), n, hs[k - 1], wsz[k - 1], c,
                                                            (unsigned char *)ga(k), hs[k], wsz[k]);
        pyr_down_u8_kernel<<<grid_for(px * c), 256, 0, s>>>(gb(k - 1), n, hs[k - 1], wsz[k - 1], c,
                                                            (unsigned char *)gb(k), hs[k], wsz[k]);
        pyr_down_f32_kernel<<<grid_for(px), 256, 0, s>>>(gm(k - 1), n, hs[k - 1], wsz[k - 1], (float *)gm(k),
                                                         hs[k], wsz[k]);
    }
    // blend + reconstruct from the top level down
    float *buf[2] = {(float *)(base + offs[0]), (float *)(base + offs[1])};
    const float *prev = nullptr;
    for (int i = levels - 1; i >= 0; --i) {
        float *dst = i == 0 ? out : buf[i & 1];
        const bool top = i == levels - 1;
        lap_level_kernel<<<grid_for((long long)n * hs[i] * wsz[i] * c), 256, 0, s>>>(
            prev, ga(i), gb(i), top ? nullptr : ga(i + 1), top ? nullptr : gb(i + 1), gm(i), n, hs[i], wsz[i], c,
            top ? 1 : hs[i + 1], top ? 1 : wsz[i + 1], i == 0 ? clip : 0, dst);
        prev = dst;
    }
    return check_launch("laplacian_blend");
}

static int resize_linear_scaled(const void *x, int n, int h, int w, int c, long long xrs, long long xis, void *y,
                                int oh, int ow, long long yrs, long long yis, int mode, double sy, double sx,
                                s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0, "resize_linear: bad args");
    S2V_REQUIRE(mode >= 0 && mode <= 4, "resize_linear: bad mode %d", mode);
    S2V_REQUIRE(xrs >= (long long)w * c && yrs >= (long long)ow * c && (n == 1 || (xis >= xrs * h && yis >= yrs * oh)),
                "resize_linear: row / image pitches smaller than the rows / images");
    const unsigned g = grid_for((long long)n * oh * ow * c);
    hipStream_t s = (hipStream_t)stream;
    switch (mode) {
        case 0: resize_linear_kernel<0><<<g, 256, 0, s>>>(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, sy, sx); break;
        case 1: resize_linear_kernel<1><<<g, 256, 0, s>>>(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, sy, sx); break;
        case 2: resize_linear_kernel<2><<<g, 256, 0, s>>>(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, sy, sx); break;
        case 3: resize_linear_kernel<3><<<g, 256, 0, s>>>(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, sy, sx); break;
        default: resize_linear_kernel<4><<<g, 256, 0, s>>>(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, sy, sx); break;
    }
    return check_launch("resize_linear");
}

extern "C" int s2v_resize_linear(const void *x, int n, int h, int w, int c, long long xrs, long long xis, void *y,
                                 int oh, int ow, long long yrs, long long yis, int mode, s2v_stream_t stream) {
    // cv::resize with dsize: inv_scale = dsize / ssize, scale = 1 / inv_scale (both double)
    return resize_linear_scaled(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, mode, 1.0 / ((double)oh / h),
                                1.0 / ((double)ow / w), stream);
}

extern "C" int s2v_resize_linear_fxfy(const void *x, int n, int h, int w, int c, long long xrs, long long xis,
                                      void *y, int oh, int ow, long long yrs, long long yis, int mode, double fx,
                                      double fy, s2v_stream_t stream) {
    // cv::resize(src, (0, 0), fx, fy): dsize = round(size * f), inv_scale = f itself
    S2V_REQUIRE(fx > 0 && fy > 0, "resize_linear_fxfy: scale factors must be positive");
    return resize_linear_scaled(x, n, h, w, c, xrs, xis, y, oh, ow, yrs, yis, mode, 1.0 / fy, 1.0 / fx, stream);
}

extern "C" int s2v_parse_mask(const float *x, int n, int h, int w, int c, long long xbs, long long ps, long long cs,
                              const unsigned char *cmap, unsigned char *out, int *cls, s2v_stream_t stream) {
    S2V_REQUIRE(x && (out || cls) && n > 0 && h > 0 && w > 0 && c > 0, "parse_mask: bad args");
    S2V_REQUIRE(!out || cmap, "parse_mask: the uint8 mask needs a colormap");
    const long long hw = (long long)h * w;
    parse_mask_kernel<<<grid_for(n * hw), 256, 0, (hipStream_t)stream>>>(x, n, hw, c, xbs, ps, cs, cmap, out, cls);
    return check_launch("parse_mask");
}

extern "C" int s2v_img_u8_to_m11(const unsigned char *x, long long pixels, int flip, float *y, int ycs,
                                 s2v_stream_t stream) {
    S2V_REQUIRE(x && y && pixels > 0 && ycs >= 3, "img_u8_to_m11: bad args");
    img_u8_to_m11_kernel<<<grid_for(pixels), 256, 0, (hipStream_t)stream>>>(x, pixels, flip, y, ycs);
    return check_launch("img_u8_to_m11");
}
