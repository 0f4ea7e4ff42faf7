// 3DMM coefficient regression front end (preprocessing/facing.py:100-130,
// third_part/face3d/util/preprocess.py:resize_n_crop_img / align_img, models/networks.py:61-105).
//
//  * pil_resize_crop_kernel: PIL's Image.resize((w, h), BICUBIC | BILINEAR) followed by
//    Image.crop((left, up, left + ow, up + oh)) on uint8 RGB frames, fused: only the pixels the
//    crop keeps are resampled.  The arithmetic is Pillow's (libImaging/Resample.c): per output
//    coordinate the filter taps are evaluated in double (precompute_coeffs), normalised by their
//    running sum, rounded to 22-bit fixed point (normalize_coeffs_8bpc); the horizontal pass
//    rounds every intermediate row to uint8 (clip8) before the vertical pass.  A column's taps do
//    not depend on the row and vice versa, so computing only the kept window is exact.  Pixels of
//    the crop box outside the resized image are 0 (Image.crop's fill).  The output is
//    float32(pixel / 255.) as facing.py:120 builds the network input, NHWC with pitch ycs.
//  * spatial_mean_kernel: AdaptiveAvgPool2d((1, 1)) of the ResNet-50 head on NHWC fp32.
#include "common.hpp"

namespace s2v {

#pragma clang fp contract(off)

constexpr int PIL_PREC = 22;      // PRECISION_BITS = 32 - 8 - 2
constexpr int PIL_KMAX = 48;      // taps per output coordinate: bicubic downscales up to 11.75x

__device__ __forceinline__ double pil_filter(int filter, double x) {
    if (x < 0.0) x = -x;
    if (filter == 3) {            // bicubic_filter, a = -0.5
        const double a = -0.5;
        if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
        if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
        return 0.0;
    }
    if (x < 1.0) return 1.0 - x;  // bilinear_filter
    return 0.0;
}

__device__ __forceinline__ int pil_clip8(int v) {
    v >>= PIL_PREC;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// precompute_coeffs + normalize_coeffs_8bpc for output coordinate xx of an in_size -> out_size
// resample (box 0..in_size): writes the count taps starting at *first, k[i * kstride].  Returns
// false when the filter needs more than PIL_KMAX taps.
__device__ bool pil_coeffs(int filter, int in_size, int out_size, int xx, int *first, int *count, int *k,
                           int kstride) {
    const double fsupport = filter == 3 ? 2.0 : 1.0;
    double scale = (double)in_size / out_size;
    double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = fsupport * filterscale;
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    if (xmax > PIL_KMAX) return false;
    double ww = 0.0;              // the running sum first; the taps are re-evaluated (same values)
    for (int x = 0; x < xmax; ++x) ww += pil_filter(filter, (x + xmin - center + 0.5) * ss);
    for (int x = 0; x < xmax; ++x) {
        double v = pil_filter(filter, (x + xmin - center + 0.5) * ss);
        if (ww != 0.0) v /= ww;
        k[x * kstride] = v < 0 ? (int)(-0.5 + v * (1 << PIL_PREC)) : (int)(0.5 + v * (1 << PIL_PREC));
    }
    *first = xmin;
    *count = xmax;
    return true;
}

// One block per (output row, image).  params[b] = (w, h, left, up).
__global__ __launch_bounds__(256) void pil_resize_crop_kernel(const unsigned char *__restrict__ x, int h0, int w0,
                                                              long long xis, const int *__restrict__ params,
                                                              int filter, float *__restrict__ y, int oh, int ow,
                                                              int ycs) {
    __shared__ int ky[PIL_KMAX];
    __shared__ int ybound[3];     // first row, row count, ok flag
    __shared__ int kx[PIL_KMAX * 256];
    const int j = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int W = params[4 * b + 0], H = params[4 * b + 1], left = params[4 * b + 2], up = params[4 * b + 3];
    const unsigned char *img = x + b * xis;
    float *out = y + ((long long)b * oh + j) * ow * ycs;
    const int Y = up + j;
    const bool need_v = H != h0, need_h = W != w0;
    if (tid == 0) {
        ybound[2] = 1;
        if (Y >= 0 && Y < H && W > 0 && H > 0) {
            if (need_v) {
                if (!pil_coeffs(filter, h0, H, Y, &ybound[0], &ybound[1], ky, 1)) ybound[2] = 0;
            } else {
                ybound[0] = Y;
                ybound[1] = 1;
                ky[0] = 1 << PIL_PREC;   // unused: no vertical pass
            }
        } else {
            ybound[1] = 0;
        }
    }
    __syncthreads();
    const int y0 = ybound[0], ny = ybound[1];
    const bool yok = ybound[2] != 0;
    for (int i = tid; i < ow; i += 256) {
        float *o = out + (long long)i * ycs;
        const int X = left + i;
        if (ny == 0 || X < 0 || X >= W) {
            for (int c = 0; c < ycs; ++c) o[c] = 0.f;
            continue;
        }
        int x0 = X, nx = 1;
        bool ok = yok;
        int *k = kx + tid;
        if (need_h) ok = ok && pil_coeffs(filter, w0, W, X, &x0, &nx, k, 256);
        if (!ok) {                                 // more taps than PIL_KMAX: loud NaN
            for (int c = 0; c < ycs; ++c) o[c] = __builtin_nanf("");
            continue;
        }
        int acc[3] = {1 << (PIL_PREC - 1), 1 << (PIL_PREC - 1), 1 << (PIL_PREC - 1)};
        int direct[3] = {0, 0, 0};
        for (int t = 0; t < ny; ++t) {
            const unsigned char *row = img + (long long)(y0 + t) * w0 * 3;
            int hv[3];
            if (need_h) {
                int s[3] = {1 << (PIL_PREC - 1), 1 << (PIL_PREC - 1), 1 << (PIL_PREC - 1)};
                for (int u = 0; u < nx; ++u) {
                    const unsigned char *p = row + (x0 + u) * 3;
                    const int kk = k[u * 256];
                    s[0] += p[0] * kk;
                    s[1] += p[1] * kk;
                    s[2] += p[2] * kk;
                }
                hv[0] = pil_clip8(s[0]);
                hv[1] = pil_clip8(s[1]);
                hv[2] = pil_clip8(s[2]);
            } else {
                const unsigned char *p = row + X * 3;
                hv[0] = p[0];
                hv[1] = p[1];
                hv[2] = p[2];
            }
            if (need_v) {
                const int kk = ky[t];
                acc[0] += hv[0] * kk;
                acc[1] += hv[1] * kk;
                acc[2] += hv[2] * kk;
            } else {
                direct[0] = hv[0];
                direct[1] = hv[1];
                direct[2] = hv[2];
            }
        }
        for (int c = 0; c < 3; ++c) {
            const int v = need_v ? pil_clip8(acc[c]) : direct[c];
            o[c] = (float)((double)v / 255.0);
        }
        for (int c = 3; c < ycs; ++c) o[c] = 0.f;
    }
}

// R output rows per block (ow <= 256): the column taps are computed once per block, and the
// horizontal pass of every input row the R rows need is computed once into LDS (uint8, as
// Pillow's intermediate image) instead of once per (output row, vertical tap).  A block whose rows
// need more than PIL_RMAX input rows (a > ~4x vertical downscale) runs the rows one by one.
constexpr int PIL_R = 4, PIL_RMAX = 40;

__device__ __forceinline__ void pil_hrow(const unsigned char *row, int X, bool need_h, int x0, int nx, const int *k,
                                         int hv[3]) {
    if (!need_h) {
        const unsigned char *p = row + X * 3;
        hv[0] = p[0];
        hv[1] = p[1];
        hv[2] = p[2];
        return;
    }
    int s0 = 1 << (PIL_PREC - 1), s1 = s0, s2 = s0;
    for (int u = 0; u < nx; ++u) {
        const unsigned char *p = row + (x0 + u) * 3;
        const int kk = k[u * 256];
        s0 += p[0] * kk;
        s1 += p[1] * kk;
        s2 += p[2] * kk;
    }
    hv[0] = pil_clip8(s0);
    hv[1] = pil_clip8(s1);
    hv[2] = pil_clip8(s2);
}

__global__ __launch_bounds__(256) void pil_resize_crop_rows(const unsigned char *__restrict__ x, int h0, int w0,
                                                            long long xis, const int *__restrict__ params,
                                                            int filter, float *__restrict__ y, int oh, int ow,
                                                            int ycs) {
    __shared__ int ky[PIL_R][PIL_KMAX];
    __shared__ int yb[PIL_R][3];                 // first row, row count, ok
    __shared__ int rng[2];                       // first input row, input row count
    __shared__ int kx[PIL_KMAX * 256];
    __shared__ unsigned char hb[PIL_RMAX * 256 * 3];
    const int j0 = blockIdx.x * PIL_R, b = blockIdx.y, tid = threadIdx.x;
    const int W = params[4 * b + 0], H = params[4 * b + 1], left = params[4 * b + 2], up = params[4 * b + 3];
    const unsigned char *img = x + b * xis;
    const bool need_v = H != h0, need_h = W != w0;
    if (tid < PIL_R) {
        const int Y = up + j0 + tid;
        yb[tid][1] = 0;
        yb[tid][2] = 1;
        if (j0 + tid < oh && Y >= 0 && Y < H && W > 0 && H > 0) {
            if (need_v) {
                if (!pil_coeffs(filter, h0, H, Y, &yb[tid][0], &yb[tid][1], ky[tid], 1)) yb[tid][2] = 0;
            } else {
                yb[tid][0] = Y;
                yb[tid][1] = 1;
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        int lo = 1 << 30, hi = -1;
        for (int t = 0; t < PIL_R; ++t)
            if (yb[t][1] > 0) {
                lo = min(lo, yb[t][0]);
                hi = max(hi, yb[t][0] + yb[t][1]);
            }
        rng[0] = lo;
        rng[1] = hi > lo ? hi - lo : 0;
    }
    // the column's taps (kept in LDS, column-major per thread)
    const int i = tid, X = left + i;
    const bool col = i < ow && X >= 0 && X < W;
    int x0 = X, nx = 1;
    bool xok = true;
    if (col && need_h) xok = pil_coeffs(filter, w0, W, X, &x0, &nx, kx + tid, 256);
    __syncthreads();
    const int rlo = rng[0], nr = rng[1];
    const bool shared_rows = nr <= PIL_RMAX;
    if (shared_rows && col && xok) {
        for (int r = 0; r < nr; ++r) {
            int hv[3];
            pil_hrow(img + (long long)(rlo + r) * w0 * 3, X, need_h, x0, nx, kx + tid, hv);
            unsigned char *d = hb + (r * 256 + i) * 3;
            d[0] = (unsigned char)hv[0];
            d[1] = (unsigned char)hv[1];
            d[2] = (unsigned char)hv[2];
        }
    }
    if (i >= ow) return;                          // no barrier follows
    for (int t = 0; t < PIL_R; ++t) {
        const int j = j0 + t;
        if (j >= oh) break;
        float *o = y + (((long long)b * oh + j) * ow + i) * ycs;
        const int ny = yb[t][1];
        if (ny == 0 || !col) {
            for (int c = 0; c < ycs; ++c) o[c] = 0.f;
            continue;
        }
        if (!xok || !yb[t][2]) {                  // more taps than PIL_KMAX: loud NaN
            for (int c = 0; c < ycs; ++c) o[c] = __builtin_nanf("");
            continue;
        }
        const int y0 = yb[t][0];
        int acc[3] = {1 << (PIL_PREC - 1), 1 << (PIL_PREC - 1), 1 << (PIL_PREC - 1)};
        int v[3] = {0, 0, 0};
        for (int k = 0; k < ny; ++k) {
            int hv[3];
            if (shared_rows) {
                const unsigned char *s = hb + ((y0 + k - rlo) * 256 + i) * 3;
                hv[0] = s[0];
                hv[1] = s[1];
                hv[2] = s[2];
            } else {
                pil_hrow(img + (long long)(y0 + k) * w0 * 3, X, need_h, x0, nx, kx + tid, hv);
            }
            if (need_v) {
                const int kk = ky[t][k];
                acc[0] += hv[0] * kk;
                acc[1] += hv[1] * kk;
                acc[2] += hv[2] * kk;
            } else {
                v[0] = hv[0];
                v[1] = hv[1];
                v[2] = hv[2];
            }
        }
        for (int c = 0; c < 3; ++c) o[c] = (float)((double)(need_v ? pil_clip8(acc[c]) : v[c]) / 255.0);
        for (int c = 3; c < ycs; ++c) o[c] = 0.f;
    }
}

// y[b][c] = mean over the hw pixels of x[b][p][c] (fp64 sum, one rounding)
__global__ __launch_bounds__(256) void spatial_mean_kernel(const float *__restrict__ x, int n, int hw, int c,
                                                           float *__restrict__ y) {
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= (long long)n * c) return;
    const int b = (int)(e / c), ch = (int)(e % c);
    const float *p = x + (long long)b * hw * c + ch;
    double s = 0.0;
    for (int i = 0; i < hw; ++i) s += p[(long long)i * c];
    y[e] = (float)(s / hw);
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_pil_resize_crop(const unsigned char *x, int n, int h0, int w0, long long xis, const int *params,
                                   int filter, float *y, int oh, int ow, int ycs, s2v_stream_t stream) {
    S2V_REQUIRE(x && params && y && n > 0 && h0 > 0 && w0 > 0 && oh > 0 && ow > 0, "pil_resize_crop: bad args");
    S2V_REQUIRE(filter == 2 || filter == 3, "pil_resize_crop: filter must be 2 (BILINEAR) or 3 (BICUBIC), got %d",
                filter);
    S2V_REQUIRE(ycs >= 3 && xis >= (long long)h0 * w0 * 3, "pil_resize_crop: pitch ycs %d / frame stride %lld", ycs,
                xis);
    S2V_REQUIRE(oh <= 65535 && n <= 65535, "pil_resize_crop: grid too large");
    if (ow <= 256)
        pil_resize_crop_rows<<<dim3(cdiv(oh, PIL_R), n), 256, 0, (hipStream_t)stream>>>(x, h0, w0, xis, params,
                                                                                       filter, y, oh, ow, ycs);
    else
        pil_resize_crop_kernel<<<dim3(oh, n), 256, 0, (hipStream_t)stream>>>(x, h0, w0, xis, params, filter, y, oh,
                                                                            ow, ycs);
    return check_launch("pil_resize_crop");
}

extern "C" int s2v_spatial_mean_nhwc(const float *x, int n, int hw, int c, float *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && hw > 0 && c > 0, "spatial_mean: bad args");
    spatial_mean_kernel<<<cdiv((long long)n * c, 256), 256, 0, (hipStream_t)stream>>>(x, n, hw, c, y);
    return check_launch("spatial_mean");
}
