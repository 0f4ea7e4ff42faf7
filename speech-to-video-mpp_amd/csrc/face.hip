// Face detection / alignment / paste-back (SURVEY.md §8f(3) and the FaceEnhancement.process
// composition, third_part/GPEN/face_enhancement.py:91-193):
//
//   * RetinaFace input (retinaface_detection.py:59-73): uint8 BGR frame -> fp32 NHWC4 minus the
//     (104, 117, 123) BGR means; the ResNet-50 stem max-pool; the prior-box decode of the fused
//     class / box / landmark head (prior_box.py:20-34, box_utils.py:209-247, softmax of
//     retinaface.py:124) with the confidence threshold applied on the device and the survivors
//     compacted (the NMS over the few survivors stays on the host, as in the reference);
//   * cv2.warpAffine (INTER_LINEAR / INTER_AREA, BORDER_CONSTANT 0) for uint8 / fp32 / fp64 images
//     in OpenCV's fixed-point coordinate scheme (AB_BITS 10, INTER_BITS 5) — warp_and_crop_face
//     (align_faces.py:264) and the paste-back warps (face_enhancement.py:143-157);
//   * the paste-back composite fused with its two warps: per frame pixel the warped soft mask is
//     compared with the running full mask and, where larger, both the mask and the warped
//     enhanced face are written (face_enhancement.py:155-157);
//   * cv2.GaussianBlur (separable, reflect-101) on fp64 / fp32 masks, with the parse-mask / 255 and
//     the 26-pixel border zeroing of mask_postprocess (:83-88) fused into the first row pass;
//   * cv2.filter2D with the 3x3 smoothing kernel on uint8 faces (:159-160); FaceGAN's img2tensor /
//     tensor2img conversions (face_gan.py:44-59); the final convertScaleAbs blends (:175-191).
//
// oracle/face.py restates every one of these on the CPU; the tests compare bit for bit where the
// arithmetic is integer and to the stated tolerance where it is floating point.  Float expressions
// are evaluated unfused in the restatement's order.
#include "common.hpp"

#pragma clang fp contract(off)

namespace s2v {
namespace {

// cv::borderInterpolate(BORDER_REFLECT_101) for any offset
__device__ __forceinline__ int bi101(int p, int n) {
    if (n == 1) return 0;
    while ((unsigned)p >= (unsigned)n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

unsigned grid_1d(long long total, int per_block = 256) {
    long long b = (total + per_block - 1) / per_block;
    if (b > 65535LL * 32) b = 65535LL * 32;
    return (unsigned)(b < 1 ? 1 : b);
}

// ------------------------------------------------------------------------------ detection input
// img = np.float32(img_raw); img -= (104, 117, 123) in fp32 (uint8 frames, or the fp32 image
// cv2.resize made of frames larger than 1500 px); channel 3 of NHWC4 is zero
template <typename TI>
__global__ __launch_bounds__(256) void bgr_mean_nhwc4_kernel(const TI *__restrict__ x, long long pixels,
                                                             float *__restrict__ y) {
    for (long long p = blockIdx.x * 256LL + threadIdx.x; p < pixels; p += (long long)gridDim.x * 256) {
        const TI *s = x + p * 3;
        float4 v;
        v.x = (float)s[0] - 104.f;
        v.y = (float)s[1] - 117.f;
        v.z = (float)s[2] - 123.f;
        v.w = 0.f;
        *(float4 *)(y + p * 4) = v;
    }
}

// F.max_pool2d(k, s, p) on NHWC fp32 (c % 4 == 0): padding never wins (implicit -inf), NaN
// propagates like torch's CPU kernel
__global__ __launch_bounds__(256) void maxpool_nhwc_kernel(const float *__restrict__ x, int n, int h, int w, int c4,
                                                           int k, int s, int p, float *__restrict__ y, int oh,
                                                           int ow) {
    const long long total = (long long)n * oh * ow * c4;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int cc = (int)(e % c4);
        long long t = e / c4;
        const int ox = (int)(t % ow);
        t /= ow;
        const int oy = (int)(t % oh);
        const int b = (int)(t / oh);
        const int y0 = oy * s - p, x0 = ox * s - p;
        float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
        for (int dy = 0; dy < k; ++dy) {
            const int yy = y0 + dy;
            if (yy < 0 || yy >= h) continue;
            for (int dx = 0; dx < k; ++dx) {
                const int xx = x0 + dx;
                if (xx < 0 || xx >= w) continue;
                const float4 v = *(const float4 *)(x + (((long long)b * h + yy) * w + xx) * (c4 * 4) + cc * 4);
                m.x = (v.x > m.x || v.x != v.x) ? v.x : m.x;
                m.y = (v.y > m.y || v.y != v.y) ? v.y : m.y;
                m.z = (v.z > m.z || v.z != v.z) ? v.z : m.z;
                m.w = (v.w > m.w || v.w != v.w) ? v.w : m.w;
            }
        }
        *(float4 *)(y + e * 4) = m;
    }
}

// ------------------------------------------------------------------------------ prior decode
struct RetinaLevels {
    const float *head[3];    // fused head output per level: NHWC [h, w, cs] with channels
                             // [box a0 (4) | box a1 (4) | cls a0 (2) | cls a1 (2) | lm a0 (10) | lm a1 (10)]
    int h[3], w[3];
    int cs;
    int step[3];
    int min_size[3][2];
    long long first[4];      // first prior index of each level (first[3] = total)
};

// one thread per prior (level-major, then row, column, anchor: PriorBox.forward's order)
__global__ __launch_bounds__(256) void retina_decode_kernel(RetinaLevels L, int im_h, int im_w, float thresh,
                                                            float *__restrict__ cand, int *__restrict__ count,
                                                            int max_cand) {
    const long long P = L.first[3];
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < P; q += (long long)gridDim.x * 256) {
        const int lv = q < L.first[1] ? 0 : (q < L.first[2] ? 1 : 2);
        const long long r = q - L.first[lv];
        const int a = (int)(r & 1);
        const long long pix = r >> 1;
        const int i = (int)(pix / L.w[lv]), j = (int)(pix % L.w[lv]);
        const float *hd = L.head[lv] + pix * L.cs;
        // softmax over the two class logits (x - max, exp, * 1 / sum)
        const float c0 = hd[8 + 2 * a], c1 = hd[8 + 2 * a + 1];
        const float mx = fmaxf(c0, c1);
        const float e0 = expf(c0 - mx), e1 = expf(c1 - mx);
        const float score = e1 * (1.f / (e0 + e1));
        if (!(score > thresh)) continue;
        // prior (cx, cy, s_kx, s_ky): python floats (double) rounded to fp32 by torch.Tensor
        const double st = (double)L.step[lv];
        const float pcx = (float)((j + 0.5) * st / im_w), pcy = (float)((i + 0.5) * st / im_h);
        const float pw = (float)((double)L.min_size[lv][a] / im_w), ph = (float)((double)L.min_size[lv][a] / im_h);
        const float *lc = hd + 4 * a;
        const float cx = pcx + lc[0] * 0.1f * pw, cy = pcy + lc[1] * 0.1f * ph;
        const float bw = pw * expf(lc[2] * 0.2f), bh = ph * expf(lc[3] * 0.2f);
        const float x1 = cx - bw / 2.f, y1 = cy - bh / 2.f;
        const float x2 = bw + x1, y2 = bh + y1;
        const int slot = atomicAdd(count, 1);
        if (slot >= max_cand) continue;
        float *o = cand + (long long)slot * 16;
        o[0] = __int_as_float((int)q);
        o[1] = x1 * (float)im_w;
        o[2] = y1 * (float)im_h;
        o[3] = x2 * (float)im_w;
        o[4] = y2 * (float)im_h;
        o[5] = score;
        const float *lm = hd + 12 + 10 * a;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            o[6 + 2 * k] = (pcx + lm[2 * k] * 0.1f * pw) * (float)im_w;
            o[7 + 2 * k] = (pcy + lm[2 * k + 1] * 0.1f * ph) * (float)im_h;
        }
    }
}

// RetinaFace.forward's outputs (retinaface.py:115-124, phase 'test'): the per-level head maps
// concatenated into loc [n,P,4], conf = softmax(logits) [n,P,2], landms [n,P,10]
__global__ __launch_bounds__(256) void retina_split_kernel(RetinaLevels L, int n, float *__restrict__ loc,
                                                           float *__restrict__ conf, float *__restrict__ lms) {
    const long long P = L.first[3];
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < (long long)n * P; e += (long long)gridDim.x * 256) {
        const long long b = e / P, q = e - b * P;
        const int lv = q < L.first[1] ? 0 : (q < L.first[2] ? 1 : 2);
        const long long r = q - L.first[lv];
        const int a = (int)(r & 1);
        const float *hd = L.head[lv] + (b * L.h[lv] * L.w[lv] + (r >> 1)) * L.cs;
#pragma unroll
        for (int k = 0; k < 4; ++k) loc[e * 4 + k] = hd[4 * a + k];
        const float c0 = hd[8 + 2 * a], c1 = hd[8 + 2 * a + 1];
        const float mx = fmaxf(c0, c1);
        const float e0 = expf(c0 - mx), e1 = expf(c1 - mx);
        const float inv = 1.f / (e0 + e1);
        conf[e * 2] = e0 * inv;
        conf[e * 2 + 1] = e1 * inv;
#pragma unroll
        for (int k = 0; k < 10; ++k) lms[e * 10 + k] = hd[12 + 10 * a + k];
    }
}

// ------------------------------------------------------------------------------ warpAffine
// cv::invertAffineTransform then WarpAffineInvoker's source coordinates for dst (x, y)
struct WarpCoord {
    int sx, sy, fx, fy;   // top-left tap, 5-bit fractions
};

__device__ __forceinline__ void invert_affine(const double *m, double *iM) {
    double D = m[0] * m[4] - m[1] * m[3];
    D = D != 0. ? 1. / D : 0.;
    const double A11 = m[4] * D, A22 = m[0] * D, A12 = -m[1] * D, A21 = -m[3] * D;
    iM[0] = A11;
    iM[1] = A12;
    iM[3] = A21;
    iM[4] = A22;
    iM[2] = -A11 * m[2] - A12 * m[5];
    iM[5] = -A21 * m[2] - A22 * m[5];
}

__device__ __forceinline__ int sat_int(double v) {
    // saturate_cast<int>(double) = cvRound (round half to even), clamped to the int range
    const double r = rint(v);
    return r >= 2147483647.0 ? 2147483647 : (r <= -2147483648.0 ? (int)-2147483648LL : (int)r);
}

__device__ __forceinline__ WarpCoord warp_coord(const double *iM, int x, int y) {
    const int adelta = sat_int(iM[0] * x * 1024.0), bdelta = sat_int(iM[3] * x * 1024.0);
    const int X0 = sat_int((iM[1] * y + iM[2]) * 1024.0) + 16;
    const int Y0 = sat_int((iM[4] * y + iM[5]) * 1024.0) + 16;
    const int X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
    WarpCoord c;
    c.sx = min(max(X >> 5, -32768), 32767);
    c.sy = min(max(Y >> 5, -32768), 32767);
    c.fx = X & 31;
    c.fy = Y & 31;
    return c;
}

// taps outside the source read the border value bv (BORDER_CONSTANT, remapBilinear's cval)
template <typename T>
__device__ __forceinline__ T tap(const T *img, long long rs, int c, int h, int w, int yy, int xx, int ch, T bv = T(0)) {
    return (yy >= 0 && yy < h && xx >= 0 && xx < w) ? img[(long long)yy * rs + (long long)xx * c + ch] : bv;
}

// uint8: 15-bit integer weights w = (32 - fy or fy) * (32 - fx or fx) * 32, (sum + 2^14) >> 15
__device__ __forceinline__ unsigned char warp_u8(const unsigned char *img, long long rs, int c, int h, int w,
                                                 const WarpCoord &q, int ch, unsigned char bv = 0) {
    const int w00 = (32 - q.fy) * (32 - q.fx) * 32, w01 = (32 - q.fy) * q.fx * 32;
    const int w10 = q.fy * (32 - q.fx) * 32, w11 = q.fy * q.fx * 32;
    const int s = tap(img, rs, c, h, w, q.sy, q.sx, ch, bv) * w00 + tap(img, rs, c, h, w, q.sy, q.sx + 1, ch, bv) * w01 +
                  tap(img, rs, c, h, w, q.sy + 1, q.sx, ch, bv) * w10 +
                  tap(img, rs, c, h, w, q.sy + 1, q.sx + 1, ch, bv) * w11;
    return (unsigned char)((s + (1 << 14)) >> 15);
}

// float: the (1 - t, t) products of initInterTab2D (exact), summed in tap order in T
template <typename T>
__device__ __forceinline__ T warp_fp(const T *img, long long rs, int c, int h, int w, const WarpCoord &q, int ch,
                                     T bv = T(0)) {
    const float tx = (float)q.fx / 32.f, ty = (float)q.fy / 32.f;
    const T w00 = (T)((1.f - ty) * (1.f - tx)), w01 = (T)((1.f - ty) * tx);
    const T w10 = (T)(ty * (1.f - tx)), w11 = (T)(ty * tx);
    T s = tap(img, rs, c, h, w, q.sy, q.sx, ch, bv) * w00;
    s = s + tap(img, rs, c, h, w, q.sy, q.sx + 1, ch, bv) * w01;
    s = s + tap(img, rs, c, h, w, q.sy + 1, q.sx, ch, bv) * w10;
    s = s + tap(img, rs, c, h, w, q.sy + 1, q.sx + 1, ch, bv) * w11;
    return s;
}

// BORDER_CONSTANT value per channel (cv::Scalar saturated to the image type)
struct WarpBorder {
    double v[4];
};

template <typename T>
__global__ __launch_bounds__(256) void warp_affine_kernel(const T *__restrict__ x, int h, int w, int c, long long xrs,
                                                          long long xis, const double *__restrict__ M, int n,
                                                          T *__restrict__ y, int oh, int ow, long long yrs,
                                                          long long yis, WarpBorder bd) {
    const long long total = (long long)n * oh * ow;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = (int)(e % ow);
        long long t = e / ow;
        const int Y = (int)(t % oh);
        const int b = (int)(t / oh);
        double iM[6];
        invert_affine(M + 6 * b, iM);
        const WarpCoord q = warp_coord(iM, X, Y);
        const T *img = x + (long long)b * xis;
        T *o = y + (long long)b * yis + (long long)Y * yrs + (long long)X * c;
        for (int ch = 0; ch < c; ++ch) {
            const T bv = (T)bd.v[ch < 4 ? ch : 3];
            if constexpr (sizeof(T) == 1) o[ch] = warp_u8((const unsigned char *)img, xrs, c, h, w, q, ch, bv);
            else o[ch] = warp_fp(img, xrs, c, h, w, q, ch, bv);
        }
    }
}

// paste-back: tmp_mask = warp(mask) (fp32), where tmp_mask > full_mask: full_mask = tmp_mask and
// full_img = warp(face) (uint8 BGR), over the frame window [y0, y0 + wh) x [x0, x0 + ww)
__global__ __launch_bounds__(256) void face_paste_kernel(const float *__restrict__ mask, const unsigned char *__restrict__ face,
                                                         int S, const double *__restrict__ M, float *__restrict__ full_mask,
                                                         unsigned char *__restrict__ full_img, int H, int W, int y0,
                                                         int x0, int wh, int ww) {
    const long long total = (long long)wh * ww;
    double iM[6];
    invert_affine(M, iM);
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = x0 + (int)(e % ww), Y = y0 + (int)(e / ww);
        const WarpCoord q = warp_coord(iM, X, Y);
        const float tm = warp_fp(mask, (long long)S, 1, S, S, q, 0);
        const long long p = (long long)Y * W + X;
        if (tm > full_mask[p]) {
            full_mask[p] = tm;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) full_img[p * 3 + ch] = warp_u8(face, (long long)S * 3, 3, S, S, q, ch);
        }
    }
}

// ------------------------------------------------------------------------------ Gaussian blur
// row pass: in = u8 / 255. (fp64) or T, zeroed outside [zb, h - zb) x [zb, w - zb) when zb > 0;
// s = k[0] x[-r] + k[1] x[-r + 1] + ... in tap order (RowFilter), reflect-101 columns
template <typename T, typename TI>
__global__ __launch_bounds__(256) void blur_row_kernel(const TI *__restrict__ x, int h, int w, int zb,
                                                       const T *__restrict__ k, int r, T *__restrict__ y) {
    const long long total = (long long)h * w;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = (int)(e % w), Y = (int)(e / w);
        const bool zrow = zb > 0 && (Y < zb || Y >= h - zb);
        const TI *row = x + (long long)Y * w;
        T s = T(0);
        for (int t = -r; t <= r; ++t) {
            const int xx = bi101(X + t, w);
            T v;
            if constexpr (sizeof(TI) == 1) v = (T)((double)row[xx] / 255.0);
            else v = (T)row[xx];
            if (zrow || (zb > 0 && (xx < zb || xx >= w - zb))) v = T(0);
            const T term = k[t + r] * v;
            s = t == -r ? term : s + term;
        }
        y[e] = s;
    }
}

// column pass (SymmColumnFilter): s = k[r] c + sum_j k[r + j] (below_j + above_j), stored as TO
template <typename T, typename TO>
__global__ __launch_bounds__(256) void blur_col_kernel(const T *__restrict__ x, int h, int w, const T *__restrict__ k,
                                                       int r, TO *__restrict__ y) {
    const long long total = (long long)h * w;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = (int)(e % w), Y = (int)(e / w);
        T s = x[e] * k[r];
        for (int j = 1; j <= r; ++j) {
            const T pair = x[(long long)bi101(Y + j, h) * w + X] + x[(long long)bi101(Y - j, h) * w + X];
            s = s + pair * k[r + j];
        }
        y[e] = (TO)s;
    }
}

// ------------------------------------------------------------------------------ uint8 helpers
// cv2.filter2D(img, -1, 3x3 fp32 kernel), BORDER_REFLECT_101: fp32 sum of the 9 products in
// row-major order, cvRound (half to even), saturated
__global__ __launch_bounds__(256) void filter3x3_u8_kernel(const unsigned char *__restrict__ x, int h, int w, int c,
                                                           const float *__restrict__ kern, unsigned char *__restrict__ y) {
    const long long total = (long long)h * w * c;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int ch = (int)(e % c);
        const long long p = e / c;
        const int X = (int)(p % w), Y = (int)(p / w);
        float s = 0.f;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
            const unsigned char *row = x + (long long)bi101(Y + dy, h) * w * c + ch;
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) s = s + kern[(dy + 1) * 3 + dx + 1] * (float)row[bi101(X + dx, w) * c];
        }
        y[e] = (unsigned char)min(max(__float2int_rn(s), 0), 255);
    }
}

// FaceGAN.img2tensor (face_gan.py:44-49): torch uint8 / 255. -> (x - 0.5) / 0.5 in fp32, HWC BGR
// -> NCHW RGB (the flip(1))
__global__ __launch_bounds__(256) void u8_to_gan_kernel(const unsigned char *__restrict__ x, long long hw, int n,
                                                        float *__restrict__ y) {
    const long long total = (long long)n * hw;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long b = e / hw, p = e - b * hw;
        const unsigned char *s = x + e * 3;
        float *o = y + b * 3 * hw + p;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) o[ch * hw] = ((float)s[2 - ch] / 255.f - 0.5f) / 0.5f;
    }
}

// FaceGAN.tensor2img (:51-59): x * 0.5 + 0.5, RGB -> BGR, np.clip(0, 1) * 255., astype(uint8)
// (truncation); NCHW fp32 -> HWC uint8
__global__ __launch_bounds__(256) void gan_to_u8_kernel(const float *__restrict__ x, long long hw, int n,
                                                        unsigned char *__restrict__ y) {
    const long long total = (long long)n * hw;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long b = e / hw, p = e - b * hw;
        const float *s = x + b * 3 * hw + p;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            float v = s[(2 - ch) * hw] * 0.5f + 0.5f;
            v = v != v ? v : fminf(fmaxf(v, 0.f), 1.f);
            y[e * 3 + ch] = (unsigned char)(int)(v * 255.f);
        }
    }
}

// mask_sharp = parse_mask / 255. (uint8 -> float64, face_enhancement.py:137)
__global__ __launch_bounds__(256) void u8_div255_f64_kernel(const unsigned char *__restrict__ x, long long n,
                                                            double *__restrict__ y) {
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
        y[e] = (double)x[e] / 255.0;
}

// mask_sharp = parse / 255. after FaceEnhancement.mask_postprocess zeroed its border in place
// (face_enhancement.py:84-85, :144-145): pixels within ``border`` of an edge are 0
__global__ __launch_bounds__(256) void u8_div255_f64_border_kernel(const unsigned char *__restrict__ x, int h, int w,
                                                                   int border, double *__restrict__ y) {
    const long long n = (long long)h * w;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int r = (int)(e / w), c = (int)(e - (long long)r * w);
        const bool in = r >= border && r < h - border && c >= border && c < w - border;
        y[e] = in ? (double)x[e] / 255.0 : 0.0;
    }
}

__device__ __forceinline__ unsigned char cvt_abs_u8(float v) {
    return (unsigned char)min(max(__float2int_rn(fabsf(v)), 0), 255);
}

// use_sr: convertScaleAbs(img_sr * (1 - full_mask) + full_img * full_mask), fp32 (:175-176)
__global__ __launch_bounds__(256) void blend_sr_kernel(const unsigned char *__restrict__ base,
                                                       const float *__restrict__ fm,
                                                       const unsigned char *__restrict__ full,
                                                       unsigned char *__restrict__ out, long long pixels) {
    for (long long p = blockIdx.x * 256LL + threadIdx.x; p < pixels; p += (long long)gridDim.x * 256) {
        const float m = fm[p], im = 1.f - m;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) out[p * 3 + ch] = cvt_abs_u8((float)base[p * 3 + ch] * im + (float)full[p * 3 + ch] * m);
    }
}

// plain: img = convertScaleAbs(ori * (1 - full_mask) + full_img * full_mask) (fp32), then
// convertScaleAbs(ori * (1 - mask_sharp) + img * mask_sharp) with the fp64 mask_sharp (:189-191)
__global__ __launch_bounds__(256) void blend_plain_kernel(const unsigned char *__restrict__ ori,
                                                          const float *__restrict__ fm,
                                                          const unsigned char *__restrict__ full,
                                                          const double *__restrict__ ms,
                                                          unsigned char *__restrict__ out, long long pixels) {
    for (long long p = blockIdx.x * 256LL + threadIdx.x; p < pixels; p += (long long)gridDim.x * 256) {
        const float m = fm[p], im = 1.f - m;
        const double s = ms[p], is = 1.0 - s;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const unsigned char o = ori[p * 3 + ch];
            const unsigned char a = cvt_abs_u8((float)o * im + (float)full[p * 3 + ch] * m);
            out[p * 3 + ch] = cvt_abs_u8((float)((double)o * is + (double)a * s));
        }
    }
}

// ------------------------------------------------------------------------------ GFPGANer restore
// basicsr tensor2img(output, rgb2bgr=True, min_max=(-1, 1)) as GFPGANer.enhance calls it
// (gfpgan/utils.py:120-121): clamp(-1, 1), (x + 1) / 2, RGB -> BGR, (x * 255.).round() (half to
// even), astype(uint8); NCHW fp32 -> HWC uint8
__global__ __launch_bounds__(256) void tensor2img_u8_kernel(const float *__restrict__ x, long long hw, int n,
                                                            unsigned char *__restrict__ y) {
    const long long total = (long long)n * hw;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long b = e / hw, p = e - b * hw;
        const float *s = x + b * 3 * hw + p;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            float v = fminf(fmaxf(s[(2 - ch) * hw], -1.f), 1.f);
            v = (v + 1.f) / 2.f;
            y[e * 3 + ch] = (unsigned char)(int)rintf(v * 255.f);
        }
    }
}

// facexlib paste_faces_to_input_image (square parse map, upscale 1): inv_mask = warpAffine(ones(S, S)
// fp32, inverse_affine) is the sum of the bilinear weights of the taps inside the crop (exact in fp32);
// inv_mask_erosion = cv2.erode(inv_mask, ones((2, 2))) (anchor (1, 1): the min over rows y-1..y and
// columns x-1..x inside the frame), over the frame window [y0, y0 + wh) x [x0, x0 + ww) (E is [wh][ww]);
// part[block] = the block's fp64 sum of the erosion (one store per block: a single-address atomic from
// ~8k blocks serialised to ~100 us at 1080p)
constexpr int RESTORE_PARTS = 512;

__global__ __launch_bounds__(256) void restore_mask_kernel(const double *__restrict__ M, int S, int y0, int x0,
                                                           int wh, int ww, float *__restrict__ E,
                                                           double *__restrict__ parts) {
    __shared__ double part[4];
    double iM[6];
    invert_affine(M, iM);
    double acc = 0.0;
    const long long total = (long long)wh * ww;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = x0 + (int)(e % ww), Y = y0 + (int)(e / ww);
        float m = INFINITY;
        for (int dy = -1; dy <= 0; ++dy) {
            const int yy = Y + dy;
            if (yy < 0) continue;
            for (int dx = -1; dx <= 0; ++dx) {
                const int xx = X + dx;
                if (xx < 0) continue;
                const WarpCoord q = warp_coord(iM, xx, yy);
                const float tx = (float)q.fx / 32.f, ty = (float)q.fy / 32.f;
                const bool x0 = q.sx >= 0 && q.sx < S, x1 = q.sx + 1 >= 0 && q.sx + 1 < S;
                const bool y0 = q.sy >= 0 && q.sy < S, y1 = q.sy + 1 >= 0 && q.sy + 1 < S;
                float v = (y0 && x0) ? (1.f - ty) * (1.f - tx) : 0.f;
                v = v + ((y0 && x1) ? (1.f - ty) * tx : 0.f);
                v = v + ((y1 && x0) ? ty * (1.f - tx) : 0.f);
                v = v + ((y1 && x1) ? ty * tx : 0.f);
                m = fminf(m, v);
            }
        }
        E[e] = m;
        acc += (double)m;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) parts[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

// area = the block partials summed in a fixed order (deterministic)
__global__ __launch_bounds__(256) void restore_area_kernel(const double *__restrict__ parts, int n,
                                                           double *__restrict__ area) {
    __shared__ double part[4];
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) acc += parts[i];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) area[0] = (part[0] + part[1]) + (part[2] + part[3]);
}

// cv2.erode with a k x k rectangle of ones (anchor (k / 2, k / 2)) as OpenCV's separable morphology:
// min over columns x - k/2 .. x - k/2 + k - 1 inside the frame (the constant border never wins), then
// the same over rows
__global__ __launch_bounds__(256) void erode_row_kernel(const float *__restrict__ x, int h, int w, int k,
                                                        float *__restrict__ y) {
    const long long total = (long long)h * w;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = (int)(e % w);
        const float *row = x + (e - X);
        const int a = max(X - k / 2, 0), b = min(X - k / 2 + k, w);
        float m = INFINITY;
        for (int t = a; t < b; ++t) m = fminf(m, row[t]);
        y[e] = m;
    }
}

__global__ __launch_bounds__(256) void erode_col_kernel(const float *__restrict__ x, int h, int w, int k,
                                                        float *__restrict__ y) {
    const long long total = (long long)h * w;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = (int)(e % w), Y = (int)(e / w);
        const int a = max(Y - k / 2, 0), b = min(Y - k / 2 + k, h);
        float m = INFINITY;
        for (int t = a; t < b; ++t) m = fminf(m, x[(long long)t * w + X]);
        y[e] = m;
    }
}

// upsample_img = inv_soft_mask * pasted_face + (1 - inv_soft_mask) * upsample_img with pasted_face =
// inv_mask_erosion * warpAffine(restored_face uint8, inverse_affine) (BORDER_CONSTANT 0), fp32; TO
// uint8 is the final astype(uint8) (truncation).  soft / E cover the window [y0, +wh) x [x0, +ww) and are
// 0 outside it, where the blend is the base itself (0 * 0 + 1 * base)
template <typename TB, typename TO>
__global__ __launch_bounds__(256) void restore_paste_kernel(const unsigned char *__restrict__ face, int S,
                                                            const double *__restrict__ M,
                                                            const float *__restrict__ soft,
                                                            const float *__restrict__ E, int y0, int x0, int wh,
                                                            int ww, const TB *base, TO *out, int H, int W) {
    double iM[6];
    invert_affine(M, iM);
    const long long total = (long long)H * W;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int X = (int)(e % W), Y = (int)(e / W);
        const int wy = Y - y0, wx = X - x0;
        if (wy < 0 || wy >= wh || wx < 0 || wx >= ww) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const float v = (float)base[e * 3 + ch];
                if constexpr (sizeof(TO) == 1) out[e * 3 + ch] = (unsigned char)(int)v;
                else out[e * 3 + ch] = v;
            }
            continue;
        }
        const long long we = (long long)wy * ww + wx;
        const WarpCoord q = warp_coord(iM, X, Y);
        const float sm = soft[we], em = E[we], ism = 1.f - sm;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const float pasted = em * (float)warp_u8(face, (long long)S * 3, 3, S, S, q, ch);
            const float v = sm * pasted + ism * (float)base[e * 3 + ch];
            if constexpr (sizeof(TO) == 1) out[e * 3 + ch] = (unsigned char)(int)v;
            else out[e * 3 + ch] = v;
        }
    }
}

}  // namespace
}  // namespace s2v

using namespace s2v;

extern "C" int s2v_bgr_mean_nhwc4(const void *x, int xtype, long long pixels, float *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && pixels > 0 && (xtype == 0 || xtype == 1), "bgr_mean_nhwc4: bad args");
    S2V_REQUIRE(((uintptr_t)y & 15) == 0, "bgr_mean_nhwc4: y must be 16-byte aligned");
    if (xtype == 0)
        bgr_mean_nhwc4_kernel<unsigned char><<<grid_1d(pixels), 256, 0, (hipStream_t)stream>>>((const unsigned char *)x, pixels, y);
    else
        bgr_mean_nhwc4_kernel<float><<<grid_1d(pixels), 256, 0, (hipStream_t)stream>>>((const float *)x, pixels, y);
    return check_launch("bgr_mean_nhwc4");
}

extern "C" int s2v_maxpool2d_nhwc(const float *x, int n, int h, int w, int c, int k, int s, int p, float *y, int oh,
                                  int ow, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && c > 0 && k > 0 && s > 0 && p >= 0, "maxpool2d: bad args");
    S2V_REQUIRE(c % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0,
                "maxpool2d: channels must be a multiple of 4 and the tensors 16-byte aligned");
    S2V_REQUIRE(oh == (h + 2 * p - k) / s + 1 && ow == (w + 2 * p - k) / s + 1 && 2 * p <= k,
                "maxpool2d: output %dx%d does not match k=%d s=%d p=%d on %dx%d", oh, ow, k, s, p, h, w);
    maxpool_nhwc_kernel<<<grid_1d((long long)n * oh * ow * (c / 4)), 256, 0, (hipStream_t)stream>>>(
        x, n, h, w, c / 4, k, s, p, y, oh, ow);
    return check_launch("maxpool2d");
}

static int retina_levels(const float *const *heads, const int *hs, const int *ws, int cs, int im_h, int im_w,
                         RetinaLevels &L) {
    S2V_REQUIRE(heads && hs && ws && im_h > 0 && im_w > 0 && cs >= 32, "retina: bad args");
    static const int steps[3] = {8, 16, 32};
    static const int mins[3][2] = {{16, 32}, {64, 128}, {256, 512}};
    L.cs = cs;
    L.first[0] = 0;
    for (int l = 0; l < 3; ++l) {
        S2V_REQUIRE(heads[l] && hs[l] > 0 && ws[l] > 0, "retina_decode: level %d missing", l);
        // PriorBox feature maps are ceil(image / step)
        S2V_REQUIRE(hs[l] == (im_h + steps[l] - 1) / steps[l] && ws[l] == (im_w + steps[l] - 1) / steps[l],
                    "retina_decode: level %d is %dx%d, the priors of a %dx%d image need ceil(size / %d)", l, hs[l],
                    ws[l], im_h, im_w, steps[l]);
        L.head[l] = heads[l];
        L.h[l] = hs[l];
        L.w[l] = ws[l];
        L.step[l] = steps[l];
        L.min_size[l][0] = mins[l][0];
        L.min_size[l][1] = mins[l][1];
        L.first[l + 1] = L.first[l] + 2LL * hs[l] * ws[l];
    }
    return S2V_OK;
}

extern "C" int s2v_retina_decode(const float *const *heads, const int *hs, const int *ws, int cs, int im_h, int im_w,
                                 float thresh, float *cand, int *count, int max_cand, s2v_stream_t stream) {
    S2V_REQUIRE(cand && count && max_cand > 0, "retina_decode: bad args");
    RetinaLevels L;
    const int rc = retina_levels(heads, hs, ws, cs, im_h, im_w, L);
    if (rc != S2V_OK) return rc;
    S2V_REQUIRE(max_cand >= L.first[3], "retina_decode: max_cand %d < %lld priors", max_cand, L.first[3]);
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(count, 0, sizeof(int), st) != hipSuccess) return check_launch("retina_decode(memset)");
    retina_decode_kernel<<<grid_1d(L.first[3]), 256, 0, st>>>(L, im_h, im_w, thresh, cand, count, max_cand);
    return check_launch("retina_decode");
}

extern "C" int s2v_retina_split(const float *const *heads, const int *hs, const int *ws, int cs, int im_h, int im_w,
                                int n, float *loc, float *conf, float *landms, s2v_stream_t stream) {
    S2V_REQUIRE(loc && conf && landms && n > 0, "retina_split: bad args");
    RetinaLevels L;
    const int rc = retina_levels(heads, hs, ws, cs, im_h, im_w, L);
    if (rc != S2V_OK) return rc;
    retina_split_kernel<<<grid_1d(n * L.first[3]), 256, 0, (hipStream_t)stream>>>(L, n, loc, conf, landms);
    return check_launch("retina_split");
}

extern "C" int s2v_warp_affine(const void *x, int n, int h, int w, int c, long long xrs, long long xis, int dtype,
                               const double *M, void *y, int oh, int ow, long long yrs, long long yis,
                               s2v_stream_t stream) {
    S2V_REQUIRE(x && y && M && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0, "warp_affine: bad args");
    S2V_REQUIRE(dtype >= 0 && dtype <= 2, "warp_affine: dtype must be 0 (uint8), 1 (fp32) or 2 (fp64)");
    S2V_REQUIRE(xrs >= (long long)w * c && yrs >= (long long)ow * c && (n == 1 || (xis >= xrs * h && yis >= yrs * oh)),
                "warp_affine: row / image pitches smaller than the rows / images");
    S2V_REQUIRE(h < 32767 && w < 32767, "warp_affine: source larger than OpenCV's int16 coordinates");
    return s2v_warp_affine_border(x, n, h, w, c, xrs, xis, dtype, M, y, oh, ow, yrs, yis, nullptr, stream);
}

extern "C" int s2v_warp_affine_border(const void *x, int n, int h, int w, int c, long long xrs, long long xis,
                                      int dtype, const double *M, void *y, int oh, int ow, long long yrs,
                                      long long yis, const double *border, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && M && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0, "warp_affine: bad args");
    S2V_REQUIRE(dtype >= 0 && dtype <= 2, "warp_affine: dtype must be 0 (uint8), 1 (fp32) or 2 (fp64)");
    // xis == 0: n warps of one source image (align_warp_face's faces of one frame)
    S2V_REQUIRE(xrs >= (long long)w * c && yrs >= (long long)ow * c &&
                    (n == 1 || ((xis == 0 || xis >= xrs * h) && yis >= yrs * oh)),
                "warp_affine: row / image pitches smaller than the rows / images");
    S2V_REQUIRE(h < 32767 && w < 32767, "warp_affine: source larger than OpenCV's int16 coordinates");
    WarpBorder bd = {{0., 0., 0., 0.}};
    for (int i = 0; border && i < 4; ++i) {
        double v = border[i < c ? i : c - 1];
        if (dtype == 0) v = v <= 0. ? 0. : (v >= 255. ? 255. : rint(v));   // saturate_cast<uchar>
        bd.v[i] = v;
    }
    const unsigned g = grid_1d((long long)n * oh * ow);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == 0)
        warp_affine_kernel<unsigned char><<<g, 256, 0, s>>>((const unsigned char *)x, h, w, c, xrs, xis, M, n,
                                                            (unsigned char *)y, oh, ow, yrs, yis, bd);
    else if (dtype == 1)
        warp_affine_kernel<float><<<g, 256, 0, s>>>((const float *)x, h, w, c, xrs, xis, M, n, (float *)y, oh, ow, yrs,
                                                    yis, bd);
    else
        warp_affine_kernel<double><<<g, 256, 0, s>>>((const double *)x, h, w, c, xrs, xis, M, n, (double *)y, oh, ow,
                                                     yrs, yis, bd);
    return check_launch("warp_affine");
}

extern "C" int s2v_face_paste(const float *mask, const unsigned char *face, int S, const double *M, float *full_mask,
                              unsigned char *full_img, int H, int W, int y0, int x0, int wh, int ww,
                              s2v_stream_t stream) {
    S2V_REQUIRE(mask && face && M && full_mask && full_img && S > 0 && H > 0 && W > 0, "face_paste: bad args");
    S2V_REQUIRE(y0 >= 0 && x0 >= 0 && wh >= 0 && ww >= 0 && y0 + wh <= H && x0 + ww <= W,
                "face_paste: window outside the frame");
    if (wh == 0 || ww == 0) return S2V_OK;
    face_paste_kernel<<<grid_1d((long long)wh * ww), 256, 0, (hipStream_t)stream>>>(mask, face, S, M, full_mask,
                                                                                     full_img, H, W, y0, x0, wh, ww);
    return check_launch("face_paste");
}

extern "C" size_t s2v_gaussian_blur_ws_bytes(int h, int w, int dtype) {
    if (h <= 0 || w <= 0) return 0;
    return (size_t)h * w * (dtype == 2 ? 8 : 4);
}

extern "C" int s2v_gaussian_blur(const void *x, int xtype, int h, int w, int zero_border, const void *kern, int ksize,
                                 void *y, int ytype, int dtype, void *ws, size_t ws_bytes, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && kern && h > 0 && w > 0 && ksize > 0 && (ksize & 1), "gaussian_blur: bad args");
    S2V_REQUIRE(dtype == 1 || dtype == 2, "gaussian_blur: work type must be 1 (fp32) or 2 (fp64)");
    S2V_REQUIRE(xtype >= 0 && xtype <= 2 && ytype >= 1 && ytype <= 2, "gaussian_blur: bad input / output type");
    S2V_REQUIRE(xtype == 0 || xtype == dtype, "gaussian_blur: fp input must have the work type");
    S2V_REQUIRE(zero_border >= 0 && 2 * zero_border <= h && 2 * zero_border <= w, "gaussian_blur: bad zero border");
    S2V_REQUIRE(ws && ws_bytes >= s2v_gaussian_blur_ws_bytes(h, w, dtype), "gaussian_blur: workspace too small");
    const int r = ksize / 2;
    const unsigned g = grid_1d((long long)h * w);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == 2) {
        const double *k = (const double *)kern;
        double *t = (double *)ws;
        if (xtype == 0) blur_row_kernel<double, unsigned char><<<g, 256, 0, s>>>((const unsigned char *)x, h, w, zero_border, k, r, t);
        else blur_row_kernel<double, double><<<g, 256, 0, s>>>((const double *)x, h, w, zero_border, k, r, t);
        if (ytype == 2) blur_col_kernel<double, double><<<g, 256, 0, s>>>(t, h, w, k, r, (double *)y);
        else blur_col_kernel<double, float><<<g, 256, 0, s>>>(t, h, w, k, r, (float *)y);
    } else {
        S2V_REQUIRE(ytype == 1, "gaussian_blur: fp32 work writes fp32");
        const float *k = (const float *)kern;
        float *t = (float *)ws;
        if (xtype == 0) blur_row_kernel<float, unsigned char><<<g, 256, 0, s>>>((const unsigned char *)x, h, w, zero_border, k, r, t);
        else blur_row_kernel<float, float><<<g, 256, 0, s>>>((const float *)x, h, w, zero_border, k, r, t);
        blur_col_kernel<float, float><<<g, 256, 0, s>>>(t, h, w, k, r, (float *)y);
    }
    return check_launch("gaussian_blur");
}

extern "C" int s2v_filter3x3_u8(const unsigned char *x, int h, int w, int c, const float *kern, unsigned char *y,
                                s2v_stream_t stream) {
    S2V_REQUIRE(x && y && kern && h > 0 && w > 0 && c > 0 && x != y, "filter3x3_u8: bad args (in place not allowed)");
    filter3x3_u8_kernel<<<grid_1d((long long)h * w * c), 256, 0, (hipStream_t)stream>>>(x, h, w, c, kern, y);
    return check_launch("filter3x3_u8");
}

extern "C" int s2v_u8_to_gan(const unsigned char *x, int n, int h, int w, float *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0, "u8_to_gan: bad args");
    const long long hw = (long long)h * w;
    u8_to_gan_kernel<<<grid_1d(n * hw), 256, 0, (hipStream_t)stream>>>(x, hw, n, y);
    return check_launch("u8_to_gan");
}

extern "C" int s2v_gan_to_u8(const float *x, int n, int h, int w, unsigned char *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0, "gan_to_u8: bad args");
    const long long hw = (long long)h * w;
    gan_to_u8_kernel<<<grid_1d(n * hw), 256, 0, (hipStream_t)stream>>>(x, hw, n, y);
    return check_launch("gan_to_u8");
}

extern "C" int s2v_u8_div255_f64(const unsigned char *x, long long n, double *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0, "u8_div255_f64: bad args");
    u8_div255_f64_kernel<<<grid_1d(n), 256, 0, (hipStream_t)stream>>>(x, n, y);
    return check_launch("u8_div255_f64");
}

extern "C" int s2v_u8_div255_f64_border(const unsigned char *x, int h, int w, int border, double *y,
                                        s2v_stream_t stream) {
    S2V_REQUIRE(x && y && h > 0 && w > 0 && border >= 0, "u8_div255_f64_border: bad args");
    u8_div255_f64_border_kernel<<<grid_1d((long long)h * w), 256, 0, (hipStream_t)stream>>>(x, h, w, border, y);
    return check_launch("u8_div255_f64_border");
}

extern "C" int s2v_face_blend(const unsigned char *base, const float *full_mask, const unsigned char *full_img,
                              const double *mask_sharp, unsigned char *out, long long pixels, s2v_stream_t stream) {
    S2V_REQUIRE(base && full_mask && full_img && out && pixels > 0, "face_blend: bad args");
    const unsigned g = grid_1d(pixels);
    if (mask_sharp)
        blend_plain_kernel<<<g, 256, 0, (hipStream_t)stream>>>(base, full_mask, full_img, mask_sharp, out, pixels);
    else
        blend_sr_kernel<<<g, 256, 0, (hipStream_t)stream>>>(base, full_mask, full_img, out, pixels);
    return check_launch("face_blend");
}

extern "C" int s2v_tensor2img_u8(const float *x, int n, int h, int w, unsigned char *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0, "tensor2img_u8: bad args");
    const long long hw = (long long)h * w;
    tensor2img_u8_kernel<<<grid_1d(n * hw), 256, 0, (hipStream_t)stream>>>(x, hw, n, y);
    return check_launch("tensor2img_u8");
}

extern "C" int s2v_restore_parts(void) { return RESTORE_PARTS; }

extern "C" int s2v_restore_mask(const double *M, int S, int H, int W, int y0, int x0, int wh, int ww,
                                float *erosion, double *area, s2v_stream_t stream) {
    S2V_REQUIRE(M && erosion && area && S > 0 && H > 0 && W > 0, "restore_mask: bad args");
    S2V_REQUIRE(y0 >= 0 && x0 >= 0 && wh > 0 && ww > 0 && y0 + wh <= H && x0 + ww <= W,
                "restore_mask: window outside the frame");
    hipStream_t s = (hipStream_t)stream;
    long long nb = ((long long)wh * ww + 255) / 256;
    const int blocks = (int)(nb < RESTORE_PARTS ? nb : RESTORE_PARTS);
    restore_mask_kernel<<<blocks, 256, 0, s>>>(M, S, y0, x0, wh, ww, erosion, area + 1);
    restore_area_kernel<<<1, 256, 0, s>>>(area + 1, blocks, area);
    return check_launch("restore_mask");
}

extern "C" int s2v_erode_rect_f32(const float *x, int h, int w, int k, float *y, float *ws, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && ws && h > 0 && w > 0 && k > 0 && ws != x && ws != y, "erode_rect_f32: bad args");
    const unsigned g = grid_1d((long long)h * w);
    hipStream_t s = (hipStream_t)stream;
    erode_row_kernel<<<g, 256, 0, s>>>(x, h, w, k, ws);
    erode_col_kernel<<<g, 256, 0, s>>>(ws, h, w, k, y);
    return check_launch("erode_rect_f32");
}

extern "C" int s2v_restore_paste(const unsigned char *face, int S, const double *M, const float *soft,
                                 const float *erosion, int y0, int x0, int wh, int ww, const void *base, int base_f32,
                                 void *out, int out_f32, int H, int W, s2v_stream_t stream) {
    S2V_REQUIRE(face && M && soft && erosion && base && out && S > 0 && H > 0 && W > 0, "restore_paste: bad args");
    S2V_REQUIRE(y0 >= 0 && x0 >= 0 && wh >= 0 && ww >= 0 && y0 + wh <= H && x0 + ww <= W,
                "restore_paste: window outside the frame");
    S2V_REQUIRE(base != out || (base_f32 && out_f32), "restore_paste: in place only on the fp32 accumulator");
    const unsigned g = grid_1d((long long)H * W);
    hipStream_t s = (hipStream_t)stream;
    if (!base_f32 && !out_f32)
        restore_paste_kernel<unsigned char, unsigned char><<<g, 256, 0, s>>>(
            face, S, M, soft, erosion, y0, x0, wh, ww, (const unsigned char *)base, (unsigned char *)out, H, W);
    else if (!base_f32)
        restore_paste_kernel<unsigned char, float><<<g, 256, 0, s>>>(face, S, M, soft, erosion, y0, x0, wh, ww,
                                                                     (const unsigned char *)base, (float *)out, H, W);
    else if (out_f32)
        restore_paste_kernel<float, float><<<g, 256, 0, s>>>(face, S, M, soft, erosion, y0, x0, wh, ww,
                                                             (const float *)base, (float *)out, H, W);
    else
        restore_paste_kernel<float, unsigned char><<<g, 256, 0, s>>>(face, S, M, soft, erosion, y0, x0, wh, ww,
                                                                     (const float *)base, (unsigned char *)out, H, W);
    return check_launch("restore_paste");
}
