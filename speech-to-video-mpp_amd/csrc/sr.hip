// Super-resolution front / back end: RealESRNet.process
// (third_part/GPEN/sr_model/real_esrnet.py:99-137) around the RRDBNet forward.
//
//   in:  uint8 HWC BGR frame -> float32 x / 255 (:100), BGR -> RGB (:101), F.pad(..., 'reflect')
//        on the bottom / right up to a multiple of the pixel-unshuffle factor (:104-115), written
//        straight into the 4-channel NHWC layout the conv engine gathers with 16-byte loads;
//   out: crop of the padded output (:126-128), clamp_(0, 1) (:129), RGB -> BGR (:130),
//        (x * 255.0).round() (NumPy round-half-even) -> uint8 (:131).
#include "common.hpp"

#pragma clang fp contract(off)

namespace s2v {

__global__ __launch_bounds__(256) void sr_u8_in_kernel(const unsigned char *__restrict__ x, int n, int h, int w,
                                                       int flip, int oh, int ow, float *__restrict__ y, int ycs) {
    const long long total = (long long)n * oh * ow;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int j = (int)(e % ow);
        const long long t = e / ow;
        const int i = (int)(t % oh);
        const int b = (int)(t / oh);
        // torch 'reflect' padding (common.hpp reflect_idx: the edge is not repeated)
        const unsigned char *px = x + (((long long)b * h + reflect_idx(i, h)) * w + reflect_idx(j, w)) * 3;
        float v[4];
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = (float)px[flip ? 2 - c : c] / 255.0f;
        v[3] = 0.f;
        float *py = y + e * ycs;
        if (ycs == 4 && ((reinterpret_cast<uintptr_t>(py) & 15) == 0)) {
            *reinterpret_cast<float4 *>(py) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int c = 0; c < 3; ++c) py[c] = v[c];
            if (ycs >= 4) py[3] = 0.f;
        }
    }
}

__global__ __launch_bounds__(256) void sr_f32_out_kernel(const float *__restrict__ x, int n, int h, int w, int xh,
                                                         int xw, int xcs, int flip, unsigned char *__restrict__ y) {
    const long long total = (long long)n * h * w;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int j = (int)(e % w);
        const long long t = e / w;
        const int i = (int)(t % h);
        const int b = (int)(t / h);
        const float *px = x + (((long long)b * xh + i) * xw + j) * xcs;
        unsigned char *py = y + e * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = fminf(fmaxf(px[flip ? 2 - c : c], 0.f), 1.f);
            py[c] = (unsigned char)rintf(v * 255.0f);
        }
    }
}

static unsigned sr_grid(long long total) {
    long long b = (total + 255) / 256;
    if (b > 65535LL * 16) b = 65535LL * 16;
    return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_sr_u8_in(const unsigned char *x, int n, int h, int w, int flip, int pad_b, int pad_r, float *y,
                            int ycs, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && ycs >= 3 && pad_b >= 0 && pad_r >= 0, "sr_u8_in: bad args");
    S2V_REQUIRE(pad_b < h && pad_r < w, "sr_u8_in: reflect padding (%d, %d) must be smaller than the image (%d, %d)",
                pad_b, pad_r, h, w);
    const int oh = h + pad_b, ow = w + pad_r;
    sr_u8_in_kernel<<<sr_grid((long long)n * oh * ow), 256, 0, (hipStream_t)stream>>>(x, n, h, w, flip, oh, ow, y,
                                                                                     ycs);
    return check_launch("sr_u8_in");
}

extern "C" int s2v_sr_f32_out(const float *x, int n, int h, int w, int xh, int xw, int xcs, int flip,
                              unsigned char *y, s2v_stream_t stream) {
    S2V_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && h <= xh && w <= xw && xcs >= 3, "sr_f32_out: bad args");
    sr_f32_out_kernel<<<sr_grid((long long)n * h * w), 256, 0, (hipStream_t)stream>>>(x, n, h, w, xh, xw, xcs, flip,
                                                                                     y);
    return check_launch("sr_f32_out");
}
