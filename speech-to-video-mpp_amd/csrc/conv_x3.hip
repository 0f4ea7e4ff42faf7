// Weight preparation for the split-fp32 convolutions (conv_x3_impl.hpp): packed fp32 weights, or
// StyleGAN2 per-sample modulated weights, written once in the [rows][kpad/32][hi 32 | lo 32]
// 16-bit layout the kernels stage into LDS unchanged.  ``scale`` (a power of two) multiplies the
// weights before the split; the conv divides it out of the accumulators (s2v_conv_params.wt_scale).
#include "conv_x3_impl.hpp"

#include <cmath>

namespace s2v {

// [rows][kpad] fp32 -> [rows][kpad/32][hi 32 | lo 32] (kpad % 32 == 0)
template <int ELT>
__global__ __launch_bounds__(256) void split_weights_kernel(const float *__restrict__ w, long long slices,
                                                            float scale, char *__restrict__ out) {
    // one thread per 4 consecutive k of one 32-k slice
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < slices * 8; e += (long long)gridDim.x * 256) {
        const long long sl = e >> 3;
        const int q = (int)(e & 7);
        const f4 v = *(const f4 *)(w + sl * 32 + q * 4) * scale;
        u32x2 hi, lo;
        split4<ELT>(v, hi, lo);
        char *o = out + sl * 128 + q * 8;
        *(u32x2 *)o = hi;
        *(u32x2 *)(o + 64) = lo;
    }
}

// StyleGAN2 per-sample weights (s2v_modulate_weights) written directly in the split layout
template <int ELT>
__global__ __launch_bounds__(256) void modulate_weights_x3_kernel(const float *__restrict__ wt, int npad, int kpad,
                                                                  int K, int cin, int cout,
                                                                  const float *__restrict__ s, int s_ns,
                                                                  const float *__restrict__ d, int d_ns, int batch,
                                                                  float scale, char *__restrict__ out) {
    const long long per = (long long)npad * kpad;
    const long long total = per * batch;
    for (long long e = (blockIdx.x * 256LL + threadIdx.x) * 4; e < total; e += (long long)gridDim.x * 256 * 4) {
        const int b = (int)(e / per);
        const long long r = e - b * per;
        const int o = (int)(r / kpad), k = (int)(r - (long long)o * kpad);
        f4 w = *(const f4 *)(wt + r);
        const float dd = ((d && o < cout) ? d[(long long)b * d_ns + o] : 1.f) * scale;
        float f[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = (k + j < K) ? s[(long long)b * s_ns + (k + j) % cin] * dd : 0.f;
        w.x *= f[0]; w.y *= f[1]; w.z *= f[2]; w.w *= f[3];
        u32x2 hi, lo;
        split4<ELT>(w, hi, lo);
        char *ob = out + (e >> 5) * 128 + (k & 31) * 2;    // slice e/32, k-offset within it
        *(u32x2 *)ob = hi;
        *(u32x2 *)(ob + 64) = lo;
    }
}

static unsigned grid_x3(long long total) {
    long long b = (total + 255) / 256;
    if (b > 65535LL * 16) b = 65535LL * 16;
    return (unsigned)(b < 1 ? 1 : b);
}

static bool pow2_scale(float s) {
    int e;
    return s > 0.f && std::frexp(s, &e) == 0.5f;
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_split_weights(const float *w, int rows, int kpad, int prec, float scale, void *out,
                                 s2v_stream_t stream) {
    S2V_REQUIRE(w && out && rows > 0 && kpad > 0 && kpad % 32 == 0, "split_weights: bad args");
    S2V_REQUIRE(prec == S2V_PREC_BF16X3 || prec == S2V_PREC_F16X3, "split_weights: prec must be BF16X3 or F16X3");
    S2V_REQUIRE(pow2_scale(scale), "split_weights: scale must be a positive power of two, got %g", scale);
    S2V_REQUIRE(((uintptr_t)w % 16) == 0 && ((uintptr_t)out % 16) == 0, "split_weights: 16-byte alignment");
    const long long slices = (long long)rows * (kpad / 32);
    if (prec == S2V_PREC_BF16X3)
        split_weights_kernel<0><<<grid_x3(slices * 8), 256, 0, (hipStream_t)stream>>>(w, slices, scale, (char *)out);
    else
        split_weights_kernel<1><<<grid_x3(slices * 8), 256, 0, (hipStream_t)stream>>>(w, slices, scale, (char *)out);
    return check_launch("split_weights");
}

extern "C" int s2v_split_weights_x3(const float *w, int rows, int kpad, void *out, s2v_stream_t stream) {
    return s2v_split_weights(w, rows, kpad, S2V_PREC_BF16X3, 1.f, out, stream);
}

extern "C" int s2v_modulate_weights_split(const float *wt, int npad, int kpad, int K, int cin, int cout,
                                          const float *s, int s_ns, const float *d, int d_ns, int batch, int prec,
                                          float scale, void *out, s2v_stream_t stream) {
    S2V_REQUIRE(wt && s && out && npad > 0 && kpad > 0 && K > 0 && K <= kpad && cin > 0 && cout > 0 && cout <= npad &&
                batch > 0 && s_ns >= cin && (!d || d_ns >= cout), "modulate_weights_split: bad args");
    S2V_REQUIRE(prec == S2V_PREC_BF16X3 || prec == S2V_PREC_F16X3, "modulate_weights_split: prec must be BF16X3 or F16X3");
    S2V_REQUIRE(pow2_scale(scale), "modulate_weights_split: scale must be a positive power of two, got %g", scale);
    S2V_REQUIRE(kpad % 32 == 0 && ((uintptr_t)wt % 16) == 0 && ((uintptr_t)out % 16) == 0,
                "modulate_weights_split: kpad %% 32 and 16-byte aligned buffers required");
    const unsigned g = grid_x3((long long)npad * kpad * batch / 4);
    if (prec == S2V_PREC_BF16X3)
        modulate_weights_x3_kernel<0><<<g, 256, 0, (hipStream_t)stream>>>(wt, npad, kpad, K, cin, cout, s, s_ns, d,
                                                                           d_ns, batch, scale, (char *)out);
    else
        modulate_weights_x3_kernel<1><<<g, 256, 0, (hipStream_t)stream>>>(wt, npad, kpad, K, cin, cout, s, s_ns, d,
                                                                           d_ns, batch, scale, (char *)out);
    return check_launch("modulate_weights_split");
}

extern "C" int s2v_modulate_weights_x3(const float *wt, int npad, int kpad, int K, int cin, int cout, const float *s,
                                       int s_ns, const float *d, int d_ns, int batch, void *out,
                                       s2v_stream_t stream) {
    return s2v_modulate_weights_split(wt, npad, kpad, K, cin, cout, s, s_ns, d, d_ns, batch, S2V_PREC_BF16X3, 1.f,
                                      out, stream);
}
