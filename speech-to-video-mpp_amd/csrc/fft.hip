// Separable 2-D real DFTs for the FourierUnit (models/ffc.py:93-126: rfftn / irfftn over (H, W),
// norm='ortho'), NHWC in, the FourierUnit's spectrum layout out.
//
//   forward:  x[n, h, w, c]  ->  spec[n, u*Wf + v, part*C + c]    (Wf = W/2 + 1, part 0 = re, 1 = im)
//   inverse:  spec[n, f, part*C + c]  ->  y[n, h, w, c] = irfft2(spec) + res[n, h, w, c]
//
// One block per (sample, group of CG channels): the tile is staged in LDS and transformed along W
// (real <-> half spectrum) and along H (complex), so a 48x48 transform costs 2*Wf*W + 4*H*H
// multiply-adds per pixel-channel instead of the 2*F*H*W of a dense 2-D DFT matrix.  The 1-D
// transform matrices come from the host (built by applying torch.fft to basis vectors, so the
// ortho scaling and the c2r treatment of the DC / Nyquist imaginary parts are exactly torch's):
//   tables = fw[W][2][Wf] | fh[H][2][H] | ih[H][2][H] | iw[Wf][2][W]
// (each matrix stored loop-invariant-index major: the inner loops of the kernels walk the last,
// contiguous index, so wave-uniform reads of a row batch into wide scalar loads).
#include "common.hpp"

namespace s2v {

struct FftTables {
    const float *fw, *fh, *ih, *iw;
};

__host__ __device__ inline FftTables fft_tables(const float *t, int H, int W) {
    const int wf = W / 2 + 1;
    FftTables r;
    r.fw = t;
    r.fh = r.fw + 2 * wf * W;
    r.ih = r.fh + 2 * H * H;
    r.iw = r.ih + 2 * H * H;
    return r;
}

// dynamic LDS: X[H][W][CG] | Y[H][Wf][2][CG] | fw[2][Wf][W] | fh[2][H][H]
__global__ __launch_bounds__(256) void rfft2_kernel(const float *__restrict__ x, int H, int W, int C, int xcs,
                                                    const float *__restrict__ tables, int CG,
                                                    float *__restrict__ spec, int scs) {
    extern __shared__ float sm[];
    const int wf = W / 2 + 1;
    const int groups = C / CG;
    const int n = blockIdx.x / groups, c0 = (blockIdx.x - n * groups) * CG;
    const int XS = W * CG + 4;   // padded row stride: the 16 rows a wave touches hit distinct banks
    float *X = sm;
    float *Y = X + H * XS;
    float *Tw = Y + H * wf * 2 * CG;
    float *Th = Tw + 2 * wf * W;
    const FftTables T = fft_tables(tables, H, W);
    for (int i = threadIdx.x; i < 2 * wf * W; i += 256) Tw[i] = T.fw[i];
    for (int i = threadIdx.x; i < 2 * H * H; i += 256) Th[i] = T.fh[i];
    const int cv = CG / 4;
    for (int i = threadIdx.x; i < H * W * cv; i += 256) {
        const int p = i / cv, q = i - p * cv;
        const int hh = p / W, ww = p - hh * W;
        *(float4 *)&X[hh * XS + ww * CG + 4 * q] = *(const float4 *)&x[((long long)n * H * W + p) * xcs + c0 + 4 * q];
    }
    __syncthreads();
    // W pass: item (h, cg) -> Y[h][v][part][cg] for all v
    for (int it = threadIdx.x; it < H * CG; it += 256) {
        const int h = it / CG, cg = it - h * CG;
        for (int v = 0; v < wf; ++v) {
            float re = 0.f, im = 0.f;
            const float *xr = X + h * XS + cg;
            for (int w = 0; w < W; ++w) {
                const float xv = xr[w * CG];
                re = fmaf(Tw[(w * 2 + 0) * wf + v], xv, re);
                im = fmaf(Tw[(w * 2 + 1) * wf + v], xv, im);
            }
            Y[((h * wf + v) * 2 + 0) * CG + cg] = re;
            Y[((h * wf + v) * 2 + 1) * CG + cg] = im;
        }
    }
    __syncthreads();
    // H pass (complex): item (v, cg, u) -> spec[n][u*wf + v][part*C + c0 + cg]
    for (int it = threadIdx.x; it < H * wf * CG; it += 256) {
        const int cg = it % CG;
        const int t = it / CG;
        const int v = t % wf, u = t / wf;
        float zr = 0.f, zi = 0.f;
        for (int h = 0; h < H; ++h) {
            const float yr = Y[((h * wf + v) * 2 + 0) * CG + cg], yi = Y[((h * wf + v) * 2 + 1) * CG + cg];
            const float fr = Th[(h * 2 + 0) * H + u], fi = Th[(h * 2 + 1) * H + u];
            zr = fmaf(fr, yr, fmaf(-fi, yi, zr));
            zi = fmaf(fi, yr, fmaf(fr, yi, zi));
        }
        float *o = spec + ((long long)n * H * wf + u * wf + v) * scs + c0 + cg;
        o[0] = zr;
        o[C] = zi;
    }
}

// dynamic LDS: Z[H][Wf][2][CG] | Y[H][Wf][2][CG] | ih[2][H][H] | iw[2][W][Wf]
__global__ __launch_bounds__(256) void irfft2_kernel(const float *__restrict__ spec, int H, int W, int C, int scs,
                                                     const float *__restrict__ tables, int CG,
                                                     const float *__restrict__ res, int rcs, float *__restrict__ y,
                                                     int ycs) {
    extern __shared__ float sm[];
    const int wf = W / 2 + 1;
    const int groups = C / CG;
    const int n = blockIdx.x / groups, c0 = (blockIdx.x - n * groups) * CG;
    float *Z = sm;
    float *Y = Z + H * wf * 2 * CG;
    float *Ti = Y + H * wf * 2 * CG;
    float *Tw = Ti + 2 * H * H;
    const FftTables T = fft_tables(tables, H, W);
    for (int i = threadIdx.x; i < 2 * H * H; i += 256) Ti[i] = T.ih[i];
    for (int i = threadIdx.x; i < 2 * W * wf; i += 256) Tw[i] = T.iw[i];
    const int cv = CG / 4;
    for (int i = threadIdx.x; i < H * wf * 2 * cv; i += 256) {
        const int q = i % cv;
        const int t = i / cv;
        const int part = t & 1, f = t >> 1;
        *(float4 *)&Z[(f * 2 + part) * CG + 4 * q] =
            *(const float4 *)&spec[((long long)n * H * wf + f) * scs + part * C + c0 + 4 * q];
    }
    __syncthreads();
    // inverse H pass (complex): item (h, v, cg)
    for (int it = threadIdx.x; it < H * wf * CG; it += 256) {
        const int cg = it % CG;
        const int t = it / CG;
        const int v = t % wf, h = t / wf;
        float yr = 0.f, yi = 0.f;
        for (int u = 0; u < H; ++u) {
            const float zr = Z[((u * wf + v) * 2 + 0) * CG + cg], zi = Z[((u * wf + v) * 2 + 1) * CG + cg];
            const float gr = Ti[(u * 2 + 0) * H + h], gi = Ti[(u * 2 + 1) * H + h];
            yr = fmaf(gr, zr, fmaf(-gi, zi, yr));
            yi = fmaf(gi, zr, fmaf(gr, zi, yi));
        }
        Y[((h * wf + v) * 2 + 0) * CG + cg] = yr;
        Y[((h * wf + v) * 2 + 1) * CG + cg] = yi;
    }
    __syncthreads();
    // c2r W pass: item (h, w, cg) -> y = sum_v iw_re[w][v] Yr + iw_im[w][v] Yi (+ res)
    for (int it = threadIdx.x; it < H * W * CG; it += 256) {
        const int cg = it % CG;
        const int t = it / CG;
        const int w = t % W, h = t / W;
        float acc = 0.f;
        for (int v = 0; v < wf; ++v)
            acc = fmaf(Tw[(v * 2 + 0) * W + w], Y[((h * wf + v) * 2 + 0) * CG + cg],
                       fmaf(Tw[(v * 2 + 1) * W + w], Y[((h * wf + v) * 2 + 1) * CG + cg], acc));
        const long long p = (long long)n * H * W + h * W + w;
        if (res) acc += res[p * rcs + c0 + cg];
        y[p * ycs + c0 + cg] = acc;
    }
}

// ---------------------------------------------------------------------------------------------
// Register-blocked variants for the LNet sizes (12, 24, 48): each thread keeps a whole output
// row / column of accumulators and the 1-D matrices are read with wave-uniform indices straight
// from global memory (scalar loads into SGPRs), so LDS carries only the data (one read per
// input element per pass) instead of one LDS read per multiply-add.
constexpr int FCG = 4;   // channels per block

template <int H, int W>
__global__ __launch_bounds__(256) void rfft2_rb(const float *__restrict__ x, int C, int xcs,
                                                const float *__restrict__ tables, float *__restrict__ spec,
                                                int scs) {
    constexpr int WF = W / 2 + 1;
    constexpr int XS = W * FCG + 4;
    constexpr int UC = H >= 24 ? H / 2 : H;          // u rows per H-pass item
    __shared__ float X[H * XS];
    __shared__ float Y[H * WF * 2 * FCG];
    const int groups = C / FCG;
    const int n = blockIdx.x / groups, c0 = (blockIdx.x - n * groups) * FCG;
    const FftTables T = fft_tables(tables, H, W);
    for (int p = threadIdx.x; p < H * W; p += 256) {
        const int hh = p / W, ww = p - hh * W;
        *(float4 *)&X[hh * XS + ww * FCG] = *(const float4 *)&x[((long long)n * H * W + p) * xcs + c0];
    }
    __syncthreads();
    if (threadIdx.x < H * FCG) {                      // W pass: item (h, cg), all WF bins
        const int h = threadIdx.x / FCG, cg = threadIdx.x % FCG;
        float re[WF], im[WF];
#pragma unroll
        for (int v = 0; v < WF; ++v) re[v] = im[v] = 0.f;
        for (int w = 0; w < W; ++w) {
            const float xv = X[h * XS + w * FCG + cg];
#pragma unroll
            for (int v = 0; v < WF; ++v) {
                re[v] = fmaf(T.fw[(w * 2 + 0) * WF + v], xv, re[v]);
                im[v] = fmaf(T.fw[(w * 2 + 1) * WF + v], xv, im[v]);
            }
        }
#pragma unroll
        for (int v = 0; v < WF; ++v) {
            Y[((h * WF + v) * 2 + 0) * FCG + cg] = re[v];
            Y[((h * WF + v) * 2 + 1) * FCG + cg] = im[v];
        }
    }
    __syncthreads();
    // H pass: item (v, cg) of u-chunk q; each chunk padded to whole waves so that u0 (and with it
    // every table index) is wave-uniform
    constexpr int IPC = (WF * FCG + 63) / 64 * 64;
    for (int it = threadIdx.x; it < IPC * (H / UC); it += 256) {
        const int q = it / IPC, r = it - q * IPC;
        if (r >= WF * FCG) continue;
        const int cg = r % FCG;
        const int v = r / FCG, u0 = q * UC;
        float zr[UC], zi[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u) zr[u] = zi[u] = 0.f;
        for (int h = 0; h < H; ++h) {
            const float yr = Y[((h * WF + v) * 2 + 0) * FCG + cg], yi = Y[((h * WF + v) * 2 + 1) * FCG + cg];
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                const float fr = T.fh[(h * 2 + 0) * H + u0 + u], fi = T.fh[(h * 2 + 1) * H + u0 + u];
                zr[u] = fmaf(fr, yr, fmaf(-fi, yi, zr[u]));
                zi[u] = fmaf(fi, yr, fmaf(fr, yi, zi[u]));
            }
        }
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            float *o = spec + ((long long)n * H * WF + (u0 + u) * WF + v) * scs + c0 + cg;
            o[0] = zr[u];
            o[C] = zi[u];
        }
    }
}

template <int H, int W>
__global__ __launch_bounds__(256) void irfft2_rb(const float *__restrict__ spec, int C, int scs,
                                                 const float *__restrict__ tables, const float *__restrict__ res,
                                                 int rcs, float *__restrict__ y, int ycs) {
    constexpr int WF = W / 2 + 1;
    constexpr int HC = H >= 24 ? H / 2 : H;          // h rows per inverse-H item
    __shared__ float Z[H * WF * 2 * FCG];
    __shared__ float Y[H * WF * 2 * FCG];
    const int groups = C / FCG;
    const int n = blockIdx.x / groups, c0 = (blockIdx.x - n * groups) * FCG;
    const FftTables T = fft_tables(tables, H, W);
    for (int i = threadIdx.x; i < H * WF * 2; i += 256) {
        const int part = i & 1, f = i >> 1;
        *(float4 *)&Z[(f * 2 + part) * FCG] = *(const float4 *)&spec[((long long)n * H * WF + f) * scs + part * C + c0];
    }
    __syncthreads();
    constexpr int IPC = (WF * FCG + 63) / 64 * 64;   // inverse H: item (v, cg) of h-chunk q (wave-uniform h0)
    for (int it = threadIdx.x; it < IPC * (H / HC); it += 256) {
        const int q = it / IPC, r = it - q * IPC;
        if (r >= WF * FCG) continue;
        const int cg = r % FCG;
        const int v = r / FCG, h0 = q * HC;
        float yr[HC], yi[HC];
#pragma unroll
        for (int h = 0; h < HC; ++h) yr[h] = yi[h] = 0.f;
        for (int u = 0; u < H; ++u) {
            const float zr = Z[((u * WF + v) * 2 + 0) * FCG + cg], zi = Z[((u * WF + v) * 2 + 1) * FCG + cg];
#pragma unroll
            for (int h = 0; h < HC; ++h) {
                const float gr = T.ih[(u * 2 + 0) * H + h0 + h], gi = T.ih[(u * 2 + 1) * H + h0 + h];
                yr[h] = fmaf(gr, zr, fmaf(-gi, zi, yr[h]));
                yi[h] = fmaf(gi, zr, fmaf(gr, zi, yi[h]));
            }
        }
#pragma unroll
        for (int h = 0; h < HC; ++h) {
            Y[(((h0 + h) * WF + v) * 2 + 0) * FCG + cg] = yr[h];
            Y[(((h0 + h) * WF + v) * 2 + 1) * FCG + cg] = yi[h];
        }
    }
    __syncthreads();
    if (threadIdx.x < H * FCG) {                      // c2r W pass: item (h, cg), all W outputs
        const int h = threadIdx.x / FCG, cg = threadIdx.x % FCG;
        float acc[W];
#pragma unroll
        for (int w = 0; w < W; ++w) acc[w] = 0.f;
        for (int v = 0; v < WF; ++v) {
            const float a = Y[((h * WF + v) * 2 + 0) * FCG + cg], b = Y[((h * WF + v) * 2 + 1) * FCG + cg];
#pragma unroll
            for (int w = 0; w < W; ++w) acc[w] = fmaf(T.iw[(v * 2 + 0) * W + w], a, fmaf(T.iw[(v * 2 + 1) * W + w], b, acc[w]));
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const long long p = (long long)n * H * W + h * W + w;
            float o = acc[w];
            if (res) o += res[p * rcs + c0 + cg];
            y[p * ycs + c0 + cg] = o;
        }
    }
}

// 4 channels per block: the most blocks (the transforms are small, parallelism matters more
// than table reuse), 16-byte channel vectors for the global loads / stores.
static int pick_cg(int C, int H, int W, size_t per_cg_floats, size_t fixed_floats) {
    (void)H; (void)W;
    return (C % 4 == 0 && (per_cg_floats * 4 + fixed_floats) * sizeof(float) <= 160 * 1024) ? 4 : 0;
}

}  // namespace s2v

using namespace s2v;

extern "C" size_t s2v_fft_tables_floats(int h, int w) {
    const int wf = w / 2 + 1;
    return (size_t)2 * wf * w + (size_t)4 * h * h + (size_t)2 * w * wf;
}

extern "C" int s2v_rfft2(const float *x, int n, int h, int w, int c, int xcs, const float *tables, float *spec,
                         int scs, s2v_stream_t stream) {
    S2V_REQUIRE(x && tables && spec && n > 0 && h > 0 && w > 1 && c > 0, "rfft2: bad args");
    S2V_REQUIRE(xcs >= c && xcs % 4 == 0 && scs >= 2 * c && scs % 4 == 0 && ((uintptr_t)x % 16) == 0 &&
                ((uintptr_t)spec % 16) == 0, "rfft2: channel pitches must be >= C (2C) and multiples of 4");
    const int wf = w / 2 + 1;
    const size_t per = (size_t)h * w + (size_t)h * wf * 2, fixed = (size_t)2 * wf * w + (size_t)2 * h * h + 4 * h;
    const int cg = pick_cg(c, h, w, per, fixed);
    S2V_REQUIRE(cg > 0, "rfft2: C %% 4 != 0 or the %dx%d tile does not fit in LDS", h, w);
    const bool aligned = xcs % 4 == 0 && ((uintptr_t)x % 16) == 0;
    hipStream_t st = (hipStream_t)stream;
    if (c % FCG == 0 && aligned && h == w && (h == 12 || h == 24 || h == 48)) {
        const unsigned grid = n * (c / FCG);
        if (h == 12) rfft2_rb<12, 12><<<grid, 256, 0, st>>>(x, c, xcs, tables, spec, scs);
        else if (h == 24) rfft2_rb<24, 24><<<grid, 256, 0, st>>>(x, c, xcs, tables, spec, scs);
        else rfft2_rb<48, 48><<<grid, 256, 0, st>>>(x, c, xcs, tables, spec, scs);
        return check_launch("rfft2");
    }
    const size_t smem = (per * cg + fixed) * sizeof(float);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)rfft2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    rfft2_kernel<<<n * (c / cg), 256, smem, (hipStream_t)stream>>>(x, h, w, c, xcs, tables, cg, spec, scs);
    return check_launch("rfft2");
}

extern "C" int s2v_irfft2(const float *spec, int n, int h, int w, int c, int scs, const float *tables,
                          const float *res, int rcs, float *y, int ycs, s2v_stream_t stream) {
    S2V_REQUIRE(spec && tables && y && n > 0 && h > 0 && w > 1 && c > 0, "irfft2: bad args");
    S2V_REQUIRE(ycs >= c && scs >= 2 * c && scs % 4 == 0 && ((uintptr_t)spec % 16) == 0 && (!res || rcs >= c),
                "irfft2: bad channel pitches");
    const int wf = w / 2 + 1;
    const size_t per = (size_t)h * wf * 4, fixed = (size_t)2 * h * h + (size_t)2 * w * wf;
    const int cg = pick_cg(c, h, w, per, fixed);
    S2V_REQUIRE(cg > 0, "irfft2: C %% 4 != 0 or the %dx%d tile does not fit in LDS", h, w);
    hipStream_t st = (hipStream_t)stream;
    if (c % FCG == 0 && h == w && (h == 12 || h == 24 || h == 48)) {
        const unsigned grid = n * (c / FCG);
        if (h == 12) irfft2_rb<12, 12><<<grid, 256, 0, st>>>(spec, c, scs, tables, res, rcs, y, ycs);
        else if (h == 24) irfft2_rb<24, 24><<<grid, 256, 0, st>>>(spec, c, scs, tables, res, rcs, y, ycs);
        else irfft2_rb<48, 48><<<grid, 256, 0, st>>>(spec, c, scs, tables, res, rcs, y, ycs);
        return check_launch("irfft2");
    }
    const size_t smem = (per * cg + fixed) * sizeof(float);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)irfft2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    irfft2_kernel<<<n * (c / cg), 256, smem, (hipStream_t)stream>>>(spec, h, w, c, scs, tables, cg, res, rcs, y, ycs);
    return check_launch("irfft2");
}
