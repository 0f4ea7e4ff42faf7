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
#include "conv_x3_impl.hpp"

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
// MFMA variants for the LNet sizes (H == W in {12, 24, 48}): one block per (image, 4-channel
// group); both 1-D passes of the tile run as small GEMMs out of LDS on v_mfma_f32_32x32x2_f32
// (exact fp32 products and sums, the k-ordered fma chains of the generic kernels):
//   rfft2   W pass  Y[(p,h)][(v,c)] = sum_w fw[w][p][v] X[h][w][c]        rows (p,v), K = w
//           H pass  Z[q][u][(v,c)]  = sum_h fh[h][u] * Y[h][(v,c)]       complex, rows u, K = h
//   irfft2  H pass  Y[p][h][(v,c)]  = sum_u ih[u][h] * Z[u][(v,c)]       complex, rows h, K = u
//           W pass  y[h][w][c]      = sum_(v,p) iw[v][p][w] Y[(p,h)][(v,c)]   rows w, K = 2v + p
// 32x32x2 f32 operand maps: lane l holds A[l & 31][k0 + (l >> 5)] and B[k0 + (l >> 5)][l & 31];
// the accumulator holds column l & 31, rows (r & 3) + 8 (r >> 2) + 4 (l >> 5).  Against the
// VALU register-blocked form this replaces (one thread per output row, 1.4M serial fmas per
// block), the waves of a block (4, or 8 at 48x48) share every pass.
typedef float mf16 __attribute__((ext_vector_type(16)));
constexpr int FCG = 4;   // channels per block (the kernels take it as a template parameter)

__device__ __forceinline__ int mf_row(int r, int lh) { return (r & 3) + 8 * (r >> 2) + 4 * lh; }

__device__ __forceinline__ mf16 mfma32(float a, float b, mf16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// (image, channel group) of block b.  The channel groups of one image go to one XCD (block b runs on
// XCD b % 8): image n on XCD n % 8 when the image count is a multiple of 8, so the pixel rows an image's
// blocks read (16 bytes of each per block) and the spectrum rows they write in 16-byte pieces stay
// in that XCD's L2 instead of being fetched / written back once per XCD (r02: rfft2_mf<48> moved 63 MB
// per launch for 14 MB of data)
__device__ __forceinline__ void fft_block(int groups, int &n, int &g) {
    const int b = blockIdx.x, nimg = gridDim.x / groups;
    if ((nimg & 7) == 0) {
        const int idx = b >> 3;
        n = (idx / groups) * 8 + (b & 7);
        g = idx - (idx / groups) * groups;
    } else {
        n = b / groups;
        g = b - n * groups;
    }
}

template <int CG> struct VecOf;
template <> struct VecOf<4> { typedef float4 T; };
template <> struct VecOf<2> { typedef float2 T; };

template <int H, int NWV, int FCG = 4>
__global__ __launch_bounds__(64 * NWV) void rfft2_mf(const float *__restrict__ x, int C, int xcs,
                                                const float *__restrict__ tables, float *__restrict__ spec,
                                                int scs) {
    constexpr int W = H, WF = W / 2 + 1;
    constexpr int XS = W * FCG + 4;                  // X row pitch: the B reads of 8 rows hit distinct banks
    constexpr int N1 = H * FCG, N2 = WF * FCG;       // W-pass columns (h, c), H-pass columns (v, c)
    constexpr int T1M = (2 * WF + 31) / 32, T1N = (N1 + 31) / 32;
    constexpr int T2M = (H + 31) / 32, T2N = (N2 + 31) / 32;
    __shared__ float X[H * XS];
    __shared__ float Y[2 * H * N2];                  // [(p, h)][(v, c)]
    __shared__ float Tw[W * 2 * WF];                 // fw[w][p][v]
    __shared__ float Th[H * 2 * H];                  // fh[h][p][u]
    int n, g;
    fft_block(C / FCG, n, g);
    const int c0 = g * FCG;
    const int tid = threadIdx.x, wave = tid >> 6, li = tid & 31, lh = (tid >> 5) & 1;
    const FftTables T = fft_tables(tables, H, W);
    for (int i = tid; i < W * 2 * WF; i += 64 * NWV) Tw[i] = T.fw[i];
    for (int i = tid; i < H * 2 * H; i += 64 * NWV) Th[i] = T.fh[i];
    for (int p = tid; p < H * W; p += 64 * NWV) {
        const int hh = p / W, ww = p - hh * W;
        typedef typename VecOf<FCG>::T V;
        *(V *)&X[hh * XS + ww * FCG] = *(const V *)&x[((long long)n * H * W + p) * xcs + c0];
    }
    __syncthreads();
    for (int t = wave; t < T1M * T1N; t += NWV) {      // W pass (real -> half spectrum)
        const int tm = t / T1N, tn = t - tm * T1N;
        const int i = tm * 32 + li, j = tn * 32 + li;
        const bool iok = i < 2 * WF, jok = j < N1;
        const float *xb = X + (j / FCG) * XS + (j % FCG);
        mf16 acc = {};
        for (int k0 = 0; k0 < W; k0 += 2) {
            const int k = k0 + lh;
            acc = mfma32(iok ? Tw[k * 2 * WF + i] : 0.f, jok ? xb[k * FCG] : 0.f, acc);
        }
        if (jok) {
            const int hh = j / FCG, cc = j % FCG;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = tm * 32 + mf_row(r, lh);
                if (row < 2 * WF) {
                    const int p = row >= WF ? 1 : 0, v = row - p * WF;
                    Y[(p * H + hh) * N2 + v * FCG + cc] = acc[r];
                }
            }
        }
    }
    __syncthreads();
    for (int t = wave; t < T2M * T2N; t += NWV) {      // H pass (complex)
        const int tm = t / T2N, tn = t - tm * T2N;
        const int u = tm * 32 + li, j = tn * 32 + li;
        const bool uok = u < H, jok = j < N2;
        mf16 zr = {}, zi = {};
        for (int k0 = 0; k0 < H; k0 += 2) {
            const int h = k0 + lh;
            const float fr = uok ? Th[(h * 2 + 0) * H + u] : 0.f, fi = uok ? Th[(h * 2 + 1) * H + u] : 0.f;
            const float yr = jok ? Y[h * N2 + j] : 0.f, yi = jok ? Y[(H + h) * N2 + j] : 0.f;
            zr = mfma32(-fi, yi, zr);
            zr = mfma32(fr, yr, zr);
            zi = mfma32(fr, yi, zi);
            zi = mfma32(fi, yr, zi);
        }
        if (jok) {
            const int v = j / FCG, cc = j % FCG;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int uu = tm * 32 + mf_row(r, lh);
                if (uu < H) {
                    float *o = spec + ((long long)n * H * WF + uu * WF + v) * scs + c0 + cc;
                    o[0] = zr[r];
                    o[C] = zi[r];
                }
            }
        }
    }
}

template <int H, int NWV, int FCG = 4>
__global__ __launch_bounds__(64 * NWV) void irfft2_mf(const float *__restrict__ spec, int C, int scs,
                                                 const float *__restrict__ tables, const float *__restrict__ res,
                                                 int rcs, float *__restrict__ y, int ycs) {
    constexpr int W = H, WF = W / 2 + 1;
    constexpr int N1 = WF * FCG, N2 = H * FCG;       // H-pass columns (v, c), W-pass columns (h, c)
    constexpr int T1M = (H + 31) / 32, T1N = (N1 + 31) / 32;
    constexpr int T2M = (W + 31) / 32, T2N = (N2 + 31) / 32;
    __shared__ float Z[2 * H * N1];                  // [(q, u)][(v, c)]
    __shared__ float Y[2 * H * N1];                  // [(p, h)][(v, c)]
    __shared__ float Ti[H * 2 * H];                  // ih[u][p][h]
    __shared__ float Tw[WF * 2 * W];                 // iw[v][p][w]
    int n, g;
    fft_block(C / FCG, n, g);
    const int c0 = g * FCG;
    const int tid = threadIdx.x, wave = tid >> 6, li = tid & 31, lh = (tid >> 5) & 1;
    const FftTables T = fft_tables(tables, H, W);
    for (int i = tid; i < H * 2 * H; i += 64 * NWV) Ti[i] = T.ih[i];
    for (int i = tid; i < WF * 2 * W; i += 64 * NWV) Tw[i] = T.iw[i];
    for (int i = tid; i < H * WF * 2; i += 64 * NWV) {
        const int q = i & 1, f = i >> 1;
        const int u = f / WF, v = f - u * WF;
        typedef typename VecOf<FCG>::T V;
        *(V *)&Z[(q * H + u) * N1 + v * FCG] = *(const V *)&spec[((long long)n * H * WF + f) * scs + q * C + c0];
    }
    __syncthreads();
    for (int t = wave; t < T1M * T1N; t += NWV) {      // inverse H pass (complex)
        const int tm = t / T1N, tn = t - tm * T1N;
        const int h = tm * 32 + li, j = tn * 32 + li;
        const bool hok = h < H, jok = j < N1;
        mf16 yr = {}, yi = {};
        for (int k0 = 0; k0 < H; k0 += 2) {
            const int u = k0 + lh;
            const float gr = hok ? Ti[(u * 2 + 0) * H + h] : 0.f, gi = hok ? Ti[(u * 2 + 1) * H + h] : 0.f;
            const float zr = jok ? Z[u * N1 + j] : 0.f, zi = jok ? Z[(H + u) * N1 + j] : 0.f;
            yr = mfma32(-gi, zi, yr);
            yr = mfma32(gr, zr, yr);
            yi = mfma32(gr, zi, yi);
            yi = mfma32(gi, zr, yi);
        }
        if (jok) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int hh = tm * 32 + mf_row(r, lh);
                if (hh < H) {
                    Y[hh * N1 + j] = yr[r];
                    Y[(H + hh) * N1 + j] = yi[r];
                }
            }
        }
    }
    __syncthreads();
    for (int t = wave; t < T2M * T2N; t += NWV) {      // c2r W pass
        const int tm = t / T2N, tn = t - tm * T2N;
        const int w = tm * 32 + li, j = tn * 32 + li;
        const bool wok = w < W, jok = j < N2;
        const int hh = j / FCG, cc = j % FCG;
        mf16 acc = {};
        for (int k0 = 0; k0 < 2 * WF; k0 += 2) {
            const int k = k0 + lh, v = k >> 1, p = k & 1;     // k = 2 v + p
            acc = mfma32(wok ? Tw[k * W + w] : 0.f, jok ? Y[(p * H + hh) * N1 + v * FCG + cc] : 0.f, acc);
        }
        if (jok) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int ww = tm * 32 + mf_row(r, lh);
                if (ww < W) {
                    const long long pix = ((long long)n * H + hh) * W + ww;
                    float o = acc[r];
                    if (res) o += res[pix * rcs + c0 + cc];
                    y[pix * ycs + c0 + cc] = o;
                }
            }
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
        // 48x48: 8 waves per block (one block per CU by LDS).  2 channels per block (twice the blocks,
        // 4 waves) measured slower on MI355X: rfft 29.7 -> 35.7 us, irfft 34.6 -> 40.5 us (r02)
        if (h == 12) rfft2_mf<12, 4><<<grid, 256, 0, st>>>(x, c, xcs, tables, spec, scs);
        else if (h == 24) rfft2_mf<24, 4><<<grid, 256, 0, st>>>(x, c, xcs, tables, spec, scs);
        else rfft2_mf<48, 8><<<grid, 512, 0, st>>>(x, c, xcs, tables, spec, scs);
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
        if (h == 12) irfft2_mf<12, 4><<<grid, 256, 0, st>>>(spec, c, scs, tables, res, rcs, y, ycs);
        else if (h == 24) irfft2_mf<24, 4><<<grid, 256, 0, st>>>(spec, c, scs, tables, res, rcs, y, ycs);
        else irfft2_mf<48, 8><<<grid, 512, 0, st>>>(spec, c, scs, tables, res, rcs, y, ycs);
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
