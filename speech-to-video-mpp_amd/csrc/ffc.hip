// LNet's FFC spectral branch and InstanceNorm as three fused kernels per FFC (gfx950).
//
// FineADAINLama (models/base_blocks.py:368-386) = FFC (models/ffc.py:176-233, ratio 0.75) + ADAIN(bn_l | bn_g)
// + LeakyReLU.  Its global branch is SpectralTransform (ffc.py:129-173):
//     t1 = relu(bn1(conv1(x_g)))                         conv1 = "st1", 1x1 cg -> cc
//     u  = irfftn(relu(bn_fu(conv_fu(rfftn(t1))))) + t1  FourierUnit (ffc.py:60-126), conv_fu 1x1 2cc -> 2cc
//     y_g = conv_l2g(x_l) + conv2(u)                     conv2 = "st2", 1x1 cc -> cg
// Run as separate launches that chain is st1 -> rfft2 -> fu -> irfft2 -> st2, five small dependent kernels
// of ~10-15 us each on MI355X (r04: 54 FFCs per forward, ~650 launches).  Here it is two kernels plus the
// norm, one block per (image, channel slice) each:
//   ffc_spec_fwd:  the st1 GEMM of the block's t1 channels over ALL pixels of its image (so the rfft of
//                  those channels needs no other block), BN + ReLU into LDS, then the rfft2 of the slice
//                  (the FourierUnit's [B, F, 2C] spectrum layout, as fft.hip);
//   ffc_spec_inv:  the fu GEMM of the slice's re / im output channels over all frequencies of the image,
//                  BN + ReLU into LDS, then the irfft2 of the slice + t1 -> u;
//   ffc_norm:      per (image, channel slice) of y = [y_l | y_g]: the l slices as written by conv_to_l,
//                  the g slices = conv_l2g output + the st2 GEMM of u (all pixels of the image: so the
//                  InstanceNorm statistics of the slice need no other block), then ADAIN + LeakyReLU (+ the
//                  FFCResnetBlock residual) and the reflect-padded copy the next FFC's 3x3 convs read.
// The GEMMs use the split-fp32 operands of conv_x3_impl.hpp (f16x3 / bf16x3 on the 16x16x32 MFMA, the
// packed split weights staged once per block in LDS, A streamed from global two load groups deep); the
// DFTs are the fp32-MFMA separable transforms of fft.hip run on the LDS tile.  Levels (H, C): (12, 1024),
// (24, 256), (48, 128); B % 8 == 0 images put all blocks of image n on XCD n % 8.
#include "conv_x3_impl.hpp"

#include <cmath>

namespace s2v {

template <int H>
struct FfcLevel {
    static constexpr int C = H == 12 ? 1024 : (H == 24 ? 256 : 128);
    static constexpr int CL = C / 4, CG = C - CL, CC = CG / 2;
    static constexpr int W = H, HW = H * W, WF = W / 2 + 1, F = H * WF;
    // channels per block: spec_fwd (t1 channels), spec_inv (u channels; the GEMM computes their re and im
    // spectra), norm
    static constexpr int CS1 = H == 12 ? 32 : (H == 24 ? 16 : 4);
    static constexpr int CS2 = H == 12 ? 16 : (H == 24 ? 16 : 4);
    static constexpr int CSO = H == 48 ? 8 : 16;
    static constexpr int NSL_G = CG / 32;           // 32-deep K slices of st1 (K = cg) and fu (K = 2cc = cg)
    static constexpr int NSL_C = (CC + 31) / 32;    // of st2 (K = cc; 48 at H = 48: a partial last slice)
};

struct FfcArgs {
    const float *a;          // GEMM A: image 0, row pitch lda floats, image stride a_bs floats
    int lda;
    long long a_bs;
    const char *wt;          // split packed weights [npad][kpad] (s2v_split_weights)
    int kpad;
    float acc_scale, x_scale;
    const float *scale, *shift;   // per GEMM output channel (folded BN), may be null
    const float *tables;     // fft_tables(H, H)
    const float *t1;         // spec_inv: the +t1 residual
    float *out, *out2;       // spec_fwd: t1, spec; spec_inv: u
    int *flag;               // f16x3 range guard: set when an accumulator is not finite
    // norm
    const float *y;
    int ycs;
    const float *gamma, *beta;
    int gb_ns;
    float eps;
    int act;
    float alpha;
    const float *res;
    int res_cs;
    float *nout;
    int nout_cs;
    float *pad;
    int pad_cs;
};

typedef float fmf16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int ffc_mf_row(int r, int lh) { return (r & 3) + 8 * (r >> 2) + 4 * lh; }
__device__ __forceinline__ fmf16 ffc_mfma32(float a, float b, fmf16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// block -> (image n, slice g): the slices of image n on XCD n % 8 when the image count is a multiple of 8
// (the blocks of an image read the same A rows and write one spectrum / u / y image: one L2)
__device__ __forceinline__ void ffc_block(int groups, int &n, int &g) {
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

// NB split weight rows (column b of the block's GEMM is weight row rowmap(b)) x NSL 32-deep K slices into
// LDS rows R = s * NB + b, 128 bytes each in the swizzled slot order of conv_x3_impl.hpp (slot_off)
// (every load of a batch of up to 8 per thread is issued before the first LDS store: the rows come from
// L2 / HBM, one round trip per batch instead of one per chunk)
template <int NB, int NSL, typename RowMap>
__device__ __forceinline__ void ffc_stage_b(char *Bs, const char *__restrict__ wt, int kpad, RowMap rowmap) {
    constexpr int TOTAL = NSL * NB * 8, PER = (TOTAL + 255) / 256, BAT = PER < 8 ? PER : 8;
#pragma unroll
    for (int i0 = 0; i0 < PER; i0 += BAT) {
        u32x4 v[BAT];
#pragma unroll
        for (int i = 0; i < BAT; ++i) {
            // unconditional loads (the index clamped into range): no branch between the loads of a batch
            const int e = min(threadIdx.x + 256 * (i0 + i), TOTAL - 1);
            const int slot = e & 7, r = e >> 3;
            const int b = r % NB, s = r / NB;
            v[i] = *(const u32x4 *)(wt + ((long long)rowmap(b) * kpad + s * 32) * 4 + slot * 16);
        }
#pragma unroll
        for (int i = 0; i < BAT; ++i) {
            // (clamped like the loads: a thread past the end rewrites the last chunk with the same bytes)
            const int e = min(threadIdx.x + 256 * (i0 + i), TOTAL - 1);
            const int slot = e & 7, r = e >> 3;
            const int b = r % NB, s = r / NB;
            *(u32x4 *)(Bs + slot_off(s * NB + b, slot)) = v[i];
        }
    }
}

// n floats (n % 4 == 0, 16-byte aligned both sides) global -> LDS, all loads of a thread in flight together
template <int N>
__device__ __forceinline__ void ffc_copy_lds(float *dst, const float *__restrict__ src) {
    constexpr int V = N / 4, PER = (V + 255) / 256;
    static_assert(N % 4 == 0, "table size");
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = *(const float4 *)(src + 4 * min((int)threadIdx.x + 256 * i, V - 1));
#pragma unroll
    for (int i = 0; i < PER; ++i) *(float4 *)(dst + 4 * min((int)threadIdx.x + 256 * i, V - 1)) = v[i];
}

// C[M x 16 NT] = A[M x K] B^T on 4 waves: 16-row strips round-robin over the waves (strip st on wave
// st % 4), A rows streamed from global (lane l: row l & 15 of the strip, k 8 (l >> 4) .. +7 of each 32-deep
// slice, the 16x16x32 MFMA's A fragment) and split in registers; B fragments from the staged LDS rows.
// Load groups of GS slices, up to D groups in flight.  epi(m, j, col, v) receives every output row m < M
// of N tile j (col = 16 j + lane % 16: fixed per lane and tile, so per-column parameters are loaded
// before the GEMM; a load in the epilogue would wait for every prefetched A group, vmcnt counting in issue
// order) with v = the raw fp32 accumulator.  Returns true when an accumulator was not finite.
template <int NT, int NSL, int ELT, typename Epi>
__device__ __forceinline__ bool ffc_strip_gemm(const float *__restrict__ A, int lda, int M, int K, float xscale,
                                               const char *Bs, Epi epi) {
    constexpr int NB = 16 * NT;
    constexpr int GS = NSL < 8 ? NSL : 8;
    constexpr int NG = (NSL + GS - 1) / GS;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, kq = lane >> 4;
    const int hs = (kq ^ swz(l16)) << 4, ls = hs ^ 64;
    const int nstrip = (M + 15) >> 4;
    const int mine = nstrip > wave ? (nstrip - wave + 3) >> 2 : 0;
    const int T = mine * NG;
    // units (strip, slice group) in flight per wave: D x GS x 8 VGPRs of A (<= 192)
    constexpr int D0 = 192 / (GS * 8);
    constexpr int D = D0 < 2 ? 2 : (D0 > 8 ? 8 : D0);
    bool bad = false;
    floatx4 acc[NT];
    f4 ra[D][GS][2];
    auto load = [&](f4(&r)[GS][2], int t) {
        const int st = wave + 4 * (t / NG), g = t - (t / NG) * NG;
        const int m = st * 16 + l16;
        const float *p = A + (long long)m * lda + 8 * kq;
#pragma unroll
        for (int u = 0; u < GS; ++u) {
            const int s = g * GS + u;
            const int k = s * 32 + 8 * kq;
            if (s < NSL && m < M && k < K) {
                r[u][0] = *(const f4 *)(p + s * 32);
                r[u][1] = *(const f4 *)(p + s * 32 + 4);
            } else {
                r[u][0] = f4{0.f, 0.f, 0.f, 0.f};
                r[u][1] = f4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto compute = [&](f4(&r)[GS][2], int t) {
        const int st = wave + 4 * (t / NG), g = t - (t / NG) * NG;
        if (g == 0) {
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < GS; ++u) {
            const int s = g * GS + u;
            if (s >= NSL) break;
            f4 v0 = r[u][0], v1 = r[u][1];
            if (xscale != 1.f) {
                v0 *= xscale;
                v1 *= xscale;
            }
            u32x2 h0, l0, h1, l1;
            split4<ELT>(v0, h0, l0);
            split4<ELT>(v1, h1, l1);
            const u32x4 ah = {h0.x, h0.y, h1.x, h1.y}, al = {l0.x, l0.y, l1.x, l1.y};
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const char *pb = Bs + (s * NB + j * 16 + l16) * 128;
                const u32x4 bh = *(const u32x4 *)(pb + hs), bl = *(const u32x4 *)(pb + ls);
                acc[j] = mfma16x16<ELT>(al, bh, acc[j]);
                acc[j] = mfma16x16<ELT>(ah, bl, acc[j]);
                acc[j] = mfma16x16<ELT>(ah, bh, acc[j]);
            }
        }
        if (g == NG - 1) {
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    const int m = st * 16 + 4 * kq + r4;
                    if (m < M) {
                        bad |= !__builtin_isfinite(acc[j][r4]);
                        epi(m, j, j * 16 + l16, acc[j][r4]);
                    }
                }
        }
    };
#pragma unroll
    for (int i = 0; i < D; ++i)
        if (i < T) load(ra[i], i);
    for (int t = 0; t < T; t += D) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            if (t + i < T) {
                compute(ra[i], t + i);
                if (t + i + D < T) load(ra[i], t + i + D);
            }
        }
    }
    return bad;
}

__device__ __forceinline__ void ffc_flag(int *flag, bool bad) {
    if (flag && bad) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------------- fwd
// t1 = relu(bn1(x_g conv1)) for CS1 channels of one image, then their rfft2 (fft.hip rfft2_mf's passes on
// the LDS tile).  LDS: X[H][W CS1 (+4)] | union(B staging, Y[2H][WF CS1]) | Tw | Th.
template <int H, int ELT>
__global__ __launch_bounds__(256, 1) void ffc_spec_fwd(FfcArgs a) {
    using L = FfcLevel<H>;
    constexpr int W = H, WF = L::WF, CS = L::CS1, CC = L::CC;
    constexpr int NT = CS > 16 ? CS / 16 : 1, NB = 16 * NT;
    constexpr int XS = W * CS + 4;
    constexpr int N1 = H * CS, N2 = WF * CS;
    constexpr int BBYTES = L::NSL_G * NB * 128, YBYTES = 2 * H * N2 * 4;
    constexpr int UBYTES = BBYTES > YBYTES ? BBYTES : YBYTES;
    __shared__ __attribute__((aligned(16))) float X[H * XS];
    __shared__ __attribute__((aligned(16))) char U[UBYTES];
    __shared__ __attribute__((aligned(16))) float Tw[W * 2 * WF];
    __shared__ __attribute__((aligned(16))) float Th[H * 2 * H];
    char *Bs = U;
    float *Y = (float *)U;
    int n, g;
    ffc_block(CC / CS, n, g);
    const int c0 = g * CS, tid = threadIdx.x;
    const float *fw = a.tables, *fh = fw + 2 * WF * W;
    ffc_copy_lds<W * 2 * WF>(Tw, fw);
    ffc_copy_lds<H * 2 * H>(Th, fh);
    ffc_stage_b<NB, L::NSL_G>(Bs, a.wt, a.kpad, [&](int b) { return c0 + b; });
    __syncthreads();
    float *t1 = a.out + (long long)n * L::HW * CC + c0;
    float sc[NT], sh[NT];                        // this lane's columns' folded BN (loaded before the GEMM)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = min(j * 16 + (tid & 15), CS - 1);
        sc[j] = (a.scale ? a.scale[c0 + col] : 1.f) * a.acc_scale;
        sh[j] = a.shift ? a.shift[c0 + col] : 0.f;
    }
    const bool bad = ffc_strip_gemm<NT, L::NSL_G, ELT>(
        a.a + (long long)n * a.a_bs, a.lda, L::HW, L::CG, a.x_scale, Bs, [&](int m, int j, int col, float v) {
            if (col < CS) {
                v = v * sc[j] + sh[j];
                v = v > 0.f ? v : 0.f;
                const int hh = m / W, ww = m - hh * W;
                X[hh * XS + ww * CS + col] = v;
                t1[(long long)m * CC + col] = v;
            }
        });
    ffc_flag(a.flag, bad);
    __syncthreads();
    // W pass (real -> half spectrum): Y[(p, h)][(v, c)] = sum_w fw[w][p][v] X[h][w][c]
    const int wave = tid >> 6, li = tid & 31, lh = (tid >> 5) & 1;
    constexpr int T1M = (2 * WF + 31) / 32, T1N = (N1 + 31) / 32;
    constexpr int T2M = (H + 31) / 32, T2N = (N2 + 31) / 32;
    for (int t = wave; t < T1M * T1N; t += 4) {
        const int tm = t / T1N, tn = t - tm * T1N;
        const int i = tm * 32 + li, j = tn * 32 + li;
        const bool iok = i < 2 * WF, jok = j < N1;
        const float *xb = X + (j / CS) * XS + (j % CS);
        fmf16 acc = {};
        for (int k0 = 0; k0 < W; k0 += 2) {
            const int k = k0 + lh;
            acc = ffc_mfma32(iok ? Tw[k * 2 * WF + i] : 0.f, jok ? xb[k * CS] : 0.f, acc);
        }
        if (jok) {
            const int hh = j / CS, cc = j % CS;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = tm * 32 + ffc_mf_row(r, lh);
                if (row < 2 * WF) {
                    const int p = row >= WF ? 1 : 0, v = row - p * WF;
                    Y[(p * H + hh) * N2 + v * CS + cc] = acc[r];
                }
            }
        }
    }
    __syncthreads();
    // H pass (complex): spec[n][u][v][(part, c)] = sum_h fh[h][u] Y[h][(v, c)]
    float *spec = a.out2 + (long long)n * L::F * 2 * CC + c0;
    for (int t = wave; t < T2M * T2N; t += 4) {
        const int tm = t / T2N, tn = t - tm * T2N;
        const int u = tm * 32 + li, j = tn * 32 + li;
        const bool uok = u < H, jok = j < N2;
        fmf16 zr = {}, zi = {};
        for (int k0 = 0; k0 < H; k0 += 2) {
            const int h = k0 + lh;
            const float fr = uok ? Th[(h * 2 + 0) * H + u] : 0.f, fi = uok ? Th[(h * 2 + 1) * H + u] : 0.f;
            const float yr = jok ? Y[h * N2 + j] : 0.f, yi = jok ? Y[(H + h) * N2 + j] : 0.f;
            zr = ffc_mfma32(-fi, yi, zr);
            zr = ffc_mfma32(fr, yr, zr);
            zi = ffc_mfma32(fr, yi, zi);
            zi = ffc_mfma32(fi, yr, zi);
        }
        if (jok) {
            const int v = j / CS, cc = j % CS;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int uu = tm * 32 + ffc_mf_row(r, lh);
                if (uu < H) {
                    float *o = spec + (long long)(uu * WF + v) * 2 * CC + cc;
                    o[0] = zr[r];
                    o[CC] = zi[r];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------- inv
// G = relu(bn_fu(spec conv_fu)) for the re / im spectra of CS2 u channels over all frequencies of one image,
// then their irfft2 + t1 -> u.  GEMM column b: b < CS2 -> output channel c0 + b (re), < 2 CS2 -> cc + c0 +
// b - CS2 (im), else padding.  LDS: Z[2H][WF CS2] | union(B staging, Y[2H][WF CS2]) | Ti | Tw.
template <int H, int ELT>
__global__ __launch_bounds__(256, 1) void ffc_spec_inv(FfcArgs a) {
    using L = FfcLevel<H>;
    constexpr int W = H, WF = L::WF, CS = L::CS2, CC = L::CC;
    constexpr int NT = 2 * CS > 16 ? 2 * CS / 16 : 1, NB = 16 * NT;
    constexpr int N1 = WF * CS, N2 = H * CS;
    constexpr int BBYTES = L::NSL_G * NB * 128, YBYTES = 2 * H * N1 * 4;
    constexpr int UBYTES = BBYTES > YBYTES ? BBYTES : YBYTES;
    __shared__ __attribute__((aligned(16))) float Z[2 * H * N1];
    __shared__ __attribute__((aligned(16))) char U[UBYTES];
    __shared__ __attribute__((aligned(16))) float Ti[H * 2 * H];
    __shared__ __attribute__((aligned(16))) float Tw[WF * 2 * W];
    char *Bs = U;
    float *Y = (float *)U;
    int n, g;
    ffc_block(CC / CS, n, g);
    const int c0 = g * CS, tid = threadIdx.x;
    const float *ih = a.tables + 2 * WF * W + 2 * H * H, *iw = ih + 2 * H * H;
    ffc_copy_lds<H * 2 * H>(Ti, ih);
    ffc_copy_lds<WF * 2 * W>(Tw, iw);
    ffc_stage_b<NB, L::NSL_G>(Bs, a.wt, a.kpad, [&](int b) {
        return b < CS ? c0 + b : (b < 2 * CS ? CC + c0 + b - CS : c0);
    });
    __syncthreads();
    float sc[NT], sh[NT];                        // this lane's columns' folded BN (loaded before the GEMM)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = min(j * 16 + (tid & 15), 2 * CS - 1);
        const int q = col >= CS ? 1 : 0, oc = q * CC + c0 + col - q * CS;
        sc[j] = (a.scale ? a.scale[oc] : 1.f) * a.acc_scale;
        sh[j] = a.shift ? a.shift[oc] : 0.f;
    }
    const bool bad = ffc_strip_gemm<NT, L::NSL_G, ELT>(
        a.a + (long long)n * a.a_bs, a.lda, L::F, L::CG, a.x_scale, Bs, [&](int m, int j, int col, float v) {
            if (col < 2 * CS) {
                const int q = col >= CS ? 1 : 0, c = col - q * CS;
                v = v * sc[j] + sh[j];
                v = v > 0.f ? v : 0.f;
                const int u = m / WF, vv = m - u * WF;
                Z[(q * H + u) * N1 + vv * CS + c] = v;
            }
        });
    ffc_flag(a.flag, bad);
    __syncthreads();
    const int wave = tid >> 6, li = tid & 31, lh = (tid >> 5) & 1;
    constexpr int T1M = (H + 31) / 32, T1N = (N1 + 31) / 32;
    constexpr int T2M = (W + 31) / 32, T2N = (N2 + 31) / 32;
    // inverse H pass (complex): Y[p][h][(v, c)] = sum_u ih[u][h] Z[u][(v, c)]
    for (int t = wave; t < T1M * T1N; t += 4) {
        const int tm = t / T1N, tn = t - tm * T1N;
        const int h = tm * 32 + li, j = tn * 32 + li;
        const bool hok = h < H, jok = j < N1;
        fmf16 yr = {}, yi = {};
        for (int k0 = 0; k0 < H; k0 += 2) {
            const int u = k0 + lh;
            const float gr = hok ? Ti[(u * 2 + 0) * H + h] : 0.f, gi = hok ? Ti[(u * 2 + 1) * H + h] : 0.f;
            const float zr = jok ? Z[u * N1 + j] : 0.f, zi = jok ? Z[(H + u) * N1 + j] : 0.f;
            yr = ffc_mfma32(-gi, zi, yr);
            yr = ffc_mfma32(gr, zr, yr);
            yi = ffc_mfma32(gr, zi, yi);
            yi = ffc_mfma32(gi, zr, yi);
        }
        if (jok) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int hh = tm * 32 + ffc_mf_row(r, lh);
                if (hh < H) {
                    Y[hh * N1 + j] = yr[r];
                    Y[(H + hh) * N1 + j] = yi[r];
                }
            }
        }
    }
    __syncthreads();
    // c2r W pass: u[h][w][c] = sum_(v, p) iw[v][p][w] Y[(p, h)][(v, c)] + t1
    const long long ibase = (long long)n * L::HW * CC + c0;
    for (int t = wave; t < T2M * T2N; t += 4) {
        const int tm = t / T2N, tn = t - tm * T2N;
        const int w = tm * 32 + li, j = tn * 32 + li;
        const bool wok = w < W, jok = j < N2;
        const int hh = j / CS, cc = j % CS;
        fmf16 acc = {};
        for (int k0 = 0; k0 < 2 * WF; k0 += 2) {
            const int k = k0 + lh, v = k >> 1, p = k & 1;
            acc = ffc_mfma32(wok ? Tw[k * W + w] : 0.f, jok ? Y[(p * H + hh) * N1 + v * CS + cc] : 0.f, acc);
        }
        if (jok) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int ww = tm * 32 + ffc_mf_row(r, lh);
                if (ww < W) {
                    const long long o = ibase + (long long)(hh * W + ww) * CC + cc;
                    a.out[o] = acc[r] + a.t1[o];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------- norm
// One block per (image, CSO channels of y): V = y_l slice, or y_g slice + (u conv2) slice (the st2 GEMM over
// all pixels of the image, y's conv_l2g output added in its epilogue), held in LDS; fp64 moments; then
// out = act((V - mean) rstd (1 + gamma) + beta) (+ res), and the reflect-padded copy (pad).
template <int H, int ELT>
__global__ __launch_bounds__(256) void ffc_norm(FfcArgs a) {
    using L = FfcLevel<H>;
    constexpr int W = H, HW = L::HW, CS = L::CSO, C = L::C, CL = L::CL;
    constexpr int NB = 16, VS = CS + 1;           // V row pitch (odd: the per-channel moment reads spread)
    __shared__ __attribute__((aligned(16))) float V[HW * VS];
    __shared__ __attribute__((aligned(16))) char Bs[L::NSL_C * NB * 128];
    __shared__ double red[256][2];
    __shared__ float coef[CS][2];
    int n, g;
    ffc_block(C / CS, n, g);
    const int c0 = g * CS, tid = threadIdx.x;
    const float *yb = a.y + (long long)n * HW * a.ycs + c0;
    const bool gslice = c0 >= CL;
    if (gslice) {
        const int o0 = c0 - CL;                    // conv2 output channel of the slice
        ffc_stage_b<NB, L::NSL_C>(Bs, a.wt, a.kpad, [&](int b) { return o0 + (b < CS ? b : 0); });
        __syncthreads();
        const bool bad = ffc_strip_gemm<1, L::NSL_C, ELT>(
            a.a + (long long)n * a.a_bs, a.lda, HW, L::CC, a.x_scale, Bs, [&](int m, int, int col, float v) {
                if (col < CS) V[m * VS + col] = v * a.acc_scale;
            });
        ffc_flag(a.flag, bad);
        __syncthreads();
    }
    // V (+)= the y slice (conv_to_l's output, or conv_l2g's beside the st2 product): float4 loads, a batch of
    // up to 8 in flight per thread
    {
        constexpr int QV = CS / 4, TOT = HW * QV, PER = (TOT + 255) / 256, BAT = PER < 8 ? PER : 8;
#pragma unroll 1
        for (int i0 = 0; i0 < PER; i0 += BAT) {
            float4 v[BAT];
            // (no guard where the slice divides into whole passes, 24^2 / 48^2: a guarded load gets sunk into its
            // branch and waited for there, one round trip per load)
            constexpr bool EXACT = TOT % 256 == 0 && PER % BAT == 0;
#pragma unroll
            for (int i = 0; i < BAT; ++i) {
                const int e = tid + 256 * (i0 + i);
                if (EXACT || (i0 + i < PER && e < TOT))
                    v[i] = *(const float4 *)(yb + (long long)(e / QV) * a.ycs + 4 * (e % QV));
            }
#pragma unroll
            for (int i = 0; i < BAT; ++i) {
                const int e = tid + 256 * (i0 + i);
                if (EXACT || (i0 + i < PER && e < TOT)) {
                    float *d = V + (e / QV) * VS + 4 * (e % QV);
                    if (gslice) {
                        d[0] += v[i].x; d[1] += v[i].y; d[2] += v[i].z; d[3] += v[i].w;
                    } else {
                        d[0] = v[i].x; d[1] = v[i].y; d[2] = v[i].z; d[3] = v[i].w;
                    }
                }
            }
        }
    }
    __syncthreads();
    // moments: thread (channel c = tid % CS, phase tid / CS) sums every (256 / CS)-th pixel
    {
        constexpr int NPH = 256 / CS;
        const int c = tid % CS, ph = tid / CS;
        double s = 0.0, q = 0.0;
        for (int p = ph; p < HW; p += NPH) {
            const double v = V[p * VS + c];
            s += v;
            q += v * v;
        }
        red[tid][0] = s;
        red[tid][1] = q;
        __syncthreads();
        if (tid < CS) {
            double sm = 0.0, sq = 0.0;
            for (int k = 0; k < NPH; ++k) {
                sm += red[k * CS + tid][0];
                sq += red[k * CS + tid][1];
            }
            const double mean = sm / HW;
            double var = sq / HW - mean * mean;
            if (var < 0.0) var = 0.0;
            const float rstd = 1.f / sqrtf((float)(var + (double)a.eps));   // fp64 moments, fp32 root (norm.hip)
            const float gm = a.gamma ? 1.f + a.gamma[(long long)n * a.gb_ns + c0 + tid] : 1.f;
            const float bt = a.beta ? a.beta[(long long)n * a.gb_ns + c0 + tid] : 0.f;
            coef[tid][0] = rstd * gm;
            coef[tid][1] = bt - (float)mean * rstd * gm;
        }
    }
    __syncthreads();
    // apply: thread (channel quad, pixel phase), float4 loads / stores
    constexpr int QB = CS / 4, NPH = 256 / QB;
    const int q4 = tid % QB, ph = tid / QB;
    float mul[4], add[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mul[j] = coef[4 * q4 + j][0];
        add[j] = coef[4 * q4 + j][1];
    }
    const float slope = a.act == S2V_ACT_LRELU ? a.alpha : (a.act == S2V_ACT_RELU ? 0.f : 1.f);
    float *ob = a.nout + (long long)n * HW * a.nout_cs + c0 + 4 * q4;
    const float *rb = a.res ? a.res + (long long)n * HW * a.res_cs + c0 + 4 * q4 : nullptr;
    float *pb = a.pad ? a.pad + (long long)n * (H + 2) * (W + 2) * a.pad_cs + c0 + 4 * q4 : nullptr;
    // the residual rows of a batch of pixels are loaded before the first store (vmcnt counts loads and
    // stores in issue order)
    constexpr int NP = (HW + NPH - 1) / NPH, RB = NP < 8 ? NP : 8;
#pragma unroll 1
    for (int i0 = 0; i0 < NP; i0 += RB) {
    constexpr bool EXACT = HW % NPH == 0 && NP % RB == 0;
    float4 rr[RB];
    if (rb) {
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int p = ph + NPH * (i0 + i);
            if (EXACT || (i0 + i < NP && p < HW)) rr[i] = *(const float4 *)(rb + (long long)p * a.res_cs);
        }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
        const int p = ph + NPH * (i0 + i);
        if (!EXACT && (i0 + i >= NP || p >= HW)) continue;
        const float *vp = V + p * VS + 4 * q4;
        float4 o;
        o.x = fmaf(vp[0], mul[0], add[0]);
        o.y = fmaf(vp[1], mul[1], add[1]);
        o.z = fmaf(vp[2], mul[2], add[2]);
        o.w = fmaf(vp[3], mul[3], add[3]);
        o.x = o.x >= 0.f ? o.x : o.x * slope;
        o.y = o.y >= 0.f ? o.y : o.y * slope;
        o.z = o.z >= 0.f ? o.z : o.z * slope;
        o.w = o.w >= 0.f ? o.w : o.w * slope;
        if (rb) {
            o.x += rr[i].x; o.y += rr[i].y; o.z += rr[i].z; o.w += rr[i].w;
        }
        *(float4 *)(ob + (long long)p * a.nout_cs) = o;
        if (pb) {
            // F.pad(..., (1, 1, 1, 1), 'reflect'): pixel (r, q) lands at (r + 1, q + 1) and, on the second /
            // second-to-last row or column, also on the mirrored border row / column (norm.hip in_apply_v)
            const int r = p / W, qq = p - r * W, W2 = W + 2;
            const int rows[2] = {r + 1, r == 1 ? 0 : (r == H - 2 ? H + 1 : -1)};
            const int cols[2] = {qq + 1, qq == 1 ? 0 : (qq == W - 2 ? W + 1 : -1)};
#pragma unroll
            for (int ri = 0; ri < 2; ++ri)
#pragma unroll
                for (int cj = 0; cj < 2; ++cj)
                    if (rows[ri] >= 0 && cols[cj] >= 0)
                        *(float4 *)(pb + ((long long)rows[ri] * W2 + cols[cj]) * a.pad_cs) = o;
        }
    }
    }
}

template <int H>
static int ffc_launch(int which, const FfcArgs &a, int n, int prec, hipStream_t s) {
    using L = FfcLevel<H>;
    const bool f16 = prec == S2V_PREC_F16X3;
    if (which == 0) {
        const unsigned grid = n * (L::CC / L::CS1);
        if (f16) ffc_spec_fwd<H, 1><<<grid, 256, 0, s>>>(a);
        else ffc_spec_fwd<H, 0><<<grid, 256, 0, s>>>(a);
    } else if (which == 1) {
        const unsigned grid = n * (L::CC / L::CS2);
        if (f16) ffc_spec_inv<H, 1><<<grid, 256, 0, s>>>(a);
        else ffc_spec_inv<H, 0><<<grid, 256, 0, s>>>(a);
    } else {
        const unsigned grid = n * (L::C / L::CSO);
        if (f16) ffc_norm<H, 1><<<grid, 256, 0, s>>>(a);
        else ffc_norm<H, 0><<<grid, 256, 0, s>>>(a);
    }
    return check_launch(which == 0 ? "ffc_spec_fwd" : (which == 1 ? "ffc_spec_inv" : "ffc_norm"));
}

static int ffc_dispatch(int which, const FfcArgs &a, int n, int h, int prec, s2v_stream_t stream) {
    S2V_REQUIRE(n > 0 && (h == 12 || h == 24 || h == 48), "ffc: h must be 12, 24 or 48 (LNet levels), got %d", h);
    S2V_REQUIRE(prec == S2V_PREC_F16X3 || prec == S2V_PREC_BF16X3,
                "ffc: split-precision arithmetic only (f16x3 / bf16x3; exact f32 takes the separate kernels)");
    hipStream_t s = (hipStream_t)stream;
    if (h == 12) return ffc_launch<12>(which, a, n, prec, s);
    if (h == 24) return ffc_launch<24>(which, a, n, prec, s);
    return ffc_launch<48>(which, a, n, prec, s);
}

static bool pow2_or_one(float v) {
    int e;
    return v > 0.f && std::frexp(v, &e) == 0.5f;
}

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_ffc_channels(int h) { return h == 12 ? 1024 : (h == 24 ? 256 : (h == 48 ? 128 : 0)); }

extern "C" int s2v_ffc_spec_fwd(const float *xg, int xcs, int n, int h, const void *w1, int w1_kpad, float wt_scale,
                                float x_scale, const float *scale, const float *shift, const float *tables, float *t1,
                                float *spec, int *flag, int prec, s2v_stream_t stream) {
    const int c = s2v_ffc_channels(h), cg = c - c / 4;
    S2V_REQUIRE(xg && w1 && tables && t1 && spec && c > 0, "ffc_spec_fwd: bad args");
    S2V_REQUIRE(xcs >= cg && xcs % 4 == 0 && ((uintptr_t)xg % 16) == 0, "ffc_spec_fwd: x_g pitch / alignment");
    S2V_REQUIRE(w1_kpad >= cg && w1_kpad % 32 == 0 && pow2_or_one(wt_scale) && pow2_or_one(x_scale),
                "ffc_spec_fwd: weights / scales");
    FfcArgs a = {};
    a.a = xg; a.lda = xcs; a.a_bs = (long long)h * h * xcs;
    a.wt = (const char *)w1; a.kpad = w1_kpad;
    a.acc_scale = 1.f / (wt_scale * x_scale); a.x_scale = x_scale;
    a.scale = scale; a.shift = shift; a.tables = tables; a.out = t1; a.out2 = spec; a.flag = flag;
    return ffc_dispatch(0, a, n, h, prec, stream);
}

extern "C" int s2v_ffc_spec_inv(const float *spec, int n, int h, const void *wfu, int wfu_kpad, float wt_scale,
                                float x_scale, const float *scale, const float *shift, const float *tables,
                                const float *t1, float *u, int *flag, int prec, s2v_stream_t stream) {
    const int c = s2v_ffc_channels(h), cg = c - c / 4;
    S2V_REQUIRE(spec && wfu && tables && t1 && u && c > 0, "ffc_spec_inv: bad args");
    S2V_REQUIRE(((uintptr_t)spec % 16) == 0, "ffc_spec_inv: spec alignment");
    S2V_REQUIRE(wfu_kpad >= cg && wfu_kpad % 32 == 0 && pow2_or_one(wt_scale) && pow2_or_one(x_scale),
                "ffc_spec_inv: weights / scales");
    const int wf = h / 2 + 1;
    FfcArgs a = {};
    a.a = spec; a.lda = cg; a.a_bs = (long long)h * wf * cg;
    a.wt = (const char *)wfu; a.kpad = wfu_kpad;
    a.acc_scale = 1.f / (wt_scale * x_scale); a.x_scale = x_scale;
    a.scale = scale; a.shift = shift; a.tables = tables; a.t1 = t1; a.out = u; a.flag = flag;
    return ffc_dispatch(1, a, n, h, prec, stream);
}

extern "C" int s2v_ffc_norm(const float *y, int ycs, int n, int h, const float *u, const void *w2, int w2_kpad,
                            float wt_scale, float x_scale, const float *gamma, const float *beta, int gb_ns, float eps,
                            int act, float alpha, const float *res, int res_cs, float *out, int out_cs, float *pad,
                            int pad_cs, int *flag, int prec, s2v_stream_t stream) {
    const int c = s2v_ffc_channels(h), cc = (c - c / 4) / 2;
    S2V_REQUIRE(y && u && w2 && out && c > 0, "ffc_norm: bad args");
    // y is read with float4 loads (and may be ``out`` itself: LNet normalises in place)
    S2V_REQUIRE(ycs >= c && ycs % 4 == 0 && ((uintptr_t)y % 16) == 0 && out_cs >= c && out_cs % 4 == 0 &&
                ((uintptr_t)out % 16) == 0 &&
                (!res || (res_cs >= c && res_cs % 4 == 0 && ((uintptr_t)res % 16) == 0)) &&
                (!pad || (pad_cs >= c && pad_cs % 4 == 0 && ((uintptr_t)pad % 16) == 0)) && ((uintptr_t)u % 16) == 0,
                "ffc_norm: channel pitches / alignment");
    S2V_REQUIRE((gamma == nullptr) == (beta == nullptr) && (!gamma || gb_ns >= c), "ffc_norm: gamma / beta");
    S2V_REQUIRE(w2_kpad >= cc && w2_kpad % 32 == 0 && pow2_or_one(wt_scale) && pow2_or_one(x_scale),
                "ffc_norm: weights / scales");
    FfcArgs a = {};
    a.a = u; a.lda = cc; a.a_bs = (long long)h * h * cc;
    a.wt = (const char *)w2; a.kpad = w2_kpad;
    a.acc_scale = 1.f / (wt_scale * x_scale); a.x_scale = x_scale; a.flag = flag;
    a.y = y; a.ycs = ycs; a.gamma = gamma; a.beta = beta; a.gb_ns = gb_ns; a.eps = eps; a.act = act; a.alpha = alpha;
    a.res = res; a.res_cs = res_cs; a.nout = out; a.nout_cs = out_cs; a.pad = pad; a.pad_cs = pad_cs;
    return ffc_dispatch(2, a, n, h, prec, stream);
}
