// Implicit-GEMM convolution / GEMM on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// GEMM view:  M = batch pixels (n, oy, ox)   N = output channels   K = (ky, kx, cin)
//   A[m][k]  gathered on the fly from the NHWC input (zero / reflect padding, nearest-x2
//            upsampling, transposed-conv scatter-as-gather), prologue act/in_scale fused;
//   B[n][k]  pre-packed weights [npad][kpad] (or an activation matrix [K][N], ``b_kn``);
//   C        NHWC output slice; epilogue fuses bias/BN/demod scale, noise, residual, act.
//
// Block = 256 threads = 4 waves laid out WAVES_M x WAVES_N; each wave owns a
// (BM/WAVES_M) x (BN/WAVES_N) sub-tile made of 32x32 MFMA tiles. K is staged through LDS in
// BK = 32 slices held K-contiguous ([row][BK+4] floats; the +4 pad makes the ds_read_b128 of 16
// consecutive rows conflict-free), so each lane feeds 4 MFMA k-steps from one 16-byte read.
// Global loads of slice t+1 are issued into registers before the MFMAs of slice t (one LDS
// buffer, register double-buffering).  Split-K writes raw partial sums to a workspace that
// ``splitk_reduce`` folds with the same epilogue.
#include "common.hpp"

#include <vector>

#include "conv_impl.hpp"

#include <cmath>

namespace s2v {

template <int ELT>   // 0 = bf16, 1 = f16 halves (conv_x3_impl.hpp; instances in conv_x3_{bf16,f16}.hip); 0 or an error
int launch_conv_x3(int tile, const ConvArgs &a, int amode, bool bkn, dim3 grid, hipStream_t s);
template <int ELT>   // LDS-DMA kernels on split-layout inputs (conv_glds.hip): cfg 0 = 256x256, 1 = 256x128
void launch_conv_glds(int cfg, const ConvArgs &a, dim3 grid, hipStream_t s);
template <int ELT>   // grouped x3 launches (conv_x3_impl.hpp conv_igemm_x3_group): 0 or an error
int launch_conv_x3_group(int cfg, const ConvGroup &g, dim3 grid, hipStream_t s);
template <int ELT>   // narrow-N register-direct-A kernel (conv_x3_nar.hip); breg: B fragments direct too
int launch_conv_x3_nar(const ConvArgs &a, bool breg, dim3 grid, hipStream_t s);
template <int ELT>   // 3x3 spatial-patch kernel with the input halo staged once per channel slice (conv_x3_halo.hip)
int launch_conv_x3_halo(const ConvArgs &a, int th, int wn, dim3 grid, hipStream_t s);

template <int BM, int BN, int AR, int BR, int BKN>
__device__ __forceinline__ void store_ab(float *As, float *Bs, int tid, const f4 (&ra)[AR],
                                         const f4 (&rb)[BR]) {
    constexpr int LDK = 36;
    const int ar = tid >> 3, ak = (tid & 7) * 4;
#pragma unroll
    for (int j = 0; j < AR; ++j) *(f4 *)&As[(ar + 32 * j) * LDK + ak] = ra[j];
    if (!BKN) {
#pragma unroll
        for (int j = 0; j < BR; ++j) *(f4 *)&Bs[(ar + 32 * j) * LDK + ak] = rb[j];
    } else {
        constexpr int NV = BN / 4, RPP = 256 / NV;
        const int kr = tid / NV, nn = (tid - (tid / NV) * NV) * 4;
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const int k = kr + RPP * j;
            Bs[(nn + 0) * LDK + k] = rb[j].x;
            Bs[(nn + 1) * LDK + k] = rb[j].y;
            Bs[(nn + 2) * LDK + k] = rb[j].z;
            Bs[(nn + 3) * LDK + k] = rb[j].w;
        }
    }
}

template <int BM, int BN, int WAVES_M, int AMODE, int BKN>
__global__ __launch_bounds__(256, 1) void conv_igemm(ConvArgs a) {
    constexpr int BK = 32, LDK = BK + 4;
    constexpr int WAVES_N = 4 / WAVES_M;
    constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int AR = BM / 32;
    constexpr int BR = BN / 32;
    constexpr int STAGE = (BM + BN) * LDK;
    static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "tile");
    launch_stamp(a, false);

    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    // XCD-aware tile order: the dispatcher deals workgroups round-robin over the 8 XCDs, so
    // remap the linear id so that each XCD owns a contiguous run of tiles (neighbouring output
    // rows share their 3x3 halo through that XCD's L2), N-tiles of one M-tile adjacent.
    int mt, nt, bz;
    {
        const int gx = gridDim.x, gy = gridDim.y;
        const int total = gx * gy * gridDim.z;
        const int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
        const int per = total >> 3, rem = total & 7;
        const int xcd = L & 7, idx = L >> 3;
        const int Lp = xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
        nt = Lp % gy;
        const int t = Lp / gy;
        mt = t % gx;
        bz = t / gx;
    }
    const int m0 = mt * BM, n0 = nt * BN;
    const int bidx = bz / a.splits, split = bz - bidx * a.splits;
    const float *__restrict__ x = a.x + (long long)bidx * a.x_bs;
    const float *__restrict__ wt = a.wt + (long long)bidx * a.w_bs;
    const int kt0 = split * a.tps;
    const int kt1 = min(a.ktiles, kt0 + a.tps);
    // AMODE 0/3: visit K-slices channel-slice-major (all taps of one 32-channel slice in a row),
    // so the 3x3 neighbourhood of a slice is re-read from L2 right away instead of after the
    // whole channel range; the weights are indexed by the same permuted slice, so the sum is
    // unchanged apart from fp32 summation order.
    const int taps = a.kh * a.kw, nsl = a.cin >> 5;
    const bool kperm = (AMODE == 0 || AMODE == 3) && !BKN && taps > 1;
    auto kmap = [&](int i) { return kperm ? (i % taps) * nsl + i / taps : i; };
    const int ar = tid >> 3, ak = (tid & 7) * 4;

    ARows<AR, AMODE> R;
    a_rows_init<AR, AMODE>(a, m0, ar, R);

    f4 ra[AR], rb[BR];
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    if (kt0 < kt1) {
        load_a<AR, AMODE>(a, x, kmap(kt0), ak, R, ra);
        load_b<BN, BR, BKN>(a, wt, kmap(kt0), n0, tid, rb);
        store_ab<BM, BN, AR, BR, BKN>(smem, smem + BM * LDK, tid, ra, rb);
        __syncthreads();
    }
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
        // prefetch slice kt+1 into registers (the last iteration re-reads its own slice: no
        // control flow around the staging registers); it lands while the MFMAs below run
        const int kn = kmap(min(kt + 1, kt1 - 1));
        load_a<AR, AMODE>(a, x, kn, ak, R, ra);
        load_b<BN, BR, BKN>(a, wt, kn, n0, tid, rb);
        __builtin_amdgcn_sched_barrier(0);   // keep the prefetch issue above the MFMA block
        const float *As = smem + buf * STAGE;
        const float *Bs = As + BM * LDK;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f4 av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                av[i] = *(const f4 *)&As[(wm * WTM + i * 32 + li) * LDK + lh * 16 + q * 4];
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bv[j] = *(const f4 *)&Bs[(wn * WTN + j * 32 + li) * LDK + lh * 16 + q * 4];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].z, bv[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].w, bv[j].w, acc[i][j], 0, 0, 0);
                }
        }
        // the other buffer was last read before the previous barrier
        float *Ad = smem + (buf ^ 1) * STAGE;
        store_ab<BM, BN, AR, BR, BKN>(Ad, Ad + BM * LDK, tid, ra, rb);
        __syncthreads();
        buf ^= 1;
    }

    // ---- epilogue (shared with the split-bf16 kernel, conv_impl.hpp)
    static_assert(BM * (BN + 4) <= 2 * STAGE, "C tile must fit in the staging LDS");
    epilogue_tile<BM, BN, WAVES_M, TM, TN>(a, acc, smem, tid, m0, n0, bz, bidx);
    launch_stamp(a, true);
}

// Split-K fold: one thread per 4 consecutive output channels (16-byte partial-sum loads) when
// cout % 4 == 0, else per channel; the epilogue is the kernels' own (one 16-byte store when ``vec``).
// 32-bit index math when the fold has < 2^31 items (the 64-bit divisions cost more VALU than the
// fold's arithmetic).
__device__ void store_epilogue4(const ConvArgs &a, int bidx, int m, int n, f4 v, bool vec, bool nt);

__global__ void splitk_reduce(ConvArgs a, int batch, int vec) {
    const int cv = (a.cout & 3) == 0 ? 4 : 1;
    const int nq = a.cout / cv;
    const long long total = (long long)batch * a.M * nq;
    const long long slab = (long long)a.M * a.cout;
    const bool small = total < (1LL << 31);
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        int q, m, bidx;
        if (small) {
            const unsigned u = (unsigned)idx, bm = u / (unsigned)nq;
            q = (int)(u - bm * (unsigned)nq);
            bidx = (int)(bm / (unsigned)a.M);
            m = (int)(bm - (unsigned)bidx * (unsigned)a.M);
        } else {
            q = (int)(idx % nq);
            const long long bm = idx / nq;
            m = (int)(bm % a.M);
            bidx = (int)(bm / a.M);
        }
        const float *src = a.ws + (long long)bidx * a.splits * slab + (long long)m * a.cout + q * cv;
        if (cv == 4) {
            f4 s = *(const f4 *)src;
            for (int sp = 1; sp < a.splits; ++sp) s += *(const f4 *)(src + sp * slab);
            store_epilogue4(a, bidx, m, 4 * q, s, vec != 0, false);
        } else {
            float s = src[0];
            for (int sp = 1; sp < a.splits; ++sp) s += src[sp * slab];
            store_epilogue(a, bidx, m, q, s);
        }
    }
}

// Split-K fold of a conv group (s2v_conv2d_group): member p folds with the blocks
// [rstart[p], rstart[p + 1]) (none when it has one split), otherwise as splitk_reduce.
__global__ void splitk_reduce_group(ConvGroup g) {
    int p = 0;
#pragma unroll
    for (int i = 1; i < kConvGroupMax; ++i)
        if (i < g.n && (int)blockIdx.x >= g.rstart[i]) p = i;
    const ConvArgs &a = g.a[p];
    const int nb = g.rstart[p + 1] - g.rstart[p];
    const int cv = (a.cout & 3) == 0 ? 4 : 1;
    const int nq = a.cout / cv;
    const long long total = (long long)a.M * nq;               // one batch entry (group members: batch 1)
    const long long slab = (long long)a.M * a.cout;
    for (long long idx = (blockIdx.x - g.rstart[p]) * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)nb * blockDim.x) {
        const unsigned u = (unsigned)idx;
        const int m = (int)(u / (unsigned)nq), q = (int)(u - (unsigned)m * (unsigned)nq);
        const float *src = a.ws + (long long)m * a.cout + q * cv;
        if (cv == 4) {
            f4 sum = *(const f4 *)src;
            for (int sp = 1; sp < a.splits; ++sp) sum += *(const f4 *)(src + sp * slab);
            store_epilogue4(a, 0, m, 4 * q, sum, g.vec[p] != 0, false);
        } else {
            float sum = src[0];
            for (int sp = 1; sp < a.splits; ++sp) sum += src[sp * slab];
            store_epilogue(a, 0, m, q, sum);
        }
    }
}

// Epilogue of 4 consecutive output channels [n, n + 4) of row m as one 16-byte store (host
// guarantees 16-byte aligned rows: ycs, res_cs % 4 == 0; n % 4 == 0); per-element otherwise.
__device__ __forceinline__ void store_epilogue4(const ConvArgs &a, int bidx, int m, int n, f4 v, bool vec,
                                                bool nt) {
    const Epi &e = a.epi;
    if (!vec || e.nc_scale || (e.res && !e.res_simple) || a.y_step > 1) {
        store_epilogue(a, bidx, m, n + 0, v.x);
        store_epilogue(a, bidx, m, n + 1, v.y);
        store_epilogue(a, bidx, m, n + 2, v.z);
        store_epilogue(a, bidx, m, n + 3, v.w);
        return;
    }
    if (e.scale) v *= *(const f4 *)(e.scale + n);
    if (e.shift) v += *(const f4 *)(e.shift + n);
    if (e.pix_add) v += e.pix_w * e.pix_add[pix_index(a, bidx, m, n)];
    f4 r = {0.f, 0.f, 0.f, 0.f};
    if (e.res) {
        r = *(const f4 *)(e.res + (long long)bidx * a.res_bs + (long long)m * e.res_cs + n);
        if (!e.res_after) v += r;
    }
    v.x = apply_act(v.x, e.act, e.alpha);
    v.y = apply_act(v.y, e.act, e.alpha);
    v.z = apply_act(v.z, e.act, e.alpha);
    v.w = apply_act(v.w, e.act, e.alpha);
    if (e.res && e.res_after) v += r;
    if (e.post_mul && n >= e.post_c0) {       // SFT (post_c0 % 4 == 0 under vec: a quad is all in or out)
        const long long q = (long long)m * e.post_cs + n - e.post_c0;
        v = v * *(const f4 *)(e.post_mul + q) + *(const f4 *)(e.post_add + q);
    }
    f4 *dst = (f4 *)(a.y + (long long)bidx * a.y_bs + (long long)m * a.ycs + n);
    if (nt) __builtin_nontemporal_store(v, dst);
    else *dst = v;
    if (e.dup_src) {
        f4 d = e.dup_a * *(const f4 *)(e.dup_src + (long long)m * e.dup_cs + n);
        if (e.dup_bias) d += *(const f4 *)(e.dup_bias + n);
        d.x = apply_act(d.x, e.act, e.alpha);
        d.y = apply_act(d.y, e.act, e.alpha);
        d.z = apply_act(d.z, e.act, e.alpha);
        d.w = apply_act(d.w, e.act, e.alpha);
        *(f4 *)(a.y + (long long)bidx * a.y_bs + (long long)m * a.ycs + e.dup_off + n) = d;
    }
}

// Small-K direct convolution (K = kh*kw*cin <= 64: the 4-channel image-input layers and the
// 4-channel StyleConv input): tppx threads per pixel group, each QPT x 4 output channels of PX
// consecutive pixels (register blocking over pixels: every weight float4 read from LDS feeds PX
// pixels, 1 LDS byte per FMA at PX = 4 instead of 4); a block walks iters x (256 / tppx) groups of
// one batch entry with that entry's filter [K][cout] staged in LDS once; one float4 of input per
// tap and channel group; fp32 VALU; 16-byte output stores.  These layers are bound by their
// output write; the implicit GEMM pads K to 32 per slice and stages every output tile through LDS
// (3-27 TFLOP/s measured on them).
#ifndef SMALLK_NT
#define SMALLK_NT 1      // streaming (non-temporal) output stores: the image-layer outputs exceed L2 / MALL
#endif
template <int QPT, int PX>
__global__ __launch_bounds__(256) void conv_smallk(ConvArgs a, int batch, int tppx, int iters, int vec) {
    extern __shared__ __attribute__((aligned(16))) float wk[];   // [K][cout]
    const int gpb = 256 / tppx;
    const long long total = (long long)batch * a.M;          // pixels (M % PX == 0: groups stay in one entry)
    const long long g0 = (long long)blockIdx.x * gpb * iters;  // first pixel group of the block
    {
        const long long p0 = g0 * PX;
        const int b0 = (int)((p0 < total ? p0 : 0) / a.M);
        const float *w0 = a.wt + (long long)b0 * a.w_bs;
        // k fastest across lanes: a wave reads whole packed rows (coalesced), LDS gets [K][cout]
        for (int e = threadIdx.x; e < a.K * a.cout; e += 256) {
            const int o = e / a.K, k = e - o * a.K;
            wk[k * a.cout + o] = w0[(long long)o * a.kpad + k];
        }
    }
    __syncthreads();
    const int tq = threadIdx.x % tppx;
    const int hw = a.oh * a.ow;
    for (int it = 0; it < iters; ++it) {
        const long long g = g0 + (long long)it * gpb + threadIdx.x / tppx;
        if (g * PX >= total) break;
        const int bidx = (int)(g * PX / a.M);
        const int mbase = (int)(g * PX - (long long)bidx * a.M);
        const float *x = a.x + (long long)bidx * a.x_bs;
        int img[PX], oy[PX], ox[PX];
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            const int m = mbase + p;
            img[p] = m / hw;
            const int rem = m - img[p] * hw;
            oy[p] = rem / a.ow;
            ox[p] = rem - oy[p] * a.ow;
        }
        f4 acc[PX][QPT];
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int q = 0; q < QPT; ++q) acc[p][q] = f4{0.f, 0.f, 0.f, 0.f};
        for (int ky = 0; ky < a.kh; ++ky)
            for (int kx = 0; kx < a.kw; ++kx) {
                const float *px[PX];
                bool ok[PX];
#pragma unroll
                for (int p = 0; p < PX; ++p) {
                    int iy, ix;
                    ok[p] = map_tap(a, oy[p], ox[p], ky, kx, iy, ix);
                    px[p] = x + ((long long)(img[p] * a.h + (ok[p] ? iy : 0)) * a.w + (ok[p] ? ix : 0)) * a.xcs;
                }
                const int kb = (ky * a.kw + kx) * a.cin;
                for (int c = 0; c < a.cin; c += 4) {
                    f4 v[PX];
#pragma unroll
                    for (int p = 0; p < PX; ++p) {
                        v[p] = ok[p] ? *(const f4 *)(px[p] + c) : f4{0.f, 0.f, 0.f, 0.f};
                        if (a.in_scale) v[p] *= *(const f4 *)(a.in_scale + (long long)img[p] * a.in_scale_ns + c);
                        if (a.pre_act) {
                            v[p].x = apply_act(v[p].x, a.pre_act, a.pre_alpha);
                            v[p].y = apply_act(v[p].y, a.pre_act, a.pre_alpha);
                            v[p].z = apply_act(v[p].z, a.pre_act, a.pre_alpha);
                            v[p].w = apply_act(v[p].w, a.pre_act, a.pre_alpha);
                        }
                        if (!ok[p]) v[p] = f4{0.f, 0.f, 0.f, 0.f};   // zero padding stays zero after the prologue
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float *wr = wk + (kb + c + e) * a.cout + 4 * tq;
#pragma unroll
                        for (int q = 0; q < QPT; ++q) {
                            const f4 w4 = *(const f4 *)(wr + 4 * tppx * q);
#pragma unroll
                            for (int p = 0; p < PX; ++p) {
                                const float ve = e == 0 ? v[p].x : e == 1 ? v[p].y : e == 2 ? v[p].z : v[p].w;
                                acc[p][q].x = fmaf(ve, w4.x, acc[p][q].x);
                                acc[p][q].y = fmaf(ve, w4.y, acc[p][q].y);
                                acc[p][q].z = fmaf(ve, w4.z, acc[p][q].z);
                                acc[p][q].w = fmaf(ve, w4.w, acc[p][q].w);
                            }
                        }
                    }
                }
            }
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int q = 0; q < QPT; ++q)
                store_epilogue4(a, bidx, mbase + p, 4 * (tq + tppx * q), acc[p][q], vec != 0, SMALLK_NT != 0);
    }
}

// 4-channel inputs with a compile-time tap count (1x1 or 3x3: ENet's conv_body_first and the first
// StyleConv on the upsampled 4-channel image): every tap's float4 is loaded before any FMA, so a
// thread has KT loads in flight instead of KT dependent round trips per pixel (the runtime-tap
// loop of conv_smallk ran the 3x3 StyleConv at 0.66 TB/s of output).
template <int QPT, int KT>
__global__ __launch_bounds__(256) void conv_smallk4(ConvArgs a, int batch, int tppx, int iters, int vec) {
    constexpr int KW = KT == 9 ? 3 : 1;
    extern __shared__ __attribute__((aligned(16))) float wk[];   // [K][cout]
    const int gpb = 256 / tppx;
    const long long total = (long long)batch * a.M;
    const long long g0 = (long long)blockIdx.x * gpb * iters;
    {
        const int b0 = (int)((g0 < total ? g0 : 0) / a.M);
        const float *w0 = a.wt + (long long)b0 * a.w_bs;
        for (int e = threadIdx.x; e < KT * 4 * a.cout; e += 256) {   // coalesced packed rows (k fastest)
            const int o = e / (KT * 4), k = e - o * (KT * 4);
            wk[k * a.cout + o] = w0[(long long)o * a.kpad + k];
        }
    }
    __syncthreads();
    const int tq = threadIdx.x % tppx;
    const int hw = a.oh * a.ow;
    if constexpr (KT == 1) {
        // 1x1, one float4 per pixel.  Software-pipelined: pixel u + 1 is loaded before pixel u is
        // stored (vmcnt counts loads and stores in issue order, so a load issued after a store
        // waits for it).  Pixel positions advance incrementally: one division per thread instead
        // of per pixel (the per-pixel 64-bit / 32-bit divisions made this loop VALU-bound, ~190
        // VALU instructions per pixel and wave, 0.65 TB/s of output).
        struct Pos { int b, m, img, oy, ox; };
        auto advance = [&](Pos &p) {
            p.m += gpb;
            p.ox += gpb;
            while (p.ox >= a.ow) { p.ox -= a.ow; ++p.oy; }
            while (p.oy >= a.oh) { p.oy -= a.oh; ++p.img; }
            while (p.img >= a.n) { p.img -= a.n; ++p.b; p.m -= a.M; }
        };
        auto load1 = [&](const Pos &p, f4 &v) {
            const float *x = a.x + (long long)p.b * a.x_bs;
            int iy, ix;
            const bool ok = map_tap(a, p.oy, p.ox, 0, 0, iy, ix);
            v = ok ? *(const f4 *)(x + ((long long)(p.img * a.h + iy) * a.w + ix) * a.xcs) : f4{0.f, 0.f, 0.f, 0.f};
            if (a.in_scale || a.pre_act) {
                v.x = prologue(a, v.x, p.img, 0);
                v.y = prologue(a, v.y, p.img, 1);
                v.z = prologue(a, v.z, p.img, 2);
                v.w = prologue(a, v.w, p.img, 3);
                if (!ok) v = f4{0.f, 0.f, 0.f, 0.f};
            }
        };
        // the epilogue's per-channel scale / shift are loaded once, before any store
        const Epi &ep = a.epi;
        const bool plain = vec && !ep.nc_scale && !ep.res && !ep.pix_add && a.y_step <= 1 && !ep.post_mul && !ep.dup_src;
        f4 esc[QPT], esh[QPT];
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            const int n = 4 * (tq + tppx * q);
            esc[q] = ep.scale ? *(const f4 *)(ep.scale + n) : f4{1.f, 1.f, 1.f, 1.f};
            esh[q] = ep.shift ? *(const f4 *)(ep.shift + n) : f4{0.f, 0.f, 0.f, 0.f};
        }
        const long long gs = g0 + threadIdx.x / tppx;
        if (gs >= total) return;
        const long long left = (total - gs + gpb - 1) / gpb;
        const int nit = left < iters ? (int)left : iters;
        Pos pl;
        pl.b = (int)(gs / a.M);
        pl.m = (int)(gs - (long long)pl.b * a.M);
        pl.img = pl.m / hw;
        {
            const int rem = pl.m - pl.img * hw;
            pl.oy = rem / a.ow;
            pl.ox = rem - pl.oy * a.ow;
        }
        Pos ps = pl;
        f4 cur = f4{0.f, 0.f, 0.f, 0.f}, nxt = f4{0.f, 0.f, 0.f, 0.f};
        load1(pl, cur);
        for (int it = 0; it < nit; ++it) {
            if (it + 1 < nit) {
                advance(pl);
                load1(pl, nxt);
            }
            f4 acc[QPT];
#pragma unroll
            for (int q = 0; q < QPT; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float ve = e == 0 ? cur.x : e == 1 ? cur.y : e == 2 ? cur.z : cur.w;
                const float *wr = wk + e * a.cout + 4 * tq;
#pragma unroll
                for (int q = 0; q < QPT; ++q) {
                    const f4 w4 = *(const f4 *)(wr + 4 * tppx * q);
                    acc[q].x = fmaf(ve, w4.x, acc[q].x);
                    acc[q].y = fmaf(ve, w4.y, acc[q].y);
                    acc[q].z = fmaf(ve, w4.z, acc[q].z);
                    acc[q].w = fmaf(ve, w4.w, acc[q].w);
                }
            }
#pragma unroll
            for (int q = 0; q < QPT; ++q) {
                const int n = 4 * (tq + tppx * q);
                if (!plain) {
                    store_epilogue4(a, ps.b, ps.m, n, acc[q], vec != 0, SMALLK_NT != 0);
                    continue;
                }
                f4 v = acc[q] * esc[q] + esh[q];
                v.x = apply_act(v.x, ep.act, ep.alpha);
                v.y = apply_act(v.y, ep.act, ep.alpha);
                v.z = apply_act(v.z, ep.act, ep.alpha);
                v.w = apply_act(v.w, ep.act, ep.alpha);
                f4 *dst = (f4 *)(a.y + (long long)ps.b * a.y_bs + (long long)ps.m * a.ycs + n);
                if (SMALLK_NT) __builtin_nontemporal_store(v, dst);
                else *dst = v;
            }
            advance(ps);
            cur = nxt;
        }
        return;
    }
    for (int it = 0; it < iters; ++it) {
        const long long g = g0 + (long long)it * gpb + threadIdx.x / tppx;
        if (g >= total) break;
        const int bidx = (int)(g / a.M);
        const int m = (int)(g - (long long)bidx * a.M);
        const float *x = a.x + (long long)bidx * a.x_bs;
        const int img = m / hw, rem = m - img * hw;
        const int oy = rem / a.ow, ox = rem - oy * a.ow;
        f4 v[KT];
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            int iy, ix;
            const bool ok = map_tap(a, oy, ox, t / KW, t % KW, iy, ix);
            v[t] = ok ? *(const f4 *)(x + ((long long)(img * a.h + iy) * a.w + ix) * a.xcs) : f4{0.f, 0.f, 0.f, 0.f};
            if (a.in_scale || a.pre_act) {
                v[t].x = prologue(a, v[t].x, img, 0);
                v[t].y = prologue(a, v[t].y, img, 1);
                v[t].z = prologue(a, v[t].z, img, 2);
                v[t].w = prologue(a, v[t].w, img, 3);
                if (!ok) v[t] = f4{0.f, 0.f, 0.f, 0.f};
            }
        }
        f4 acc[QPT];
#pragma unroll
        for (int q = 0; q < QPT; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float ve = e == 0 ? v[t].x : e == 1 ? v[t].y : e == 2 ? v[t].z : v[t].w;
                const float *wr = wk + (t * 4 + e) * a.cout + 4 * tq;
#pragma unroll
                for (int q = 0; q < QPT; ++q) {
                    const f4 w4 = *(const f4 *)(wr + 4 * tppx * q);
                    acc[q].x = fmaf(ve, w4.x, acc[q].x);
                    acc[q].y = fmaf(ve, w4.y, acc[q].y);
                    acc[q].z = fmaf(ve, w4.z, acc[q].z);
                    acc[q].w = fmaf(ve, w4.w, acc[q].w);
                }
            }
#pragma unroll
        for (int q = 0; q < QPT; ++q)
            store_epilogue4(a, bidx, m, 4 * (tq + tppx * q), acc[q], vec != 0, SMALLK_NT != 0);
    }
}

// Direct VALU convolution for tiny Cout (final RGB / flow heads, ToRGB): one thread per output
// pixel, all CO outputs per thread.  Per filter tap the block stages W[:, tap, c0:c0+CCH] in LDS,
// so every weight read is an LDS broadcast (all lanes read the same address).
template <int CO>
__global__ __launch_bounds__(256) void conv_direct_small(ConvArgs a, int batch) {
    constexpr int CCH = 512;                  // channels staged per pass
    __shared__ __attribute__((aligned(16))) float wsm[CO * CCH];
    const long long total = (long long)batch * a.M;
    const long long gid = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const bool live = gid < total;
    const int bidx = live ? (int)(gid / a.M) : 0;
    const int m = live ? (int)(gid - (long long)bidx * a.M) : 0;
    const int hw = a.oh * a.ow;
    const int img = m / hw;
    const int rem = m - img * hw;
    const int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
    const float *x = a.x + (long long)bidx * a.x_bs;
    const float *wt = a.wt + (long long)bidx * a.w_bs;
    float acc[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[o] = 0.f;
    const bool vec = (a.cin % 4 == 0) && (a.xcs % 4 == 0) && !a.in_scale && !a.pre_act &&
                     (((uintptr_t)x & 15) == 0);
    for (int ky = 0; ky < a.kh; ++ky)
        for (int kx = 0; kx < a.kw; ++kx) {
            int iy = 0, ix = 0;
            const bool ok = live && map_tap(a, oy, ox, ky, kx, iy, ix);
            const float *px = x + ((long long)(img * a.h + iy) * a.w + ix) * a.xcs;
            const int kb = (ky * a.kw + kx) * a.cin;
            for (int c0 = 0; c0 < a.cin; c0 += CCH) {
                const int cn = min(CCH, a.cin - c0);
                __syncthreads();
                for (int e = threadIdx.x; e < CO * cn; e += 256) {
                    const int o = e / cn, c = e - (e / cn) * cn;
                    wsm[o * CCH + c] = o < a.cout ? wt[(long long)o * a.kpad + kb + c0 + c] : 0.f;
                }
                __syncthreads();
                if (!ok) continue;
                if (vec) {
                    for (int c = 0; c < cn; c += 4) {
                        const float4 v = *(const float4 *)(px + c0 + c);
#pragma unroll
                        for (int o = 0; o < CO; ++o) {
                            const float4 wv = *(const float4 *)&wsm[o * CCH + c];
                            acc[o] = fmaf(v.x, wv.x, acc[o]);
                            acc[o] = fmaf(v.y, wv.y, acc[o]);
                            acc[o] = fmaf(v.z, wv.z, acc[o]);
                            acc[o] = fmaf(v.w, wv.w, acc[o]);
                        }
                    }
                } else {
                    for (int c = 0; c < cn; ++c) {
                        const float v = prologue(a, px[c0 + c], img, c0 + c);
#pragma unroll
                        for (int o = 0; o < CO; ++o) acc[o] = fmaf(v, wsm[o * CCH + c], acc[o]);
                    }
                }
            }
        }
    if (!live) return;
#pragma unroll
    for (int o = 0; o < CO; ++o)
        if (o < a.cout) store_epilogue(a, bidx, m, o, acc[o]);
}

// Small-Cout conv, channel-parallel form: TPP lanes share one output pixel, each owns 4 input
// channels (16-byte loads; consecutive lanes read consecutive bytes of the pixel row, so a wave
// reads 64/TPP neighbouring pixels contiguously), partial dot products are combined with
// shuffles.  Requires cin % 4 == 0 and 16-byte aligned rows.
// LW: the block's filter (CO x K floats of one batch entry) is staged in LDS first, so the per-tap
// weight reads are LDS broadcasts instead of CO global loads per input float4.
template <int CO, int TPP, bool LW>
__global__ __launch_bounds__(256) void conv_small_cpar(ConvArgs a, int batch) {
    extern __shared__ __attribute__((aligned(16))) float wsm_dyn[];
    const long long total = (long long)batch * a.M;
    const unsigned blk = xcd_block(blockIdx.x, gridDim.x);      // stencil rows share one XCD's L2
    const long long gid = (blk * 256LL + threadIdx.x) / TPP;
    const int sub = threadIdx.x % TPP;
    const bool live = gid < total;
    const int bidx = live ? (int)(gid / a.M) : 0;
    const int m = live ? (int)(gid - (long long)bidx * a.M) : 0;
    const int hw = a.oh * a.ow;
    const int img = m / hw;
    const int rem = m - img * hw;
    const int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
    const float *x = a.x + (long long)bidx * a.x_bs;
    const float *wt = a.wt + (long long)bidx * a.w_bs;
    int wstride = a.kpad;
    if (LW) {
        // every pixel of the block belongs to the batch entry of its first pixel (the host
        // guarantees M % (256 / TPP) == 0 when the weights are per batch entry)
        const long long g0 = blk * (256LL / TPP);
        const int b0 = (int)((g0 < total ? g0 : 0) / a.M);
        const float *w0 = a.wt + (long long)b0 * a.w_bs;
        for (int e = threadIdx.x; e < CO * a.K; e += 256) {
            const int o = e / a.K, k = e - (e / a.K) * a.K;
            wsm_dyn[e] = o < a.cout ? w0[(long long)o * a.kpad + k] : 0.f;
        }
        __syncthreads();
        wt = wsm_dyn;
        wstride = a.K;
    }
    float acc[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[o] = 0.f;
    if (live) {
        for (int ky = 0; ky < a.kh; ++ky)
            for (int kx = 0; kx < a.kw; ++kx) {
                int iy, ix;
                if (!map_tap(a, oy, ox, ky, kx, iy, ix)) continue;
                const float *px = x + ((long long)(img * a.h + iy) * a.w + ix) * a.xcs;
                const int kb = (ky * a.kw + kx) * a.cin;
                for (int c = sub * 4; c < a.cin; c += TPP * 4) {
                    f4 v = *(const f4 *)(px + c);
                    if (a.in_scale) v *= *(const f4 *)(a.in_scale + (long long)img * a.in_scale_ns + c);
                    if (a.pre_act) {
                        v.x = apply_act(v.x, a.pre_act, a.pre_alpha);
                        v.y = apply_act(v.y, a.pre_act, a.pre_alpha);
                        v.z = apply_act(v.z, a.pre_act, a.pre_alpha);
                        v.w = apply_act(v.w, a.pre_act, a.pre_alpha);
                    }
#pragma unroll
                    for (int o = 0; o < CO; ++o) {
                        const f4 wv = *(const f4 *)(wt + (long long)o * wstride + kb + c);
                        acc[o] = fmaf(v.x, wv.x, fmaf(v.y, wv.y, fmaf(v.z, wv.z, fmaf(v.w, wv.w, acc[o]))));
                    }
                }
            }
    }
#pragma unroll
    for (int o = 0; o < CO; ++o)
#pragma unroll
        for (int off = TPP / 2; off > 0; off >>= 1) acc[o] += __shfl_xor(acc[o], off, 64);
    if (!live || sub != 0) return;
#pragma unroll
    for (int o = 0; o < CO; ++o)
        if (o < a.cout) store_epilogue(a, bidx, m, o, acc[o]);
}

// LDS weights when the filter is small next to the block's input (<= 16 KB: ToRGB 1x1s); the 7x7
// heads keep global (L1-resident) weight reads.  Per-batch-entry weights need every block inside
// one entry (M % pixels-per-block == 0).  s2v_conv2d_plan reports the same flag.
static bool cpar_lw(int co, int K, long long w_bs, int batch, int M, int tpp) {
    return (size_t)co * K * sizeof(float) <= 16 * 1024 && (w_bs == 0 || batch == 1 || M % (256 / tpp) == 0);
}

template <int CO, int TPP>
static void launch_cpar(const ConvArgs &a, int batch, hipStream_t s) {
    const long long total = (long long)batch * a.M;
    const unsigned grid = cdiv(total * TPP, 256);
    const size_t wbytes = (size_t)CO * a.K * sizeof(float);
    if (cpar_lw(CO, a.K, a.w_bs, batch, a.M, TPP)) conv_small_cpar<CO, TPP, true><<<grid, 256, wbytes, s>>>(a, batch);
    else conv_small_cpar<CO, TPP, false><<<grid, 256, 0, s>>>(a, batch);
}

// lanes per output pixel of conv_small_cpar (launch_small and the plan report share it)
static int cpar_lanes(int cin) { return cin >= 128 ? 8 : cin >= 64 ? 4 : cin >= 32 ? 2 : 4; }

template <int CO>
static void launch_small(const ConvArgs &a, int batch, bool cpar, hipStream_t s) {
    const long long total = (long long)batch * a.M;
    if (!cpar) {
        conv_direct_small<CO><<<cdiv(total, 256), 256, 0, s>>>(a, batch);
        return;
    }
    // 8 lanes per pixel (each lane walks cin/32 float4s): 3 shuffle levels per output instead of
    // 5-6 with one float4 per lane, 128-byte contiguous row pieces per load instruction.  Below 128
    // channels fewer lanes share a pixel so every lane still has >= 4 float4s in flight per tap:
    // with one float4 per lane (32-channel ToRGB heads at 2048^2, RealESRNet's conv_last) the
    // kernel was latency-bound at 1.5 TB/s.
    switch (cpar_lanes(a.cin)) {
        case 8: launch_cpar<CO, 8>(a, batch, s); break;
        case 2: launch_cpar<CO, 2>(a, batch, s); break;
        default: launch_cpar<CO, 4>(a, batch, s); break;
    }
}


// Halo-tiled direct conv for Cout <= 4 heads with a wide square filter (DNet's 7x7 64 -> 3 tanh
// head at 256^2, LNet's 7x7 64 -> 3 sigmoid head): a block owns an 8 x 128 output tile; per chunk
// of 4 input channels it stages the (8 + KS - 1) x (128 + KS - 1) input halo once in LDS (planar
// per channel), and each thread computes 4 horizontally adjacent pixels x CO outputs from 16-byte
// LDS row reads, so every staged value feeds up to 4 * KS taps.  The per-pixel gather of
// conv_small_cpar re-read each input pixel KS^2 times from L1/L2 (DNet head: 1.5 ms per 16 frames
// at 185 GB/s).  Filter values are block-uniform (scalar loads).  fp32 VALU, exact products.
template <int CO, int KS>
__global__ __launch_bounds__(256) void conv_halo_small(ConvArgs a, int tiles_x, int tiles_y) {
    constexpr int TH = 8, PX = 4, TW = 32 * PX;
    constexpr int IH = TH + KS - 1, IW = TW + KS - 1, IWP = (IW + 3) / 4 * 4;
    constexpr int NV = (PX + KS - 1 + 3) / 4;                 // float4 row reads per (channel, ky)
    static_assert(4 * 31 + 4 * NV <= IWP, "halo row reads stay inside the padded LDS row");
    __shared__ __attribute__((aligned(16))) float tile[4][IH][IWP];
    const int tid = threadIdx.x, r = tid >> 5, cg = tid & 31;
    int t = blockIdx.x;
    const int txi = t % tiles_x;
    t /= tiles_x;
    const int tyi = t % tiles_y, img = t / tiles_y;
    const int oy0 = tyi * TH, ox0 = txi * TW;
    const float *xb = a.x + (long long)img * a.h * a.w * a.xcs;
    const float *__restrict__ wt = a.wt;
    // channel split (gridDim.y = a.splits, a.tps channels each): raw partial sums to the split-K
    // workspace, folded by splitk_reduce with the epilogue (small images: too few tiles otherwise)
    const int cb = blockIdx.y * a.tps, ce = min(a.cin, cb + a.tps);
    float acc[PX][CO];
#pragma unroll
    for (int p = 0; p < PX; ++p)
#pragma unroll
        for (int o = 0; o < CO; ++o) acc[p][o] = 0.f;
    const bool refl = a.pad_mode == S2V_PAD_REFLECT;
    for (int c0 = cb; c0 < ce; c0 += 4) {
        __syncthreads();                                      // the previous chunk has been consumed
        for (int e = tid; e < IH * IW; e += 256) {
            const int iy = e / IW, ix = e - iy * IW;
            int gy = oy0 + iy - a.ph, gx = ox0 + ix - a.pw;
            if (refl) {
                gy = reflect_idx(gy, a.h);
                gx = reflect_idx(gx, a.w);
            }
            // halo rows / columns past the image (tiles overhanging the bottom / right edge, or
            // beyond a single reflection) feed only outputs that are never stored
            const bool ok = (unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w;
            f4 v = f4{0.f, 0.f, 0.f, 0.f};
            if (ok) v = *(const f4 *)(xb + ((long long)gy * a.w + gx) * a.xcs + c0);
            tile[0][iy][ix] = v.x;
            tile[1][iy][ix] = v.y;
            tile[2][iy][ix] = v.z;
            tile[3][iy][ix] = v.w;
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int ky = 0; ky < KS; ++ky) {
                float row[4 * NV];
                const float *src = &tile[c][r + ky][4 * cg];
#pragma unroll
                for (int j = 0; j < NV; ++j) *(f4 *)&row[4 * j] = *(const f4 *)(src + 4 * j);
#pragma unroll
                for (int kx = 0; kx < KS; ++kx) {
                    const long long k = (long long)(ky * KS + kx) * a.cin + c0 + c;
                    float wv[CO];
#pragma unroll
                    for (int o = 0; o < CO; ++o) wv[o] = wt[(long long)o * a.kpad + k];
#pragma unroll
                    for (int p = 0; p < PX; ++p)
#pragma unroll
                        for (int o = 0; o < CO; ++o) acc[p][o] = fmaf(row[p + kx], wv[o], acc[p][o]);
                }
            }
        }
    }
    const int oy = oy0 + r;
    if (oy >= a.oh) return;
#pragma unroll
    for (int p = 0; p < PX; ++p) {
        const int ox = ox0 + 4 * cg + p;
        if (ox >= a.ow) continue;
        const int m = (img * a.oh + oy) * a.ow + ox;
        if (a.splits > 1) {
            float *w = a.ws + ((long long)blockIdx.y * a.M + m) * a.cout;
#pragma unroll
            for (int o = 0; o < CO; ++o) w[o] = acc[p][o];
            continue;
        }
#pragma unroll
        for (int o = 0; o < CO; ++o) store_epilogue(a, 0, m, o, acc[p][o]);
    }
}

// The halo kernel serves plain stride-1 square-filter heads: direct input, zero or reflect
// padding (pad < filter), no prologue scaling, one shared filter, 16-byte channel quads.
// planner knobs (s2v_tune; defaults, or S2V_HALO_MIN_BLOCKS / S2V_GLDS_TILE from the environment)
static long long g_tune[S2V_TUNE_COUNT];
static bool g_tune_init = false;
static long long tune_value(int key) {
    if (!g_tune_init) {
        const char *e = getenv("S2V_HALO_MIN_BLOCKS");
        g_tune[S2V_TUNE_HALO_MIN_BLOCKS] = e ? atoll(e) : 0;
        e = getenv("S2V_GLDS_TILE");
        g_tune[S2V_TUNE_GLDS_TILE] = e ? atoll(e) : -1;
        e = getenv("S2V_SMALLK_TILE");
        g_tune[S2V_TUNE_SMALLK_TILE] = e ? atoll(e) : 1;
        e = getenv("S2V_X3_RATE_512");
        g_tune[S2V_TUNE_X3_RATE_512] = e ? atoll(e) : 0;
        e = getenv("S2V_IN_FUSED");
        g_tune[S2V_TUNE_IN_FUSED] = e ? atoll(e) : 576;   // max plane pixels of the one-launch InstanceNorm
        e = getenv("S2V_RESIZE_UP2");
        g_tune[S2V_TUNE_RESIZE_UP2] = e ? atoll(e) : 1;
        g_tune_init = true;
    }
    return g_tune[key];
}

// CUs the planner fills (split-K factors, tile choice): the device's
static int plan_cus() { return device_cus() > 0 ? device_cus() : 256; }

long long tune_get(int key) { return tune_value(key); }

static int halo_ks(const s2v_conv_params *p) {
    const int batch = p->batch > 0 ? p->batch : 1;
    if (p->cout > 4 || p->kh != p->kw || (p->kh != 3 && p->kh != 5 && p->kh != 7)) return 0;
    if (p->in_mode != S2V_IN_DIRECT || p->sh != 1 || p->sw != 1 || p->dh != 1 || p->dw != 1) return 0;
    if (p->in_scale || p->pre_act || p->w_bs || batch != 1 || p->b_kn || p->out_step > 1) return 0;
    if (p->ph >= p->kh || p->pw >= p->kw || p->cin % 4 || p->xcs % 4 || ((uintptr_t)p->x % 16)) return 0;
    if (p->pad_mode == S2V_PAD_REFLECT && (p->ph >= p->h || p->pw >= p->w)) return 0;
    // 8 x 128 output tiles: on small images (LNet's 96^2 RGB head, DNet's 64^2 flow head) too few
    // blocks cover the chip and a 128-wide tile runs part empty; the channel-parallel kernel (lanes
    // split K per pixel) has the parallelism there.  S2V_HALO_MIN_BLOCKS overrides (tuning).
    const long long blocks = (long long)p->n * cdiv(p->ow, 128) * cdiv(p->oh, 8);
    if (blocks < tune_value(S2V_TUNE_HALO_MIN_BLOCKS)) return 0;
    return p->kh;
}

// Split-precision heads (conv_head.hip): Cout <= 4, a square 5x5 / 7x7 stride-1 filter over 32 / 64
// channels, direct input with zero or reflect padding, no prologue scaling, one shared filter
// (S2V_HEAD_X3=0: the fp32 VALU kernels instead)
int launch_conv_head_x3(const ConvArgs &a, int prec, int co, int ks, int ncs, int th, hipStream_t s);
static bool head_x3_on() {
    static const int on = [] { const char *e = getenv("S2V_HEAD_X3"); return e ? atoi(e) : 1; }();
    return on != 0;
}
static bool head_x3_ok(const s2v_conv_params *p) {
    const int batch = p->batch > 0 ? p->batch : 1;
    if (!head_x3_on() || p->prec == S2V_PREC_F32 || p->x_split || p->force_tile || !p->wt_x3 || ((uintptr_t)p->wt_x3 % 16))
        return false;
    if (p->cout > 4 || p->kh != p->kw || (p->kh != 7 && p->kh != 5) || (p->cin != 32 && p->cin % 64) || p->cin > 512)
        return false;
    if (p->in_mode != S2V_IN_DIRECT || p->sh != 1 || p->sw != 1 || p->dh != 1 || p->dw != 1) return false;
    if (p->in_scale || p->pre_act || p->w_bs || batch != 1 || p->b_kn || p->out_step > 1 || p->out_pool || p->d2s_cout)
        return false;
    if (p->ph >= p->kh || p->pw >= p->kw || p->xcs % 4 || ((uintptr_t)p->x % 16)) return false;
    if (p->pad_mode == S2V_PAD_REFLECT && (p->ph >= p->h || p->pw >= p->w)) return false;
    return true;
}
// output rows per conv_head_x3 block: 16, halved while the grid is under two blocks per CU (>= 4)
static int head_rows(const s2v_conv_params *p) {
    const long long strips = cdiv(p->ow, 32 - p->kw + 1);
    int th = 16;
    const long long groups = p->cin > 64 ? p->cin / 64 : 1;
    while (th > 4 && (long long)p->n * strips * groups * cdiv(p->oh, th) < 2LL * device_cus()) th /= 2;
    return th;
}

// channel splits of the halo kernel: about three blocks per CU, at least 8 channels per split
static int halo_splits(const s2v_conv_params *p, int &per) {
    const long long blocks = (long long)p->n * cdiv(p->ow, 128) * cdiv(p->oh, 8);
    const int cus = plan_cus();
    const int quads = p->cin / 4;
    int s = blocks >= 3LL * cus ? 1 : (int)((3LL * cus + blocks - 1) / blocks);
    if (s > quads / 2) s = quads / 2;
    if (s < 1) s = 1;
    per = 4 * ((quads + s - 1) / s);
    return (p->cin + per - 1) / per;
}

template <int CO>
static void launch_halo(const ConvArgs &a, int ks, hipStream_t s) {
    const int tiles_x = (int)cdiv(a.ow, 128), tiles_y = (int)cdiv(a.oh, 8);
    const dim3 grid((unsigned)((long long)a.n * tiles_x * tiles_y), (unsigned)a.splits);
    if (ks == 3) conv_halo_small<CO, 3><<<grid, 256, 0, s>>>(a, tiles_x, tiles_y);
    else if (ks == 5) conv_halo_small<CO, 5><<<grid, 256, 0, s>>>(a, tiles_x, tiles_y);
    else conv_halo_small<CO, 7><<<grid, 256, 0, s>>>(a, tiles_x, tiles_y);
}

// ------------------------------------------------------------------ host side
struct TileCfg {
    int bm, bn, wm, nw, ks, pf;   // nw / ks / pf: waves, K-slices per stage, prefetch sets (x3 kernel)
};
static const TileCfg kTiles[] = {
    {128, 128, 2, 4, 1, 2}, {128, 64, 2, 4, 1, 2}, {64, 128, 2, 4, 1, 2}, {64, 64, 2, 4, 1, 2}, {256, 32, 4, 4, 1, 2},
    {128, 32, 4, 4, 1, 2}};
// split-fp32 (S2V_PREC_BF16X3 / F16X3) configurations, conv_x3_impl.hpp launch_conv_x3, with the sustained
// throughput each reaches on a full chip (TFLOP/s fp32-equivalent, MI355X, tools/conv_micro.py r01)
// and resident blocks per CU (LDS / waves) for the planner's cost model
// (512x128: 360, set end to end on MI355X r03 — lipsync 29.11 -> 28.35 ms, its 400^2 N = 128 StyleConvs;
// 420 also displaces the 256x256 tile on N = 256 layers: 28.80 ms)
struct X3Cfg {
    TileCfg t;
    float tflops;
    int bpc;
    int kind = 0;    // 1 / 2: conv_x3_nar (register-direct A / A and B fragments), 3 / 4: conv_x3_halo (4 / 8 rows)
};
static const X3Cfg kX3Tiles[] = {
    {{256, 256, 2, 8, 1, 1}, 400.f, 1}, {{128, 128, 2, 8, 1, 1}, 330.f, 2}, {{64, 128, 2, 8, 1, 1}, 260.f, 3},
    {{128, 64, 2, 4, 1, 1}, 290.f, 3},  {{64, 64, 2, 4, 1, 1}, 265.f, 4},   {{128, 32, 4, 4, 1, 1}, 235.f, 4},
    {{256, 128, 4, 8, 1, 1}, 335.f, 1}, {{256, 64, 8, 8, 1, 1}, 300.f, 2},  {{512, 128, 4, 8, 1, 1}, 360.f, 1},
    // narrow-N tiles with 64-row waves (r04, tools/r04_nsweep.sh on MI355X, graph-timed 3x3 64-channel
    // convs): 4x512^2 128 -> 64 199 (256x64 8-wave) -> 225 (512x64) / 233 (256x64 4-wave) TFLOP/s,
    // 16x256^2 64 -> 64 156 -> 171 / 183; at 96^2 and below 128x64 stays ahead (more blocks).  The
    // rates keep that order in the planner's model.  256x32 (4-wave): no faster than 128x32, forced-only.
    {{512, 64, 8, 8, 1, 1}, 335.f, 1},  {{256, 64, 4, 4, 1, 1}, 350.f, 2},  {{256, 32, 4, 4, 1, 1}, 0.f, 2},
    // deep-stage 4-wave tiles (r05): 2 or 4 K-slices per LDS stage, so a latency-bound small-grid conv (LNet's
    // 12^2 - 48^2 layers: one block per CU, K loops of 6 - 72 slices) waits on half / a quarter as many
    // load round trips; one block per CU by LDS.  Forced-only until measured (tools/lnet_convs.py --tiles)
    {{64, 64, 2, 4, 4, 1}, 0.f, 1},     {{128, 64, 2, 4, 2, 1}, 0.f, 1},   {{128, 32, 4, 4, 2, 1}, 0.f, 1},
    // 256 x 64 with A fragments loaded by each lane straight into registers, B alone through LDS
    // (conv_x3_nar.hip): direct zero-padded convs, cin % 32 == 0, no pooled epilogue, 2^31-byte offsets
    {{256, 64, 4, 4, 1, 1}, 0.f, 2, 1},
    // ... with the B fragments loaded by every wave into registers too: no LDS, no barrier per slice
    {{256, 64, 4, 4, 1, 1}, 0.f, 2, 2},
    // 4 x 64 output patches, 64 channels, the 6 x 66 input halo per channel slice staged once
    // (conv_x3_halo.hip): 3x3 stride-1 zero-padded convs (ragged images: partly empty last patches)
    {{256, 64, 4, 4, 1, 1}, 0.f, 2, 3},
    // ... 8 x 64 patches, one 512-thread block per CU (oh % 8 == 0)
    {{512, 64, 8, 8, 1, 1}, 0.f, 1, 4},
    // ... 4 x 64 patches x 128 output channels (two 64-channel wave columns), one 512-thread block per CU
    {{256, 128, 4, 8, 1, 1}, 0.f, 1, 5}};
constexpr int kNumX3 = sizeof(kX3Tiles) / sizeof(kX3Tiles[0]);

static const TileCfg &tile_cfg(const s2v_conv_params *p, int tile);
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

struct Plan {
    int tile;   // index into kTiles, or -1 for the direct small-N kernel
    int splits, tps, ktiles;
    int kslab = 1;   // split-K granularity in K-slices (9 for conv_x3_halo: whole channel slices)
};

// 16-byte epilogue stores are possible (store_epilogue4's vec): aligned rows and per-channel vectors
static int epi_vec4(const s2v_conv_params *p) {
    return p->cout % 4 == 0 && p->ycs % 4 == 0 && ((uintptr_t)p->y % 16) == 0 && p->y_bs % 4 == 0 &&
           (!p->res || (p->res_cs % 4 == 0 && ((uintptr_t)p->res % 16) == 0 && p->res_bs % 4 == 0)) &&
           (!p->scale || ((uintptr_t)p->scale % 16) == 0) && (!p->shift || ((uintptr_t)p->shift % 16) == 0) &&
           (!p->post_mul || (p->post_cs % 4 == 0 && p->post_c0 % 4 == 0 && ((uintptr_t)p->post_mul % 16) == 0 &&
                             ((uintptr_t)p->post_add % 16) == 0)) &&
           (!p->dup_src || (p->dup_cs % 4 == 0 && p->dup_off % 4 == 0 && ((uintptr_t)p->dup_src % 16) == 0 &&
                            (!p->dup_bias || ((uintptr_t)p->dup_bias % 16) == 0)));
}

static bool use_direct(const s2v_conv_params *p) { return p->cout <= 4 && !p->b_kn; }

// 4-channel 1x1 / 3x3 convs on the exact-fp32 MFMA kernel (conv_k4.hip) in every precision mode: stride 1,
// zero "same" padding, 32k <= 256 output channels, a plain epilogue (scale, shift, per-pixel add, activation);
// S2V_K4=0: the split-precision tiles / conv_smallk4 instead
int launch_conv_k4(const ConvArgs &a, int batch, int kt, hipStream_t s);
static bool k4_ok(const s2v_conv_params *p) {
    static const int on = [] { const char *e = getenv("S2V_K4"); return e ? atoi(e) : 1; }();
    if (!on || p->cin != 4 || p->kh != p->kw || (p->kh != 1 && p->kh != 3) || p->force_tile || p->b_kn || p->x_split)
        return false;
    if (p->in_mode != S2V_IN_DIRECT || p->pad_mode != S2V_PAD_ZERO || p->sh != 1 || p->sw != 1 || p->dh != 1 ||
        p->dw != 1 || p->ph != p->kh / 2 || p->pw != p->kw / 2)
        return false;
    if (p->cout % 32 || p->cout > 256 || p->in_scale || p->pre_act != S2V_ACT_NONE || p->nc_scale || p->res ||
        p->post_mul || p->dup_src || p->out_pool || p->out_step > 1 || p->d2s_cout > 0)
        return false;
    if (!p->wt || p->kpad < p->kh * p->kw * 4 || p->xcs % 4 || ((uintptr_t)p->x % 16) || p->x_bs % 4) return false;
    return (long long)p->n * p->oh * p->ow < (1LL << 31);
}

static bool vec4_input(const s2v_conv_params *p) {
    return (p->cin % 4 == 0) && (p->xcs % 4 == 0) && (((uintptr_t)p->x % 16) == 0) && (p->x_bs % 4 == 0) &&
           (!p->in_scale || (p->in_scale_ns % 4 == 0 && ((uintptr_t)p->in_scale % 16) == 0));
}

static int smallk_px(int M);

// conv_smallk geometry: threads per pixel (cout / 4 channel quads, at most 64) and quads per thread
static bool smallk_cfg(const s2v_conv_params *p, int M, int K, int &tppx, int &qpt) {
    if (p->b_kn || p->force_tile || p->out_pool || p->cout < 8 || (p->cout & 3) || K > 64 || !vec4_input(p)) return false;
    // multi-tap filters on 4k-channel inputs go to the split-precision implicit GEMM even at K <= 64
    // (measured on MI355X, r02: 3x3 4 -> 256 at 200^2 776 -> 336 us, 4 -> 64 at 512^2 602 -> 361 us,
    // at 96^2 74 -> 32 us; the 1x1 4 -> 256 layer stays here, 415 us against 491 us)
    if (p->prec != S2V_PREC_F32 && p->kh * p->kw > 1) return false;
    // 1x1 convs on >= 32 channels too (ResNet-50 layer1 64 -> 64 / 64 -> 256 at 56^2: VALU-bound here)
    if (p->prec != S2V_PREC_F32 && K >= 32) return false;
    const int quads = p->cout / 4;
    if (quads & (quads - 1)) return false;                       // power of two
    // one output quad per thread, up to 64 threads per pixel (measured on MI355X: 64 lanes x 1 quad
    // beat 4 lanes x 16 quads and 4-pixel register blocking on the 256-channel image layers, r02)
    tppx = quads < 64 ? quads : 64;
    qpt = quads / tppx;
    if (qpt > 2 || (size_t)K * p->cout * sizeof(float) > 64 * 1024) return false;
    const int batch = p->batch > 0 ? p->batch : 1;
    return p->w_bs == 0 || batch == 1 || (M / smallk_px(M)) % (256 / tppx) == 0;
}

// pixels per thread group: 4 when M % 4 == 0 (register blocking over pixels), else 1
static int smallk_px(int M) { (void)M; return 1; }

// groups per block = iters x (256 / tppx): up to 16 iterations, and a divisor of M / px when each
// batch entry has its own weights (a block never straddles two entries)
static int smallk_iters(const s2v_conv_params *p, int M, int tppx) {
    const int batch = p->batch > 0 ? p->batch : 1;
    const bool per_entry = p->w_bs != 0 && batch > 1;
    const int px = smallk_px(M);
    int it = 16;
    while (it > 1 && per_entry && (M / px) % (it * (256 / tppx)) != 0) it /= 2;
    return it;
}

// the split-bf16 kernel reads the pre-split packed weights; b_kn matrices are split on the fly
static bool smallk_cfg(const s2v_conv_params *p, int M, int K, int &tppx, int &qpt);

static bool is_smallk(const s2v_conv_params *p) {
    const long long m = (long long)p->n * p->oh * p->ow, k = (long long)p->kh * p->kw * p->cin;
    int tppx, qpt;
    return m < (1LL << 31) && k <= 64 && smallk_cfg(p, (int)m, (int)k, tppx, qpt);
}
static bool tiled_x3(const s2v_conv_params *p) {
    return p->prec != S2V_PREC_F32 && !(use_direct(p) && !p->force_tile) && !is_smallk(p) && !k4_ok(p);
}
static bool uses_x3(const s2v_conv_params *p) { return tiled_x3(p) && !p->b_kn; }

static int a_mode(const s2v_conv_params *p);
static bool nar_ok(const s2v_conv_params *p);
static bool x3_kind_ok(const s2v_conv_params *p, int kind);
static bool halo_ok(const s2v_conv_params *p);
static double halo_fill(const s2v_conv_params *p, int th);


static const TileCfg &tile_cfg(const s2v_conv_params *p, int tile) {
    return tiled_x3(p) ? kX3Tiles[tile].t : kTiles[tile];
}

static void finish_plan(Plan &pl, int splits) {
    if (pl.kslab > 1) {                  // splits over whole groups of kslab K-slices (conv_x3_halo: 9 taps)
        const int groups = pl.ktiles / pl.kslab;
        if (splits > groups) splits = groups;
        if (splits < 1) splits = 1;
        pl.tps = (groups + splits - 1) / splits * pl.kslab;
        pl.splits = (pl.ktiles + pl.tps - 1) / pl.tps;
        return;
    }
    if (splits > pl.ktiles) splits = pl.ktiles;
    if (splits < 1) splits = 1;
    pl.tps = (pl.ktiles + splits - 1) / splits;
    pl.splits = (pl.ktiles + pl.tps - 1) / pl.tps;
}

// Split-bf16 planner: minimise a simple time model over (tile, split-K):
//   T = ceil(blocks / (CUs * bpc)) * t_block + splitk_reduce
// with t_block = one block's share of the tile's sustained full-chip rate (kX3Tiles).
static Plan make_plan_x3(const s2v_conv_params *p, int M, Plan pl) {
    const int batch = p->batch > 0 ? p->batch : 1;
    const int cus = plan_cus();
    if (p->force_tile > 0) {
        pl.tile = p->force_tile - 1;
        if (kX3Tiles[pl.tile].kind >= 3) pl.kslab = 9;
        const TileCfg &t = kX3Tiles[pl.tile].t;
        const long long blocks = (long long)cdiv(M, t.bm) * cdiv(p->cout, t.bn) * batch;
        int splits = p->force_splits;
        if (splits <= 0) {
            splits = 1;
            if (blocks < 2LL * cus) splits = (int)((2LL * cus + blocks - 1) / blocks);
            if (splits > pl.ktiles / 8) splits = pl.ktiles / 8;
        }
        finish_plan(pl, splits);
        return pl;
    }
    // 3x3 stride-1 layers of <= 128 output channels over 64-wide rows (the enhancers' and DNet's 128^2 -
    // 512^2 layers): the halo-staged spatial patch kernel, measured 20-30 % faster than every implicit-GEMM
    // tile on them (4x512^2 64 -> 64: 356 vs 444 us, 128 -> 64: 547 vs 697, 4x256^2 128 -> 128: 292 vs 381,
    // profiles/r05_halo_sweep.txt), whenever the grid fills the chip without split-K
    // (<= 32 output channels stay on the 32-column tiles: half of a 64-column halo block would be idle,
    // 4x512^2 64 -> 32: 320 us against 277 us on 128x32)
    if (halo_ok(p) && p->cout > 32 && p->cout <= 128 && halo_fill(p, 4) >= 0.85) {
        const int batch = p->batch > 0 ? p->batch : 1;
        const long long blocks = (long long)p->n * cdiv(p->oh, 4) * cdiv(p->ow, 64) * cdiv(p->cout, 64) * batch;
        // 65..128 output channels: one block per 128 columns (two 64-channel wave columns share the halo):
        // 4x256^2 128 -> 128 279 vs 291 us (profiles/r05_halo_sweep.txt); <= 64: the 4-wave 64-column block
        const int kind = p->cout > 64 && x3_kind_ok(p, 5) ? 5 : 3;
        // ... but large 65..128-channel layers stay on 512x128: 16x400^2 128 -> 128 2189 us there against
        // 2595 / 2418 us on the halo blocks (profiles/r05_halo_sweep.txt)
        const bool big_n128 = p->cout > 64 && (long long)p->n * p->oh * p->ow * batch >= (1LL << 20);
        if (blocks >= 2LL * plan_cus() && !big_n128) {
            for (int i = 0; i < kNumX3; ++i)
                if (kX3Tiles[i].kind == kind) {
                    pl.tile = i;
                    pl.kslab = 9;
                    finish_plan(pl, 1);
                    return pl;
                }
        }
    }
    if (pl.ktiles <= 4 && !p->b_kn && tune_value(S2V_TUNE_SMALLK_TILE)) {
        // K <= 128 (image-input layers): the launch is output-write / gather bound, the throughput
        // model does not apply.  One N tile covering cout reads A once; measured on MI355X (r02):
        // 4 -> 256 3x3 at 200^2 256x256 336 us (128x128 497), 4 -> 64 at 96^2 64x64 32 us (128x64 43)
        // (small M — LNet's 12^2 1x1 convs — keeps the throughput model: it needs the blocks)
        int t = p->cout > 128 ? 0 : (p->cout > 64 ? 1 : 4);
        const TileCfg &c = kX3Tiles[t].t;
        const long long blocks = (long long)cdiv(M, c.bm) * cdiv(p->cout, c.bn) * batch;
        if ((long long)cdiv(p->cout, c.bn) * c.bn <= p->npad && blocks >= 4LL * cus) {
            pl.tile = t;
            finish_plan(pl, 1);
            return pl;
        }
    }
    double best = 1e30;
    int bt = 8, bs = 1;                                      // 512x128: the planner's fallback
    const int am = a_mode(p);
    for (int i = 0; i < kNumX3; ++i) {
        const X3Cfg &c = kX3Tiles[i];
        if (c.tflops <= 0.f) continue;                          // forced-only configurations
        if (!x3_kind_ok(p, c.kind)) continue;
        if (p->b_kn && c.t.nw != 4) continue;
        if (c.t.bm >= 256 && c.t.bn >= 128 && am != 0 && am != 3) continue;   // generic gathers spill there
        // the 256 / 512-row narrow-N tiles on per-row gathers: measured slower than 128x64 (256x64, r02)
        if (c.t.bm >= 256 && c.t.bn <= 64 && am != 0) continue;
        if (!p->b_kn && (long long)cdiv(p->cout, c.t.bn) * c.t.bn > p->npad) continue;   // weight rows
        const long long tiles = (long long)cdiv(M, c.t.bm) * cdiv(p->cout, c.t.bn) * batch;
        const double slots = (double)cus * c.bpc;
        for (int s = 1; s <= 16; s *= 2) {
            if (s > 1 && (p->force_splits > 0 || s > pl.ktiles / 4)) break;
            if (p->force_splits > 0) s = p->force_splits;
            const int tps = (pl.ktiles + s - 1) / s;
            const long long r512 = (c.t.bm == 512) ? tune_value(S2V_TUNE_X3_RATE_512) : 0;
            const double rate = r512 > 0 ? (double)r512 : c.tflops;
            const double t_block = 2.0 * c.t.bm * c.t.bn * 32.0 * tps / (rate * 1e12 / slots);
            double t = std::ceil((double)(tiles * s) / slots) * t_block;
            if (s > 1) t += 4e-6 + (double)batch * M * p->cout * 4.0 * (s + 1) / 4e12;
            if (t < best * 0.97) {   // prefer the earlier (larger) tile / fewer splits on near ties
                best = t;
                bt = i;
                bs = s;
            }
            if (p->force_splits > 0) break;
        }
    }
    pl.tile = bt;
    if (kX3Tiles[bt].kind >= 3) pl.kslab = 9;
    finish_plan(pl, bs);
    return pl;
}

// LDS-DMA kernels (x_split inputs): 256 x BN tiles, BN = 256 when the weight rows allow, else 128
struct GldsCfg {
    int bm, bn, wm, nst;
};
static const GldsCfg kGlds[] = {{256, 256, 2, 2}, {256, 128, 4, 3}, {512, 128, 4, 2}};

static int glds_cfg(const s2v_conv_params *p) {
    const int forced = (int)tune_value(S2V_TUNE_GLDS_TILE);   // tuning override (tools/glds_sweep.sh)
    if (forced >= 0 && forced < (int)(sizeof(kGlds) / sizeof(kGlds[0]))) {
        const GldsCfg &c = kGlds[forced];
        if ((long long)cdiv(p->cout, c.bn) * c.bn <= p->npad) return forced;
    }
    if (p->cout > 128 && (long long)cdiv(p->cout, 256) * 256 <= p->npad) return 0;
    // N <= 128: 512x128 (128x64 per wave) over 256x128 (64x64 per wave, 33 % more LDS reads per
    // MFMA): 400^2 256 -> 128 4330 vs 4648 us, 128 -> 128 2543 vs 2749 us (r02)
    const long long m = (long long)p->n * p->oh * p->ow * (p->batch > 0 ? p->batch : 1);
    return m >= 512LL * 1024 ? 2 : 1;
}

static Plan make_plan_glds(const s2v_conv_params *p, int M, Plan pl) {
    const int batch = p->batch > 0 ? p->batch : 1;
    const int cus = plan_cus();
    pl.tile = glds_cfg(p);
    const GldsCfg &c = kGlds[pl.tile];
    const long long blocks = (long long)cdiv(M, c.bm) * cdiv(p->cout, c.bn) * batch;
    int splits = p->force_splits;
    if (splits <= 0) {
        splits = 1;
        if (blocks < cus) splits = (int)((2LL * cus + blocks - 1) / blocks);
        if (splits > pl.ktiles / 8) splits = pl.ktiles / 8;
    }
    finish_plan(pl, splits);
    return pl;
}

static Plan make_plan(const s2v_conv_params *p_in, int M, int K) {
    s2v_conv_params q = *p_in;
    if (q.out_pool) q.force_splits = 1;          // the pooled epilogue needs whole-K tiles
    const s2v_conv_params *p = &q;
    Plan pl{};
    pl.ktiles = (K + 31) / 32;
    if (p->x_split) return make_plan_glds(p, M, pl);
    if (head_x3_ok(p)) {
        pl.tile = -3;
        pl.splits = p->cin > 64 ? p->cin / 64 : 1;     // 64-channel groups, folded by splitk_reduce
        pl.tps = pl.ktiles;
        return pl;
    }
    if (use_direct(p) && !p->force_tile) {
        pl.tile = -1;
        pl.splits = 1;
        pl.tps = pl.ktiles;
        if (halo_ks(p)) pl.splits = halo_splits(p, pl.tps);   // tps: channels per split
        return pl;
    }
    if (k4_ok(p)) {                                   // conv_k4_mfma (fp32 MFMA, no split-K)
        pl.tile = -4;
        pl.splits = 1;
        pl.tps = pl.ktiles;
        return pl;
    }
    int tppx, qpt;
    if (smallk_cfg(p, M, K, tppx, qpt)) {
        pl.tile = -2;
        pl.splits = 1;
        pl.tps = pl.ktiles;
        return pl;
    }
    if (tiled_x3(p)) return make_plan_x3(p, M, pl);
    const int batch = p->batch > 0 ? p->batch : 1;
    const long long target = 2LL * plan_cus();
    int cands[kNumTiles];
    int nc = 0;
    if (p->force_tile > 0) {
        cands[nc++] = p->force_tile - 1;
    } else if (p->cout <= 32) {
        cands[nc++] = 5;
    } else if (p->cout <= 64) {
        cands[nc++] = 1; cands[nc++] = 3;
    } else {
        cands[nc++] = 0; cands[nc++] = 1; cands[nc++] = 2; cands[nc++] = 3;
    }
    pl.tile = cands[nc - 1];
    long long blocks = 0;
    for (int i = 0; i < nc; ++i) {
        const TileCfg &t = kTiles[cands[i]];
        blocks = (long long)cdiv(M, t.bm) * cdiv(p->cout, t.bn) * batch;
        if (blocks >= target) {
            pl.tile = cands[i];
            break;
        }
    }
    const TileCfg &t = kTiles[pl.tile];
    blocks = (long long)cdiv(M, t.bm) * cdiv(p->cout, t.bn) * batch;
    int splits = 1;
    if (p->force_splits > 0) {
        splits = p->force_splits;
    } else if (blocks < target) {
        splits = (int)((target + blocks - 1) / blocks);
        int maxs = pl.ktiles / 8;
        if (splits > maxs) splits = maxs;
        if (splits < 1) splits = 1;
    }
    finish_plan(pl, splits);
    return pl;
}

static int validate(const s2v_conv_params *p, int &M, int &K) {
    S2V_REQUIRE(p && p->x && p->y, "conv2d: null pointer");
    {
        int e;
        S2V_REQUIRE(p->x_scale == 0.f || (p->x_scale > 0.f && std::frexp(p->x_scale, &e) == 0.5f),
                    "conv2d: x_scale must be 0 or a positive power of two, got %g", p->x_scale);
        S2V_REQUIRE(!p->x_split || p->x_scale == 0.f || p->x_scale == 1.f,
                    "conv2d: split-layout inputs carry no x_scale (split them already scaled)");
    }
    S2V_REQUIRE(!p->stamps || (p->stamp_ctr && p->stamp_reps > 0 && p->stamp_slot >= 0 &&
                               p->stamp_slot < p->stamp_stride),
                "conv2d: launch stamps need stamp_ctr, stamp_reps > 0 and 0 <= stamp_slot < stamp_stride");
    S2V_REQUIRE(p->prec == S2V_PREC_F32 || p->prec == S2V_PREC_BF16X3 || p->prec == S2V_PREC_F16X3,
                "conv2d: bad prec %d", p->prec);
    {
        int e;
        S2V_REQUIRE(p->wt_scale == 0.f || (p->wt_scale > 0.f && std::frexp(p->wt_scale, &e) == 0.5f),
                    "conv2d: wt_scale must be 0 or a positive power of two, got %g", p->wt_scale);
    }
    S2V_REQUIRE(p->force_tile >= 0 && p->force_tile <= (tiled_x3(p) ? kNumX3 : kNumTiles),
                "conv2d: bad force_tile %d", p->force_tile);
    S2V_REQUIRE(!(tiled_x3(p) && p->b_kn && p->force_tile > 0 && kX3Tiles[p->force_tile - 1].t.nw != 4),
                "conv2d: b_kn operands need a 4-wave split-bf16 tile (force_tile 4..6)");
    S2V_REQUIRE(!(tiled_x3(p) && p->force_tile > 0 && !x3_kind_ok(p, kX3Tiles[p->force_tile - 1].kind)),
                "conv2d: force_tile %d (conv_x3_nar / conv_x3_halo) needs a direct zero-padded conv, cin %% 32 == 0, "
                "<= 32 taps, no pooling, packed weights over whole 64-row slabs, 2^31-byte offsets and, with "
                "in_scale, oh * ow %% 256 == 0; conv_x3_halo also 3x3 stride 1 pad 1 (ragged images run partly empty "
                "patches), and its 8-row form oh %% 8 == 0",
                p->force_tile);
    if (tiled_x3(p) && p->force_tile > 0) {
        // a forced tile must not read weight rows past the packed [npad] rows (the planner never
        // picks such a tile: the kernels load whole BN-row slabs of B without a row guard)
        const TileCfg &t = kX3Tiles[p->force_tile - 1].t;
        S2V_REQUIRE(!p->b_kn ? (long long)cdiv(p->cout, t.bn) * t.bn <= p->npad : true,
                    "conv2d: force_tile %d (BN %d) needs npad >= %d, got %d", p->force_tile, t.bn,
                    cdiv(p->cout, t.bn) * t.bn, p->npad);
    }
    if (p->x_split) {
        S2V_REQUIRE(p->prec == S2V_PREC_BF16X3 || p->prec == S2V_PREC_F16X3, "conv2d: x_split needs prec BF16X3 / F16X3");
        S2V_REQUIRE(!p->b_kn && p->in_mode == S2V_IN_DIRECT && p->pad_mode == S2V_PAD_ZERO && p->cin % 32 == 0 &&
                        p->kh * p->kw <= 32 && !p->in_scale && p->pre_act == S2V_ACT_NONE && p->xcs % 4 == 0 &&
                        ((uintptr_t)p->x % 16) == 0 && p->x_bs % 4 == 0 && p->force_tile == 0,
                    "conv2d: x_split needs a direct zero-padded conv, cin %% 32 == 0, <= 32 taps, packed weights, "
                    "no in_scale / pre_act / force_tile, xcs %% 4 == 0 and a 16-byte aligned x");
        S2V_REQUIRE(p->wt_x3 && ((uintptr_t)p->wt_x3 % 16) == 0, "conv2d: x_split needs 16B-aligned wt_x3");
    } else if (uses_x3(p))
        S2V_REQUIRE(p->wt_x3 && ((uintptr_t)p->wt_x3 % 16) == 0, "conv2d: split precisions need 16B-aligned wt_x3");
    else
        S2V_REQUIRE(p->wt != nullptr, "conv2d: null weights");
    S2V_REQUIRE(p->n > 0 && p->h > 0 && p->w > 0 && p->cin > 0 && p->cout > 0 && p->oh > 0 && p->ow > 0,
                "conv2d: bad shape n=%d h=%d w=%d cin=%d cout=%d oh=%d ow=%d", p->n, p->h, p->w, p->cin,
                p->cout, p->oh, p->ow);
    S2V_REQUIRE(p->kh > 0 && p->kw > 0 && p->sh > 0 && p->sw > 0 && p->dh > 0 && p->dw > 0, "conv2d: bad kernel");
    S2V_REQUIRE(p->xcs >= p->cin && p->ycs >= (p->d2s_cout > 0 ? p->d2s_cout : p->cout),
                "conv2d: channel stride smaller than channels");
    S2V_REQUIRE(p->in_mode >= 0 && p->in_mode <= 2, "conv2d: bad in_mode %d", p->in_mode);
    S2V_REQUIRE(!(p->pad_mode == S2V_PAD_REFLECT && p->in_mode == S2V_IN_TRANSPOSED),
                "conv2d: reflect padding only with direct or nearest-x2 input");
    {
        const int up = p->in_mode == S2V_IN_NEAREST_UP2 ? 2 : 1;   // reflection happens in the upsampled frame
        S2V_REQUIRE(!(p->pad_mode == S2V_PAD_REFLECT && (p->ph >= up * p->h || p->pw >= up * p->w)),
                    "conv2d: reflect pad must be smaller than the input");
    }
    const long long m = (long long)p->n * p->oh * p->ow;
    const long long k = (long long)p->kh * p->kw * p->cin;
    S2V_REQUIRE(m < (1LL << 31) && k < (1LL << 31), "conv2d: problem too large");
    M = (int)m;
    K = (int)k;
    if (p->b_kn) {
        S2V_REQUIRE(p->ldb >= p->cout, "conv2d: ldb < cout");
        S2V_REQUIRE(p->ldb % 4 == 0 && ((uintptr_t)p->wt % 16) == 0, "conv2d: b_kn needs ldb%%4==0, 16B aligned");
    } else {
        S2V_REQUIRE(p->kpad >= k && p->kpad % 32 == 0, "conv2d: kpad=%d must be >= K=%lld and %%32", p->kpad, k);
        S2V_REQUIRE(p->npad >= p->cout && p->npad % 128 == 0, "conv2d: npad=%d must be >= cout and %%128", p->npad);
        S2V_REQUIRE(uses_x3(p) || ((uintptr_t)p->wt % 16) == 0, "conv2d: weights must be 16B aligned");
    }
    if (p->res) S2V_REQUIRE(p->res_cs >= p->cout, "conv2d: res_cs < cout");
    if (p->out_pool) {
        S2V_REQUIRE(p->oh % 2 == 0 && p->ow % 2 == 0, "conv2d: out_pool needs even output sizes");
        S2V_REQUIRE(!p->res && !p->nc_scale && !p->pix_add && p->out_step <= 1 && p->force_splits <= 1,
                    "conv2d: out_pool takes no res / nc_scale / pix_add / strided output / K split");
        S2V_REQUIRE(p->x_split || (!(use_direct(p) && !p->force_tile) && !is_smallk(p)),
                    "conv2d: out_pool needs the implicit-GEMM path");
    }
    if (p->post_mul || p->dup_src) {
        S2V_REQUIRE(p->out_step <= 1 && !p->out_pool && p->d2s_cout <= 0 && p->batch <= 1 && p->cout > 4,
                    "conv2d: post_mul / dup_src need a dense output (no strided / pooled / depth-to-space / batched) "
                    "and cout > 4");
        S2V_REQUIRE(!p->post_mul || (p->post_add && p->post_c0 >= 0 && p->post_c0 < p->cout &&
                                     p->post_cs >= p->cout - p->post_c0),
                    "conv2d: post_mul needs post_add, 0 <= post_c0 < cout and post_cs >= cout - post_c0");
        S2V_REQUIRE(!p->dup_src || (p->dup_cs >= p->cout && p->dup_off >= p->cout && p->dup_off + p->cout <= p->ycs),
                    "conv2d: dup_src needs dup_cs >= cout and cout <= dup_off <= ycs - cout");
    }
    if (p->d2s_cout > 0)
        S2V_REQUIRE(p->out_step == 2 && p->cout == 4 * p->d2s_cout && !p->res && !p->out_pool && !p->nc_scale,
                    "conv2d: depth-to-space output needs out_step 2, cout == 4 * d2s_cout, no res / pool / nc_scale");
    if (p->out_step > 1) {
        S2V_REQUIRE(!p->pix_add || p->d2s_cout > 0, "conv2d: strided output cannot take pix_add");
        S2V_REQUIRE(!p->res || (p->res == p->y && p->res_cs == p->ycs && p->res_oy == 0 && p->res_ox == 0),
                    "conv2d: strided output only takes an in-place residual (res == y)");
        S2V_REQUIRE(p->cout > 4 || p->x_split, "conv2d: strided output needs the implicit-GEMM path (cout > 4)");
        S2V_REQUIRE(p->out_full_h >= (p->oh - 1) * p->out_step + 1 && p->out_full_w >= (p->ow - 1) * p->out_step + 1,
                    "conv2d: strided output exceeds out_full_h/w");
    }
    return 0;
}

static ConvArgs make_args(const s2v_conv_params *p, int M, int K, const Plan &pl) {
    ConvArgs a{};
    a.x = p->x; a.n = p->n; a.h = p->h; a.w = p->w; a.cin = p->cin; a.xcs = p->xcs;
    a.in_mode = p->in_mode; a.pad_mode = p->pad_mode; a.pre_act = p->pre_act; a.pre_alpha = p->pre_alpha;
    a.in_scale = p->in_scale; a.in_scale_ns = p->in_scale_ns;
    a.kh = p->kh; a.kw = p->kw; a.sh = p->sh; a.sw = p->sw; a.ph = p->ph; a.pw = p->pw; a.dh = p->dh; a.dw = p->dw;
    a.wt = p->wt; a.kpad = p->kpad; a.cout = p->cout; a.ldb = p->ldb;
    a.y = p->y; a.oh = p->oh; a.ow = p->ow; a.ycs = p->ycs;
    Epi &e = a.epi;
    e.scale = p->scale; e.shift = p->shift; e.nc_scale = p->nc_scale; e.nc_ns = p->nc_scale_ns;
    e.pix_add = p->pix_add; e.pix_w = p->pix_w; e.res = p->res; e.res_cs = p->res_cs;
    e.res_h = p->res_h > 0 ? p->res_h : p->oh; e.res_w = p->res_w > 0 ? p->res_w : p->ow;
    e.res_oy = p->res_oy; e.res_ox = p->res_ox; e.res_after = p->res_after_act;
    e.res_simple = (e.res_h == p->oh && e.res_w == p->ow && p->res_oy == 0 && p->res_ox == 0);
    e.act = p->act; e.alpha = p->alpha;
    e.post_mul = p->post_mul; e.post_add = p->post_add; e.post_cs = p->post_cs; e.post_c0 = p->post_c0;
    e.dup_src = p->dup_src; e.dup_bias = p->dup_bias; e.dup_a = p->dup_a; e.dup_cs = p->dup_cs; e.dup_off = p->dup_off;
    a.x_bs = p->x_bs; a.w_bs = p->w_bs; a.y_bs = p->y_bs; a.res_bs = p->res_bs;
    a.M = M; a.K = K; a.ktiles = pl.ktiles; a.splits = pl.splits; a.tps = pl.tps; a.ws = p->ws;
    a.y_step = p->out_step > 1 ? p->out_step : 1; a.y_h = p->out_full_h; a.y_w = p->out_full_w;
    a.d2s_c = p->d2s_cout > 0 ? p->d2s_cout : 0;
    a.acc_scale = ((p->x_split || tiled_x3(p)) && !p->b_kn && p->wt_scale > 0.f) ? 1.f / p->wt_scale : 1.f;
    a.pool = p->out_pool != 0;
    a.stamps = p->stamps; a.stamp_ctr = p->stamp_ctr; a.stamp_slot = p->stamp_slot;
    a.stamp_stride = p->stamp_stride; a.stamp_reps = p->stamp_reps > 0 ? p->stamp_reps : 1;
    a.x_scale = 1.f;
    a.nonfinite = p->nonfinite;
    static const bool vec4_on = [] { const char *e = getenv("S2V_EPI_VEC4"); return !e || atoi(e) != 0; }();
    a.vec4 = vec4_on && epi_vec4(p) && (!p->nc_scale || (p->nc_scale_ns % 4 == 0 && ((uintptr_t)p->nc_scale % 16) == 0)) &&
             (p->d2s_cout <= 0 || p->d2s_cout % 4 == 0);
    if (tiled_x3(p) && !p->b_kn && !p->x_split && p->x_scale > 0.f && p->x_scale != 1.f) {
        a.x_scale = p->x_scale;
        a.acc_scale /= p->x_scale;
    }
    return a;
}

template <int BM, int BN, int WM>
static void launch_tile(const ConvArgs &a, int amode, bool bkn, dim3 grid, hipStream_t s) {
    switch (amode * 2 + (bkn ? 1 : 0)) {
        case 0: conv_igemm<BM, BN, WM, 0, 0><<<grid, 256, 0, s>>>(a); break;
        case 1: conv_igemm<BM, BN, WM, 0, 1><<<grid, 256, 0, s>>>(a); break;
        case 2: conv_igemm<BM, BN, WM, 1, 0><<<grid, 256, 0, s>>>(a); break;
        case 3: conv_igemm<BM, BN, WM, 1, 1><<<grid, 256, 0, s>>>(a); break;
        case 4: conv_igemm<BM, BN, WM, 2, 0><<<grid, 256, 0, s>>>(a); break;
        case 5: conv_igemm<BM, BN, WM, 2, 1><<<grid, 256, 0, s>>>(a); break;
        default: conv_igemm<BM, BN, WM, 3, 0><<<grid, 256, 0, s>>>(a); break;   // 6 (reflect, packed B)
    }
}

// 0: fast direct path, 1: generic float4 gather, 2: scalar gather
static int a_mode(const s2v_conv_params *p) {
    const bool vec = (p->cin % 4 == 0) && (p->xcs % 4 == 0) && (((uintptr_t)p->x % 16) == 0) && (p->x_bs % 4 == 0);
    if (!vec) return 2;
    const bool simple_pre = (p->pre_act == S2V_ACT_NONE || p->pre_act == S2V_ACT_RELU || p->pre_act == S2V_ACT_LRELU) &&
                            (!p->in_scale || (p->in_scale_ns % 4 == 0 && ((uintptr_t)p->in_scale % 16) == 0));
    if (p->cin % 32 == 0 && p->in_mode != S2V_IN_TRANSPOSED && simple_pre && !p->b_kn)
        return (p->pad_mode == S2V_PAD_ZERO && p->in_mode == S2V_IN_DIRECT) ? 0 : 3;
    if (p->cin % 32 == 0 && p->in_mode == S2V_IN_DIRECT && p->pad_mode == S2V_PAD_ZERO && simple_pre) return 0;
    return 1;
}

// The split-precision kernels' A-operand mode: AMODE 0 becomes 4 (buffer loads, conv_x3_impl.hpp)
// when the tile stages A wide (BM a multiple of 16 * waves), the filter has <= 32 taps and the x
// slab / packed weights fit the 2^31-byte offsets.
static long long x_extent_bytes(const s2v_conv_params *p) {
    return ((long long)p->n * p->h * p->w - 1) * p->xcs * 4 + (long long)p->cin * 4;
}

// 1x1 convs over cin % 8 == 0 (not % 32) channels take the buffer-load path too: the last 32-channel
// K-slice is partial and the lanes whose 8 channels lie past cin load zeros (r04: LNet's 48^2 st2 over
// 48 channels ran the per-row float4 gather)
static bool x3_partial_1x1(const s2v_conv_params *p) {
    return p->kh == 1 && p->kw == 1 && p->cin % 8 == 0 && p->cin % 32 != 0 && p->in_mode == S2V_IN_DIRECT &&
           p->pad_mode == S2V_PAD_ZERO && !p->b_kn && !p->x_split && a_mode(p) == 1 && p->pre_act == S2V_ACT_NONE &&
           !p->in_scale;   // (an input scale would be read past cin by the masked lanes' prologue)
}

static int x3_amode(const s2v_conv_params *p, const TileCfg &t) {
    const int am = x3_partial_1x1(p) ? 0 : a_mode(p);
    if (am != 0 || p->b_kn || p->kh * p->kw > 32 || t.bm % (16 * t.nw) != 0) return a_mode(p);
    // past the 2^31-byte buffer offsets: the gather path the conv would take without buffer loads (a_mode,
    // never AMODE 0 for a partial 1x1, which assumes whole 32-channel K-slices)
    if (x_extent_bytes(p) >= (1LL << 31) || (long long)p->npad * p->kpad * 4 >= (1LL << 31)) return a_mode(p);
    return 4;
}

// conv_x3_nar's conditions: the AMODE 4 addressing (direct zero-padded conv, whole 32-channel slices,
// <= 32 taps, 2^31-byte offsets), packed weights covering every 64-row B slab, no pooled epilogue, and
// with an input modulation every 256-row tile inside one image (its s[n, c] loads are per tile)
static bool nar_ok(const s2v_conv_params *p) {
    return tiled_x3(p) && !p->b_kn && !p->x_split && a_mode(p) == 0 && p->cin % 32 == 0 && !p->out_pool &&
           p->kh * p->kw <= 32 && x_extent_bytes(p) < (1LL << 31) && (long long)p->npad * p->kpad * 4 < (1LL << 31) &&
           (long long)cdiv(p->cout, 64) * 64 <= p->npad && (!p->in_scale || (p->oh * p->ow) % 256 == 0);
}

// conv_x3_halo's conditions (and nar_ok's addressing / weight conditions)
static bool halo_ok(const s2v_conv_params *p) {
    // the nar_ok conditions without its in_scale one (a halo patch never straddles two images)
    return tiled_x3(p) && !p->b_kn && !p->x_split && a_mode(p) == 0 && p->cin % 32 == 0 && !p->out_pool &&
           x_extent_bytes(p) < (1LL << 31) && (long long)p->npad * p->kpad * 4 < (1LL << 31) &&
           (long long)cdiv(p->cout, 64) * 64 <= p->npad && p->kh == 3 && p->kw == 3 && p->sh == 1 &&
           p->sw == 1 && p->dh == 1 && p->dw == 1 && p->ph == 1 && p->pw == 1;
}

// output pixels / patch-grid pixels of conv_x3_halo's TH x 64 patches (ragged images run part-empty patches)
static double halo_fill(const s2v_conv_params *p, int th) {
    return (double)p->oh * p->ow / ((double)cdiv(p->oh, th) * th * cdiv(p->ow, 64) * 64);
}

static bool x3_kind_ok(const s2v_conv_params *p, int kind) {
    if (kind == 4) return halo_ok(p) && p->oh % 8 == 0;
    if (kind == 5) return halo_ok(p) && (long long)cdiv(p->cout, 128) * 128 <= p->npad;
    return kind == 0 || (kind == 3 ? halo_ok(p) : nar_ok(p));
}

// Persistent blocks of a launch under s2v_conv_params.grid_cap: the 256x256 buffer-load split-precision
// tile only (conv_x3_impl.hpp x3_has_persist), when the tile grid exceeds the cap; 0 = one block per tile
static int persist_blocks(const s2v_conv_params *p, const Plan &pl, int M) {
    // (not with the SFT / second-output extras: the persistent kernel is built without them)
    if (p->grid_cap <= 0 || !tiled_x3(p) || p->b_kn || p->x_split || pl.tile != 0 || p->post_mul || p->dup_src) return 0;
    const TileCfg &t = kX3Tiles[0].t;
    if (x3_amode(p, t) != 4) return 0;
    const long long cap = p->grid_cap & ~7LL;
    const int batch = p->batch > 0 ? p->batch : 1;
    const long long tiles = (long long)cdiv(M, t.bm) * cdiv(p->cout, t.bn) * batch * pl.splits;
    return cap > 0 && tiles > cap ? (int)cap : 0;
}

// ------------------------------------------------------------------ grouped launches
// A group of independent split-precision convs (s2v_conv2d_group: LNet's FFC conv_to_l, l2g and the
// spectral branch's first 1x1, which all read the block input) as one launch on one tile
// configuration, each member with its own split-K factor, plus one launch folding every member's
// partials.  Plan: minimise  rounds * (T0 + max_p tps_p * t_slice) + [reduce]  over the grouped tiles
// and per-member splits in {1, 2, 4, 8, 16}, where t_slice = max(the tile's per-slice latency floor,
// its share of the full-chip rate) — the latency floor is what one block alone on a CU takes per
// 32-deep K slice (measured on MI355X r04, graph-timed: 0.5 us for the 4-wave tiles).
struct GroupPlan {
    int cfg;
    int splits[kConvGroupMax];
    Plan plan[kConvGroupMax];
    int M[kConvGroupMax];
};

static bool group_member_ok(const s2v_conv_params *p, int cfg) {
    return tiled_x3(p) && !p->b_kn && !p->x_split && p->grid_cap == 0 && p->force_tile == 0 && !p->out_pool &&
           (p->batch <= 1) && x3_amode(p, kX3Tiles[cfg].t) == 4 && !p->in_scale && p->pre_act == S2V_ACT_NONE &&
           !p->post_mul && !p->dup_src;       // the grouped kernel is built without the epilogue extras
}

static int group_plan(const s2v_conv_params *ps, int n, GroupPlan &gp) {
    S2V_REQUIRE(ps && n >= 1 && n <= kConvGroupMax, "conv2d_group: 1..%d members", kConvGroupMax);
    int K[kConvGroupMax];
    for (int i = 0; i < n; ++i) {
        const int rc = validate(&ps[i], gp.M[i], K[i]);
        if (rc) return rc;
        S2V_REQUIRE(ps[i].prec == ps[0].prec, "conv2d_group: members of one precision");
    }
    // candidate tiles (kX3Tiles indices; S2V_GROUP_TILES overrides, e.g. "0,6,4,3,1")
    static const std::vector<int> cands = [] {
        std::vector<int> v;
        const char *e = getenv("S2V_GROUP_TILES");
        if (e && *e) {
            for (const char *q = e; *q;) {
                const int t = atoi(q);
                if (t == 0 || t == 1 || t == 3 || t == 4 || t == 6) v.push_back(t);
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
        }
        if (v.empty()) v = {4, 3, 1};
        return v;
    }();
    const int cus = plan_cus();
    double best = 1e30;
    gp.cfg = -1;
    for (int cfg : cands) {
        bool ok = true;
        for (int i = 0; i < n && ok; ++i) ok = group_member_ok(&ps[i], cfg) &&
                                              (long long)cdiv(ps[i].cout, kX3Tiles[cfg].t.bn) * kX3Tiles[cfg].t.bn <= ps[i].npad;
        if (!ok) continue;
        const X3Cfg &c = kX3Tiles[cfg];
        const double lat = c.t.nw == 4 ? 0.5e-6 : 0.6e-6;
        const double slots = (double)cus * c.bpc;
        int s[kConvGroupMax] = {1, 1, 1, 1};
        long long tiles[kConvGroupMax];
        for (int i = 0; i < n; ++i) tiles[i] = (long long)cdiv(gp.M[i], c.t.bm) * cdiv(ps[i].cout, c.t.bn);
        int combos = 1;
        for (int i = 0; i < n; ++i) combos *= 5;
        for (int cb = 0; cb < combos; ++cb) {
            int v = cb;
            long long blocks = 0;
            int maxtps = 0;
            double red = 0.0;
            bool any_split = false, bad = false;
            for (int i = 0; i < n; ++i) {
                s[i] = 1 << (v % 5);
                v /= 5;
                const int kt = (K[i] + 31) / 32;
                if (s[i] > 1 && s[i] > kt / 4) { bad = true; break; }
                const int tps = (kt + s[i] - 1) / s[i];
                blocks += tiles[i] * s[i];
                maxtps = tps > maxtps ? tps : maxtps;
                if (s[i] > 1) {
                    any_split = true;
                    red += (double)gp.M[i] * ps[i].cout * 4.0 * (s[i] + 1) / 4e12;
                }
            }
            if (bad) continue;
            const double conc = blocks < slots ? (double)blocks : slots;
            const double thr = 2.0 * c.t.bm * c.t.bn * 32.0 / (c.tflops * 1e12 / (conc > cus ? conc : cus));
            const double rounds = std::ceil((double)blocks / slots);
            double t = rounds * (2e-6 + maxtps * (thr > lat ? thr : lat));
            if (any_split) t += 7e-6 + red;
            if (t < best * 0.97) {
                best = t;
                gp.cfg = cfg;
                for (int i = 0; i < n; ++i) gp.splits[i] = s[i];
            }
        }
    }
    S2V_REQUIRE(gp.cfg >= 0, "conv2d_group: members need the split-precision buffer-load path (direct zero-padded "
                "conv, cin %% 32 == 0, <= 32 taps, no in_scale / pre_act / pool / grid_cap / force_tile / post / dup, batch 1)");
    for (int i = 0; i < n; ++i) {
        Plan &pl = gp.plan[i];
        pl.tile = gp.cfg;
        pl.ktiles = (K[i] + 31) / 32;
        finish_plan(pl, gp.splits[i]);
        gp.splits[i] = pl.splits;
    }
    return 0;
}

static size_t group_ws_bytes(const s2v_conv_params *ps, int n, const GroupPlan &gp) {
    size_t b = 0;
    for (int i = 0; i < n; ++i)
        if (gp.plan[i].splits > 1) b += ((size_t)gp.plan[i].splits * gp.M[i] * ps[i].cout * sizeof(float) + 255) / 256 * 256;
    return b;
}

}  // namespace s2v

using namespace s2v;

extern "C" size_t s2v_conv2d_group_ws_bytes(const s2v_conv_params *ps, int n) {
    GroupPlan gp;
    if (group_plan(ps, n, gp)) return 0;
    return group_ws_bytes(ps, n, gp);
}

extern "C" int s2v_conv2d_group_plan(const s2v_conv_params *ps, int n, int *out) {
    GroupPlan gp;
    const int rc = group_plan(ps, n, gp);
    if (rc) return rc;
    out[0] = gp.cfg;
    for (int i = 0; i < n; ++i) out[1 + i] = gp.plan[i].splits;
    return 0;
}

extern "C" int s2v_conv2d_group(const s2v_conv_params *ps, int n, s2v_stream_t stream) {
    GroupPlan gp;
    int rc = group_plan(ps, n, gp);
    if (rc) return rc;
    const size_t need = group_ws_bytes(ps, n, gp);
    if (need && (!ps[0].ws || ps[0].ws_bytes < need)) {
        set_error("conv2d_group: split-K workspace of %zu bytes required in member 0 (have %zu)", need, ps[0].ws_bytes);
        return S2V_E_WORKSPACE;
    }
    ConvGroup g{};
    g.n = n;
    const TileCfg &t = kX3Tiles[gp.cfg].t;
    long long blocks = 0, rblocks = 0;
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        const s2v_conv_params *p = &ps[i];
        ConvArgs &a = g.a[i];
        a = make_args(p, gp.M[i], p->kh * p->kw * p->cin, gp.plan[i]);
        a.wt = (const float *)p->wt_x3;
        a.x_bytes = (unsigned)x_extent_bytes(p);
        a.w_bytes = (unsigned)((long long)p->npad * p->kpad * 4);
        a.stamps = nullptr;
        if (gp.plan[i].splits > 1) {
            a.ws = (float *)((char *)ps[0].ws + off);
            off += ((size_t)gp.plan[i].splits * gp.M[i] * p->cout * sizeof(float) + 255) / 256 * 256;
        }
        g.gx[i] = (int)cdiv(gp.M[i], t.bm);
        g.gy[i] = (int)cdiv(p->cout, t.bn);
        g.start[i] = (int)blocks;
        blocks += (long long)g.gx[i] * g.gy[i] * gp.plan[i].splits;
        g.rstart[i] = (int)rblocks;
        if (gp.plan[i].splits > 1) {
            long long items = (long long)gp.M[i] * (p->cout % 4 == 0 ? p->cout / 4 : p->cout);
            long long rb = (items + 255) / 256;
            if (rb > 1024) rb = 1024;
            rblocks += rb;
        }
        g.vec[i] = epi_vec4(p);
    }
    for (int i = n; i <= kConvGroupMax; ++i) {
        g.start[i] = (int)blocks;
        g.rstart[i] = (int)rblocks;
    }
    S2V_REQUIRE(blocks < (1LL << 31), "conv2d_group: too many tiles");
    hipStream_t s = (hipStream_t)stream;
    rc = ps[0].prec == S2V_PREC_BF16X3 ? launch_conv_x3_group<0>(gp.cfg, g, dim3((unsigned)blocks), s)
                                       : launch_conv_x3_group<1>(gp.cfg, g, dim3((unsigned)blocks), s);
    if (rc) return rc;
    rc = check_launch("conv2d_group");
    if (rc || rblocks == 0) return rc;
    splitk_reduce_group<<<(unsigned)rblocks, 256, 0, s>>>(g);
    return check_launch("splitk_reduce_group");
}

extern "C" int s2v_tune(int key, long long value, long long *old_value) {
    S2V_REQUIRE(key >= 0 && key < S2V_TUNE_COUNT, "tune: bad key %d", key);
    const long long prev = tune_value(key);
    if (old_value) *old_value = prev;
    g_tune[key] = value;
    return 0;
}

extern "C" size_t s2v_conv2d_ws_bytes(const s2v_conv_params *p) {
    int M, K;
    if (validate(p, M, K) != 0) return 0;
    Plan pl = make_plan(p, M, K);
    if (pl.splits <= 1 || pl.tile == -2 || pl.tile == -4) return 0;
    const int batch = p->batch > 0 ? p->batch : 1;
    return (size_t)batch * pl.splits * (size_t)M * p->cout * sizeof(float);
}

extern "C" int s2v_conv2d_plan(const s2v_conv_params *p, int *out6) {
    for (int i = 6; i < 11; ++i) out6[i] = 0;
    int M, K;
    int rc = validate(p, M, K);
    if (rc) return rc;
    Plan pl = make_plan(p, M, K);
    if (p->x_split) {                                   // conv_glds_x3<BM, BN, WM, NST, prec-1>
        const GldsCfg &c = kGlds[pl.tile];
        out6[0] = c.bm; out6[1] = c.bn; out6[2] = c.wm; out6[3] = 5; out6[4] = 0; out6[5] = pl.splits;
        out6[6] = p->prec; out6[7] = 8; out6[8] = c.nst; out6[9] = 0;
        return 0;
    }
    if (pl.tile == -4) {                                // conv_k4_mfma<KT> (reported as 4000 + KT)
        out6[0] = 0; out6[1] = p->cout; out6[2] = 0; out6[3] = 0;
        out6[4] = 4000 + p->kh * p->kw; out6[5] = 1;
        return 0;
    }
    if (pl.tile == -2) {
        int tppx, qpt;
        smallk_cfg(p, M, K, tppx, qpt);
        out6[0] = 0; out6[1] = p->cout; out6[2] = -qpt;
        out6[3] = smallk_px(M); out6[5] = 1;
        // conv_smallk4<QPT, KT> for 4-channel 1x1 / 3x3 inputs (reported as 2000 + KT)
        out6[4] = p->cin == 4 && p->kh == p->kw && (p->kh == 1 || p->kh == 3) ? 2000 + p->kh * p->kw : 0;
        return 0;
    }
    if (pl.tile == -3) {                                // conv_head_x3<prec - 1, CO, KS, cin / 32>
        out6[0] = 0; out6[1] = p->cout; out6[2] = p->cin == 32 ? 1 : 2; out6[3] = 0;
        out6[4] = 3000 + p->kh; out6[5] = pl.splits; out6[6] = p->prec;
        return 0;
    }
    if (pl.tile < 0 && halo_ks(p)) {
        out6[0] = 0; out6[1] = p->cout < 4 ? p->cout : 4;
        out6[2] = 0; out6[3] = 0;
        out6[4] = 1000 + halo_ks(p); out6[5] = pl.splits;  // conv_halo_small<CO, KS>
        return 0;
    }
    if (pl.tile < 0) {
        const bool cpar = (p->cin % 4 == 0) && (p->xcs % 4 == 0) && (((uintptr_t)p->x % 16) == 0) &&
                          (p->x_bs % 4 == 0) && (!p->in_scale || (p->in_scale_ns % 4 == 0 &&
                                                                  ((uintptr_t)p->in_scale % 16) == 0));
        const int co = p->cout < 4 ? p->cout : 4, tpp = cpar_lanes(p->cin);
        const int batch = p->batch > 0 ? p->batch : 1;
        out6[0] = 0; out6[1] = co;
        out6[2] = !cpar ? 0 : tpp;
        out6[3] = cpar && cpar_lw(co, K, p->w_bs, batch, M, tpp);
        out6[4] = 0; out6[5] = 1;
        return 0;
    }
    const TileCfg &t = tile_cfg(p, pl.tile);
    out6[0] = t.bm; out6[1] = t.bn; out6[2] = t.wm;
    out6[3] = tiled_x3(p) ? (kX3Tiles[pl.tile].kind >= 1 ? 5 + kX3Tiles[pl.tile].kind : x3_amode(p, t)) : a_mode(p);
    if (tiled_x3(p) && kX3Tiles[pl.tile].kind >= 4) out6[3] = 8;   // conv_x3_halo<ELT, TH, WN>: bm / bn tell them apart
    out6[4] = p->b_kn != 0;
    out6[5] = pl.splits;
    out6[6] = tiled_x3(p) ? p->prec : 0;
    out6[7] = t.nw; out6[8] = t.ks; out6[9] = t.pf;
    out6[10] = persist_blocks(p, pl, M);
    return 0;
}

extern "C" int s2v_conv2d(const s2v_conv_params *p, s2v_stream_t stream) {
    int M, K;
    int rc = validate(p, M, K);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int batch = p->batch > 0 ? p->batch : 1;
    Plan pl = make_plan(p, M, K);
    ConvArgs a = make_args(p, M, K, pl);
    if (pl.tile == -4) {
        rc = launch_conv_k4(a, batch, p->kh * p->kw, s);
        if (rc) return rc;
        return check_launch("conv_k4");
    }
    if (pl.tile == -2) {
        int tppx, qpt;
        smallk_cfg(p, M, K, tppx, qpt);
        const int iters = smallk_iters(p, M, tppx);
        const int px = smallk_px(M);
        const long long groups = (long long)batch * M / px;
        const unsigned grid = cdiv(groups, (256 / tppx) * iters);
        const size_t lds = (size_t)K * p->cout * sizeof(float);
        const int vec = epi_vec4(p);
        const int kt = p->cin == 4 && p->kh == p->kw && (p->kh == 1 || p->kh == 3) ? p->kh * p->kw : 0;
        if (kt == 9 && qpt == 1) conv_smallk4<1, 9><<<grid, 256, lds, s>>>(a, batch, tppx, iters, vec);
        else if (kt == 9) conv_smallk4<2, 9><<<grid, 256, lds, s>>>(a, batch, tppx, iters, vec);
        else if (kt == 1 && qpt == 1) conv_smallk4<1, 1><<<grid, 256, lds, s>>>(a, batch, tppx, iters, vec);
        else if (kt == 1) conv_smallk4<2, 1><<<grid, 256, lds, s>>>(a, batch, tppx, iters, vec);
        else if (qpt == 1) conv_smallk<1, 1><<<grid, 256, lds, s>>>(a, batch, tppx, iters, vec);
        else conv_smallk<2, 1><<<grid, 256, lds, s>>>(a, batch, tppx, iters, vec);
        return check_launch("conv_smallk");
    }
    if (pl.tile == -3) {
        a.wt = (const float *)p->wt_x3;
        a.acc_scale = p->wt_scale > 0.f ? 1.f / p->wt_scale : 1.f;
        if (p->x_scale > 0.f && p->x_scale != 1.f) {
            a.x_scale = p->x_scale;
            a.acc_scale /= p->x_scale;
        }
        if (pl.splits > 1) {
            const size_t need = (size_t)pl.splits * (size_t)M * p->cout * sizeof(float);
            if (!p->ws || p->ws_bytes < need) {
                set_error("conv2d: split workspace of %zu bytes required (have %zu)", need, p->ws_bytes);
                return S2V_E_WORKSPACE;
            }
        }
        rc = launch_conv_head_x3(a, p->prec, p->cout, p->kh, p->cin == 32 ? 1 : 2, head_rows(p), s);
        if (rc) return rc;
        rc = check_launch("conv_head_x3");
        if (rc || pl.splits <= 1) return rc;
        splitk_reduce<<<cdiv((long long)M * p->cout, 256), 256, 0, s>>>(a, 1, epi_vec4(p));
        return check_launch("splitk_reduce");
    }
    if (pl.tile < 0 && halo_ks(p)) {
        if (pl.splits > 1) {
            const size_t need = (size_t)pl.splits * (size_t)M * p->cout * sizeof(float);
            if (!p->ws || p->ws_bytes < need) {
                set_error("conv2d: split workspace of %zu bytes required (have %zu)", need, p->ws_bytes);
                return S2V_E_WORKSPACE;
            }
        }
        switch (p->cout) {
            case 1: launch_halo<1>(a, halo_ks(p), s); break;
            case 2: launch_halo<2>(a, halo_ks(p), s); break;
            case 3: launch_halo<3>(a, halo_ks(p), s); break;
            default: launch_halo<4>(a, halo_ks(p), s); break;
        }
        rc = check_launch("conv_halo_small");
        if (rc || pl.splits <= 1) return rc;
        splitk_reduce<<<cdiv((long long)M * p->cout, 256), 256, 0, s>>>(a, 1, epi_vec4(p));
        return check_launch("splitk_reduce");
    }
    if (pl.tile < 0) {
        const bool cpar = (p->cin % 4 == 0) && (p->xcs % 4 == 0) && (((uintptr_t)p->x % 16) == 0) &&
                          (p->x_bs % 4 == 0) && (!p->in_scale || (p->in_scale_ns % 4 == 0 &&
                                                                  ((uintptr_t)p->in_scale % 16) == 0));
        S2V_REQUIRE(cpar || p->w_bs == 0 || batch == 1 || M % 256 == 0,
                    "conv2d: per-batch weights on the LDS-staged small-Cout path need M %% 256 == 0");
        switch (p->cout) {
            case 1: launch_small<1>(a, batch, cpar, s); break;
            case 2: launch_small<2>(a, batch, cpar, s); break;
            case 3: launch_small<3>(a, batch, cpar, s); break;
            default: launch_small<4>(a, batch, cpar, s); break;
        }
        return check_launch("conv_small");
    }
    if (pl.splits > 1) {
        const size_t need = (size_t)batch * pl.splits * (size_t)M * p->cout * sizeof(float);
        if (!p->ws || p->ws_bytes < need) {
            set_error("conv2d: split-K workspace of %zu bytes required (have %zu)", need, p->ws_bytes);
            return S2V_E_WORKSPACE;
        }
    }
    if (p->x_split) {
        const GldsCfg &c = kGlds[pl.tile];
        dim3 grid(cdiv(M, c.bm), cdiv(p->cout, c.bn), batch * pl.splits);
        a.wt = (const float *)p->wt_x3;
        if (p->prec == S2V_PREC_BF16X3) launch_conv_glds<0>(pl.tile, a, grid, s);
        else launch_conv_glds<1>(pl.tile, a, grid, s);
    } else {
    const int amode = a_mode(p);
    const bool bkn = p->b_kn != 0;
    const TileCfg &t = tile_cfg(p, pl.tile);
    dim3 grid(cdiv(M, t.bm), cdiv(p->cout, t.bn), batch * pl.splits);
    if (tiled_x3(p) && kX3Tiles[pl.tile].kind >= 3) {   // conv_x3_halo: one block per (image, patch)
        const int th = kX3Tiles[pl.tile].kind == 4 ? 8 : 4;
        grid.x = (unsigned)((long long)p->n * cdiv(p->oh, th) * cdiv(p->ow, 64));
    }
    if (tiled_x3(p)) {
        if (!bkn) a.wt = (const float *)p->wt_x3;
        if (kX3Tiles[pl.tile].kind >= 1) {         // conv_x3_nar / _halo (conditions: planner / validate)
            a.x_bytes = (unsigned)x_extent_bytes(p);
            a.w_bytes = (unsigned)((long long)p->npad * p->kpad * 4);
            const int kind = kX3Tiles[pl.tile].kind;
            if (kind >= 3)
                rc = p->prec == S2V_PREC_BF16X3
                         ? launch_conv_x3_halo<0>(a, kind == 4 ? 8 : 4, kind == 5 ? 2 : 1, grid, s)
                         : launch_conv_x3_halo<1>(a, kind == 4 ? 8 : 4, kind == 5 ? 2 : 1, grid, s);
            else
                rc = p->prec == S2V_PREC_BF16X3 ? launch_conv_x3_nar<0>(a, kind == 2, grid, s)
                                                : launch_conv_x3_nar<1>(a, kind == 2, grid, s);
        } else {
        const int am = x3_amode(p, t);
        if (am == 4) {
            a.x_bytes = (unsigned)x_extent_bytes(p);
            a.w_bytes = (unsigned)((long long)p->npad * p->kpad * 4);
        }
        const int cap = persist_blocks(p, pl, M);
        if (cap > 0) {                              // persistent blocks over the tile grid (s2v.h grid_cap)
            a.vgrid_x = (int)grid.x;
            a.vgrid_y = (int)grid.y;
            a.vgrid_z = (int)grid.z;
            grid = dim3((unsigned)cap, 1, 1);
        }
        rc = p->prec == S2V_PREC_BF16X3 ? launch_conv_x3<0>(pl.tile, a, am, bkn, grid, s)
                                        : launch_conv_x3<1>(pl.tile, a, am, bkn, grid, s);
        }
        if (rc) return rc;
    } else switch (pl.tile) {
        case 0: launch_tile<128, 128, 2>(a, amode, bkn, grid, s); break;
        case 1: launch_tile<128, 64, 2>(a, amode, bkn, grid, s); break;
        case 2: launch_tile<64, 128, 2>(a, amode, bkn, grid, s); break;
        case 3: launch_tile<64, 64, 2>(a, amode, bkn, grid, s); break;
        case 4: launch_tile<256, 32, 4>(a, amode, bkn, grid, s); break;
        default: launch_tile<128, 32, 4>(a, amode, bkn, grid, s); break;
    }
    }
    rc = check_launch("conv_igemm");
    if (rc || pl.splits <= 1) return rc;
    const long long total = (long long)batch * M * (p->cout % 4 == 0 ? p->cout / 4 : p->cout);
    unsigned blocks = cdiv(total, 256);
    if (blocks > 65535u * 4u) blocks = 65535u * 4u;
    splitk_reduce<<<blocks, 256, 0, s>>>(a, batch, epi_vec4(p));
    return check_launch("splitk_reduce");
}
