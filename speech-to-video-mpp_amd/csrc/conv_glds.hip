// Split-fp32 implicit-GEMM convolution with both operands staged by LDS-DMA (global_load_lds).
//
// The x3 kernels (conv_x3_impl.hpp) split the fp32 activations into 16-bit halves after their
// global load, in registers, then write them to LDS: per 32-deep K-slice a thread spends ~30 VALU
// and 8 ds_write_b128 on the A tile, and holds the staged slice in ~32 VGPRs.  When the producer
// writes its activation already split — the "split" layout, same bytes and pitch as the fp32
// tensor: per pixel and 32-channel block, 32 hi halves (64 B) then 32 lo halves (64 B), exactly
// the 128-byte LDS row of a K-slice — both operands can go global -> LDS without touching a
// register: one global_load_lds_dwordx4 per 8 tile rows and thread, the row swizzle applied on the
// source address (the LDS image is lane-linear; cdna_hip_programming.md §5.4 rule 21).
//
// Pipeline: NST LDS stages (2 for 256x256 tiles, 3 for 256x128), slices issued NST-1 ahead, a
// counted `s_waitcnt vmcnt` (never 0 inside the loop with 3 stages) and a raw s_barrier per slice
// (a __syncthreads() would drain the DMA queue: "Pipelining across barriers").
// Out-of-image filter taps and rows past M read a 256-byte zero line (the DMA writes zeros).
// Same GEMM view, K-slice order, XCD-aware tile order, 16x16x32 fragment reads and epilogue as the
// x3 kernels; only AMODE-0 convolutions (direct, zero padding, cin % 32 == 0, no prologue).
#include "conv_x3_impl.hpp"

namespace s2v {

__device__ __attribute__((aligned(256))) char g_zero_line[256];

// timing ablations (never in the shipped build): 1 = no DMA inside the loop, 2 = no wait / barrier,
// 3 = neither — results are wrong, only the loop's cost without that piece is measured
#ifndef GLDS_ABL
#define GLDS_ABL 0
#endif

typedef const __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

__device__ __forceinline__ void glds16(const char *src, char *lds_wave_base) {
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_wave_base, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else static_assert(N < 0, "wait_vm: add the count");
}

template <int BM, int BN, int WAVES_M, int NST, int ELT>
__global__ __launch_bounds__(512, 1) void conv_glds_x3(ConvArgs a) {
    constexpr int NW = 8;
    constexpr int WAVES_N = NW / WAVES_M;
    constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    constexpr int TM16 = WTM / 16, TN16 = WTN / 16;
    constexpr int RP = 8 * NW;                      // tile rows per DMA pass (8 rows of 128 B per wave)
    constexpr int AP = BM / RP, BP = BN / RP;       // DMA passes per slice
    constexpr int G = AP + BP;                      // DMA instructions per slice and thread
    constexpr int SUB = (BM + BN) * 128;
    constexpr int OPS = NST * SUB;
    constexpr int CH = x3_chunk(BM, BN, OPS > 65536 ? OPS : 65536);
    constexpr int CBYTES = CH * (BN + 4) * 4;
    constexpr int SMEM = OPS > CBYTES ? OPS : CBYTES;
    static_assert(BM % RP == 0 && BN % RP == 0 && WTM % 16 == 0 && WTN % 16 == 0, "tile");
    static_assert(SMEM <= 160 * 1024, "LDS");
    static_assert(NST == 2 || NST == 3, "stages");

    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    launch_stamp(a, false);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    int mt, nt, bz;
    {   // XCD-aware tile order (see conv.hip)
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
    const char *__restrict__ xb = (const char *)(a.x + (long long)bidx * a.x_bs);
    const char *__restrict__ wb = (const char *)(a.wt + (long long)bidx * a.w_bs);
    const int kt0 = split * a.tps;
    const int kt1 = min(a.ktiles, kt0 + a.tps);
    const int taps = a.kh * a.kw, nsl = a.cin >> 5;
    const bool kperm = taps > 1;

    // DMA geometry: in pass j a wave fills rows j*RP + wave*8 .. +7 (1 KB, lane-linear); lane l
    // writes position l & 7 of row (l >> 3), which holds slot (l & 7) ^ swz(row) of the data
    const int prow = wave * 8 + (lane >> 3);
    const int sbyte = (((lane & 7) ^ swz(prow)) << 4);   // swz depends on row bits 1..3 only: same for every pass
    ARows<AP, 0> R;
    {
        int rows[AP];
#pragma unroll
        for (int j = 0; j < AP; ++j) rows[j] = j * RP + prow;
        a_rows_init_at<AP, 0>(a, m0, rows, R);
    }
    const char *arow[AP];
    unsigned tmask[AP];
#pragma unroll
    for (int j = 0; j < AP; ++j) {
        arow[j] = xb + R.base[j] * 4 + sbyte;
        unsigned m = 0;
        if (R.ok[j])
            for (int ky = 0; ky < a.kh; ++ky)
                for (int kx = 0; kx < a.kw; ++kx)
                    if ((unsigned)(R.iy0[j] + ky * a.dh) < (unsigned)a.h && (unsigned)(R.ix0[j] + kx * a.dw) < (unsigned)a.w)
                        m |= 1u << (ky * a.kw + kx);
        tmask[j] = m;
    }
    const char *zline = g_zero_line + sbyte;
    const char *brow = wb + (long long)(n0 + prow) * a.kpad * 4 + sbyte;
    const long long bpass = (long long)RP * a.kpad * 4;

    SliceIt ld;
    ld.init(kt0, kperm, taps, nsl, a.kw);
    auto issue = [&](int buf) {
        char *st = smem + buf * SUB + wave * 8 * 128;
        const long long toff = ((long long)(ld.ky * a.dh * a.w + ld.kx * a.dw) * a.xcs + ld.cs * 32) * 4;
#pragma unroll
        for (int j = 0; j < AP; ++j) {
            const char *src = ((tmask[j] >> ld.tap) & 1u) ? arow[j] + toff : zline;
            glds16(src, st + j * RP * 128);
        }
        const char *bs = brow + (long long)ld.kt(nsl) * 128;
#pragma unroll
        for (int j = 0; j < BP; ++j) glds16(bs + j * bpass, st + BM * 128 + j * RP * 128);
        if (ld.i < kt1 - 1) ld.next(kperm, taps, nsl, a.kw);
    };

    floatx4 acc4[TM16][TN16];
#pragma unroll
    for (int i = 0; i < TM16; ++i)
#pragma unroll
        for (int j = 0; j < TN16; ++j) acc4[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int l16 = lane & 15;
    const int hs16 = ((lane >> 4) ^ swz(l16)) << 4, ls16 = hs16 ^ 64;
    auto compute = [&](const char *As) {
        const char *Bs = As + BM * 128;
        u32x4 bh[TN16], bl[TN16];
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
            const char *p = Bs + (wn * WTN + j * 16 + l16) * 128;
            bh[j] = *(const u32x4 *)(p + hs16);
            bl[j] = *(const u32x4 *)(p + ls16);
        }
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const char *p = As + (wm * WTM + i * 16 + l16) * 128;
            const u32x4 ah = *(const u32x4 *)(p + hs16);
            const u32x4 al = *(const u32x4 *)(p + ls16);
#pragma unroll
            for (int j = 0; j < TN16; ++j) {
                acc4[i][j] = mfma16x16<ELT>(al, bh[j], acc4[i][j]);
                acc4[i][j] = mfma16x16<ELT>(ah, bl[j], acc4[i][j]);
                acc4[i][j] = mfma16x16<ELT>(ah, bh[j], acc4[i][j]);
            }
        }
    };

    const int n = kt1 - kt0;
    if (n > 0) {
        // prologue: slices 0 .. NST-2 in flight
#pragma unroll
        for (int s = 0; s < NST - 1; ++s)
            if (s < n) issue(s);
        int cbuf = 0;                // stage of slice t
        int ibuf = NST - 1;          // stage slice t + NST - 1 goes to
        for (int t = 0; t < n; ++t) {
            // slice t landed (this thread's DMAs; slices t+1 .. t+NST-2 may stay in flight), then
            // every wave's: the barrier also retires all reads of the stage reissued below
#if GLDS_ABL != 2 && GLDS_ABL != 3
            if constexpr (NST == 3) {
                if (t + 1 < n) wait_vm<G>();
                else wait_vm<0>();
            } else {
                wait_vm<0>();
            }
            __builtin_amdgcn_s_barrier();
#endif
            __builtin_amdgcn_sched_barrier(0);
#if GLDS_ABL != 1 && GLDS_ABL != 3
            if (t + NST - 1 < n) issue(ibuf);
#endif
            compute(smem + cbuf * SUB);
            cbuf = cbuf == NST - 1 ? 0 : cbuf + 1;
            ibuf = ibuf == NST - 1 ? 0 : ibuf + 1;
        }
    }
    // epilogue (its first __syncthreads() orders the last slice's reads before the C staging)
    epilogue_tile_fn<BM, BN, NW, CH>(a, (float *)smem, tid, m0, n0, bz, bidx, [&](float *Cs, int c0) {
        constexpr int LDC = BN + 4;
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const int r0 = wm * WTM + i * 16 - c0;
            if (r0 < 0 || r0 >= CH) continue;
#pragma unroll
            for (int j = 0; j < TN16; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cs[(r0 + 4 * (lane >> 4) + r) * LDC + wn * WTN + j * 16 + l16] = acc4[i][j][r] * a.acc_scale;
        }
    });    launch_stamp(a, true);
}

// fp32 NHWC [pixels][xcs] -> split layout (same pitch): per 32-channel block 32 hi halves then 32 lo
template <int ELT>
__global__ __launch_bounds__(256) void split_act_kernel(const float *__restrict__ x, long long pixels, int c, int xcs,
                                                        char *__restrict__ out, int ocs) {
    const int q4 = c >> 2;
    const long long total = pixels * q4;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long p = e / q4;
        const int ch = (int)(e - p * q4) * 4;
        const f4 v = *(const f4 *)(x + p * xcs + ch);
        u32x2 hi, lo;
        split4<ELT>(v, hi, lo);
        char *o = out + (p * ocs + (ch & ~31)) * 4 + (ch & 31) * 2;
        *(u32x2 *)o = hi;
        *(u32x2 *)(o + 64) = lo;
    }
}

// glds configurations (conv.hip kGlds): 0 = 256x256 (2 stages), 1 = 256x128 (3 stages),
// 2 = 512x128 (2 stages, 128x64 per wave).  Measured and dropped (r02, tools/glds_sweep.sh): s_setprio
// for the younger half / around the MFMA clusters (+-1 %), 4-wave blocks with 128x128 wave tiles
// (-11 % at 256x256, -11 % at 512x128).
template <int ELT>
void launch_conv_glds(int cfg, const ConvArgs &a, dim3 grid, hipStream_t s) {
    switch (cfg) {
        case 0: conv_glds_x3<256, 256, 2, 2, ELT><<<grid, 512, 0, s>>>(a); break;
        case 1: conv_glds_x3<256, 128, 4, 3, ELT><<<grid, 512, 0, s>>>(a); break;
        default: conv_glds_x3<512, 128, 4, 2, ELT><<<grid, 512, 0, s>>>(a); break;
    }
}
template void launch_conv_glds<0>(int, const ConvArgs &, dim3, hipStream_t);
template void launch_conv_glds<1>(int, const ConvArgs &, dim3, hipStream_t);

}  // namespace s2v

using namespace s2v;

extern "C" int s2v_split_act(const float *x, long long pixels, int c, int xcs, int prec, float *out, int ocs,
                             s2v_stream_t stream) {
    S2V_REQUIRE(x && out && pixels > 0 && c > 0 && c % 32 == 0 && xcs >= c && ocs >= c && xcs % 4 == 0 &&
                    ocs % 32 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 128) == 0,
                "split_act: C %% 32, pitches (ocs %% 32) and alignment (x 16 B, out 128 B) required");
    S2V_REQUIRE(prec == S2V_PREC_BF16X3 || prec == S2V_PREC_F16X3, "split_act: prec must be BF16X3 or F16X3");
    S2V_REQUIRE((const void *)x != (const void *)out, "split_act: not in place");
    const long long total = pixels * (c / 4);
    long long b = (total + 255) / 256;
    if (b > 65535LL * 16) b = 65535LL * 16;
    if (prec == S2V_PREC_BF16X3)
        split_act_kernel<0><<<(unsigned)b, 256, 0, (hipStream_t)stream>>>(x, pixels, c, xcs, (char *)out, ocs);
    else
        split_act_kernel<1><<<(unsigned)b, 256, 0, (hipStream_t)stream>>>(x, pixels, c, xcs, (char *)out, ocs);
    return check_launch("split_act");
}

// Both f16 split variants of conv_x3_impl.hpp (X3_F16_MIX 1: v_fma_mix residuals; 0: widen + subtract +
// pack) on the same inputs: counts the float4s whose hi or lo halves differ (a self-check of the variant
// the library is not built with; they must be bit-identical).
__global__ __launch_bounds__(256) void f16_split_check_kernel(const float *__restrict__ x, long long n4,
                                                              int *__restrict__ mismatch) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const f4 v = ((const f4 *)x)[i];
        u32x2 h1, l1, h0, l0;
        split4<1, 1>(v, h1, l1);
        split4<1, 0>(v, h0, l0);
        if (h1.x != h0.x || h1.y != h0.y || l1.x != l0.x || l1.y != l0.y) atomicAdd(mismatch, 1);
    }
}

extern "C" int s2v_f16_split_check(const float *x, long long n, int *mismatch, s2v_stream_t stream) {
    S2V_REQUIRE(x && mismatch && n > 0 && n % 4 == 0 && ((uintptr_t)x % 16) == 0,
                "f16_split_check: n %% 4 == 0 floats, 16-byte aligned");
    const long long n4 = n / 4;
    const unsigned grid = (unsigned)std::min<long long>((n4 + 255) / 256, 4096);
    f16_split_check_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, n4, mismatch);
    return check_launch("f16_split_check");
}
