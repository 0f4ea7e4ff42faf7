// Split-fp32 implicit-GEMM convolution with a deep LDS-DMA ring ("ring" kernels) for the
// latency-bound convolutions: small output tiles with long K loops (LNet's FFC 3x3 / 1x1 convs at
// 12^2-48^2, the DNet / enhancer convs whose tile count does not fill the chip).
//
// Why a third kernel family: the register-staged x3 kernels (conv_x3_impl.hpp) keep one K-slice in
// flight per block; a 4-wave block (one wave per SIMD) then waits the full L2 / Infinity-Cache load
// latency on every 32-deep slice (~0.8 us per slice measured on LNet's 12^2 convs, r03), and their
// two-set prefetch variant lost its overlap to the compiler's vmcnt placement.  Here both operands go
// global -> LDS by global_load_lds (no VGPRs held, no ds_write) into an NST-stage ring, NST - 1
// slices in flight ahead of the one being multiplied, with counted `s_waitcnt vmcnt` waits and one
// raw s_barrier per slice (cdna_hip_programming.md, "Pipelining across barriers"):
//   * A (activations) lands as fp32 rows of 128 B (one 32-channel slice of one filter tap per output
//     pixel; out-of-image taps and rows past M read a zero line);
//   * B (packed weights, pre-split [npad][kpad/32][hi 32 | lo 32]) lands as 128-B split rows;
//   * each wave owns BM/4 full rows of the tile (4 waves stacked along M), so every A fragment is read
//     and split into f16 / bf16 hi + lo halves by exactly one wave, in registers, right before its
//     MFMAs (no redundant split, no LDS round trip of the halves).
// The LDS image is lane-linear (LDS-DMA writes 16 B per lane at M0 + 16 lane); the row swizzles are
// applied on the source address: B rows use the x3 kernels' slot swizzle, A rows a swizzle chosen for
// the fp32 fragment reads (lane l reads row l & 15, 16-byte chunks 2 (l >> 4) and 2 (l >> 4) + 1;
// conflict-free for all four ds_read_b128 lane groups).
// Same GEMM view, K-slice order (channel-slice-major over the taps), XCD-aware tile order, split-K
// partials and LDS-staged epilogue as the x3 kernels: identical sums up to the fp32 accumulation order
// of the 16x16x32 MFMA (the same instruction the x3 kernels use).
#include "conv_x3_impl.hpp"

namespace s2v {

__device__ __attribute__((aligned(256))) char g_ring_zero[256];

typedef const __attribute__((address_space(1))) void *ring_gptr_t;
typedef __attribute__((address_space(3))) void *ring_lptr_t;

__device__ __forceinline__ void ring_dma16(const char *src, char *lds_wave_base) {
    __builtin_amdgcn_global_load_lds((ring_gptr_t)src, (ring_lptr_t)lds_wave_base, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void ring_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// fp32 A row swizzle: 16-byte chunk c of tile row r sits at LDS position c ^ ring_aswz(r)
// (bits 1, 2, 3 of r -> 2, 1, 4: every ds_read_b128 lane group of the fragment reads hits 16
// distinct 4-bank groups)
__device__ __forceinline__ int ring_aswz(int r) { return (((r >> 1) & 1) << 1) | ((r >> 2) & 1) | (((r >> 3) & 1) << 2); }

// 8 fp32 -> 8 hi halves + 8 lo halves (ELT 1: f16 with the v_fma_mix residual; 0: bf16)
template <int ELT>
__device__ __forceinline__ void ring_split8(const f4 &a0, const f4 &a1, u32x4 &hi, u32x4 &lo) {
    u32x2 h0, l0, h1, l1;
    split4<ELT>(a0, h0, l0);
    split4<ELT>(a1, h1, l1);
    hi = u32x4{h0.x, h0.y, h1.x, h1.y};
    lo = u32x4{l0.x, l0.y, l1.x, l1.y};
}

// BM x BN tile, 4 waves stacked along M (WTM = BM / 4 rows each, all BN columns), NST ring stages.
template <int BM, int BN, int NST, int ELT>
__global__ __launch_bounds__(256) void conv_ring_x3(ConvArgs a) {
    constexpr int NW = 4, NT = 256;
    constexpr int WTM = BM / NW;
    constexpr int TM16 = WTM / 16, TN16 = BN / 16;
    constexpr int RP = 8 * NW;                      // tile rows per DMA pass (8 rows of 128 B per wave)
    constexpr int AP = BM / RP, BP = BN / RP;       // DMA passes per slice
    constexpr int G = AP + BP;                      // DMA instructions per slice and thread
    constexpr int SUB = (BM + BN) * 128;
    constexpr int OPS = NST * SUB;
    constexpr int CH = x3_chunk(BM, BN, OPS > 32768 ? OPS : 32768);
    constexpr int CBYTES = CH * (BN + 4) * 4;
    constexpr int SMEM = OPS > CBYTES ? OPS : CBYTES;
    static_assert(BM % RP == 0 && BN % RP == 0 && WTM % 16 == 0, "tile");
    static_assert(SMEM <= 160 * 1024, "LDS");
    static_assert(NST >= 3 && (NST - 2) * G < 64, "stages");

    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    launch_stamp(a, false);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    int mt, nt, bz;
    {   // XCD-aware tile order (conv.hip): L & 7 is the XCD of the block that runs tile L
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

    // DMA geometry: in pass j wave w fills rows j*RP + w*8 .. +7 (1 KB, lane-linear); lane l writes
    // LDS position l & 7 of row (l >> 3), which holds 16-byte chunk (l & 7) ^ swz(row) of that row
    // (the swizzles depend on row bits 1..3 only: the same for every pass)
    const int prow = wave * 8 + (lane >> 3);
    const int pos = lane & 7;
    const int abyte = (pos ^ ring_aswz(prow)) << 4;
    const int bbyte = (pos ^ swz(prow)) << 4;
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
        arow[j] = xb + R.base[j] * 4 + abyte;
        unsigned m = 0;
        if (R.ok[j])
            for (int ky = 0; ky < a.kh; ++ky)
                for (int kx = 0; kx < a.kw; ++kx)
                    if ((unsigned)(R.iy0[j] + ky * a.dh) < (unsigned)a.h && (unsigned)(R.ix0[j] + kx * a.dw) < (unsigned)a.w)
                        m |= 1u << (ky * a.kw + kx);
        tmask[j] = m;
    }
    const char *zline = g_ring_zero + abyte;
    const char *brow = wb + (long long)(n0 + prow) * a.kpad * 4 + bbyte;
    const long long bpass = (long long)RP * a.kpad * 4;

    SliceIt ld;
    ld.init(kt0, kperm, taps, nsl, a.kw);
    auto issue = [&](int buf) {
        char *st = smem + buf * SUB + wave * 8 * 128;
        const long long toff = ((long long)(ld.ky * a.dh * a.w + ld.kx * a.dw) * a.xcs + ld.cs * 32) * 4;
#pragma unroll
        for (int j = 0; j < AP; ++j) {
            const char *src = ((tmask[j] >> ld.tap) & 1u) ? arow[j] + toff : zline;
            ring_dma16(src, st + j * RP * 128);
        }
        const char *bs = brow + (long long)ld.kt(nsl) * 128;
#pragma unroll
        for (int j = 0; j < BP; ++j) ring_dma16(bs + j * bpass, st + BM * 128 + j * RP * 128);
        if (ld.i < kt1 - 1) ld.next(kperm, taps, nsl, a.kw);
    };

    floatx4 acc4[TM16][TN16];
#pragma unroll
    for (int i = 0; i < TM16; ++i)
#pragma unroll
        for (int j = 0; j < TN16; ++j) acc4[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int l16 = lane & 15, q = lane >> 4;
    const int hs16 = (q ^ swz(l16)) << 4, ls16 = hs16 ^ 64;          // B: hi / lo slot of the fragment
    const int ac0 = ((2 * q) ^ ring_aswz(l16)) << 4;                  // A: fp32 chunks 2q, 2q + 1
    const int ac1 = ((2 * q + 1) ^ ring_aswz(l16)) << 4;
    const bool xs = a.x_scale != 1.f;
    auto compute = [&](const char *As) {
        const char *Bs = As + BM * 128;
        u32x4 ah[TM16], al[TM16];
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const char *p = As + (wave * WTM + i * 16 + l16) * 128;
            f4 a0 = *(const f4 *)(p + ac0);
            f4 a1 = *(const f4 *)(p + ac1);
            if (xs) {                          // activation range pre-scale (exact: a power of two)
                a0 *= a.x_scale;
                a1 *= a.x_scale;
            }
            ring_split8<ELT>(a0, a1, ah[i], al[i]);
        }
        u32x4 bh[TN16], bl[TN16];
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
            const char *p = Bs + (j * 16 + l16) * 128;
            bh[j] = *(const u32x4 *)(p + hs16);
            bl[j] = *(const u32x4 *)(p + ls16);
        }
        // the halves of the last split feed the MFMAs below: a VALU-written operand needs wait states
        // before an MFMA reads it, which the hazard pass does not see through the inline-asm residual
        // (lo terms lost when the MFMA followed the split directly)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 4");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM16; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j) {
                acc4[i][j] = mfma16x16<ELT>(al[i], bh[j], acc4[i][j]);
                acc4[i][j] = mfma16x16<ELT>(ah[i], bl[j], acc4[i][j]);
                acc4[i][j] = mfma16x16<ELT>(ah[i], bh[j], acc4[i][j]);
            }
    };

    const int n = kt1 - kt0;
    if (n > 0) {
#pragma unroll
        for (int s = 0; s < NST - 1; ++s)
            if (s < n) issue(s);
        int cbuf = 0;                 // stage of slice t
        int ibuf = NST - 1;           // stage slice t + NST - 1 goes to
#pragma unroll 1
        for (int t = 0; t < n; ++t) {
            // slice t landed (this thread's DMAs; up to NST - 2 younger slices stay in flight), then
            // every wave's: the barrier also retires every wave's reads of the stage reissued below
            if (t + NST - 2 < n) ring_wait_vm<(NST - 2) * G>();
            else ring_wait_vm<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (t + NST - 1 < n) issue(ibuf);
            compute(smem + cbuf * SUB);
            __builtin_amdgcn_sched_barrier(0);
            cbuf = cbuf == NST - 1 ? 0 : cbuf + 1;
            ibuf = ibuf == NST - 1 ? 0 : ibuf + 1;
        }
    }
    if (a.nonfinite) {                 // range guard: any non-finite accumulator flags the launch
        bool bad = false;
#pragma unroll
        for (int i = 0; i < TM16; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) bad |= !__builtin_isfinite(acc4[i][j][r]);
        if (bad) __hip_atomic_store(a.nonfinite, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // epilogue (its first __syncthreads() orders the last slice's reads before the C staging; every
    // DMA was waited for by the last iteration's vmcnt(0))
    epilogue_tile_fn<BM, BN, NW, CH>(a, (float *)smem, tid, m0, n0, bz, bidx, [&](float *Cs, int c0) {
        constexpr int LDC = BN + 4;
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const int r0 = wave * WTM + i * 16 - c0;
            if (r0 < 0 || r0 >= CH) continue;
#pragma unroll
            for (int j = 0; j < TN16; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cs[(r0 + 4 * (lane >> 4) + r) * LDC + j * 16 + l16] = acc4[i][j][r] * a.acc_scale;
        }
    });
    launch_stamp(a, true);
}

// ring configurations (conv.hip kX3Tiles entries with ring = id + 1)
template <int ELT>
void launch_conv_ring(int cfg, const ConvArgs &a, dim3 grid, hipStream_t s) {
    switch (cfg) {
        case 0: conv_ring_x3<64, 64, 6, ELT><<<grid, 256, 0, s>>>(a); break;
        case 1: conv_ring_x3<128, 64, 5, ELT><<<grid, 256, 0, s>>>(a); break;
        case 2: conv_ring_x3<64, 128, 5, ELT><<<grid, 256, 0, s>>>(a); break;
        case 3: conv_ring_x3<128, 128, 4, ELT><<<grid, 256, 0, s>>>(a); break;
        case 4: conv_ring_x3<64, 32, 8, ELT><<<grid, 256, 0, s>>>(a); break;
        default: conv_ring_x3<128, 32, 6, ELT><<<grid, 256, 0, s>>>(a); break;
    }
}
template void launch_conv_ring<0>(int, const ConvArgs &, dim3, hipStream_t);
template void launch_conv_ring<1>(int, const ConvArgs &, dim3, hipStream_t);

}  // namespace s2v
