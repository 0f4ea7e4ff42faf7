// Narrow-N split-precision convolution with register-direct A fragments (conv_x3_nar).
//
// The tiled split-fp32 kernels (conv_x3_impl.hpp) stage both operands through LDS: every K-slice of A
// is loaded to registers, split into hi | lo halves and written to LDS, then read back as MFMA
// fragments.  For a 64-channel output (the enhancers' 256^2 / 512^2 StyleConvs and U-Net blocks, DNet's
// and ENet's wide-image 64-channel layers) the 256 x 64 tile's waves each cover all 64 output columns,
// so no A fragment is shared between waves, and the LDS round trip is pure overhead: per K-slice the A
// stores (32 KB of ds_write_b128 at ~79 B/clk/CU) and reads (32 KB) cost as many LDS cycles as the
// slice's 48 MFMAs per wave take (768 cycles per SIMD; MI355X_MICROARCH.md §LDS) — measured 150 - 235
// TFLOP/s (0.18 - 0.28 of the x3 peak) on those layers, tools/gpu_s23.sh.
//
// Here each lane loads exactly its own 16x16x32 A fragments: row (lane & 15) of each 16-row block,
// channels 8 (lane >> 4) .. + 7 of the K-slice (two 16-byte buffer loads per row block, the AMODE 4
// addressing: per-row offsets and in-image tap masks, out-of-image taps read zeros), splits them in
// registers (the same split4 as the LDS path, so results are bit-identical to conv_igemm_x3 with the
// same K order) and feeds them to the MFMAs.  Only B (the pre-split packed weights, 8 KB per slice,
// shared by the four waves) goes through LDS, double-buffered.  The next slice's loads (A, B and the
// modulation s[n, c] of its channels) are in flight while the current one is multiplied.  Epilogue: conv_impl.hpp epilogue_tile_fn (every fused
// epilogue, split-K partials, the range guard's non-finite flag).
//
// Measured on MI355X (r05, profiles/r05_nar_sweep.txt, graph-timed, f16x3): parity bit-identical to
// the LDS tile; speed within +-5 % of the best LDS tile (4x512^2 64 -> 64: 441 vs 433 us for 128x64,
// 128 -> 64: 712 vs 672 us; 4x256^2 256 -> 64: 347 vs 360 us): the LDS round trip is not what holds these
// layers at 0.2 of the x3 peak.  With BREG = 1 (six more wave-loads per K-slice, no LDS, no barrier) the
// launches are 1.4-1.5x slower: the bound is the L2 -> CU operand stream, which conv_x3_halo.hip cuts
// (the input loaded once per channel slice instead of once per tap).  Kept forced-only (force_tile 16 / 17).
#include "conv_x3_impl.hpp"

namespace s2v {

// NAR_ABL (timing ablation, never in the shipped build): 1 = every slice re-reads the first tap's A
// (L1-resident loads, wrong results)
#ifndef NAR_ABL
#define NAR_ABL 0
#endif

// BREG = 1: B fragments also straight to registers (every wave loads its own; the four waves' loads of
// a slice hit the same lines): no LDS and no barrier in the main loop
template <int ELT, int BREG>
__global__ __launch_bounds__(256, 2) void conv_x3_nar(ConvArgs a) {
    launch_stamp(a, false);
    constexpr int BM = 256, BN = 64, NW = 4, TM16 = 4, TN16 = 4, RS = 32, BR = 2;
    constexpr int BSUB = BN * 128;                     // one K-slice of B (bytes)
    constexpr int CH = 64;                             // epilogue chunk rows
    constexpr int CBYTES = CH * (BN + 4) * 4;
    constexpr int SMEM = 2 * BSUB > CBYTES ? 2 * BSUB : CBYTES;
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int total = gridDim.x * gridDim.y * gridDim.z;
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    int mt, nt, bz;
    {   // XCD-aware tile order, as conv_x3_tile
        const int per = total >> 3, rem = total & 7;
        const int xcd = L & 7, idx = L >> 3;
        const int Lp = xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
        nt = Lp % gridDim.y;
        const int t = Lp / gridDim.y;
        mt = t % gridDim.x;
        bz = t / gridDim.x;
    }
    const int m0 = mt * BM, n0 = nt * BN;
    const int bidx = bz / a.splits, split = bz - bidx * a.splits;
    const float *__restrict__ x = a.x + (long long)bidx * a.x_bs;
    const char *__restrict__ wtb = (const char *)(a.wt + (long long)bidx * a.w_bs);
    const int kt0 = split * a.tps;
    const int kt1 = min(a.ktiles, kt0 + a.tps);
    const int taps = a.kh * a.kw, nsl = a.cin >> 5;
    const bool kperm = taps > 1;
    const int l16 = lane & 15, kg = lane >> 4;

    // this lane's A rows: row l16 of the wave's four 16-row blocks
    ARows<TM16, 0> R;
    {
        int rows[TM16];
#pragma unroll
        for (int i = 0; i < TM16; ++i) rows[i] = wave * 64 + i * 16 + l16;
        a_rows_init_at<TM16, 0>(a, m0, rows, R);
    }
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)a.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)wtb, 0, (int)a.w_bytes, 0x00020000);
    int rowoff[TM16];
    unsigned tmask[TM16];
#pragma unroll
    for (int i = 0; i < TM16; ++i) {
        rowoff[i] = (int)((R.base[i] + 8 * kg) * 4);
        unsigned m = 0;
        if (R.ok[i])
            for (int ky = 0; ky < a.kh; ++ky)
                for (int kx = 0; kx < a.kw; ++kx)
                    if ((unsigned)(R.iy0[i] + ky * a.dh) < (unsigned)a.h && (unsigned)(R.ix0[i] + kx * a.dw) < (unsigned)a.w)
                        m |= 1u << (ky * a.kw + kx);
        tmask[i] = m;
    }
    int boff[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) boff[j] = ((n0 + (tid >> 3) + RS * j) * a.kpad) * 4 + (tid & 7) * 16;

    // input modulation s[n, c] of the tile's image (the host allows in_scale only when every 256-row
    // tile lies in one image: oh * ow % 256 == 0), loaded with each slice
    const int hw_img = a.oh * a.ow;
    const float *sc_base = a.in_scale ? a.in_scale + (long long)(m0 / hw_img) * a.in_scale_ns : a.x;
    const __amdgpu_buffer_rsrc_t srs =
        __builtin_amdgcn_make_buffer_rsrc((void *)sc_base, 0, a.in_scale ? a.cin * 4 : 0, 0x00020000);

    floatx4 acc[TM16][TN16];
#pragma unroll
    for (int i = 0; i < TM16; ++i)
#pragma unroll
        for (int j = 0; j < TN16; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

    SliceIt ld;
    ld.init(kt0, kperm, taps, nsl, a.kw);
    // one slice's operands in registers: B staging (two 16-byte slots), A fragments (8 channels of 4 rows)
    struct Ops {
        u32x4 b[BREG ? 1 : BR];
        u32x4 bh[BREG ? TN16 : 1], bl[BREG ? TN16 : 1];   // BREG: the next slice's B fragments
        f4 v[2 * TM16];
        f4 s0, s1;       // modulation of the slice's channels (one-image tiles), loaded with the slice
        int cs;
    };
    // BREG: this lane's B fragment rows n0 + 16 j + l16, hi slot kg and lo slot kg + 4 of the slice
    int bfr[BREG ? TN16 : 1];
#pragma unroll
    for (int j = 0; j < (BREG ? TN16 : 1); ++j) bfr[j] = ((n0 + 16 * j + l16) * a.kpad) * 4 + kg * 16;
    auto issue_b = [&](Ops &o) {
        const int kt = ld.kt(nsl);
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
            o.bh[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, bfr[j], kt * 128, 0));
            o.bl[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, bfr[j] + 64, kt * 128, 0));
        }
    };
    auto issue = [&](Ops &o) {
        const int kt = ld.kt(nsl);
        if constexpr (!BREG) {
#pragma unroll
            for (int j = 0; j < BR; ++j)
                o.b[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, boff[j], kt * 128, 0));
        }
        const int toff = NAR_ABL == 1 ? 0 : ((ld.ky * a.dh * a.w + ld.kx * a.dw) * a.xcs + ld.cs * 32) * 4;
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const int vo = ((tmask[i] >> ld.tap) & 1u) ? rowoff[i] + toff : (int)0x80000000;
            o.v[2 * i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 0, 0));
            o.v[2 * i + 1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo + 16, 0, 0));
        }
        {   // modulation of the slice's channels: zeros (never read) without in_scale
            const int so = a.in_scale ? (ld.cs * 32 + 8 * kg) * 4 : (int)0x80000000;
            o.s0 = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(srs, so, 0, 0));
            o.s1 = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(srs, so + 16, 0, 0));
        }
        o.cs = ld.cs;
        if (ld.i < kt1 - 1) ld.next(kperm, taps, nsl, a.kw);
    };
    auto store_b = [&](char *Bs, const Ops &o) {
#pragma unroll
        for (int j = 0; j < BR; ++j) *(u32x4 *)(Bs + slot_off((tid >> 3) + RS * j, tid & 7)) = o.b[j];
    };
    const int hs16 = (kg ^ swz(l16)) << 4, ls16 = hs16 ^ 64;
    // A of the staged slice: modulation, pre-activation and range pre-scale, then the split (registers)
    auto split_a = [&](Ops &o, u32x4 (&ah)[TM16], u32x4 (&al)[TM16]) {
        if (a.in_scale) {
#pragma unroll
            for (int i = 0; i < TM16; ++i) {
                o.v[2 * i] *= o.s0;
                o.v[2 * i + 1] *= o.s1;
            }
        }
        if (a.pre_act) {
#pragma unroll
            for (int i = 0; i < 2 * TM16; ++i) pre_act4(a, o.v[i]);
        }
        if (a.x_scale != 1.f) {
#pragma unroll
            for (int i = 0; i < 2 * TM16; ++i) o.v[i] *= a.x_scale;
        }
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            u32x2 h0, l0, h1, l1;
            split4<ELT>(o.v[2 * i], h0, l0);
            split4<ELT>(o.v[2 * i + 1], h1, l1);
            ah[i] = u32x4{h0.x, h0.y, h1.x, h1.y};
            al[i] = u32x4{l0.x, l0.y, l1.x, l1.y};
        }
    };
    auto mma = [&](const char *Bs, const u32x4 (&ah)[TM16], const u32x4 (&al)[TM16]) {
        // column block j outer: only one B fragment pair (plus the next one's reads) live at a time
        u32x4 bh[2], bl[2];
        bh[0] = *(const u32x4 *)(Bs + l16 * 128 + hs16);
        bl[0] = *(const u32x4 *)(Bs + l16 * 128 + ls16);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
            const int c = j & 1;
            if (j + 1 < TN16) {
                const char *p = Bs + ((j + 1) * 16 + l16) * 128;
                bh[c ^ 1] = *(const u32x4 *)(p + hs16);
                bl[c ^ 1] = *(const u32x4 *)(p + ls16);
            }
#pragma unroll
            for (int i = 0; i < TM16; ++i) {
                acc[i][j] = mfma16x16<ELT>(al[i], bh[c], acc[i][j]);
                acc[i][j] = mfma16x16<ELT>(ah[i], bl[c], acc[i][j]);
                acc[i][j] = mfma16x16<ELT>(ah[i], bh[c], acc[i][j]);
            }
        }
        __builtin_amdgcn_s_setprio(0);
    };

    const int n = kt1 - kt0;
    if (n > 0) {
        // One register set: slice g's A is split (the only loads in flight are its own, issued a whole
        // MFMA phase earlier) before slice g + 1's loads reuse the registers; those then fly under slice
        // g's MFMAs.  (Issuing them before the split made the split's vmcnt waits, which count loads in
        // issue order, drain the next slice's loads too: load latency and MFMAs in series.)  B of slice
        // g + 1 is loaded first, so its LDS store waits for those two loads only.  A second register set
        // (two slices in flight) does not fit 256 VGPRs at two waves per SIMD without the compiler
        // merging the sets (r05).
        if constexpr (BREG) {
            // step g: B(g + 1) loads go out first (the split's in-order waits on A(g) leave them in
            // flight), then A(g + 1); the MFMAs use B(g) held since the previous step
            Ops o;
            u32x4 bh[TN16], bl[TN16];
            issue_b(o);
            issue(o);
#pragma unroll
            for (int j = 0; j < TN16; ++j) {
                bh[j] = o.bh[j];
                bl[j] = o.bl[j];
            }
#pragma unroll 1
            for (int g = 0; g < n; ++g) {
                issue_b(o);                                    // slice g + 1 (past the end: re-load, unused)
                u32x4 ah[TM16], al[TM16];
                split_a(o, ah, al);
                __builtin_amdgcn_sched_barrier(0);
                issue(o);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int j = 0; j < TN16; ++j)
#pragma unroll
                    for (int i = 0; i < TM16; ++i) {
                        acc[i][j] = mfma16x16<ELT>(al[i], bh[j], acc[i][j]);
                        acc[i][j] = mfma16x16<ELT>(ah[i], bl[j], acc[i][j]);
                        acc[i][j] = mfma16x16<ELT>(ah[i], bh[j], acc[i][j]);
                    }
                __builtin_amdgcn_s_setprio(0);
#pragma unroll
                for (int j = 0; j < TN16; ++j) {
                    bh[j] = o.bh[j];
                    bl[j] = o.bl[j];
                }
            }
        } else {
            Ops o;
            issue(o);
            store_b(smem, o);
            __syncthreads();
#pragma unroll 1
            for (int g = 0; g < n; ++g) {
                u32x4 ah[TM16], al[TM16];
                split_a(o, ah, al);
                __builtin_amdgcn_sched_barrier(0);
                issue(o);                                      // past the last slice: re-loads it, unused
                __builtin_amdgcn_sched_barrier(0);
                mma(smem + (g & 1) * BSUB, ah, al);
                store_b(smem + ((g + 1) & 1) * BSUB, o);
                __syncthreads();
            }
        }
    }
    if (a.nonfinite) {                         // range guard: any non-finite accumulator flags the launch
        bool bad = false;
#pragma unroll
        for (int i = 0; i < TM16; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) bad |= !__builtin_isfinite(acc[i][j][r]);
        if (bad) __hip_atomic_store(a.nonfinite, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    epilogue_tile_fn<BM, BN, NW, CH>(a, (float *)smem, tid, m0, n0, bz, bidx, [&](float *Cs, int c0) {
        constexpr int LDC = BN + 4;
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const int r0 = wave * 64 + i * 16 - c0;
            if (r0 < 0 || r0 >= CH) continue;
#pragma unroll
            for (int j = 0; j < TN16; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cs[(r0 + 4 * kg + r) * LDC + j * 16 + l16] = acc[i][j][r] * a.acc_scale;
        }
    });
    launch_stamp(a, true);
}

template <int ELT>
int launch_conv_x3_nar(const ConvArgs &a, bool breg, dim3 grid, hipStream_t s) {
    if (breg) conv_x3_nar<ELT, 1><<<grid, 256, 0, s>>>(a);
    else conv_x3_nar<ELT, 0><<<grid, 256, 0, s>>>(a);
    return 0;
}

template int launch_conv_x3_nar<0>(const ConvArgs &, bool, dim3, hipStream_t);
template int launch_conv_x3_nar<1>(const ConvArgs &, bool, dim3, hipStream_t);

}  // namespace s2v
