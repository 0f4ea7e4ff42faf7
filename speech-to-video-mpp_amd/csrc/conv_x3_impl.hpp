// Implicit-GEMM convolution on gfx950 16-bit MFMA with split-fp32 operands ("x3" kernels).
//
// Every fp32 operand v is carried as two 16-bit halves, hi = T(v) and lo = T(v - hi) (round to
// nearest even both; v - hi is exact in fp32), and a product as hi*hi + hi*lo + lo*hi accumulated
// in fp32 by a 32x32x16 MFMA (16-bit x 16-bit products are exact in fp32).  T is the element type
// ELT of the instance:
//   ELT 0, bf16 (v_mfma_f32_32x32x16_bf16): 8 significant bits per half, |v - hi - lo| <= 2^-16 |v|
//          and the dropped |lo*lo| <= 2^-16 |a*b|: <= 3 * 2^-16 relative per product, any fp32 range;
//   ELT 1, f16 (v_mfma_f32_32x32x16_f16): 11 significant bits per half, <= 3 * 2^-22 relative per
//          product (64x tighter; the exact-fp32 MFMA rounds each product-sum at 2^-24) for |v| in
//          the f16 normal range.  Below it the halves are f16 subnormals (absolute spacing 2^-24),
//          above 65504 they overflow, so the host pre-scales the packed weights by a power of two
//          (ConvArgs::acc_scale undoes it exactly); activations are conv inputs after norms /
//          activations (|v| << 65504 on every path of this model family).
// Both cost three 16-bit MFMAs (96 cycles per 32x32x16 block against 512 for eight
// v_mfma_f32_32x32x2_f32) and the same VALU work to split an operand (v_cvt_pk_{bf16,f16}_f32 ...).
//
// Same GEMM view, gather loaders, K-slice order, XCD-aware tile order and epilogue as the fp32
// kernel (conv.hip / conv_impl.hpp).  Differences:
//   * B (packed weights) is pre-split on the device once into [npad][kpad/32][hi 32 | lo 32] 16-bit
//     (s2v_split_weights / s2v_modulate_weights_split: same bytes as fp32), so a 128-byte weight
//     row slice lands in LDS unchanged;
//   * A is split in registers after its global load, while the MFMAs of the previous slice run;
//   * LDS rows are 128 B (eight 16-byte slots: hi k0-7, k8-15, k16-23, k24-31, then lo), slot s of
//     row r stored at s ^ ((r >> 1) & 7): the 16 rows of each ds_read_b128 lane group hit 16
//     distinct slots of the 256-byte bank row (conflict-free operand reads).
#pragma once
#include "conv_impl.hpp"

namespace s2v {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// f16 lo halves by v_fma_mix (1): one VALU per half, written into the halves of one register; 0: widen the
// hi halves (v_cvt_f32_f16), subtract, pack (as the bf16 path does).  0 failed the modulated depth-to-space
// test's f16x3 bound in r04 (1.2e-4).  Cause (r05, from the ISA of split4<1> built with 0): the compiler
// folded "widen the packed hi halves" into a second conversion of the fp32 inputs — v_cvt_f16_f32 +
// v_cvt_f32_f16 per value beside the v_cvt_pk_f16_f32 that produced the stored hi — so the lo halves were
// residuals against a separately rounded copy of hi, not against the hi that is stored: whenever the two
// conversions round differently, hi + lo misses the input by one f16 ulp.  The hi register now goes
// through an empty asm, which the compiler cannot see through, so the widening reads the stored halves;
// s2v_f16_split_check asserts both variants bit-identical (tests/test_ops_gpu.py).
#ifndef X3_F16_MIX
#define X3_F16_MIX 1
#endif

// two fp32 -> two 16-bit halves of type ELT (RNE): v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32
template <int ELT>
__device__ __forceinline__ unsigned pack2(float a, float b) {
    if constexpr (ELT == 0) {
        bf16x2 v = {(__bf16)a, (__bf16)b};
        return __builtin_bit_cast(unsigned, v);
    } else {
        f16x2 v = {(_Float16)a, (_Float16)b};
        return __builtin_bit_cast(unsigned, v);
    }
}

template <int ELT>
__device__ __forceinline__ void unpack2(unsigned u, float &a, float &b) {
    if constexpr (ELT == 0) {
        a = __uint_as_float(u << 16);
        b = __uint_as_float(u & 0xffff0000u);
    } else {
        const f16x2 v = __builtin_bit_cast(f16x2, u);
        a = (float)v.x;
        b = (float)v.y;
    }
}

// f16 residual pair: {f16(a - h.lo), f16(b - h.hi)} with one rounding each (v_fma_mix computes
// -h + a exactly from the f16 source and rounds once): 2 VALU instead of unpack + subtract + pack
__device__ __forceinline__ unsigned f16_residual2(unsigned h, float a, float b) {
    unsigned r;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(a));
    asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(r) : "v"(h), "v"(b));
    return r;
}

// 4 fp32 -> 4 hi halves (8 bytes) + 4 lo halves (8 bytes)
template <int ELT, int MIX = X3_F16_MIX>
__device__ __forceinline__ void split4(const f4 &v, u32x2 &hi, u32x2 &lo) {
    hi.x = pack2<ELT>(v.x, v.y);
    hi.y = pack2<ELT>(v.z, v.w);
    if constexpr (ELT == 1 && MIX) {
        lo.x = f16_residual2(hi.x, v.x, v.y);
        lo.y = f16_residual2(hi.y, v.z, v.w);
    } else {
        if constexpr (ELT == 1) asm volatile("" : "+v"(hi.x), "+v"(hi.y));   // widen THESE halves (see X3_F16_MIX)
        float h0, h1, h2, h3;
        unpack2<ELT>(hi.x, h0, h1);
        unpack2<ELT>(hi.y, h2, h3);
        lo.x = pack2<ELT>(v.x - h0, v.y - h1);
        lo.y = pack2<ELT>(v.z - h2, v.w - h3);
    }
}

// Main-loop MFMA shape: 16x16x32 (default) or 32x32x16 (X3_MFMA16=0).  Same FLOP per cycle and
// the same LDS reads per MFMA cycle; on MI355X the 16x16x32 loop holds a higher clock under load
// (MI355X_MICROARCH.md, DVFS give-back item 7): 256x256 f16x3 372 -> 389 TFLOP/s, 128x128 291 -> 309
// (tools/conv_micro.py, 16x200x200x256 3x3).
// Waves raise their issue priority over the MFMA block of a K-slice: always in the 4-wave tiles
// (measured on MI355X: 16x12^2x1024 -> 256, 128x64 tile, 74 -> 68 us), X3_PRIO=1 also in the 8-wave
// tiles (no change there: their two waves per SIMD already run the phases staggered)
#ifndef X3_PRIO
#define X3_PRIO 0
#endif
#ifndef X3_MFMA16
#define X3_MFMA16 1
#endif
#ifndef X3_APIPE
#define X3_APIPE 1
#endif
typedef float floatx4 __attribute__((ext_vector_type(4)));

// one 16x16x32 MFMA on 16-byte fragments holding 8 halves of type ELT each
template <int ELT>
__device__ __forceinline__ floatx4 mfma16x16(const u32x4 &a, const u32x4 &b, const floatx4 &c) {
    if constexpr (ELT == 0)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                     0, 0, 0);
}

// one 32x32x16 MFMA on 16-byte fragments holding 8 halves of type ELT each
template <int ELT>
__device__ __forceinline__ floatx16 mfma16(const u32x4 &a, const u32x4 &b, const floatx16 &c) {
    if constexpr (ELT == 0)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                     0, 0, 0);
}

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// byte offset of 16-byte slot ``slot`` (0..7) of LDS row ``row``
__device__ __forceinline__ int slot_off(int row, int slot) { return row * 128 + ((slot ^ swz(row)) << 4); }

// A rows ar + RS*j of the tile: 4 k-values per thread (slot q>>1, bytes (q&1)*8)
template <int AR, int RS, int ELT>
__device__ __forceinline__ void store_a_x3(char *As, int tid, const f4 (&ra)[AR]) {
    const int ar = tid >> 3, q = tid & 7;
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int row = ar + RS * j;
        u32x2 hi, lo;
        split4<ELT>(ra[j], hi, lo);
        const int off = slot_off(row, q >> 1) + (q & 1) * 8;
        *(u32x2 *)(As + off) = hi;
        *(u32x2 *)(As + (off ^ 64)) = lo;          // slot ^ 4 == the lo slot (slot < 4)
    }
}

// Wide A staging (AMODE 0/3): a thread owns 8 consecutive k (two float4 loads) of AR8 rows and
// writes each as one 16-byte hi slot + one 16-byte lo slot (ds_write_b128).  Lane t of a pass
// takes row 16 (t >> 6) + ((t >> 3) & 7) + 8 ((t >> 2) & 1): the two rows of every 8-lane store
// group are r and r + 8, whose swizzles differ in bit 2, so their four slots land in disjoint
// halves of the 128-byte bank window (no write conflicts); 4 lanes cover a 128-byte row piece.
template <int NT>
__device__ __forceinline__ int a_row8(int t, int j) {
    return j * (NT / 4) + ((t >> 6) << 4) + ((t >> 3) & 7) + 8 * ((t >> 2) & 1);
}

template <int AR8, int NT, int ELT>
__device__ __forceinline__ void store_a8_x3(char *As, int tid, const f4 (&ra)[2 * AR8]) {
    const int q = tid & 3;
#pragma unroll
    for (int j = 0; j < AR8; ++j) {
        u32x2 h0, l0, h1, l1;
        split4<ELT>(ra[2 * j], h0, l0);
        split4<ELT>(ra[2 * j + 1], h1, l1);
        const u32x4 hi = {h0.x, h0.y, h1.x, h1.y}, lo = {l0.x, l0.y, l1.x, l1.y};
        const int off = slot_off(a_row8<NT>(tid, j), q);
        *(u32x4 *)(As + off) = hi;
        *(u32x4 *)(As + (off ^ 64)) = lo;
    }
}

// pre-split packed weights: thread loads 16 bytes (one slot) of rows br + RS j
template <int BR, int RS>
__device__ __forceinline__ void load_b_x3(const ConvArgs &a, const char *__restrict__ wt, int kt, int n0, int tid,
                                          u32x4 (&rb)[BR]) {
    const int br = tid >> 3, sl = tid & 7;
    const char *p = wt + ((long long)(n0 + br) * a.kpad + kt * 32) * 4 + sl * 16;
#pragma unroll
    for (int j = 0; j < BR; ++j) rb[j] = *(const u32x4 *)(p + (long long)RS * j * a.kpad * 4);
}

template <int BR, int RS>
__device__ __forceinline__ void store_b_x3(char *Bs, int tid, const u32x4 (&rb)[BR]) {
    const int br = tid >> 3, sl = tid & 7;
#pragma unroll
    for (int j = 0; j < BR; ++j) *(u32x4 *)(Bs + slot_off(br + RS * j, sl)) = rb[j];
}

// activation B ([K][ldb] fp32, b_kn, 256 threads): split on the fly, scattered 2-byte stores
// (small GEMMs only)
template <int BN, int BR, int ELT>
__device__ __forceinline__ void store_b_kn_x3(char *Bs, int tid, const f4 (&rb)[BR]) {
    constexpr int NV = BN / 4, RPP = 256 / NV;
    const int kr = tid / NV, nn = (tid - (tid / NV) * NV) * 4;
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int k = kr + RPP * j;
        u32x2 hi, lo;
        split4<ELT>(rb[j], hi, lo);
        const unsigned hs[4] = {hi.x & 0xffffu, hi.x >> 16, hi.y & 0xffffu, hi.y >> 16};
        const unsigned ls[4] = {lo.x & 0xffffu, lo.x >> 16, lo.y & 0xffffu, lo.y >> 16};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int off = slot_off(nn + e, k >> 3) + (k & 7) * 2;
            *(unsigned short *)(Bs + off) = (unsigned short)hs[e];
            *(unsigned short *)(Bs + (off ^ 64)) = (unsigned short)ls[e];
        }
    }
}

// K-slice cursor.  Slice kt = tap * nsl + cs covers channels [32 cs, 32 cs + 32) of filter tap
// ``tap`` = ky * kw + kx.  With ``kperm`` (AMODE 0/3 multi-tap convs) slices are visited
// channel-slice-major — all taps of one 32-channel slice in a row, so a 3x3 neighbourhood is
// re-read from L2 right away; the weights are indexed by the same kt, so the sum is the same up
// to fp32 summation order.  Otherwise in natural k order.  Advancing needs no division.
struct SliceIt {
    int i, tap, cs, ky, kx;
    __device__ __forceinline__ void init(int i0, bool kperm, int taps, int nsl, int kw) {
        i = i0;
        if (kperm) { tap = i0 % taps; cs = i0 / taps; }
        else if (nsl > 0) { tap = i0 / nsl; cs = i0 - tap * nsl; }
        else { tap = 0; cs = 0; }                 // generic gathers only use i
        ky = tap / kw;
        kx = tap - ky * kw;
    }
    __device__ __forceinline__ void next(bool kperm, int taps, int nsl, int kw) {
        ++i;
        if (kperm) {
            ++tap; ++kx;
            if (kx == kw) { kx = 0; ++ky; }
            if (tap == taps) { tap = 0; ky = 0; kx = 0; ++cs; }
        } else {
            ++cs;
            if (cs == nsl) { cs = 0; ++tap; ++kx; if (kx == kw) { kx = 0; ++ky; } }
        }
    }
    __device__ __forceinline__ int kt(int nsl) const { return tap * nsl + cs; }
};

constexpr int x3_chunk(int bm, int bn, int smem) {
    int ch = bm;
    while (ch > 32 && ch * (bn + 4) * 4 > smem) ch /= 2;
    return ch;
}

// BM x BN tile, NW waves (WAVES_M x NW/WAVES_M), KS 32-deep K-slices per LDS stage (two stages),
// PF register stages of prefetch (1: slice group t+1 in flight during group t; 2: t+2).
// Measured on MI355X (tools/conv_micro.py, r01): KS = 1, PF = 1 with 8 waves (two or more waves
// per SIMD hide each other's load waits) beats deeper register prefetch (PF = 2 costs ~64 VGPRs and
// drops to one wave per SIMD: -40 %) and BK = 64 stages (KS = 2: LDS for one block per CU: -40 %).
// AMODE 4 is AMODE 0 (direct conv, zero padding, cin % 32 == 0, wide A staging) with buffer loads:
// per A row a precomputed 32-bit offset and a mask of the filter taps that land inside the image
// (out-of-image taps load from an offset past the buffer's extent, which returns zeros — no
// branches, no zero fills), the tap / channel-slice offset a wave-uniform scalar; the B rows as
// loop-invariant offsets plus a scalar K offset.  The host picks it when the x slab and the weights
// fit 2^31 bytes and the filter has <= 32 taps.
// One output tile: L is its linear index in the (gx, gy, total / (gx gy)) tile grid.
// EXTRA = false: the persistent and grouped forms, which the host never gives the SFT / second-output
// extras (their registers pushed the persistent 256x256 tile from 6 to 21 spilled VGPRs)
template <int BM, int BN, int WAVES_M, int NW, int KS, int PF, int AMODE_, int BKN, int ELT, bool EXTRA = true>
__device__ __forceinline__ void conv_x3_tile(const ConvArgs &a, int L, int gx, int gy, int total) {
    constexpr bool BUF = AMODE_ == 4;
    constexpr int AMODE = BUF ? 0 : AMODE_;
    constexpr int NT = 64 * NW, RS = NT / 8;
    constexpr int WAVES_N = NW / WAVES_M;
    constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int AR = BM / RS;
    constexpr int BR = BN / RS;
    constexpr int SUB = (BM + BN) * 128;                      // one K-slice of A and B (bytes)
    constexpr int STAGE = KS * SUB;
    constexpr int OPS = 2 * STAGE;
    constexpr int CH = x3_chunk(BM, BN, OPS > 65536 ? OPS : 65536);
    constexpr int CBYTES = CH * (BN + 4) * 4;                 // epilogue C staging
    constexpr int SMEM = OPS > CBYTES ? OPS : CBYTES;
    static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0 && AR >= 1 && BR >= 1, "tile");
    static_assert(!BKN || NW == 4, "b_kn operands only with 4 waves");
    static_assert(SMEM <= 160 * 1024, "LDS");
    constexpr int BKR = BKN ? BN / 32 : 1;                    // b_kn loader rows (256 threads)

    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    int mt, nt, bz;
    {   // XCD-aware tile order (see conv.hip): L & 7 is the XCD of the block that runs tile L
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
    const float *__restrict__ wtf = a.wt + (long long)bidx * a.w_bs;      // fp32 view (b_kn)
    const char *__restrict__ wtb = (const char *)wtf;                      // split view (packed)
    const int kt0 = split * a.tps;
    const int kt1 = min(a.ktiles, kt0 + a.tps);
    // buffer loads: a partial last channel slice (1x1, cin % 8 == 0, conv.hip x3_partial_1x1)
    const int taps = a.kh * a.kw, nsl = BUF ? (a.cin + 31) >> 5 : a.cin >> 5;
    const bool kperm = (AMODE == 0 || AMODE == 3) && !BKN && taps > 1;
    const int ak = (tid & 7) * 4;

    constexpr bool A8 = (AMODE == 0 || AMODE == 3) && !BKN && BM % (NT / 4) == 0;
    constexpr int AR8 = A8 ? BM / (NT / 4) : 1;
    ARows<A8 ? AR8 : AR, AMODE> R;
    if constexpr (A8) {
        int rows[AR8];
#pragma unroll
        for (int j = 0; j < AR8; ++j) rows[j] = a_row8<NT>(tid, j);
        a_rows_init_at<AR8, AMODE>(a, m0, rows, R);
    } else {
        a_rows_init<AR, AMODE, RS>(a, m0, tid >> 3, R);
    }
    static_assert(!A8 || 2 * AR8 == AR, "wide A staging: same float4 count");
    static_assert(!BUF || (A8 && !BKN), "buffer loads: wide A staging, packed B");

    // buffer-load state (AMODE 4)
    __amdgpu_buffer_rsrc_t xrs, wrs;
    int rowoff[BUF ? AR8 : 1];
    unsigned tmask[BUF ? AR8 : 1];
    int boff[BUF ? BR : 1];
    if constexpr (BUF) {
        xrs = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)a.x_bytes, 0x00020000);
        wrs = __builtin_amdgcn_make_buffer_rsrc((void *)wtb, 0, (int)a.w_bytes, 0x00020000);
#pragma unroll
        for (int j = 0; j < AR8; ++j) {
            rowoff[j] = (int)((R.base[j] + 8 * (tid & 3)) * 4);
            unsigned m = 0;
            if (R.ok[j])
                for (int ky = 0; ky < a.kh; ++ky)
                    for (int kx = 0; kx < a.kw; ++kx)
                        if ((unsigned)(R.iy0[j] + ky * a.dh) < (unsigned)a.h &&
                            (unsigned)(R.ix0[j] + kx * a.dw) < (unsigned)a.w)
                            m |= 1u << (ky * a.kw + kx);
            tmask[j] = m;
        }
#pragma unroll
        for (int j = 0; j < BR; ++j) boff[j] = ((n0 + (tid >> 3) + RS * j) * a.kpad) * 4 + (tid & 7) * 16;
    }

    f4 ra[PF][KS][AR];
    int rc[PF][KS];                  // A8: channel base of the staged slice (for the deferred prologue)
    // input scale s[n, c] (StyleGAN2 modulation with shared weights) loaded with the A operand in issue()
    // instead of in the store phase, where its load was waited for right away (one memory round trip per
    // K-slice); only in tiles with register room (the 256-row / 512-row tiles keep the old path)
    constexpr bool PSC = A8 && KS == 1 && PF == 1 && (BM * BN <= 128 * 128 || (BN == 64 && AR8 <= 4 && NW == 4));
    static_assert(!PSC || (PF == 1 && KS == 1), "the input-scale registers follow one in-flight slice");
    f4 rsc[PF][KS][PSC ? 2 * AR8 : 1];
    // a tile whose rows all lie in one image (every tile of the 256^2 / 512^2 enhancer and DNet layers)
    // needs one s[n, c8 .. c8 + 7] pair per thread, reloaded only when the channel slice changes (every
    // kh * kw K-slices in the channel-slice-major order), instead of two loads per row per slice
    // (the 256 / 512-row tiles: the smaller ones keep their register budget and the per-row loads)
    constexpr bool PSC1 = PSC && BM >= 256;
    const int hw_img = a.oh * a.ow;
    const bool one_img = PSC1 && a.in_scale && m0 / hw_img == (min(m0 + BM, a.M) - 1) / hw_img;
    const float *sc_base = PSC1 && a.in_scale ? a.in_scale + (long long)(m0 / hw_img) * a.in_scale_ns : nullptr;
    f4 sc0 = {1.f, 1.f, 1.f, 1.f}, sc1 = {1.f, 1.f, 1.f, 1.f};
    int sc_cs = -1;
    u32x4 rbp[PF][KS][BKN ? 1 : BR];
    f4 rbk[PF][KS][BKN ? BKR : 1];
    constexpr bool M16 = X3_MFMA16;
    constexpr int TM16 = WTM / 16, TN16 = WTN / 16;
    floatx16 acc[M16 ? 1 : TM][M16 ? 1 : TN];
    floatx4 acc4[M16 ? TM16 : 1][M16 ? TN16 : 1];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) if (!M16) acc[i][j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < TM16; ++i)
#pragma unroll
        for (int j = 0; j < TN16; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) if (M16) acc4[i][j][r] = 0.f;

    SliceIt ld;                      // the next K-slice to load
    ld.init(kt0, kperm, taps, nsl, a.kw);
    // load one group of KS slices into register set p (slices past the end re-load the last one;
    // their products are never formed)
    auto issue = [&](int p) {
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            const int kt = (AMODE == 0 || AMODE == 3) ? ld.kt(nsl) : ld.i;
            if constexpr (BUF) {
                const int c8 = ld.cs * 32 + 8 * (tid & 3);
                const bool cok = c8 < a.cin;             // false only in a partial last slice
                rc[p][u] = c8;
                if constexpr (PSC) {
                    if (PSC1 && one_img) {
                        if (ld.cs != sc_cs) {
                            if (cok) {
                                sc0 = *(const f4 *)(sc_base + c8);
                                sc1 = *(const f4 *)(sc_base + c8 + 4);
                            }
                            sc_cs = ld.cs;
                        }
                    } else if (a.in_scale && cok) {
#pragma unroll
                        for (int j = 0; j < AR8; ++j) {
                            const float *sp = a.in_scale + (long long)R.img[j] * a.in_scale_ns + c8;
                            rsc[p][u][2 * j] = *(const f4 *)sp;
                            rsc[p][u][2 * j + 1] = *(const f4 *)(sp + 4);
                        }
                    }
                }
                const int toff = ((ld.ky * a.dh * a.w + ld.kx * a.dw) * a.xcs + ld.cs * 32) * 4;
#pragma unroll
                for (int j = 0; j < AR8; ++j) {
                    const int vo = (cok && ((tmask[j] >> ld.tap) & 1u)) ? rowoff[j] + toff : (int)0x80000000;
                    ra[p][u][2 * j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 0, 0));
                    ra[p][u][2 * j + 1] =
                        __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo + 16, 0, 0));
                }
#pragma unroll
                for (int j = 0; j < BR; ++j)
                    rbp[p][u][j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, boff[j], kt * 128, 0));
            } else if constexpr (A8) {
                f4 t0[AR8], t1[AR8];
                const int c8 = ld.cs * 32 + 8 * (tid & 3);
                rc[p][u] = c8;
                if constexpr (PSC) {
                    if (PSC1 && one_img) {
                        if (ld.cs != sc_cs) {
                            sc0 = *(const f4 *)(sc_base + c8);
                            sc1 = *(const f4 *)(sc_base + c8 + 4);
                            sc_cs = ld.cs;
                        }
                    } else if (a.in_scale) {
#pragma unroll
                        for (int j = 0; j < AR8; ++j) {
                            const float *sp = a.in_scale + (long long)R.img[j] * a.in_scale_ns + c8;
                            rsc[p][u][2 * j] = *(const f4 *)sp;
                            rsc[p][u][2 * j + 1] = *(const f4 *)(sp + 4);
                        }
                    }
                }
                load_a_tap<AR8, AMODE, false>(a, x, ld.ky, ld.kx, c8, R, t0);
                load_a_tap<AR8, AMODE, false>(a, x, ld.ky, ld.kx, c8 + 4, R, t1);
#pragma unroll
                for (int j = 0; j < AR8; ++j) {
                    ra[p][u][2 * j] = t0[j];
                    ra[p][u][2 * j + 1] = t1[j];
                }
            } else if constexpr (AMODE == 0 || AMODE == 3) {
                load_a_tap<AR, AMODE>(a, x, ld.ky, ld.kx, ld.cs * 32 + ak, R, ra[p][u]);
            } else {
                load_a<AR, AMODE>(a, x, kt, ak, R, ra[p][u]);
            }
            if constexpr (BKN) load_b<BN, BKR, 1>(a, wtf, kt, n0, tid, rbk[p][u]);
            else if constexpr (!BUF) load_b_x3<BR, RS>(a, wtb, kt, n0, tid, rbp[p][u]);
            if (ld.i < kt1 - 1) ld.next(kperm, taps, nsl, a.kw);
        }
    };
    auto store = [&](char *st, int p) {
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            char *sb = st + u * SUB;
            if constexpr (A8) {
                if constexpr (PSC) {
                    if (PSC1 && one_img) {
#pragma unroll
                        for (int j = 0; j < AR8; ++j) {
                            ra[p][u][2 * j] *= sc0;
                            ra[p][u][2 * j + 1] *= sc1;
                        }
                    } else if (a.in_scale) {
#pragma unroll
                        for (int j = 0; j < 2 * AR8; ++j) ra[p][u][j] *= rsc[p][u][j];
                    }
                    if (a.pre_act) {
#pragma unroll
                        for (int j = 0; j < 2 * AR8; ++j) pre_act4(a, ra[p][u][j]);
                    }
                } else if (a.in_scale || a.pre_act) {
#pragma unroll
                    for (int j = 0; j < AR8; ++j) {
                        prologue4<AR8, AMODE>(a, R, j, rc[p][u], ra[p][u][2 * j]);
                        prologue4<AR8, AMODE>(a, R, j, rc[p][u] + 4, ra[p][u][2 * j + 1]);
                    }
                }
            }
            if (a.x_scale != 1.f) {            // activation range pre-scale (exact: a power of two)
#pragma unroll
                for (int j = 0; j < AR; ++j) ra[p][u][j] *= a.x_scale;
            }
            if constexpr (A8) store_a8_x3<AR8, NT, ELT>(sb, tid, ra[p][u]);
            else store_a_x3<AR, RS, ELT>(sb, tid, ra[p][u]);
            if constexpr (BKN) store_b_kn_x3<BN, BKR, ELT>(sb + BM * 128, tid, rbk[p][u]);
            else store_b_x3<BR, RS>(sb + BM * 128, tid, rbp[p][u]);
        }
    };

    const int li = lane & 31, lh = lane >> 5;
    const int rsw = swz(li);     // rows wm*WTM + i*32 + li share li's swizzle (tile bases are multiples of 32)
    // 16x16x32 fragments: lane l reads row l & 15, hi slot l >> 4 (k 8(l>>4) .. +7) and its lo slot
    const int l16 = lane & 15;
    const int hs16 = ((lane >> 4) ^ swz(l16)) << 4, ls16 = hs16 ^ 64;
    // multiply ``nv`` (<= KS) slices of one stage
    auto compute = [&](const char *st, int nv) {
        if constexpr (X3_PRIO || NW == 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            if (u >= nv) break;
            const char *As = st + u * SUB;
            const char *Bs = As + BM * 128;
            if constexpr (M16) {
                // A fragments double-buffered: row block i + 1 is read from LDS before the MFMAs of row
                // block i are issued, so its LDS latency hides under them (X3_APIPE; with one buffer
                // each row block waited lgkmcnt(0) on reads issued after the previous block's MFMAs)
                u32x4 bh[TN16], bl[TN16];
                u32x4 ah[X3_APIPE ? 2 : 1], al[X3_APIPE ? 2 : 1];
                const char *pa = As + (wm * WTM + l16) * 128;
                if constexpr (X3_APIPE) {
                    ah[0] = *(const u32x4 *)(pa + hs16);
                    al[0] = *(const u32x4 *)(pa + ls16);
                }
#pragma unroll
                for (int j = 0; j < TN16; ++j) {
                    const char *p = Bs + (wn * WTN + j * 16 + l16) * 128;
                    bh[j] = *(const u32x4 *)(p + hs16);
                    bl[j] = *(const u32x4 *)(p + ls16);
                }
#pragma unroll
                for (int i = 0; i < TM16; ++i) {
                    const int c = X3_APIPE ? (i & 1) : 0;
                    if constexpr (X3_APIPE) {
                        if (i + 1 < TM16) {
                            ah[c ^ 1] = *(const u32x4 *)(pa + (i + 1) * 16 * 128 + hs16);
                            al[c ^ 1] = *(const u32x4 *)(pa + (i + 1) * 16 * 128 + ls16);
                        }
                    } else {
                        ah[0] = *(const u32x4 *)(pa + i * 16 * 128 + hs16);
                        al[0] = *(const u32x4 *)(pa + i * 16 * 128 + ls16);
                    }
#pragma unroll
                    for (int j = 0; j < TN16; ++j) {
                        acc4[i][j] = mfma16x16<ELT>(al[c], bh[j], acc4[i][j]);
                        acc4[i][j] = mfma16x16<ELT>(ah[c], bl[j], acc4[i][j]);
                        acc4[i][j] = mfma16x16<ELT>(ah[c], bh[j], acc4[i][j]);
                    }
                }
                continue;
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int hs = ((2 * s + lh) ^ rsw) << 4, ls = hs ^ 64;
                u32x4 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const char *p = As + (wm * WTM + i * 32 + li) * 128;
                    ah[i] = *(const u32x4 *)(p + hs);
                    al[i] = *(const u32x4 *)(p + ls);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const char *p = Bs + (wn * WTN + j * 32 + li) * 128;
                    bh[j] = *(const u32x4 *)(p + hs);
                    bl[j] = *(const u32x4 *)(p + ls);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        acc[i][j] = mfma16<ELT>(al[i], bh[j], acc[i][j]);
                        acc[i][j] = mfma16<ELT>(ah[i], bl[j], acc[i][j]);
                        acc[i][j] = mfma16<ELT>(ah[i], bh[j], acc[i][j]);
                    }
            }
        }
        if constexpr (X3_PRIO || NW == 4) __builtin_amdgcn_s_setprio(0);
    };

    const int n = kt1 - kt0;
    const int ng = (n + KS - 1) / KS;            // stage groups
    if (ng > 0) {
        issue(0);
        store(smem, 0);
        __syncthreads();
        if (PF == 1) {
            // group g: load g+1 into the registers, multiply stage g%2, store g+1 into the other
            // stage (last read before the previous barrier).  In 8-wave blocks the two waves that
            // share a SIMD run each step in opposite phase orders (the upper half: store the group
            // loaded one step earlier, load the next, multiply), so one wave's split + LDS-store
            // phase overlaps its partner's MFMAs instead of both leaving the matrix pipe idle at
            // the same time (MI355X_MICROARCH.md, two waves per SIMD, item 9).  Either order stores
            // into the buffer last read before the previous barrier and multiplies the one
            // completed before it.
            const bool late = NW == 8 && __builtin_amdgcn_readfirstlane(wave) >= NW / 2;
            if (late) {
                issue(0);                                        // group 1
                for (int g = 0; g < ng; ++g) {
                    store(smem + ((g + 1) & 1) * STAGE, 0);       // group g+1
                    issue(0);                                    // group g+2
                    __builtin_amdgcn_sched_barrier(0);
                    compute(smem + (g & 1) * STAGE, min(KS, n - g * KS));
                    __syncthreads();
                }
            } else {
                for (int g = 0; g < ng; ++g) {
                    issue(0);
                    __builtin_amdgcn_sched_barrier(0);
                    compute(smem + (g & 1) * STAGE, min(KS, n - g * KS));
                    store(smem + ((g + 1) & 1) * STAGE, 0);
                    __syncthreads();
                }
            }
        } else {
            issue(PF - 1);
            // group g: load g+2 into set g%2, multiply stage g%2, store set (g+1)%2 (group g+1)
            for (int g = 0; g < ng; g += 2) {
                issue(0);
                __builtin_amdgcn_sched_barrier(0);
                compute(smem, min(KS, n - g * KS));
                store(smem + STAGE, PF - 1);
                __syncthreads();
                if (g + 1 >= ng) break;
                issue(PF - 1);
                __builtin_amdgcn_sched_barrier(0);
                compute(smem + STAGE, min(KS, n - (g + 1) * KS));
                store(smem, 0);
                __syncthreads();
            }
        }
    }
    if constexpr (M16) {
        // stage the 16x16 accumulators (col = lane & 15, row = 4 (lane >> 4) + r) chunk by chunk
        if (a.nonfinite) {                     // range guard: any non-finite accumulator flags the launch
            bool bad = false;
#pragma unroll
            for (int i = 0; i < TM16; ++i)
#pragma unroll
                for (int j = 0; j < TN16; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) bad |= !__builtin_isfinite(acc4[i][j][r]);
            if (bad) __hip_atomic_store(a.nonfinite, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        epilogue_tile_fn<BM, BN, NW, CH, EXTRA>(a, (float *)smem, tid, m0, n0, bz, bidx, [&](float *Cs, int c0) {
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
        });
    } else {
        epilogue_tile<BM, BN, WAVES_M, TM, TN, NW, CH, EXTRA>(a, acc, (float *)smem, tid, m0, n0, bz, bidx);
    }
}

// One block per tile.
template <int BM, int BN, int WAVES_M, int NW, int KS, int PF, int AMODE_, int BKN, int ELT>
__global__ __launch_bounds__(64 * NW, 1) void conv_igemm_x3(ConvArgs a) {
    launch_stamp(a, false);
    conv_x3_tile<BM, BN, WAVES_M, NW, KS, PF, AMODE_, BKN, ELT>(
        a, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), gridDim.x, gridDim.y,
        gridDim.x * gridDim.y * gridDim.z);
    launch_stamp(a, true);
}

// Persistent form (s2v_conv_params.grid_cap, a.vgrid_*): gridDim.x blocks, block b running tiles b,
// b + gridDim.x, ...; gridDim.x is a multiple of 8, so every tile of a block has the block's XCD
// (b & 7) in the tile order's sense.  A kernel of its own: folding the loop (or a branch to it) into
// conv_igemm_x3 cost every one-block-per-tile launch 3-10 % (LNet 11.4 -> 11.9 ms, enhance 18.0 ->
// 19.8 ms, MI355X A/B of the builds, r03).
template <int BM, int BN, int WAVES_M, int NW, int KS, int PF, int AMODE_, int BKN, int ELT>
__global__ __launch_bounds__(64 * NW, 1) void conv_igemm_x3_persist(ConvArgs a) {
    launch_stamp(a, false);
    const int total = a.vgrid_x * a.vgrid_y * a.vgrid_z;
#pragma unroll 1
    for (int L = blockIdx.x; L < total; L += gridDim.x) {
        conv_x3_tile<BM, BN, WAVES_M, NW, KS, PF, AMODE_, BKN, ELT, false>(a, L, a.vgrid_x, a.vgrid_y, total);
        __syncthreads();     // the epilogue's LDS reads end before the next tile's operand stores
    }
    launch_stamp(a, true);
}

// Grouped form (s2v_conv2d_group): member p of the group runs the blocks [start[p], start[p + 1]) as
// its own tile grid.  The member index is block-uniform; the ConvArgs are read from the kernarg
// segment at that index (scalar loads).
template <int BM, int BN, int WAVES_M, int NW, int KS, int PF, int ELT>
__global__ __launch_bounds__(64 * NW, 1) void conv_igemm_x3_group(ConvGroup g) {
    const int L = blockIdx.x;
    int p = 0;
#pragma unroll
    for (int i = 1; i < kConvGroupMax; ++i)
        if (i < g.n && L >= g.start[i]) p = i;
    conv_x3_tile<BM, BN, WAVES_M, NW, KS, PF, 4, 0, ELT, false>(g.a[p], L - g.start[p], g.gx[p], g.gy[p],
                                                         g.start[p + 1] - g.start[p]);
}

template <int BM, int BN, int WM, int NW, int KS, int PF, int ELT>
static bool launch_x3(const ConvArgs &a, int amode, bool bkn, dim3 grid, hipStream_t s) {
    constexpr int NT = 64 * NW;
    if constexpr (KS > 1) {
        // the deep-stage tiles exist for the buffer-load A path only (compile time: 2 instances, not 10)
        if (bkn || amode != 4) return false;
        conv_igemm_x3<BM, BN, WM, NW, KS, PF, 4, 0, ELT><<<grid, NT, 0, s>>>(a);
        return true;
    }
    if (bkn) {
        if constexpr (NW == 4) {
            if (amode == 0) conv_igemm_x3<BM, BN, WM, NW, KS, PF, 0, 1, ELT><<<grid, NT, 0, s>>>(a);
            else if (amode == 1) conv_igemm_x3<BM, BN, WM, NW, KS, PF, 1, 1, ELT><<<grid, NT, 0, s>>>(a);
            else conv_igemm_x3<BM, BN, WM, NW, KS, PF, 2, 1, ELT><<<grid, NT, 0, s>>>(a);
            return true;
        }
        return false;
    }
    switch (amode) {
        case 4:
            if constexpr (BM % (16 * NW) == 0) conv_igemm_x3<BM, BN, WM, NW, KS, PF, 4, 0, ELT><<<grid, NT, 0, s>>>(a);
            else return false;
            break;
        case 0: conv_igemm_x3<BM, BN, WM, NW, KS, PF, 0, 0, ELT><<<grid, NT, 0, s>>>(a); break;
        case 1: conv_igemm_x3<BM, BN, WM, NW, KS, PF, 1, 0, ELT><<<grid, NT, 0, s>>>(a); break;
        case 2: conv_igemm_x3<BM, BN, WM, NW, KS, PF, 2, 0, ELT><<<grid, NT, 0, s>>>(a); break;
        default: conv_igemm_x3<BM, BN, WM, NW, KS, PF, 3, 0, ELT><<<grid, NT, 0, s>>>(a); break;
    }
    return true;
}

// x3 kernel configurations (index = the host planner's tile id, conv.hip kX3Tiles)
// the persistent form exists for the 256x256 tile with buffer-load A (the ENet style encoder's
// layers; conv.hip only sets a.vgrid_* for that configuration)
constexpr bool x3_has_persist(int cfg, int amode, bool bkn) { return cfg == 0 && amode == 4 && !bkn; }

// The tile configurations are instantiated in three parts (conv_x3_{f16,bf16}{,_1,_2}.hip) so the six
// translation units compile in parallel: part 0 = configurations 0 - 5, 1 = 6 - 11, 2 = 12 - 14.
template <int ELT, int PART>
bool launch_conv_x3_part(int cfg, const ConvArgs &a, int amode, bool bkn, dim3 grid, hipStream_t s) {
    if constexpr (PART == 0) {
        switch (cfg) {
            case 0: return launch_x3<256, 256, 2, 8, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 1: return launch_x3<128, 128, 2, 8, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 2: return launch_x3<64, 128, 2, 8, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 3: return launch_x3<128, 64, 2, 4, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 4: return launch_x3<64, 64, 2, 4, 1, 1, ELT>(a, amode, bkn, grid, s);
            default: return launch_x3<128, 32, 4, 4, 1, 1, ELT>(a, amode, bkn, grid, s);
        }
    } else if constexpr (PART == 1) {
        switch (cfg) {
            case 6: return launch_x3<256, 128, 4, 8, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 7: return launch_x3<256, 64, 8, 8, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 8: return launch_x3<512, 128, 4, 8, 1, 1, ELT>(a, amode, bkn, grid, s);   // N = 128 layers
            // narrow-N tiles whose waves each cover 64 rows (r04): fewer LDS operand reads per MFMA than the
            // 256x64 / 128x32 tiles (A fragments reused over all of N): 64-channel layers at 256^2 / 512^2
            case 9: return launch_x3<512, 64, 8, 8, 1, 1, ELT>(a, amode, bkn, grid, s);
            case 10: return launch_x3<256, 64, 4, 4, 1, 1, ELT>(a, amode, bkn, grid, s);
            default: return launch_x3<256, 32, 4, 4, 1, 1, ELT>(a, amode, bkn, grid, s);
        }
    } else {
        // deep-stage 4-wave tiles (KS 4 / 2 / 2): fewer load round trips in latency-bound small grids
        switch (cfg) {
            case 12: return launch_x3<64, 64, 2, 4, 4, 1, ELT>(a, amode, bkn, grid, s);
            case 13: return launch_x3<128, 64, 2, 4, 2, 1, ELT>(a, amode, bkn, grid, s);
            default: return launch_x3<128, 32, 4, 4, 2, 1, ELT>(a, amode, bkn, grid, s);
        }
    }
}

template <int ELT>
int launch_conv_x3(int cfg, const ConvArgs &a, int amode, bool bkn, dim3 grid, hipStream_t s) {
    if (a.vgrid_x > 0) {
        // a persistent launch of a configuration without the persistent kernel would leave the output
        // unwritten: an error, never a silent no-op (the planner only sets vgrid_* where it exists)
        S2V_REQUIRE(x3_has_persist(cfg, amode, bkn),
                    "conv2d: persistent launch (grid_cap) of x3 configuration %d / A mode %d, which has no "
                    "persistent kernel", cfg, amode);
        conv_igemm_x3_persist<256, 256, 2, 8, 1, 1, 4, 0, ELT><<<grid, 512, 0, s>>>(a);
        return 0;
    }
    const bool ok = cfg < 6 ? launch_conv_x3_part<ELT, 0>(cfg, a, amode, bkn, grid, s)
                  : cfg < 12 ? launch_conv_x3_part<ELT, 1>(cfg, a, amode, bkn, grid, s)
                             : launch_conv_x3_part<ELT, 2>(cfg, a, amode, bkn, grid, s);
    // a configuration / A-mode pair without a kernel would leave the output unwritten: an error
    S2V_REQUIRE(ok, "conv2d: x3 configuration %d has no kernel for A mode %d%s", cfg, amode, bkn ? " (b_kn)" : "");
    return 0;
}

// grouped launches exist for the 4-wave 64x64 / 128x64 and the 8-wave 128x128 buffer-load tiles
constexpr bool x3_has_group(int cfg) { return cfg == 1 || cfg == 3 || cfg == 4; }

template <int ELT>
int launch_conv_x3_group(int cfg, const ConvGroup &g, dim3 grid, hipStream_t s) {
    switch (cfg) {
        case 0: conv_igemm_x3_group<256, 256, 2, 8, 1, 1, ELT><<<grid, 512, 0, s>>>(g); break;
        case 1: conv_igemm_x3_group<128, 128, 2, 8, 1, 1, ELT><<<grid, 512, 0, s>>>(g); break;
        case 6: conv_igemm_x3_group<256, 128, 4, 8, 1, 1, ELT><<<grid, 512, 0, s>>>(g); break;
        case 3: conv_igemm_x3_group<128, 64, 2, 4, 1, 1, ELT><<<grid, 256, 0, s>>>(g); break;
        case 4: conv_igemm_x3_group<64, 64, 2, 4, 1, 1, ELT><<<grid, 256, 0, s>>>(g); break;
        default: S2V_REQUIRE(false, "conv2d_group: x3 configuration %d has no grouped kernel", cfg);
    }
    return 0;
}

}  // namespace s2v
