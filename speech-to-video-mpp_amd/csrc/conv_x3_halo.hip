// Spatially tiled 3x3 split-precision convolution with the input halo staged once per channel slice
// (conv_x3_halo).
//
// Why: the implicit-GEMM tiles (conv_x3_impl.hpp, conv_x3_nar.hip) load a K-slice of A per filter tap,
// so a 3x3 conv streams its input nine times from L2 into the CU.  At 64 output channels that is 40 KB
// of global -> register traffic per 256 x 64 x 32 K-slice (192 MFMAs per block), and the narrow layers
// run at the L2 -> CU rate, not the MFMA rate: a variant that also loaded B per wave (6 more
// wave-loads per slice) was 1.4-1.5x slower, one without the A tile's LDS round trip no faster
// (profiles/r05_nar_sweep.txt).  Here a block owns a 4-row x 64-column patch of output pixels
// (BM = 256, one wave per output row) and BN = 64 output channels.  Per 32-channel slice it loads the
// (4 + 2) x (64 + 2) input halo once (50.7 KB, 1.55x the patch instead of 9x), splits it into hi | lo
// halves once, stores it to LDS, and runs the nine taps' MFMAs on shifted views of it; only the 8 KB
// of pre-split weights per tap still come from L2 (double-buffered LDS stages, one barrier per tap).
// The next channel slice's halo is loaded into registers during the first taps.
//
// Conditions (conv.hip halo_ok): 3x3, stride 1, dilation 1, zero padding 1, direct input, cin % 32 == 0,
// packed weights over whole 64-row slabs, 2^31-byte offsets, no pooled epilogue; ragged images run
// partly empty last patches (the planner requires >= 85 % of the patch grid to be image).  Same products and the same per-slice MFMA order as conv_igemm_x3, but the K order is
// channel-slice major over taps in the natural order (conv_x3_impl's kperm order is the same: tap
// fastest), so results equal the LDS tiles bit for bit (tests/test_ops_gpu.py).
#include "conv_x3_impl.hpp"

namespace s2v {

// TH output rows per patch, WN waves per row each owning 64 of the BN = 64 WN output channels
// (TH 4 / WN 1: 256 threads, two blocks per CU; TH 8 / WN 1 and TH 4 / WN 2: 512 threads, one block per
// CU, the halo's edge rows resp. the halo itself amortised over twice the outputs)
template <int ELT, int TH, int WN>
__global__ __launch_bounds__(64 * TH * WN, TH * WN == 4 ? 2 : 1) void conv_x3_halo(ConvArgs a) {
    launch_stamp(a, false);
    constexpr int NT = 64 * TH * WN;
    constexpr int TW = 64, BN = 64 * WN, TM16 = TW / 16, TN16 = 4, RS = NT / 8, BR = BN / RS;
    constexpr int HW_ = TW + 2, HPX = (TH + 2) * HW_;   // halo row width, pixels
    constexpr int ITEMS = HPX * 4;                      // (pixel, 8-channel group) items per slice
    constexpr int NIT = (ITEMS + NT - 1) / NT;
    constexpr int HALO = HPX * 128;                     // split hi | lo halo of one 32-channel slice
    constexpr int BSUB = BN * 128;
    constexpr int CH = 64;
    constexpr int CBYTES = CH * (BN + 4) * 4;
    constexpr int OPS = HALO + 2 * BSUB;
    constexpr int SMEM = OPS > CBYTES ? OPS : CBYTES;
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    char *halo = smem;
    char *bst = smem + HALO;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WN, wc = wave - wr * WN;          // patch row, 64-channel column group
    const int l16 = lane & 15, kg = lane >> 4;
    const int total = gridDim.x * gridDim.y * gridDim.z;
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    int mt, nt, bz;
    {   // XCD-aware tile order, as conv_x3_tile: consecutive patches (one row band) on one XCD
        const int per = total >> 3, rem = total & 7;
        const int xcd = L & 7, idx = L >> 3;
        const int Lp = xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
        nt = Lp % gridDim.y;
        const int t = Lp / gridDim.y;
        mt = t % gridDim.x;
        bz = t / gridDim.x;
    }
    const int ntx = (a.ow + TW - 1) / TW, nty = (a.oh + TH - 1) / TH;   // ragged last patches: rows / columns
                                                                          // past the image are not stored
    const int img = mt / (ntx * nty), rr = mt - img * (ntx * nty);
    const int y0 = (rr / ntx) * TH, x0 = (rr % ntx) * TW;
    const int n0 = nt * BN;
    const int bidx = bz / a.splits, split = bz - bidx * a.splits;
    const float *__restrict__ x = a.x + (long long)bidx * a.x_bs;
    const char *__restrict__ wtb = (const char *)(a.wt + (long long)bidx * a.w_bs);
    const int nsl = a.cin >> 5;
    // split-K over channel slices (the host makes tps a multiple of 9)
    const int cs0 = split * (a.tps / 9), cs1 = min(nsl, cs0 + a.tps / 9);

    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)a.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void *)wtb, 0, (int)a.w_bytes, 0x00020000);
    const float *sc_base = a.in_scale ? a.in_scale + (long long)img * a.in_scale_ns : a.x;
    const __amdgpu_buffer_rsrc_t srs =
        __builtin_amdgcn_make_buffer_rsrc((void *)sc_base, 0, a.in_scale ? a.cin * 4 : 0, 0x00020000);

    // halo items of this thread: item q = tid + NT j -> pixel q >> 2, channel group q & 3 (= tid & 3)
    int hoff[NIT];        // byte offset of the item's 8 channels at channel slice 0, or -1 (zeros)
    int hlds[NIT];        // LDS byte offset of its hi slot, or -1 (no item)
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
        const int q = tid + NT * j;
        hoff[j] = -1;
        hlds[j] = -1;
        if (q < ITEMS) {
            const int px = q >> 2, grp = q & 3;
            const int hy = px / HW_, hx = px - hy * HW_;
            const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
            hlds[j] = slot_off(px, grp);
            if ((unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w)
                hoff[j] = (int)((((long long)img * a.h + iy) * a.w + ix) * a.xcs + 8 * grp) * 4;
        }
    }
    int boff[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) boff[j] = ((n0 + (tid >> 3) + RS * j) * a.kpad) * 4 + (tid & 7) * 16;

    floatx4 acc[TM16][TN16];
#pragma unroll
    for (int i = 0; i < TM16; ++i)
#pragma unroll
        for (int j = 0; j < TN16; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

    f4 hr[NIT][2];        // the next channel slice's halo items
    f4 s0, s1;            // its modulation s[n, c] (channels 8 (tid & 3) .. + 7 of the slice)
    auto issue_halo = [&](int cs) {
        const int co = cs * 128;
#pragma unroll
        for (int j = 0; j < NIT; ++j) {
            const int vo = hoff[j] >= 0 ? hoff[j] + co : (int)0x80000000;
            hr[j][0] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 0, 0));
            hr[j][1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo + 16, 0, 0));
        }
        const int so = a.in_scale ? (cs * 32 + 8 * (tid & 3)) * 4 : (int)0x80000000;
        s0 = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(srs, so, 0, 0));
        s1 = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(srs, so + 16, 0, 0));
    };
    auto store_halo = [&]() {
#pragma unroll
        for (int j = 0; j < NIT; ++j) {
            f4 v0 = hr[j][0], v1 = hr[j][1];
            if (a.in_scale) {
                v0 *= s0;
                v1 *= s1;
            }
            if (a.pre_act) {
                pre_act4(a, v0);
                pre_act4(a, v1);
            }
            if (a.x_scale != 1.f) {
                v0 *= a.x_scale;
                v1 *= a.x_scale;
            }
            u32x2 h0, lo0, h1, lo1;
            split4<ELT>(v0, h0, lo0);
            split4<ELT>(v1, h1, lo1);
            if (hlds[j] >= 0) {
                *(u32x4 *)(halo + hlds[j]) = u32x4{h0.x, h0.y, h1.x, h1.y};
                *(u32x4 *)(halo + (hlds[j] ^ 64)) = u32x4{lo0.x, lo0.y, lo1.x, lo1.y};
            }
        }
    };
    u32x4 rb[BR];
    auto issue_b = [&](int cs, int tap) {
        const int kt = tap * nsl + cs;
#pragma unroll
        for (int j = 0; j < BR; ++j)
            rb[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, boff[j], kt * 128, 0));
    };
    auto store_b = [&](char *Bs) {
#pragma unroll
        for (int j = 0; j < BR; ++j) *(u32x4 *)(Bs + slot_off((tid >> 3) + RS * j, tid & 7)) = rb[j];
    };
    // tap (ky, kx): row block i of wave w reads halo pixels (w + ky) * HW_ + 16 i + kx + l16
    auto mma = [&](const char *Bs, int ky, int kx) {
        u32x4 bh[TN16], bl[TN16];
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
            const char *p = Bs + (wc * 64 + j * 16 + l16) * 128;
            const int hs = (kg ^ swz(l16)) << 4;
            bh[j] = *(const u32x4 *)(p + hs);
            bl[j] = *(const u32x4 *)(p + (hs ^ 64));
        }
        const int pbase = (wr + ky) * HW_ + kx + l16;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM16; ++i) {
            const int px = pbase + 16 * i;
            const int hs = (kg ^ swz(px)) << 4;
            const u32x4 ah = *(const u32x4 *)(halo + px * 128 + hs);
            const u32x4 al = *(const u32x4 *)(halo + px * 128 + (hs ^ 64));
#pragma unroll
            for (int j = 0; j < TN16; ++j) {
                acc[i][j] = mfma16x16<ELT>(al, bh[j], acc[i][j]);
                acc[i][j] = mfma16x16<ELT>(ah, bl[j], acc[i][j]);
                acc[i][j] = mfma16x16<ELT>(ah, bh[j], acc[i][j]);
            }
        }
        __builtin_amdgcn_s_setprio(0);
    };

    if (cs1 > cs0) {
        // prologue: channel slice cs0's halo and its tap-0 weights
        issue_b(cs0, 0);
        issue_halo(cs0);
        store_b(bst);
        store_halo();
        __syncthreads();
        int g = 0;                                    // global tap step (B stage g & 1)
#pragma unroll 1
        for (int cs = cs0; cs < cs1; ++cs) {
            const int csn = min(cs + 1, cs1 - 1);     // past the last slice: re-load it, unused
#pragma unroll 1
            for (int t = 0; t < 9; ++t, ++g) {
                // next weights first: their LDS store below then waits for these two loads only
                // (loads count in issue order); the next halo goes out at tap 0, so the store at
                // the end of tap 1 is the first to drain it
                if (t < 8) issue_b(cs, t + 1);
                else issue_b(csn, 0);
                if (t == 0) issue_halo(csn);
                __builtin_amdgcn_sched_barrier(0);
                mma(bst + (g & 1) * BSUB, t / 3, t - (t / 3) * 3);
                store_b(bst + ((g + 1) & 1) * BSUB);
                if (t == 8) {
                    __syncthreads();                  // every wave's tap-8 reads of the halo are done
                    store_halo();
                }
                __syncthreads();
            }
        }
    }
    if (a.nonfinite) {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < TM16; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) bad |= !__builtin_isfinite(acc[i][j][r]);
        if (bad) __hip_atomic_store(a.nonfinite, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // chunk c0 = wave row c0 / 64 of the patch: 64 consecutive output pixels
    const long long mrow0 = ((long long)img * a.oh + y0) * a.ow + x0;
    epilogue_tile_map<TH * TW, BN, TH * WN, CH>(
        a, (float *)smem, tid, n0, bz, bidx,
        [&](float *Cs, int c0) {
            constexpr int LDC = BN + 4;
            if (wr * 64 != c0) return;
#pragma unroll
            for (int i = 0; i < TM16; ++i)
#pragma unroll
                for (int j = 0; j < TN16; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        Cs[(i * 16 + 4 * kg + r) * LDC + wc * 64 + j * 16 + l16] = acc[i][j][r] * a.acc_scale;
        },
        [&](int c0) { return (int)(mrow0 + (long long)(c0 / 64) * a.ow); },
        [&](int c0) { return y0 + c0 / 64 < a.oh ? min(CH, a.ow - x0) : 0; });
    launch_stamp(a, true);
}

template <int ELT>
int launch_conv_x3_halo(const ConvArgs &a, int th, int wn, dim3 grid, hipStream_t s) {
    if (wn == 2) conv_x3_halo<ELT, 4, 2><<<grid, 512, 0, s>>>(a);
    else if (th == 8) conv_x3_halo<ELT, 8, 1><<<grid, 512, 0, s>>>(a);
    else conv_x3_halo<ELT, 4, 1><<<grid, 256, 0, s>>>(a);
    return 0;
}

template int launch_conv_x3_halo<0>(const ConvArgs &, int, int, dim3, hipStream_t);
template int launch_conv_x3_halo<1>(const ConvArgs &, int, int, dim3, hipStream_t);

}  // namespace s2v
