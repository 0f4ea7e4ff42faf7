// 4-channel-input convolutions with a short K on exact fp32 MFMA (v_mfma_f32_32x32x2f32): ENet's
// conv_body_first (1x1 3(+1) -> 256 at 256^2, models/ENet.py:94) and its first StyleConv (3x3 over the x2-upsampled
// 4-channel low-res image, K = 36, -> 256 at 200^2, models/ENet.py:122, base_blocks.py:487-533).
//
// These layers write 0.66 / 1.07 GB per B = 16 launch and do 9 / 1 MACs per output byte: they are bound by their
// output stores.  As implicit GEMMs on the split-precision tiles they reached ~2 TB/s (one 256x256 block per CU
// alternating a short main loop with a long LDS-staged epilogue, 48 % of wave cycles waiting,
// profiles/r06_pmc_first_styleconv_shape.json), and as the fp32 VALU kernel (conv_smallk4) less: every FMA read its
// weight from LDS.  Here each wave owns 64 output channels for the whole block and keeps their filter in VGPRs
// (K/2 k-steps x 2 column blocks, 36 VGPRs at 3x3), a block walks TILES 32-pixel tiles of one image, and each tile
// is 2 K/2 MFMAs from A values the lanes gather straight from the 16-byte NHWC pixels (lane l: pixel l % 32, the
// channels of parity l / 32) to C fragments that are stored without staging: for each of the 16 C rows, lanes
// 0-31 write 32 consecutive channels of one pixel (one 128-byte line) and lanes 32-63 those of another.  Exact fp32
// in every precision mode (the products are fp32 MFMA: more precise than the split modes, the same as f32).
#include "conv_impl.hpp"

namespace s2v {

constexpr int kK4Tiles = 8;   // 32-pixel tiles per block

// PF: the next tile's A loads issued before this tile's MFMAs (software pipelining; more VGPRs)
template <int KT, bool PF>
__global__ __launch_bounds__(256) void conv_k4_mfma(ConvArgs a, int chunks) {
    constexpr int KS = 2 * KT;                        // k-steps of 2 over K = 4 KT
    constexpr int KW = KT == 9 ? 3 : 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const int g = blockIdx.x / chunks, chunk = blockIdx.x - (blockIdx.x / chunks) * chunks;   // image, pixel chunk
    const int bidx = g / a.n, img = g - (g / a.n) * a.n;
    const int hw = a.oh * a.ow;
    // waves over channels (64 each) x waves over the block's tiles: a narrow layer (Cout <= 64: GFPGAN's / GPEN's
    // 1x1 RGB input convs) gives all four waves their own tiles instead of leaving three idle
    const int WN = (a.cout + 63) / 64, WM = 4 / WN;
    const int wn = wave % WN, wm = wave / WN;
    if (wm >= WM) return;                             // (no barriers below)
    const int n0 = wn * 64;                           // this wave's 64 output channels: blocks n0 .. n0 + 31, + 32 ..
    // filter fragments: B[k][n] = W[n][k] for k = 2 s + lh, the wave's two 32-column blocks
    const float *__restrict__ w = a.wt + (long long)bidx * a.w_bs;
    float b[KS][2];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + 32 * j + li;
            b[s][j] = n < a.cout ? w[(long long)n * a.kpad + 2 * s + lh] : 0.f;
        }
    const Epi &e = a.epi;
    float sc[2], sh[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + 32 * j + li;
        sc[j] = (e.scale && n < a.cout) ? e.scale[n] : 1.f;
        sh[j] = (e.shift && n < a.cout) ? e.shift[n] : 0.f;
    }
    const float slope = e.act == S2V_ACT_RELU ? 0.f : (e.act == S2V_ACT_LRELU ? e.alpha : 1.f);
    const float *__restrict__ xb = a.x + (long long)bidx * a.x_bs + (long long)img * a.h * a.w * a.xcs;
    float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + (long long)img * hw * a.ycs;
    const float *__restrict__ pix = e.pix_add ? e.pix_add + ((long long)bidx * a.n + img) * hw : nullptr;
    bool bad = false;
    // A: pixel p0 + li, channels lh and lh + 2 of every tap (k = 4 tap + c: k-step 2 tap + u takes c = 2 u + lh)
    auto load_a = [&](int p0, f4 (&v)[KT]) {
        const int p = p0 + li;
        const int oy = p / a.ow, ox = p - (p / a.ow) * a.ow;
#pragma unroll
        for (int tap = 0; tap < KT; ++tap) {
            const int iy = oy - a.ph + tap / KW, ix = ox - a.pw + tap % KW;
            v[tap] = f4{0.f, 0.f, 0.f, 0.f};
            if (p < hw && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w)
                v[tap] = *(const f4 *)(xb + ((long long)iy * a.w + ix) * a.xcs);
        }
    };
    f4 vn[KT];
    if (PF) load_a((chunk * kK4Tiles + wm) * 32, vn);
#pragma unroll 1
    for (int t = wm; t < kK4Tiles; t += WM) {
        const int p0 = (chunk * kK4Tiles + t) * 32;
        if (p0 >= hw) break;
        f4 vc[KT];
        if (PF) {
#pragma unroll
            for (int tap = 0; tap < KT; ++tap) vc[tap] = vn[tap];
            if (t + WM < kK4Tiles && p0 + 32 * WM < hw) load_a(p0 + 32 * WM, vn);
        } else {
            load_a(p0, vc);
        }
        float av[KS];
#pragma unroll
        for (int tap = 0; tap < KT; ++tap) {
            av[2 * tap] = lh ? vc[tap].y : vc[tap].x;
            av[2 * tap + 1] = lh ? vc[tap].w : vc[tap].z;
        }
        floatx16 acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], b[s][j], acc[j], 0, 0, 0);
        // C: column li of each 32-column block, rows (r & 3) + 8 (r >> 2) + 4 lh of the tile.  One 64-bit row base
        // per tile and 32-bit row steps; the pixel's noise loaded once for both column blocks; bounds checks only in
        // an image's last, partial tile (the per-value index / address VALU had made the epilogue the kernel's bound)
        const bool full = p0 + 32 <= hw;
        const bool jv1 = n0 + 32 < a.cout;            // (cout % 32 == 0: whole blocks)
        float *__restrict__ yt = yb + (long long)(p0 + 4 * lh) * a.ycs + n0 + li;
        const float *__restrict__ pt = pix ? pix + p0 + 4 * lh : nullptr;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int dr = (r & 3) + 8 * (r >> 2);
            if (!full && p0 + 4 * lh + dr >= hw) continue;
            const float pv = pt ? e.pix_w * pt[dr] : 0.f;
            float *__restrict__ yr = yt + dr * a.ycs;
            float v0 = fast_act(fmaf(acc[0][r], sc[0], sh[0]) + pv, e.act, slope);
            yr[0] = v0;
            bad |= !__builtin_isfinite(v0);
            if (jv1) {
                float v1 = fast_act(fmaf(acc[1][r], sc[1], sh[1]) + pv, e.act, slope);
                yr[32] = v1;
                bad |= !__builtin_isfinite(v1);
            }
        }
    }
    if (bad && a.nonfinite) __hip_atomic_store(a.nonfinite, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// host launcher (conv.hip): one block per (batch entry x image, chunk of kK4Tiles x 32 pixels)
int launch_conv_k4(const ConvArgs &a, int batch, int kt, hipStream_t s) {
    const int hw = a.oh * a.ow;
    const int chunks = (int)cdiv(hw, 32 * kK4Tiles);
    const long long blocks = (long long)batch * a.n * chunks;
    S2V_REQUIRE(blocks < (1LL << 31), "conv_k4: grid too large");
    static const bool pf = [] { const char *e = getenv("S2V_K4_PF"); return e && atoi(e) != 0; }();
    if (kt == 9 && pf) conv_k4_mfma<9, true><<<(unsigned)blocks, 256, 0, s>>>(a, chunks);
    else if (kt == 9) conv_k4_mfma<9, false><<<(unsigned)blocks, 256, 0, s>>>(a, chunks);
    else if (pf) conv_k4_mfma<1, true><<<(unsigned)blocks, 256, 0, s>>>(a, chunks);
    else conv_k4_mfma<1, false><<<(unsigned)blocks, 256, 0, s>>>(a, chunks);
    return 0;
}

}  // namespace s2v
