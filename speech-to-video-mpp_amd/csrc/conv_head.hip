// Wide-filter small-Cout output heads on the split-precision MFMA: DNet's 7x7 64 -> 3 tanh output conv
// (models/DNet.py:77-86, FinalBlock2d base_blocks.py:444-457, 16 x 256^2) and LNet's 7x7 64 -> 3
// sigmoid head (models/LNet.py:77, 16 x 96^2).
//
// A Cout <= 4 conv is a GEMM with N = Cout: as an implicit GEMM it wastes the MFMA's N dimension, and
// as a direct VALU conv (conv_halo_small) it is bound by fp32 FMA issue and by re-staging the input
// in 4-channel chunks (each 256-byte NHWC pixel read 16 bytes at a time: 13x the input in fetched
// lines at the DNet head).  Here the filter column kx moves into N and the row ky into K:
//
//   P[p, (o, kx)] = sum_{ky, c} x[oy - ph + ky, x0 + p, c] * W[o, ky, kx, c]     (N = Cout * KS <= 32)
//   y[oy, x0 + q, o] = sum_kx P[q + kx, (o, kx)]                                 (shift-sum over kx)
//
// One block owns a strip of TW = 32 - KS + 1 output columns (32 input columns: two 16-row MFMA
// blocks x two 16-column filter blocks, one per wave) and a band of output rows; at 61 KB of LDS
// (7 x 32 x 64 split channels + P) two blocks share a CU, so one block's shift-sum / barrier phase
// runs under the other's MFMAs (64-column strips with one 123 KB block per CU: 173 vs ? us).  The KS input rows an output row reads live in an
// LDS ring, each staged ONCE per block as split hi | lo halves (the whole 32-channel slice of a pixel
// is one 128-byte row: every fetched line is used whole); an output row stages one new input row,
// prefetched into registers under the previous row's MFMAs.  The filter (K = KS * cin, N = 32) stays
// in VGPRs for the whole block as pre-split fragments (112 VGPRs per wave at KS = 7, cin = 64), so the row
// loop reads only LDS.  Products are split-fp32 (hi*hi + hi*lo + lo*hi on 16x16x32 MFMAs, fp32
// accumulate) exactly as the implicit-GEMM kernels (conv_x3_impl.hpp), and so are the activation
// pre-scale (x_scale), the weight pre-scale (acc_scale) and the non-finite flag of the range guard.
#include "conv_x3_impl.hpp"

namespace s2v {

constexpr int kHeadM = 32;    // input columns of a strip (2 MFMA row blocks of 16)
constexpr int kHeadT = kHeadM * 8;   // threads: 2 waves per row block (one per 16 filter columns)

// RPI output rows per loop iteration (1 or 2): with 2, the KS + 1 ring rows of two output rows are each read
// from LDS once and feed both rows' MFMA chains (six independent accumulators), and the P / barrier phase runs
// once per two rows
template <int ELT, int CO, int KS, int NCS, int RPI>
__global__ __launch_bounds__(kHeadT) void conv_head_x3(ConvArgs a, int strips, int th) {
    constexpr int RING = KS + RPI - 1;        // staged input rows
    constexpr int TW = kHeadM - KS + 1;       // output columns per strip
    constexpr int NSL = KS * NCS;             // K-slices: (ky, 32-channel slice)
    constexpr int SLB = kHeadM * 128;         // bytes of one 32-channel slice of a staged row
    constexpr int ROWB = NCS * SLB;           // bytes of one staged input row
    constexpr int PLD = 33;                   // P row pitch (floats)
    static_assert(CO * KS <= 32, "N = Cout * KS must fit two 16-column blocks");
    static_assert(TW * CO <= kHeadT, "one shift-sum output per thread");
    __shared__ __attribute__((aligned(16))) char ring[RING * ROWB];
    __shared__ float P[RPI][kHeadM * PLD];

    launch_stamp(a, false);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // wave w multiplies the strip's 16-row block w >> 1 by the 16 filter columns (w & 1) * 16 .. + 15
    const int mb = wave >> 1, nb = wave & 1;
    int b = blockIdx.x;
    const int strip = b % strips;
    b /= strips;
    const int bands = (a.oh + th - 1) / th;
    const int band = b % bands, img = b / bands;
    const int ox0 = strip * TW, oy0 = band * th;
    const int oy1 = min(oy0 + th, a.oh);
    const int base = oy0 - a.ph;              // input row of ring row 0
    const bool refl = a.pad_mode == S2V_PAD_REFLECT;
    // channel group blockIdx.y: channels [32 NCS g, 32 NCS (g + 1)) (a.splits groups; partial sums to the
    // split-K workspace, folded with the epilogue by splitk_reduce)
    const int cg = blockIdx.y, nsl_all = a.cin >> 5;
    const float *__restrict__ xb = a.x + (long long)img * a.h * a.w * a.xcs + 32 * NCS * cg;

    // ---- filter fragments of this wave's 16 columns: B[n][k], n = o * KS + kx (n >= CO * KS: zero),
    // K-slice s = ky * NCS + cs holds W[o][(ky * KS + kx) * cin + 32 (NCS g + cs) + k] = packed split row o,
    // 32-k group (ky * KS + kx) * cin / 32 + NCS g + cs
    const char *__restrict__ wtb = (const char *)a.wt;
    u32x4 bh[NSL], bl[NSL];
    {
        const int n = nb * 16 + (lane & 15);
        const int o = n / KS, kx = n - (n / KS) * KS;
#pragma unroll
        for (int s = 0; s < NSL; ++s) {
            const int ky = s / NCS, cs = s - (s / NCS) * NCS;
            u32x4 h = {0u, 0u, 0u, 0u}, l = {0u, 0u, 0u, 0u};
            if (o < CO) {
                const char *p = wtb + ((long long)o * a.kpad + (long long)((ky * KS + kx) * nsl_all + NCS * cg + cs) * 32) * 4 +
                                16 * (lane >> 4);
                h = *(const u32x4 *)p;
                l = *(const u32x4 *)(p + 64);
            }
            bh[s] = h;
            bl[s] = l;
        }
    }

    // ---- input rows: thread t stages channel octet t & 7 (slice (t & 7) >> 2, slot (t & 7) & 3) of
    // pixel t >> 3; with one 32-channel slice the upper four octets are idle
    const int sp = tid >> 3, so = tid & 7, scs = so >> 2, sq = so & 3;
    const bool sact = scs < NCS;
    int gx = ox0 - a.pw + sp;
    if (refl) gx = reflect_idx(gx, a.w);
    const bool xok = (unsigned)gx < (unsigned)a.w && sact;
    const float *__restrict__ xcol = xb + (long long)gx * a.xcs + 32 * scs + 8 * sq;
    // the last ring row an output row of this band reads: with RPI = 2 an odd band's last iteration stages one
    // row past it, which is never read and (under reflect padding of a small image) may reflect out of range
    const int rlast = (oy1 - oy0 - 1) + KS - 1;
    auto load_row = [&](int r, f4 (&v)[2]) {  // ring row r = input row base + r
        int gy = base + r;
        if (refl) gy = reflect_idx(gy, a.h);
        v[0] = f4{0.f, 0.f, 0.f, 0.f};
        v[1] = f4{0.f, 0.f, 0.f, 0.f};
        if (xok && r <= rlast && (unsigned)gy < (unsigned)a.h) {
            const float *src = xcol + (long long)gy * a.w * a.xcs;
            v[0] = *(const f4 *)src;
            v[1] = *(const f4 *)(src + 4);
        }
    };
    auto store_row = [&](int r, const f4 (&v)[2]) {
        if (!sact) return;
        u32x2 h0, l0, h1, l1;
        split4<ELT>(v[0] * a.x_scale, h0, l0);
        split4<ELT>(v[1] * a.x_scale, h1, l1);
        const u32x4 hi = {h0.x, h0.y, h1.x, h1.y}, lo = {l0.x, l0.y, l1.x, l1.y};
        const int off = (r % RING) * ROWB + scs * SLB + slot_off(sp, sq);
        *(u32x4 *)(ring + off) = hi;
        *(u32x4 *)(ring + (off ^ 64)) = lo;
    };
    {   // the first iteration's RING input rows: all loads in flight at once
        f4 v[RING][2];
#pragma unroll
        for (int r = 0; r < RING; ++r) load_row(r, v[r]);
#pragma unroll
        for (int r = 0; r < RING; ++r) store_row(r, v[r]);
    }
    __syncthreads();

    const int l16 = lane & 15;
    const int aoff = slot_off(mb * 16 + l16, lane >> 4);   // hi slot; lo = aoff ^ 64 (rows are 128-B multiples)
    bool bad = false;
    // shift-sum outputs: thread t owns strip column t / CO, channel t % CO (TW * CO <= 512); the plain
    // epilogue (scale, shift, activation) inline with its two per-channel values loaded once per block
    const Epi &e = a.epi;
    const bool plain = !e.nc_scale && !e.pix_add && !e.res && !e.post_mul && !e.dup_src;
    float *__restrict__ wsp = a.splits > 1 ? a.ws + (long long)cg * a.M * a.cout : nullptr;
    const int oq = tid / CO, oo = tid - (tid / CO) * CO;
    const bool owner = tid < TW * CO && ox0 + oq < a.ow;
    const float esc = (owner && e.scale) ? e.scale[oo] : 1.f, esh = (owner && e.shift) ? e.shift[oo] : 0.f;
    float *__restrict__ yrow = a.y + (long long)img * a.oh * a.ow * a.ycs + (long long)(ox0 + oq) * a.ycs + oo;
    for (int oy = oy0; oy < oy1; oy += RPI) {
        const int rr = oy - oy0;              // ring row of ky = 0 of the iteration's first output row
        const bool more = oy + RPI < oy1;
        f4 nxt[RPI][2];
        if (more) {                           // the next iteration's new input rows, under the MFMAs
#pragma unroll
            for (int j = 0; j < RPI; ++j) load_row(rr + RING + j, nxt[j]);
        }
        // the three split products of each row in separate accumulators: 3 RPI independent MFMA chains
        floatx4 acc[RPI][3];
#pragma unroll
        for (int j = 0; j < RPI; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) acc[j][q] = floatx4{0.f, 0.f, 0.f, 0.f};
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int t = 0; t < RING; ++t)
#pragma unroll
            for (int cs = 0; cs < NCS; ++cs) {
                const int ro = ((rr + t) % RING) * ROWB + cs * SLB;
                const u32x4 ah = *(const u32x4 *)(ring + ro + aoff), al = *(const u32x4 *)(ring + ro + (aoff ^ 64));
#pragma unroll
                for (int j = 0; j < RPI; ++j) {
                    const int ky = t - j;     // ring row t is filter row t - j of output row oy + j
                    if (ky < 0 || ky >= KS) continue;
                    const int s = ky * NCS + cs;
                    acc[j][0] = mfma16x16<ELT>(al, bh[s], acc[j][0]);
                    acc[j][1] = mfma16x16<ELT>(ah, bl[s], acc[j][1]);
                    acc[j][2] = mfma16x16<ELT>(ah, bh[s], acc[j][2]);
                }
            }
        __builtin_amdgcn_s_setprio(0);
        // C layout: column lane & 15, rows 4 (lane >> 4) + r of the wave's 16-row block
#pragma unroll
        for (int j = 0; j < RPI; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                P[j][(mb * 16 + 4 * (lane >> 4) + r) * PLD + nb * 16 + l16] =
                    ((acc[j][0][r] + acc[j][1][r]) + acc[j][2][r]) * a.acc_scale;
        __syncthreads();                      // P complete; ring rows rr .. rr + RPI - 1 no longer read
        if (owner) {
#pragma unroll
            for (int j = 0; j < RPI; ++j) {
                if (oy + j >= oy1) break;
                float v = 0.f;
#pragma unroll
                for (int kx = 0; kx < KS; ++kx) v += P[j][(oq + kx) * PLD + oo * KS + kx];
                bad |= !__builtin_isfinite(v);
                const int oyj = oy + j;
                if (wsp) wsp[(long long)((img * a.oh + oyj) * a.ow + ox0 + oq) * a.cout + oo] = v;
                else if (plain) yrow[(long long)oyj * a.ow * a.ycs] = apply_act(v * esc + esh, e.act, e.alpha);
                else store_epilogue(a, 0, (img * a.oh + oyj) * a.ow + ox0 + oq, oo, v);
            }
        }
        if (more) {                           // into the ring slots of rows rr .. rr + RPI - 1
#pragma unroll
            for (int j = 0; j < RPI; ++j) store_row(rr + RING + j, nxt[j]);
        }
        __syncthreads();                      // P reads done; the new ring rows visible
    }
    if (bad && a.nonfinite) __hip_atomic_store(a.nonfinite, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    launch_stamp(a, true);
}

template <int ELT, int CO, int RPI>
static int launch_head_rpi(const ConvArgs &a, int ks, int ncs, dim3 grid, int strips, int th, hipStream_t s) {
    if (ks == 7 && ncs == 2) conv_head_x3<ELT, CO, 7, 2, RPI><<<grid, kHeadT, 0, s>>>(a, strips, th);
    else if (ks == 7 && ncs == 1) conv_head_x3<ELT, CO, 7, 1, RPI><<<grid, kHeadT, 0, s>>>(a, strips, th);
    else if (ks == 5 && ncs == 2) conv_head_x3<ELT, CO, 5, 2, RPI><<<grid, kHeadT, 0, s>>>(a, strips, th);
    else if (ks == 5 && ncs == 1) conv_head_x3<ELT, CO, 5, 1, RPI><<<grid, kHeadT, 0, s>>>(a, strips, th);
    else S2V_REQUIRE(false, "conv_head_x3: no kernel for a %dx%d filter over %d channels", ks, ks, 32 * ncs);
    return 0;
}

// S2V_HEAD_RPI: output rows per loop iteration (1 or 2, default 2)
static int head_rpi() {
    static const int r = [] { const char *e = getenv("S2V_HEAD_RPI"); return e && atoi(e) == 1 ? 1 : 2; }();
    return r;
}

template <int ELT, int CO>
static int launch_head_co(const ConvArgs &a, int ks, int ncs, dim3 grid, int strips, int th, hipStream_t s) {
    return head_rpi() == 1 ? launch_head_rpi<ELT, CO, 1>(a, ks, ncs, grid, strips, th, s)
                           : launch_head_rpi<ELT, CO, 2>(a, ks, ncs, grid, strips, th, s);
}

// host launcher (conv.hip): prec 1 = bf16x3, 2 = f16x3
// ncs: 32-channel slices per block (1 or 2); a.splits channel groups of 32 ncs channels
int launch_conv_head_x3(const ConvArgs &a, int prec, int co, int ks, int ncs, int th, hipStream_t s) {
    const int tw = kHeadM - ks + 1;
    const int strips = (int)cdiv(a.ow, tw);
    const int bands = (int)cdiv(a.oh, th);
    const dim3 grid((unsigned)((long long)a.n * bands * strips), (unsigned)a.splits);
#define S2V_HEAD(ELT)                                                                         \
    switch (co) {                                                                             \
        case 1: return launch_head_co<ELT, 1>(a, ks, ncs, grid, strips, th, s);              \
        case 2: return launch_head_co<ELT, 2>(a, ks, ncs, grid, strips, th, s);              \
        case 3: return launch_head_co<ELT, 3>(a, ks, ncs, grid, strips, th, s);              \
        default: return launch_head_co<ELT, 4>(a, ks, ncs, grid, strips, th, s);             \
    }
    if (prec == S2V_PREC_BF16X3) { S2V_HEAD(0) }
    S2V_HEAD(1)
#undef S2V_HEAD
}

}  // namespace s2v
