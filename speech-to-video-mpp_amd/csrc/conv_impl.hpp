// Device-side pieces shared by the fp32 (conv.hip) and split-bf16 (conv_x3.hip) implicit-GEMM
// convolutions: argument block, epilogue, tap mapping and the A/B operand gather loaders.
#pragma once
#include "common.hpp"

namespace s2v {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));   // register-native 16-byte vector

struct Epi {
    const float *scale, *shift, *nc_scale, *pix_add, *res;
    int nc_ns;
    float pix_w;
    int res_cs, res_h, res_w, res_oy, res_ox, res_after, res_simple;
    int act;
    float alpha;
    const float *post_mul, *post_add;   // SFT on channels >= post_c0 (s2v_conv_params)
    int post_cs, post_c0;
    const float *dup_src, *dup_bias;    // second output at channel offset dup_off
    float dup_a;
    int dup_cs, dup_off;
};

struct ConvArgs {
    const float *x;
    int n, h, w, cin, xcs;
    int in_mode, pad_mode, pre_act;
    float pre_alpha;
    const float *in_scale;
    int in_scale_ns;
    int kh, kw, sh, sw, ph, pw, dh, dw;
    const float *wt;
    int kpad, cout, ldb;
    float *y;
    int oh, ow, ycs;
    Epi epi;
    long long x_bs, w_bs, y_bs, res_bs;
    int M, K, ktiles, splits, tps;
    float *ws;
    int y_step, y_h, y_w;   // strided (polyphase) output, y_step > 1
    int d2s_c;              // depth-to-space output (s2v_conv_params.d2s_cout), 0 = off
    float acc_scale;        // accumulator factor before the epilogue (1 / the split weights' pre-scale)
    unsigned x_bytes, w_bytes;   // buffer-load extents of one batch slab of x / of the weights (AMODE 4)
    int pool;               // 2x2 average-pooled output: M runs over 2x2 output quads (quad-major),
                            // the epilogue writes act(v) averaged over each quad to pixel m / 4
    unsigned long long *stamps;            // launch timer (s2v_conv_params.stamps), or null
    const unsigned long long *stamp_ctr;
    int stamp_slot, stamp_stride, stamp_reps;
    float x_scale;          // split-precision A operand pre-scale (power of two; 1 = none)
    int *nonfinite;         // set to 1 when an accumulator is non-finite (or null)
    int vec4;               // the tile epilogues may write 4-channel quads (cout, ycs, y_bs multiples of 4, 16-byte
                            // aligned y / scale / shift / res / nc_scale rows: conv.hip epi_vec4)
    int vgrid_x, vgrid_y, vgrid_z;   // x3 persistent launch: the tile grid gridDim.x blocks loop over
                                     // (s2v_conv_params.grid_cap); vgrid_x == 0: one block per tile
};

// A group of independent convolutions launched as one kernel (s2v_conv2d_group): member p owns the
// blocks [start[p], start[p + 1]) of the launch, laid out as its own (gx, gy, gz) tile grid; the
// split-K fold of the members with splits > 1 owns the reduce blocks [rstart[p], rstart[p + 1]).
constexpr int kConvGroupMax = 4;
struct ConvGroup {
    ConvArgs a[kConvGroupMax];
    int start[kConvGroupMax + 1];
    int gx[kConvGroupMax], gy[kConvGroupMax];
    int rstart[kConvGroupMax + 1];
    int vec[kConvGroupMax];
    int n;
};

// Launch timer: block start (atomic min) / end (atomic max) of the device real-time clock into the
// slot of the current replay.  One lane per block; vector-memory 64-bit atomics.
__device__ __forceinline__ void launch_stamp(const ConvArgs &a, bool end) {
    if (a.stamps == nullptr) return;
    if (threadIdx.x == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        const unsigned long long r = __hip_atomic_load(a.stamp_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long *p = a.stamps + 2 * ((long long)(r % (unsigned long long)a.stamp_reps) * a.stamp_stride +
                                                a.stamp_slot);
        if (end) atomicMax(p + 1, t);
        else atomicMin(p, t);
    }
}

// Element offset of output row m (flattened n, oy, ox) for channel 0.
__device__ __forceinline__ long long out_row(const ConvArgs &a, long long m) {
    if (a.y_step <= 1) return m * a.ycs;
    const int hw = a.oh * a.ow;
    const long long img = m / hw;
    const int rem = (int)(m - img * hw);
    const int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
    return ((img * a.y_h + (long long)oy * a.y_step) * a.y_w + (long long)ox * a.y_step) * a.ycs;
}

// Element offset of output column n relative to out_row(): n, or under depth-to-space
// (a.d2s_c > 0) the output channel n % d2s_c at the parity-class pixel cls = n / d2s_c
__device__ __forceinline__ long long out_col(const ConvArgs &a, int n) {
    if (a.d2s_c <= 0) return n;
    const int cls = n / a.d2s_c;
    return ((long long)(cls >> 1) * a.y_w + (cls & 1)) * a.ycs + (n - cls * a.d2s_c);
}

// pix_add element of output row m (conv pixel) and column n
__device__ __forceinline__ long long pix_index(const ConvArgs &a, int bidx, int m, int n) {
    if (a.d2s_c <= 0) return (long long)bidx * a.oh * a.ow * a.n + m;
    const int hw = a.oh * a.ow;
    const int img = m / hw, rem = m - img * hw;
    const int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
    const int cls = n / a.d2s_c;
    return (long long)bidx * a.y_h * a.y_w * a.n + ((long long)img * a.y_h + 2 * oy + (cls >> 1)) * a.y_w + 2 * ox +
           (cls & 1);
}

// EXTRA = false: a kernel that never carries the SFT / second-output extras (host-checked), so their
// registers are not allocated in it
template <bool EXTRA = true>
__device__ __forceinline__ void store_epilogue(const ConvArgs &a, int bidx, int m, int n, float v) {
    const Epi &e = a.epi;
    const int hw = a.oh * a.ow;
    int img = 0, oy = 0, ox = 0;
    if (e.nc_scale || (e.res && !e.res_simple)) {
        img = m / hw;
        int rem = m - img * hw;
        oy = rem / a.ow;
        ox = rem - oy * a.ow;
    }
    if (e.scale) v *= e.scale[n];
    if (e.nc_scale) v *= e.nc_scale[(long long)img * e.nc_ns + n];
    if (e.shift) v += e.shift[n];
    if (e.pix_add) v += e.pix_w * e.pix_add[pix_index(a, bidx, m, n)];
    float r = 0.f;
    if (e.res) {
        long long off = a.y_step > 1 ? out_row(a, m)     // in-place residual on a strided output
            : e.res_simple
            ? (long long)m * e.res_cs
            : ((long long)(img * e.res_h + oy + e.res_oy) * e.res_w + ox + e.res_ox) * e.res_cs;
        r = e.res[(long long)bidx * a.res_bs + off + n];
        if (!e.res_after) v += r;
    }
    v = apply_act(v, e.act, e.alpha);
    if (e.res && e.res_after) v += r;
    if (EXTRA && e.post_mul && n >= e.post_c0) {
        const long long q = (long long)m * e.post_cs + n - e.post_c0;
        v = v * e.post_mul[q] + e.post_add[q];
    }
    a.y[(long long)bidx * a.y_bs + out_row(a, m) + out_col(a, n)] = v;
    if (EXTRA && e.dup_src) {
        float d = e.dup_a * e.dup_src[(long long)m * e.dup_cs + n];
        if (e.dup_bias) d += e.dup_bias[n];
        a.y[(long long)bidx * a.y_bs + out_row(a, m) + e.dup_off + n] = apply_act(d, e.act, e.alpha);
    }
}

// Map an output pixel + filter tap to an input pixel; false -> zero padding.
__device__ __forceinline__ bool map_tap(const ConvArgs &a, int oy, int ox, int ky, int kx, int &iy, int &ix) {
    if (a.in_mode == S2V_IN_DIRECT) {
        iy = oy * a.sh - a.ph + ky * a.dh;
        ix = ox * a.sw - a.pw + kx * a.dw;
        if (a.pad_mode == S2V_PAD_REFLECT) {
            iy = reflect_idx(iy, a.h);
            ix = reflect_idx(ix, a.w);
            return true;
        }
        return (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    } else if (a.in_mode == S2V_IN_NEAREST_UP2) {
        int uy = oy * a.sh - a.ph + ky * a.dh;
        int ux = ox * a.sw - a.pw + kx * a.dw;
        if (a.pad_mode == S2V_PAD_REFLECT) {   // reflected in the upsampled frame (ParseNet, blocks.py:92-96)
            uy = reflect_idx(uy, 2 * a.h);
            ux = reflect_idx(ux, 2 * a.w);
        }
        if ((unsigned)uy >= (unsigned)(2 * a.h) || (unsigned)ux >= (unsigned)(2 * a.w)) return false;
        iy = uy >> 1;
        ix = ux >> 1;
        return true;
    } else {  // transposed
        int ty = oy + a.ph - ky * a.dh;
        int tx = ox + a.pw - kx * a.dw;
        if (ty < 0 || tx < 0) return false;
        iy = ty / a.sh;
        ix = tx / a.sw;
        return iy * a.sh == ty && ix * a.sw == tx && iy < a.h && ix < a.w;
    }
}

__device__ __forceinline__ float prologue(const ConvArgs &a, float v, int img, int c) {
    if (a.in_scale) v *= a.in_scale[(long long)img * a.in_scale_ns + c];
    if (a.pre_act) v = apply_act(v, a.pre_act, a.pre_alpha);
    return v;
}

// Branch-light activation for the epilogue hot path: NONE / RELU / LRELU are one select; the
// transcendental ones go through an out-of-line call so 64 unrolled copies stay small.
static __device__ __noinline__ float act_complex(float v, int act) { return apply_act(v, act, 0.f); }

__device__ __forceinline__ float fast_act(float v, int act, float slope) {
    if (act > S2V_ACT_LRELU) return act_complex(v, act);
    return v >= 0.f ? v : v * slope;
}

// A operand loaders.  AMODE 0: direct conv, zero padding, no prologue, cin % 32 == 0 (a whole
// K-slice lies in one filter tap: the tap offset is tile-uniform).  AMODE 1: any input mode,
// cin % 4 == 0 (one tap per float4).  AMODE 2: anything (scalar gather).
template <int AR, int AMODE>
struct ARows {
    long long base[AR];  // AMODE 0: element offset of (img, iy0, ix0) (may point outside the image)
    int iy0[AR], ix0[AR];
    int img[AR], oy[AR], ox[AR];
    bool ok[AR];
};

// tile rows rows[j] (j < AR): output pixel m0 + rows[j]
template <int AR, int AMODE>
__device__ __forceinline__ void a_rows_init_at(const ConvArgs &a, int m0, const int (&rows)[AR], ARows<AR, AMODE> &R) {
    const int hw = a.oh * a.ow;
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int m = m0 + rows[j];
        R.ok[j] = m < a.M;
        const int mm = R.ok[j] ? m : 0;
        int img, oy, ox;
        if (a.pool) {       // quad-major order: m = 4 * pooled pixel + (dy * 2 + dx)
            const int q = mm >> 2, hq = hw >> 2, wq = a.ow >> 1;
            img = q / hq;
            const int rq = q - img * hq;
            const int qy = rq / wq;
            oy = 2 * qy + ((mm >> 1) & 1);
            ox = 2 * (rq - qy * wq) + (mm & 1);
        } else {
            img = mm / hw;
            const int rem = mm - img * hw;
            oy = rem / a.ow;
            ox = rem - oy * a.ow;
        }
        R.img[j] = img;
        R.oy[j] = oy;
        R.ox[j] = ox;
        R.iy0[j] = oy * a.sh - a.ph;
        R.ix0[j] = ox * a.sw - a.pw;
        R.base[j] = AMODE == 3 ? (long long)img * a.h * a.w * a.xcs
                               : ((long long)(img * a.h + R.iy0[j]) * a.w + R.ix0[j]) * a.xcs;
    }
}

// rows m0 + ar + RS * j of the tile (RS = rows covered by one load pass of the block)
template <int AR, int AMODE, int RS = 32>
__device__ __forceinline__ void a_rows_init(const ConvArgs &a, int m0, int ar, ARows<AR, AMODE> &R) {
    int rows[AR];
#pragma unroll
    for (int j = 0; j < AR; ++j) rows[j] = ar + RS * j;
    a_rows_init_at<AR, AMODE>(a, m0, rows, R);
}

// pre-activation of 4 gathered values (NONE / RELU / LRELU: max(v, slope v) for slopes in [0, 1])
__device__ __forceinline__ void pre_act4(const ConvArgs &a, f4 &v) {
    const float sl = a.pre_act == S2V_ACT_RELU ? 0.f : a.pre_alpha;
    v.x = v.x >= 0.f ? v.x : v.x * sl;
    v.y = v.y >= 0.f ? v.y : v.y * sl;
    v.z = v.z >= 0.f ? v.z : v.z * sl;
    v.w = v.w >= 0.f ? v.w : v.w * sl;
}

// prologue of 4 gathered channels [c, c + 4) of tile row j: StyleGAN2 input modulation s[n, c]
// (zero padding stays zero), then the pre-activation (NONE / RELU / LRELU only on these paths)
template <int AR, int AMODE>
__device__ __forceinline__ void prologue4(const ConvArgs &a, const ARows<AR, AMODE> &R, int j, int c, f4 &v) {
    if (a.in_scale) v *= *(const f4 *)(a.in_scale + (long long)R.img[j] * a.in_scale_ns + c);
    if (a.pre_act) {
        const float sl = a.pre_act == S2V_ACT_RELU ? 0.f : a.pre_alpha;
        v.x = v.x >= 0.f ? v.x : v.x * sl;
        v.y = v.y >= 0.f ? v.y : v.y * sl;
        v.z = v.z >= 0.f ? v.z : v.z * sl;
        v.w = v.w >= 0.f ? v.w : v.w * sl;
    }
}

// AMODE 0 / 3 gather of one K-slice: filter tap (ky, kx), channels [c, c + 4) per row (the tap is
// tile-uniform: scalar math).  PRO = false leaves the prologue to the caller (the bf16x3 kernel applies it when it stores the
// slice to LDS, so the global loads stay in flight under the MFMAs instead of being waited for
// right after issue)
template <int AR, int AMODE, bool PRO = true>
__device__ __forceinline__ void load_a_tap(const ConvArgs &a, const float *__restrict__ x, int ky, int kx, int c,
                                           const ARows<AR, AMODE> &R, f4 (&ra)[AR]) {
    const int dy = ky * a.dh, dx = kx * a.dw;
    if (AMODE == 0) {
        const long long toff = ((long long)dy * a.w + dx) * a.xcs + c;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const bool ok = R.ok[j] && (unsigned)(R.iy0[j] + dy) < (unsigned)a.h &&
                            (unsigned)(R.ix0[j] + dx) < (unsigned)a.w;
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (ok) v = *(const f4 *)(x + R.base[j] + toff);
            ra[j] = v;
        }
    } else {
        // AMODE 3: per-row index math — reflect padding and / or a nearest-x2 upsampled input
        // (tap coordinates in the upsampled frame, source pixel = coordinate >> 1); the mode
        // branches are tile-uniform
        const bool up = a.in_mode == S2V_IN_NEAREST_UP2, refl = a.pad_mode == S2V_PAD_REFLECT;
        const int uh = up ? 2 * a.h : a.h, uw = up ? 2 * a.w : a.w, sh = up ? 1 : 0;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            int uy = R.iy0[j] + dy, ux = R.ix0[j] + dx;
            bool ok = R.ok[j];
            if (refl) {
                uy = reflect_idx(uy, uh);
                ux = reflect_idx(ux, uw);
            } else {
                ok = ok && (unsigned)uy < (unsigned)uh && (unsigned)ux < (unsigned)uw;
            }
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (ok) v = *(const f4 *)(x + R.base[j] + ((long long)(uy >> sh) * a.w + (ux >> sh)) * a.xcs + c);
            ra[j] = v;
        }
    }
    if (PRO && (a.in_scale || a.pre_act)) {
#pragma unroll
        for (int j = 0; j < AR; ++j) prologue4<AR, AMODE>(a, R, j, c, ra[j]);
    }
}

template <int AR, int AMODE>
__device__ __forceinline__ void load_a(const ConvArgs &a, const float *__restrict__ x, int kt, int ak,
                                       const ARows<AR, AMODE> &R, f4 (&ra)[AR]) {
    const int kbase = kt * 32;
    if (AMODE == 0 || AMODE == 3) {
        const int tap = kbase / a.cin;
        const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
        load_a_tap<AR, AMODE>(a, x, ky, kx, kbase - tap * a.cin + ak, R, ra);
    } else if (AMODE == 1) {
        const int k = kbase + ak;
        const bool kok = k < a.K;
        const int tap = k / a.cin;
        const int c = k - tap * a.cin;
        const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            f4 v = {0.f, 0.f, 0.f, 0.f};
            int iy, ix;
            if (R.ok[j] && kok && map_tap(a, R.oy[j], R.ox[j], ky, kx, iy, ix)) {
                v = *(const f4 *)(x + ((long long)(R.img[j] * a.h + iy) * a.w + ix) * a.xcs + c);
                if (a.in_scale || a.pre_act) {
                    v.x = prologue(a, v.x, R.img[j], c);
                    v.y = prologue(a, v.y, R.img[j], c + 1);
                    v.z = prologue(a, v.z, R.img[j], c + 2);
                    v.w = prologue(a, v.w, R.img[j], c + 3);
                }
            }
            ra[j] = v;
        }
    } else {
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            float vv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = kbase + ak + e;
                float v = 0.f;
                if (R.ok[j] && k < a.K) {
                    const int tap = k / a.cin;
                    const int c = k - tap * a.cin;
                    const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
                    int iy, ix;
                    if (map_tap(a, R.oy[j], R.ox[j], ky, kx, iy, ix)) {
                        v = x[((long long)(R.img[j] * a.h + iy) * a.w + ix) * a.xcs + c];
                        v = prologue(a, v, R.img[j], c);
                    }
                }
                vv[e] = v;
            }
            ra[j] = f4{vv[0], vv[1], vv[2], vv[3]};
        }
    }
}

template <int BN, int BR, int BKN>
__device__ __forceinline__ void load_b(const ConvArgs &a, const float *__restrict__ wt, int kt, int n0, int tid,
                                       f4 (&rb)[BR]) {
    const int kbase = kt * 32;
    if (!BKN) {
        const int ar = tid >> 3, ak = (tid & 7) * 4;
        const float *p = wt + (long long)(n0 + ar) * a.kpad + kbase + ak;
#pragma unroll
        for (int j = 0; j < BR; ++j) rb[j] = *(const f4 *)(p + (long long)32 * j * a.kpad);
    } else {
        constexpr int NV = BN / 4, RPP = 256 / NV;
        const int kr = tid / NV, nn = (tid - (tid / NV) * NV) * 4;
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const int k = kbase + kr + RPP * j;
            const int n = n0 + nn;
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (k < a.K) {
                const float *src = wt + (long long)k * a.ldb + n;
                if (n + 3 < a.cout) {
                    v = *(const f4 *)src;
                } else {
                    if (n < a.cout) v.x = src[0];
                    if (n + 1 < a.cout) v.y = src[1];
                    if (n + 2 < a.cout) v.z = src[2];
                }
            }
            rb[j] = v;
        }
    }
}

// Epilogue of one BM x BN output tile.  The accumulators are staged through LDS (``Cs``, at least
// CH*(BN+4) floats) CH rows at a time by ``stage(Cs, c0)`` (rows [c0, c0 + CH) of the tile, static
// register indices), then every thread walks the chunk row by row (consecutive threads ->
// consecutive output channels: coalesced stores).  Split-K launches write raw partial sums to the
// workspace instead.
// ``base(c0)``: the GEMM row (output pixel m) of chunk row 0 — a chunk's CH rows are consecutive m;
// ``rows(c0)``: how many of them exist.  epilogue_tile_fn is the linear tile (rows m0, m0 + 1, ...);
// the spatial halo tile (conv_x3_halo.hip) maps each 64-row chunk to one output row segment.
// EXTRA = false drops the SFT / second-output code (store_epilogue<EXTRA>).
template <int BM, int BN, int NW, int CH, bool EXTRA = true, class Stage, class Base, class Rows>
__device__ __forceinline__ void epilogue_tile_map(const ConvArgs &a, float *Cs, int tid, int n0, int bz, int bidx,
                                                  Stage stage, Base base, Rows rows);

template <int BM, int BN, int NW, int CH, bool EXTRA = true, class Stage>
__device__ __forceinline__ void epilogue_tile_fn(const ConvArgs &a, float *Cs, int tid, int m0, int n0, int bz,
                                                 int bidx, Stage stage) {
    const int mlim = min(BM, a.M - m0);
    epilogue_tile_map<BM, BN, NW, CH, EXTRA>(a, Cs, tid, n0, bz, bidx, stage, [&](int c0) { return m0 + c0; },
                                             [&](int c0) { return min(CH, mlim - c0); });
}

template <int BM, int BN, int NW, int CH, bool EXTRA, class Stage, class Base, class Rows>
__device__ __forceinline__ void epilogue_tile_map(const ConvArgs &a, float *Cs, int tid, int n0, int bz, int bidx,
                                                  Stage stage, Base base, Rows rows) {
    constexpr int NT = 64 * NW;
    constexpr int LDC = BN + 4;
    static_assert(CH % 16 == 0 && BM % CH == 0, "epilogue chunk");
    const Epi &e = a.epi;
    constexpr int TPR = BN < NT ? BN : NT;   // threads per tile row
    constexpr int RSTEP = NT / TPR;
    const int cn = tid % TPR;
    const int n = n0 + cn;
    const bool live = n < a.cout;
    const bool extra = EXTRA && (e.post_mul || e.dup_src);
    const bool simple = !e.nc_scale && !e.pix_add && (!e.res || e.res_simple) && !extra;
    const float sc = (live && e.scale) ? e.scale[n] : 1.f;
    const float sh = (live && e.shift) ? e.shift[n] : 0.f;
    const float slope = e.act == S2V_ACT_RELU ? 0.f : (e.act == S2V_ACT_LRELU ? e.alpha : 1.f);
    // 4-channel quads per thread (a.vec4): one LDS read, one 16-byte store and one address update per four
    // outputs instead of per output (the per-element index / act VALU was ~40 % of the non-MFMA vector work
    // of the 256x256 StyleConv launches, PMC profiles/r06_pmc_headline_conv.json)
    constexpr int TQ = BN / 4 < NT ? BN / 4 : NT;    // threads per tile row
    constexpr int RS4 = NT / TQ;
    const bool vq = a.vec4 && !a.pool && a.splits <= 1 && BN % 4 == 0 && (BN / 4) % TQ == 0 &&
                    (a.y_step > 1 ? !e.nc_scale && !e.post_mul && !e.dup_src : (!e.res || e.res_simple));
    const int cq = tid % TQ, nq = n0 + 4 * cq;
    const bool liveq = nq < a.cout;
    f4 sc4 = {1.f, 1.f, 1.f, 1.f}, sh4 = {0.f, 0.f, 0.f, 0.f};
    if (vq && liveq && e.scale) sc4 = *(const f4 *)(e.scale + nq);
    if (vq && liveq && e.shift) sh4 = *(const f4 *)(e.shift + nq);
    f4 dsb4 = {0.f, 0.f, 0.f, 0.f};
    if (EXTRA && vq && liveq && e.dup_src && e.dup_bias) dsb4 = *(const f4 *)(e.dup_bias + nq);
#pragma unroll 1
    for (int c0 = 0; c0 < BM; c0 += CH) {
        __syncthreads();   // operand stages (first chunk) / the previous chunk are no longer read
        stage(Cs, c0);
        __syncthreads();
        const int clim = rows(c0);
        const int cb = base(c0);
        if (vq) {
            if (!liveq || clim <= 0) continue;
            const int hw = a.oh * a.ow;
            const int rr0 = tid / TQ;
            int m = cb + rr0;
            int img = m / hw, rem = m - img * hw;
            auto act4 = [&](f4 v) {
                v.x = fast_act(v.x, e.act, slope); v.y = fast_act(v.y, e.act, slope);
                v.z = fast_act(v.z, e.act, slope); v.w = fast_act(v.w, e.act, slope);
                return v;
            };
            if (a.y_step > 1) {
                // strided / depth-to-space output: quads stay inside one parity class (d2s_c % 4 == 0)
                const int cls = a.d2s_c > 0 ? nq / a.d2s_c : 0;
                const int oc = a.d2s_c > 0 ? nq - cls * a.d2s_c : nq;
                const int dy = cls >> 1, dx = cls & 1, ys = a.y_step;
                int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
                float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + oc;
                const float *pix = e.pix_add ? e.pix_add + (long long)bidx * a.y_h * a.y_w * a.n : nullptr;
                const float *rsrc = e.res ? e.res + (long long)bidx * a.res_bs + oc : nullptr;
#pragma unroll 1
                for (int rr = rr0; rr < clim; rr += RS4) {
                    const long long q = ((long long)img * a.y_h + oy * ys + dy) * a.y_w + ox * ys + dx;
                    ox += RS4;
                    while (ox >= a.ow) {
                        ox -= a.ow;
                        if (++oy == a.oh) { oy = 0; ++img; }
                    }
                    f4 v = *(const f4 *)&Cs[rr * LDC + 4 * cq] * sc4 + sh4;
                    if (pix) v += e.pix_w * pix[q];
                    f4 rv = {0.f, 0.f, 0.f, 0.f};
                    if (rsrc) rv = *(const f4 *)(rsrc + q * a.ycs);
                    if (!e.res_after) v += rv;
                    v = act4(v);
                    if (e.res_after) v += rv;
                    *(f4 *)(yb + q * a.ycs) = v;
                }
            } else {
                float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + nq;
                const float *pix = e.pix_add ? e.pix_add + (long long)bidx * a.oh * a.ow * a.n : nullptr;
                const float *rsrc = e.res ? e.res + (long long)bidx * a.res_bs + nq : nullptr;
#pragma unroll 1
                for (int rr = rr0; rr < clim; rr += RS4, m += RS4, rem += RS4) {
                    while (rem >= hw) { rem -= hw; ++img; }
                    f4 v = *(const f4 *)&Cs[rr * LDC + 4 * cq] * sc4;
                    if (e.nc_scale) v *= *(const f4 *)(e.nc_scale + (long long)img * e.nc_ns + nq);
                    v += sh4;
                    if (pix) v += e.pix_w * pix[m];
                    f4 rv = {0.f, 0.f, 0.f, 0.f};
                    if (rsrc) rv = *(const f4 *)(rsrc + (long long)m * e.res_cs);
                    if (!e.res_after) v += rv;
                    v = act4(v);
                    if (e.res_after) v += rv;
                    if (EXTRA && e.post_mul && nq >= e.post_c0) {
                        const long long q = (long long)m * e.post_cs + nq - e.post_c0;
                        v = v * *(const f4 *)(e.post_mul + q) + *(const f4 *)(e.post_add + q);
                    }
                    *(f4 *)(yb + (long long)m * a.ycs) = v;
                    if (EXTRA && e.dup_src) {
                        f4 d = e.dup_a * *(const f4 *)(e.dup_src + (long long)m * e.dup_cs + nq) + dsb4;
                        *(f4 *)(yb + (long long)m * a.ycs + e.dup_off) = act4(d);
                    }
                }
            }
            continue;
        }
        if (!live || clim <= 0) continue;
        if (a.pool) {
            // 2x2 average of the activated outputs (ResBlock: lrelu(conv1) then bilinear x0.5 ==
            // the quad mean, base_blocks.py:40-49); rows 4r..4r+3 of the chunk are one quad
            float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + n;
#pragma unroll 1
            for (int rq = tid / TPR; 4 * rq < clim; rq += RSTEP) {
                float v = 0.f;
#pragma unroll
                for (int d = 0; d < 4; ++d) v += fast_act(Cs[(4 * rq + d) * LDC + cn] * sc + sh, e.act, slope);
                yb[(long long)(cb / 4 + rq) * a.ycs] = 0.25f * v;
            }
            continue;
        }
        if (a.splits > 1) {
            float *w = a.ws + (long long)bz * a.M * a.cout;
#pragma unroll 1
            for (int rr = tid / TPR; rr < clim; rr += RSTEP)
                w[(long long)(cb + rr) * a.cout + n] = Cs[rr * LDC + cn];
        } else if (simple && a.y_step <= 1) {
            float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + out_col(a, n);
            const float *rsrc = e.res ? e.res + (long long)bidx * a.res_bs + n : nullptr;
            int rr0 = tid / TPR;
            if (rsrc && a.y_step <= 1) {
                // residual rows: four loads in flight before their adds (a dependent load per
                // row left the store loop latency-bound)
                // ... and the next group's loads are issued before this group's stores (vmcnt counts
                // loads and stores in issue order: a load issued after a store waits for it)
                float rv[4];
                if (rr0 + 3 * RSTEP < clim) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) rv[q] = rsrc[(long long)(cb + rr0 + q * RSTEP) * e.res_cs];
                }
#pragma unroll 1
                for (; rr0 + 3 * RSTEP < clim; rr0 += 4 * RSTEP) {
                    const bool more = rr0 + 7 * RSTEP < clim;
                    float rn[4];
                    if (more) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            rn[q] = rsrc[(long long)(cb + rr0 + (4 + q) * RSTEP) * e.res_cs];
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const long long m = cb + rr0 + q * RSTEP;
                        float v = Cs[(rr0 + q * RSTEP) * LDC + cn] * sc + sh;
                        if (!e.res_after) v += rv[q];
                        v = fast_act(v, e.act, slope);
                        if (e.res_after) v += rv[q];
                        yb[m * a.ycs] = v;
                    }
                    if (more) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) rv[q] = rn[q];
                    }
                }
            }
#pragma unroll 1
            for (int rr = rr0; rr < clim; rr += RSTEP) {
                const long long m = cb + rr;
                float v = Cs[rr * LDC + cn] * sc + sh;
                float rv = 0.f;
                if (rsrc) {
                    rv = rsrc[a.y_step > 1 ? out_row(a, m) : m * e.res_cs];
                    if (!e.res_after) v += rv;
                }
                v = fast_act(v, e.act, slope);
                if (rsrc && e.res_after) v += rv;
                yb[out_row(a, m)] = v;
            }
        } else if (a.y_step > 1 && !e.nc_scale) {
            // strided (polyphase transposed) / depth-to-space (polyphase x2 StyleConv) output: the output
            // pixel of each row advances incrementally (one division per chunk instead of out_row's and
            // pix_index's per element), and the noise plane / residual of four rows is loaded ahead of
            // their stores
            const int cls = a.d2s_c > 0 ? n / a.d2s_c : 0;
            const int oc = a.d2s_c > 0 ? n - cls * a.d2s_c : n;
            const int dy = cls >> 1, dx = cls & 1, ys = a.y_step;
            const int hw = a.oh * a.ow;
            int m = cb + tid / TPR;
            int img = m / hw, rem = m - img * hw;
            int oy = rem / a.ow, ox = rem - (rem / a.ow) * a.ow;
            float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + oc;
            const float *pix = e.pix_add ? e.pix_add + (long long)bidx * a.y_h * a.y_w * a.n : nullptr;
            const float *rsrc = e.res ? e.res + (long long)bidx * a.res_bs + oc : nullptr;   // in place (validate)
            auto pixel = [&]() {
                const long long q = ((long long)img * a.y_h + oy * ys + dy) * a.y_w + ox * ys + dx;
                ox += RSTEP;
                while (ox >= a.ow) {
                    ox -= a.ow;
                    if (++oy == a.oh) { oy = 0; ++img; }
                }
                return q;
            };
            int rr = tid / TPR;
#pragma unroll 1
            for (; rr + 3 * RSTEP < clim; rr += 4 * RSTEP) {
                long long q[4];
                float pv[4] = {0.f, 0.f, 0.f, 0.f}, rv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; ++j) q[j] = pixel();
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (pix) pv[j] = pix[q[j]];
                    if (rsrc) rv[j] = rsrc[q[j] * a.ycs];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v = Cs[(rr + j * RSTEP) * LDC + cn] * sc + sh + e.pix_w * pv[j];
                    if (!e.res_after) v += rv[j];
                    v = fast_act(v, e.act, slope);
                    if (e.res_after) v += rv[j];
                    yb[q[j] * a.ycs] = v;
                }
            }
#pragma unroll 1
            for (; rr < clim; rr += RSTEP) {
                const long long q = pixel();
                float v = Cs[rr * LDC + cn] * sc + sh;
                if (pix) v += e.pix_w * pix[q];
                float rv = rsrc ? rsrc[q * a.ycs] : 0.f;
                if (!e.res_after) v += rv;
                v = fast_act(v, e.act, slope);
                if (e.res_after) v += rv;
                yb[q * a.ycs] = v;
            }
        } else if (a.y_step <= 1 && a.d2s_c <= 0 && (!e.res || e.res_simple) && !extra) {
            // per-(image, channel) scale and / or per-pixel add on a dense output (GPEN / GFPGAN StyledConv:
            // demod scale + noise): the row's image index advances incrementally instead of a division per
            // element (store_epilogue), which made the epilogue as long as the main loop of a 64-channel tile
            const int hw = a.oh * a.ow;
            const int rr0 = tid / TPR;
            int m = cb + rr0;
            int img = m / hw, rem = m - img * hw;
            float *__restrict__ yb = a.y + (long long)bidx * a.y_bs + out_col(a, n);
            const float *pix = e.pix_add ? e.pix_add + (long long)bidx * a.oh * a.ow * a.n : nullptr;
            const float *rsrc = e.res ? e.res + (long long)bidx * a.res_bs + n : nullptr;
            int rr = rr0;
            if (!e.nc_scale) {
                // the noise plane (and residual) of four rows loaded ahead of their stores
#pragma unroll 1
                for (; rr + 3 * RSTEP < clim; rr += 4 * RSTEP, m += 4 * RSTEP) {
                    float pv[4] = {0.f, 0.f, 0.f, 0.f}, rv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (pix) pv[j] = pix[m + j * RSTEP];
                        if (rsrc) rv[j] = rsrc[(long long)(m + j * RSTEP) * e.res_cs];
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float v = Cs[(rr + j * RSTEP) * LDC + cn] * sc + sh + e.pix_w * pv[j];
                        if (!e.res_after) v += rv[j];
                        v = fast_act(v, e.act, slope);
                        if (e.res_after) v += rv[j];
                        yb[(long long)(m + j * RSTEP) * a.ycs] = v;
                    }
                }
                rem = m - img * hw;
            }
#pragma unroll 1
            for (; rr < clim; rr += RSTEP, m += RSTEP, rem += RSTEP) {
                while (rem >= hw) { rem -= hw; ++img; }
                float v = Cs[rr * LDC + cn] * sc;
                if (e.nc_scale) v *= e.nc_scale[(long long)img * e.nc_ns + n];
                v += sh;
                if (pix) v += e.pix_w * pix[m];
                float rv = 0.f;
                if (rsrc) {
                    rv = rsrc[(long long)m * e.res_cs];
                    if (!e.res_after) v += rv;
                }
                v = fast_act(v, e.act, slope);
                if (rsrc && e.res_after) v += rv;
                yb[(long long)m * a.ycs] = v;
            }
        } else {
#pragma unroll 1
            for (int rr = tid / TPR; rr < clim; rr += RSTEP) store_epilogue<EXTRA>(a, bidx, cb + rr, n, Cs[rr * LDC + cn]);
        }
    }
}

// 32x32 MFMA accumulators (C/D map: lane owns column li of each tile, rows (r&3) + 8(r>>2) + 4 lh)
// held by NW waves laid out WAVES_M x NW/WAVES_M
template <int BM, int BN, int WAVES_M, int TM, int TN, int NW = 4, int CH = BM, bool EXTRA = true>
__device__ __forceinline__ void epilogue_tile(const ConvArgs &a, const floatx16 (&acc)[TM][TN], float *Cs, int tid,
                                              int m0, int n0, int bz, int bidx) {
    constexpr int WAVES_N = NW / WAVES_M;
    constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    constexpr int LDC = BN + 4;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int li = lane & 31, lh = lane >> 5;
    epilogue_tile_fn<BM, BN, NW, CH, EXTRA>(a, Cs, tid, m0, n0, bz, bidx, [&](float *C, int c0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int r0 = wm * WTM + i * 32 - c0;
            if (r0 < 0 || r0 >= CH) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    C[(r0 + (r & 3) + 8 * (r >> 2) + 4 * lh) * LDC + wn * WTN + j * 32 + li] = acc[i][j][r] * a.acc_scale;
        }
    });
}

}  // namespace s2v
