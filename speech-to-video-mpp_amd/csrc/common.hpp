// Shared device/host helpers for libs2v (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/s2v.h"

namespace s2v {

void set_error(const char *fmt, ...);
int check_launch(const char *what);
int device_cus();
long long tune_get(int key);   // s2v_tune knobs (conv.hip)

#define S2V_REQUIRE(cond, ...)            \
    do {                                  \
        if (!(cond)) {                    \
            ::s2v::set_error(__VA_ARGS__);\
            return S2V_E_INVALID;         \
        }                                 \
    } while (0)

__device__ __forceinline__ float apply_act(float v, int act, float alpha) {
    switch (act) {
        case S2V_ACT_RELU: return v > 0.f ? v : 0.f;
        case S2V_ACT_LRELU: return v >= 0.f ? v : v * alpha;
        case S2V_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
        case S2V_ACT_TANH: return tanhf(v);
        case S2V_ACT_GELU_TANH: {
            const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
            return 0.5f * v * (1.f + tanhf(k0 * (v + 0.044715f * v * v * v)));
        }
        default: return v;
    }
}

// F.pad(mode='reflect') index map for one reflection (pad < n)
// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8), each with its own L2.
// Remap a 1-D grid so that XCD j runs the j-th contiguous eighth of the logical blocks: blocks that
// share input (the rows above / below of a 3x3 stencil) then meet in one L2 instead of eight.
__device__ __forceinline__ unsigned xcd_block(unsigned L, unsigned total) {
    const unsigned per = total >> 3, rem = total & 7;
    const unsigned xcd = L & 7, idx = L >> 3;
    return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

__device__ __forceinline__ int reflect_idx(int i, int n) {
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

inline unsigned cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

}  // namespace s2v
