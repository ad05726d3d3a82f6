// Keras-v1 Adam arithmetic shared by every embedding-table path (ncf_update.hip's sweeps, updates,
// replays and flush): one definition, so every path rounds identically.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ncf_internal.h"

namespace ncf {

__device__ inline float adam_lr_t(float lr, float b1, float b2, int t) {
    const float ft = (float)t;
    return lr * (sqrtf(1.0f - powf(b2, ft)) / (1.0f - powf(b1, ft)));
}

// lr_t * m / (sqrt(v) + eps) with the hardware square root and reciprocal (v_sqrt_f32,
// v_rcp_f32: ~1 ulp each) instead of the correctly rounded sequences (~20 VALU instructions):
// the zero-gradient replays of the deferred decay are VALU-bound chains of these.  Every
// embedding Adam path (dense sweep, touched-row update, replays, flush, sharded update) goes
// through it, so they still round identically; against the correctly rounded quotient the step
// term differs by a few ulp (the oracle tolerances hold it).
__device__ __forceinline__ float adam_term(float lr_t, float m, float v, float eps) {
#pragma clang fp contract(off)
    return (lr_t * m) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) + eps);
}

// One Adam step of one float4 element (Keras v1 update, see top of file).  Every sweep of the
// table goes through this one function, so the dense sweep, the touched-row update and the
// zero-gradient replay round identically.
__device__ __forceinline__ void adam4(float4& p, float4& m, float4& v, const float4& g, float lr_t, float b1,
                                      float b2, float eps) {
    // no FMA contraction: which product an fma would absorb depends on how the surrounding
    // kernel got scheduled, and every caller must round identically
#pragma clang fp contract(off)
    const float c1 = 1.0f - b1, c2 = 1.0f - b2;
    m.x = b1 * m.x + c1 * g.x; m.y = b1 * m.y + c1 * g.y;
    m.z = b1 * m.z + c1 * g.z; m.w = b1 * m.w + c1 * g.w;
    v.x = b2 * v.x + c2 * (g.x * g.x); v.y = b2 * v.y + c2 * (g.y * g.y);
    v.z = b2 * v.z + c2 * (g.z * g.z); v.w = b2 * v.w + c2 * (g.w * g.w);
    p.x -= adam_term(lr_t, m.x, v.x, eps); p.y -= adam_term(lr_t, m.y, v.y, eps);
    p.z -= adam_term(lr_t, m.z, v.z, eps); p.w -= adam_term(lr_t, m.w, v.w, eps);
}

// One component of adam4, the same expression: the replay below runs one element per lane and
// rounds exactly like the float4 sweeps.
__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, float lr_t, float b1, float b2,
                                      float eps) {
#pragma clang fp contract(off)
    const float c1 = 1.0f - b1, c2 = 1.0f - b2;
    m = b1 * m + c1 * g;
    v = b2 * v + c2 * (g * g);
    p -= adam_term(lr_t, m, v, eps);
}

// adam1 with g = 0 (the deferred decay's replayed steps): c1 * 0 and c2 * (0 * 0) are +0 for the
// finite c1, c2 of any valid beta, so b1*m + c1*g rounds like b1*m + 0 — bitwise adam1(..., 0, ...)
// with three multiplies less per replayed step
__device__ __forceinline__ void adam1_zero(float& p, float& m, float& v, float lr_t, float b1, float b2, float eps) {
#pragma clang fp contract(off)
    m = b1 * m + 0.0f;
    v = b2 * v + 0.0f;
    p -= adam_term(lr_t, m, v, eps);
}

// adam1_zero on two neighbouring elements: the multiplies and adds as packed fp32 (v_pk_mul_f32,
// v_pk_add_f32: IEEE per component, so bitwise adam1_zero per element), half the VALU issue of the
// moment updates and the step term's products in the replays
typedef float f32x2 __attribute__((ext_vector_type(2)));
// v's "+ 0" is dropped: v >= +0 always (never -0), so b2 * v + 0 rounds to b2 * v exactly; m keeps
// it (b1 * m can be -0, which + 0 turns into the dense sweep's +0)
__device__ __forceinline__ f32x2 rcp_sqrt_eps2(f32x2 v, float eps) {
    const f32x2 q = f32x2{__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)} + eps;
    return f32x2{__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
}
__device__ __forceinline__ void adam2_zero(f32x2& p, f32x2& m, f32x2& v, float lr_t, float b1, float b2, float eps) {
#pragma clang fp contract(off)
    m = m * b1 + 0.0f;
    v = v * b2;
    p -= (m * lr_t) * rcp_sqrt_eps2(v, eps);
}

// adam4's moment updates with g = 0: b1*m + c1*0 and b2*v + c2*0 round like b1*m + 0, b2*v + 0
__device__ __forceinline__ void decay4(float4& m, float4& v, float b1, float b2) {
#pragma clang fp contract(off)
    m.x = b1 * m.x + 0.0f; m.y = b1 * m.y + 0.0f; m.z = b1 * m.z + 0.0f; m.w = b1 * m.w + 0.0f;
    v.x = b2 * v.x + 0.0f; v.y = b2 * v.y + 0.0f; v.z = b2 * v.z + 0.0f; v.w = b2 * v.w + 0.0f;
}

// decay4 on an element pair (adam2_zero's moment updates: bitwise)
__device__ __forceinline__ void decay2(f32x2& m, f32x2& v, float b1, float b2) {
#pragma clang fp contract(off)
    m = m * b1 + 0.0f;
    v = v * b2;
}

// Whole wave: each lane's row `key` (-1: none) behind step t (0 <= row_step < t; a P-ahead mark or a
// pristine row is not) is claimed by CAS — a row repeated in the wave or across waves replays once —
// and the wave replays its claimed rows fully (p, m, v to step t, row_step = t), one after another,
// two elements per lane
__device__ inline void claim_replay(float* __restrict__ embf, float* __restrict__ mf, float* __restrict__ vf, int W,
                                    int32_t* row_step, int key, int t, float lr, float b1, float b2, float eps) {
    const int lane = threadIdx.x & 63;
    bool claim = false;
    int s0 = t;
    if (key >= 0) {
        int sv = row_step[key];
        while (sv >= 0 && sv < t) {
            const int prev = atomicCAS(&row_step[key], sv, t);
            if (prev == sv) {
                claim = true;
                s0 = sv;
                break;
            }
            sv = prev;
        }
    }
    uint64_t cm = __ballot(claim);
    while (cm) {
        const int src = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int r = __shfl(key, src, 64);
        const int s = __shfl(s0, src, 64);
        for (int q = lane; 2 * q < W; q += 64) {
            const size_t e = (size_t)r * W + 2 * q;
            f32x2 p = *reinterpret_cast<const f32x2*>(embf + e);
            f32x2 m = *reinterpret_cast<const f32x2*>(mf + e);
            f32x2 v = *reinterpret_cast<const f32x2*>(vf + e);
            for (int st = s + 1; st <= t; ++st) adam2_zero(p, m, v, adam_lr_t(lr, b1, b2, st), b1, b2, eps);
            *reinterpret_cast<f32x2*>(embf + e) = p;
            *reinterpret_cast<f32x2*>(mf + e) = m;
            *reinterpret_cast<f32x2*>(vf + e) = v;
        }
    }
}


}  // namespace ncf
