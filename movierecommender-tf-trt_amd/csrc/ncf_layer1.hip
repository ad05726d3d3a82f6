// First dense layer of the layer-by-layer path (config D: MLP [256,128,64,32] + GMF 128) on
// hand-written fp32 MFMA (v_mfma_f32_16x16x4_f32), its gather and scatter fused in.
//
// rocBLAS ran this layer as a [n x 256] x [256 x 128] GEMM with the gather (X0, GMF product) and
// bias + ReLU as separate HBM passes before it, and dX = G1 W1^T as a GEMM with the gradient-row
// scatter after it (profiles/r03_c/tl_D_step.txt: 112 + 103 us per 65,536-sample step).  Here W1
// (128 KB at config D) sits in LDS once per workgroup, in the operand layout of ncf_wave.hip
// (column c of a row at position (c mod 16) B1 + c / 16, row stride 16 B1 + 4), and every wave
// streams its own 16-sample units through it:
//
//   k_lay_l1f  rows -> registers (lane (sample li, lane group lq) holds MLP-input features
//              XQ lq + q, q < XQ = L0 / 4), H1 = relu(W1^T x + b1) as B1 16 x 16 accumulator
//              tiles [feature][sample] over L0 / 4 k-steps of B1 MFMAs, then X0, GMF product
//              (u_g * i_g) and H1 written row-major for the GEMM layers behind it
//              (model.py:159-181; masked samples: zero X0 and GMF, as k_lay_gather)
//   k_lay_l1b  G1 rows -> registers (lane (li, lq): features 16 t + 4 lq + r), dX = W1 G1 as
//              L0 / 16 tiles over 4 B1 k-steps each, written straight into the per-sample
//              gradient rows gs[2i] / gs[2i + 1] together with their GMF part
//              dz w_gmf * (the other side's GMF vector) (k_lay_scatter's rows, model.py:159-188)
//
// Two units in flight per wave (their loads alternate between two register sets, no copies).
// Both kernels are HBM-bound more than MFMA-bound at config D: the forward reads the two rows
// (1 KB of MLP input + 1 KB of GMF vectors per sample) and writes X0, the GMF product and H1 for the
// GEMM layers (2 KB), the backward reads G1 and the GMF vectors and writes the two gradient rows.
// Outputs are those of the replaced kernels, so the GEMM layers, the slab reduction and the
// optimizer launches are unchanged.

#include <cstdlib>

// 1 (the default): with user-row folding the layer-1 forward computes the user half once per group
// (k_lay_l1f_gu); 0: per sample (A/B)
#ifndef NCF_LAYERED_GU
#define NCF_LAYERED_GU 1
#endif
// timing diagnostic (wrong results): 1 = layer 1's user half skipped in all three kernels (the
// work a per-group user half would leave)
#ifndef NCF_DIAG_DHALF
#define NCF_DIAG_DHALF 0
#endif

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int L0_, int L1_, int G_>
struct L1Shape {
    static constexpr int L0 = L0_, L1 = L1_, G = G_, D0 = L0 / 2, W = G + D0;
    static constexpr int B1 = L1 / 16, XQ = L0 / 4, GQ = G / 4, B0 = L0 / 16;
    static constexpr int S1 = 16 * B1 + 4;            // LDS row stride of W1 (floats)
    static constexpr int SB = L0 * S1;                // b1 after W1
    static constexpr size_t LDS = (size_t)(SB + L1) * 4;
    static_assert(L0 % 64 == 0 && L1 % 16 == 0 && B1 <= 8 && (B1 & (B1 - 1)) == 0 && G % 16 == 0, "layer-1 shape");
    static_assert(LDS <= 163840, "W1 must fit the LDS");
};

// W1 [L0][L1] (flat Keras kernel at offset 0) and b1 into the LDS operand layout.  Every float4 a
// thread moves is loaded in one batch before any LDS store (a load-store loop waits one memory
// round trip per float4: 32 of them per thread at config D)
template <class S, int NT>
__device__ __forceinline__ void load_w1(float* wl, const float* __restrict__ mlp) {
    constexpr int L0 = S::L0, L1 = S::L1, B1 = S::B1, NV = L0 * L1 / 4 / NT;
    static_assert(L0 * L1 % (4 * NT) == 0, "W1 in whole float4 rounds");
    const float4* w4 = reinterpret_cast<const float4*>(mlp);
    float4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = w4[threadIdx.x + NT * j];
    const float bv = threadIdx.x < L1 ? mlp[L0 * L1 + threadIdx.x] : 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int e = threadIdx.x + NT * j;
        const int i = (4 * e) / L1, c0 = (4 * e) % L1;
        float* row = wl + i * S::S1;
        row[((c0 + 0) & 15) * B1 + ((c0 + 0) >> 4)] = v[j].x;
        row[((c0 + 1) & 15) * B1 + ((c0 + 1) >> 4)] = v[j].y;
        row[((c0 + 2) & 15) * B1 + ((c0 + 2) >> 4)] = v[j].z;
        row[((c0 + 3) & 15) * B1 + ((c0 + 3) >> 4)] = v[j].w;
    }
    static_assert(L1 <= NT, "b1 by one pass");
    if (threadIdx.x < L1) wl[S::SB + threadIdx.x] = bv;
    __syncthreads();
}

// sum over this lane's group of FOLD consecutive sample lanes (DPP quad butterfly, ds_swizzle for the
// third step): every lane of the group gets it, the group head's association is ((s0 + s1) + (s2 +
// s3)) as the fused kernels fold (ncf_wave.hip fold_sum)
template <int FOLD>
__device__ __forceinline__ float fold_sum(float x) {
    static_assert(FOLD == 2 || FOLD == 4 || FOLD == 8, "fold width");
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    if constexpr (FOLD >= 4)
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    if constexpr (FOLD >= 8) x += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x1F | (4 << 10)));
    return x;
}

template <int NB>
__device__ __forceinline__ void ldsv(const float* p, float (&o)[NB]) {
    if constexpr (NB == 8) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(p), y = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = x[i], o[4 + i] = y[i];
    } else if constexpr (NB == 4) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = x[i];
    } else if constexpr (NB == 2) {
        o[0] = p[0], o[1] = p[1];
    } else {
        o[0] = p[0];
    }
}

// NW waves per workgroup (8: two per SIMD, one unit's registers each; 4: one per SIMD with two
// units' loads in flight)
// GMF: also write the GMF product (the rocBLAS layers' output pass reads it; k_lay_mid forms it
// from the rows itself)
template <class S, int NW, bool GMF>
__global__ __launch_bounds__(64 * NW, 1) void k_lay_l1f(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                    const int32_t* __restrict__ users,
                                                    const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                    float* __restrict__ x0, float* __restrict__ gmf,
                                                    float* __restrict__ h1) {
    constexpr int L0 = S::L0, L1 = S::L1, G = S::G, W = S::W, B1 = S::B1, XQ = S::XQ, GQ = S::GQ;
    extern __shared__ __attribute__((aligned(16))) float wl[];
    load_w1<S, 64 * NW>(wl, mlp);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    const int64_t nunits = (n + 15) / 16, ustride = (int64_t)gridDim.x * NW;
    float bias[B1][4];
#pragma unroll
    for (int t = 0; t < B1; ++t) ldsv<4>(wl + S::SB + 16 * t + 4 * g, bias[t]);

    struct Unit {
        float x[XQ];
        bool ok;
        int urow, irow;
    };
    // the unit's ids and MLP-input rows (lane group lq < 2: the user half, else the item half)
    auto load = [&](int64_t u, Unit& U) {
        const int64_t s = u * 16 + li;
        const bool in = s < n;
        const int cu = in ? users[s] : 0, cv = in ? items[s] : 0;
        U.ok = in && (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
        U.urow = U.ok ? cu : 0;
        U.irow = U.ok ? ids.ibase + cv : 0;
        const float4* xs =
            reinterpret_cast<const float4*>(emb + (size_t)(g < 2 && !NCF_DIAG_DHALF ? U.urow : U.irow) * W + G + (g & 1) * XQ);
#pragma unroll
        for (int k = 0; k < (NCF_DIAG_DHALF ? XQ / 8 : XQ / 4); ++k) {
            const float4 v = xs[k];
            U.x[4 * k] = v.x, U.x[4 * k + 1] = v.y, U.x[4 * k + 2] = v.z, U.x[4 * k + 3] = v.w;
        }
    };
    auto process = [&](int64_t u, Unit& U) {
        const int64_t s = u * 16 + li;
        const bool in = s < n;
        // the GMF slices (dims GQ lq .. GQ lq + GQ - 1) go out now, under the MFMAs
        float4 pu[GQ / 4], pi[GQ / 4];
        if constexpr (GMF) {
            const float4* gu = reinterpret_cast<const float4*>(emb + (size_t)U.urow * W + GQ * g);
            const float4* gi = reinterpret_cast<const float4*>(emb + (size_t)U.irow * W + GQ * g);
#pragma unroll
            for (int k = 0; k < GQ / 4; ++k) pu[k] = gu[k], pi[k] = gi[k];
        }
#pragma unroll
        for (int q = 0; q < XQ; ++q) U.x[q] = U.ok ? U.x[q] : 0.f;  // masked sample: zero input
        f32x4 h[B1];
#pragma unroll
        for (int t = 0; t < B1; ++t) h[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        // k-step q: feature XQ lq + q from lane group lq (A: W1 row XQ lq + q, all B1 blocks in one read)
        float a[2][B1];
        ldsv<B1>(wl + (XQ * g) * S::S1 + li * B1, a[0]);
#pragma unroll
        for (int q = 0; q < (NCF_DIAG_DHALF ? XQ / 2 : XQ); ++q) {
            if (q + 1 < XQ) ldsv<B1>(wl + (XQ * g + q + 1) * S::S1 + li * B1, a[(q + 1) & 1]);
#pragma unroll
            for (int t = 0; t < B1; ++t) h[t] = mfma16(a[q & 1][t], U.x[q], h[t]);
        }
        if (in) {
            float* xo = x0 + s * L0 + XQ * g;
#pragma unroll
            for (int k = 0; k < XQ / 4; ++k)
                *reinterpret_cast<float4*>(xo + 4 * k) = make_float4(U.x[4 * k], U.x[4 * k + 1], U.x[4 * k + 2], U.x[4 * k + 3]);
            float* ho = h1 + s * L1 + 4 * g;
#pragma unroll
            for (int t = 0; t < B1; ++t)
                *reinterpret_cast<float4*>(ho + 16 * t) =
                    make_float4(fmaxf(h[t][0] + bias[t][0], 0.f), fmaxf(h[t][1] + bias[t][1], 0.f),
                                fmaxf(h[t][2] + bias[t][2], 0.f), fmaxf(h[t][3] + bias[t][3], 0.f));
            // GMF product of the two rows
            if constexpr (GMF) {
                float4* go = reinterpret_cast<float4*>(gmf + s * G + GQ * g);
#pragma unroll
                for (int k = 0; k < GQ / 4; ++k) {
                    const float4 p = pu[k], r = pi[k];
                    go[k] = U.ok ? make_float4(p.x * r.x, p.y * r.y, p.z * r.z, p.w * r.w) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
    };
    const int64_t u0 = (int64_t)blockIdx.x * NW + wv;
    if constexpr (NW == 8) {
        Unit A;
        for (int64_t u = u0; u < nunits; u += ustride) {
            load(u, A);
            process(u, A);
        }
    } else {
        Unit A, B;
        if (u0 < nunits) load(u0, A);
        for (int64_t u = u0; u < nunits; u += 2 * ustride) {
            const bool hb = u + ustride < nunits;
            if (hb) load(u + ustride, B);
            process(u, A);
            if (u + 2 * ustride < nunits) load(u + 2 * ustride, A);
            if (hb) process(u + ustride, B);
        }
    }
}

// Group-user form of the layer-1 forward (user-row folding, FOLD 2, 4, 8): the reference's batches
// are groups of FOLD samples sharing one user (data_pipeline.py:141), and layer 1 is linear in the
// user half of its input: W1^T [x_u; x_i] = W1_u^T x_u + W1_i^T x_i.  Phase 0: each wave computes
// P_u = W1_u^T x_u of the group heads of its units, 16 groups per MFMA tile (column li: group
// li % NGU of the wave's unit tau FOLD + li / NGU), into gpart [n / FOLD][L1], and writes X0's user
// half for the group heads (k_lay_dw1<FOLD> contracts the user half per group from the heads' rows).  Per unit: the accumulators start from
// the sample's group's P_u and only the item half is contracted (128 instead of 256 k-features at
// config D).  A unit holding a sample whose user is not its head's, or a masked sample, runs the
// per-sample form (k_lay_l1f's), so any batch stays exact.  Same sums, reassociated.
template <class S, int NW, int FOLD>
__global__ __launch_bounds__(64 * NW, 1) void k_lay_l1f_gu(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                       const int32_t* __restrict__ users,
                                                       const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                       float* __restrict__ x0, float* __restrict__ h1,
                                                       float* __restrict__ gpart) {
    constexpr int L0 = S::L0, L1 = S::L1, G = S::G, W = S::W, B1 = S::B1, XQ = S::XQ, D0 = S::D0;
    constexpr int XH = D0 / 4;       // features of one half per lane group
    constexpr int NGU = 16 / FOLD;   // groups per unit
    static_assert(FOLD == 2 || FOLD == 4 || FOLD == 8, "fold width");
    extern __shared__ __attribute__((aligned(16))) float wl[];
    load_w1<S, 64 * NW>(wl, mlp);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    const int64_t nunits = (n + 15) / 16, ustride = (int64_t)gridDim.x * NW;
    float bias[B1][4];
#pragma unroll
    for (int t = 0; t < B1; ++t) ldsv<4>(wl + S::SB + 16 * t + 4 * g, bias[t]);
    const int64_t u0 = (int64_t)blockIdx.x * NW + wv;
    const int64_t nown = u0 < nunits ? (nunits - u0 + ustride - 1) / ustride : 0;

    // ---- phase 0
    const int64_t ntile = (nown + FOLD - 1) / FOLD;
    for (int64_t tau = 0; tau < ntile; ++tau) {
        const int64_t k = tau * FOLD + li / NGU;
        const int64_t hs = (u0 + k * ustride) * 16 + (li % NGU) * FOLD;
        const bool hv = k < nown && hs < n;
        const int hu = hv ? users[hs] : 0;
        const int row = hv && (unsigned)hu < (unsigned)ids.ubound ? hu : 0;
        float xu[XH];
        {
            const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)row * W + G + XH * g);
#pragma unroll
            for (int k4 = 0; k4 < XH / 4; ++k4) {
                const float4 v = xs[k4];
                xu[4 * k4] = v.x, xu[4 * k4 + 1] = v.y, xu[4 * k4 + 2] = v.z, xu[4 * k4 + 3] = v.w;
            }
        }
        f32x4 acc[B1];
#pragma unroll
        for (int t = 0; t < B1; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        float a[2][B1];
        ldsv<B1>(wl + (XH * g) * S::S1 + li * B1, a[0]);
#pragma unroll
        for (int q = 0; q < XH; ++q) {
            if (q + 1 < XH) ldsv<B1>(wl + (XH * g + q + 1) * S::S1 + li * B1, a[(q + 1) & 1]);
#pragma unroll
            for (int t = 0; t < B1; ++t) acc[t] = mfma16(a[q & 1][t], xu[q], acc[t]);
        }
        if (hv) {
            float* pg = gpart + (hs / FOLD) * L1 + 4 * g;
#pragma unroll
            for (int t = 0; t < B1; ++t) *reinterpret_cast<f32x4*>(pg + 16 * t) = acc[t];
            // X0's user half of the group head (k_lay_dw1<FOLD> reads the heads' only in units of the
            // group form; a unit that takes the per-sample form rewrites all of its X0 rows)
            {
                float4* xo = reinterpret_cast<float4*>(x0 + hs * L0 + XH * g);
#pragma unroll
                for (int k4 = 0; k4 < XH / 4; ++k4)
                    xo[k4] = make_float4(xu[4 * k4], xu[4 * k4 + 1], xu[4 * k4 + 2], xu[4 * k4 + 3]);
            }
        }
    }
    // the P_u rows are read back by other lanes of this wave (a fence emits no vmcnt wait on gfx950)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

    struct Unit {
        float x[XH];      // the item half (lane group lq: item features XH lq + q)
        f32x4 pu[B1];     // the sample's group's P_u
        bool ok, grp;     // grp: every sample of the unit valid and its user its head's
        int irow;
    };
    auto load = [&](int64_t u, Unit& U) {
        const int64_t s = u * 16 + li;
        const bool in = s < n;
        const int cu = in ? users[s] : 0, cv = in ? items[s] : 0;
        const int hu = in ? users[s & ~(int64_t)(FOLD - 1)] : 0;
        U.ok = in && (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
        U.grp = __ballot(in && (!U.ok || cu != hu)) == 0;
        U.irow = U.ok ? ids.ibase + cv : 0;
        const float* xr = emb + (size_t)U.irow * W + G + XH * g;   // the item row's MLP half: features XH lq ..
#pragma unroll
        for (int k4 = 0; k4 < XH / 4; ++k4) {
            const float4 v = reinterpret_cast<const float4*>(xr)[k4];
            U.x[4 * k4] = v.x, U.x[4 * k4 + 1] = v.y, U.x[4 * k4 + 2] = v.z, U.x[4 * k4 + 3] = v.w;
        }
        const float* pg = gpart + ((in ? s : 0) / FOLD) * L1 + 4 * g;
#pragma unroll
        for (int t = 0; t < B1; ++t) U.pu[t] = *reinterpret_cast<const f32x4*>(pg + 16 * t);
    };
    auto store_h1 = [&](int64_t s, const f32x4 (&h)[B1]) {
        float* ho = h1 + s * L1 + 4 * g;
#pragma unroll
        for (int t = 0; t < B1; ++t)
            *reinterpret_cast<float4*>(ho + 16 * t) =
                make_float4(fmaxf(h[t][0] + bias[t][0], 0.f), fmaxf(h[t][1] + bias[t][1], 0.f),
                            fmaxf(h[t][2] + bias[t][2], 0.f), fmaxf(h[t][3] + bias[t][3], 0.f));
    };
    auto process = [&](int64_t u, Unit& U) {
        const int64_t s = u * 16 + li;
        const bool in = s < n;
        f32x4 h[B1];
        if (U.grp) {
#pragma unroll
            for (int t = 0; t < B1; ++t) h[t] = U.pu[t];
            float a[2][B1];
            ldsv<B1>(wl + (D0 + XH * g) * S::S1 + li * B1, a[0]);
#pragma unroll
            for (int q = 0; q < XH; ++q) {
                if (q + 1 < XH) ldsv<B1>(wl + (D0 + XH * g + q + 1) * S::S1 + li * B1, a[(q + 1) & 1]);
#pragma unroll
                for (int t = 0; t < B1; ++t) h[t] = mfma16(a[q & 1][t], U.x[q], h[t]);
            }
            if (in) {
                float4* xo = reinterpret_cast<float4*>(x0 + s * L0 + D0 + XH * g);
#pragma unroll
                for (int k4 = 0; k4 < XH / 4; ++k4)
                    xo[k4] = make_float4(U.x[4 * k4], U.x[4 * k4 + 1], U.x[4 * k4 + 2], U.x[4 * k4 + 3]);
                store_h1(s, h);
            }
        } else {
            // the per-sample form (k_lay_l1f): lane group lq holds MLP-input features XQ lq + q
            const int cu = in ? users[s] : 0, cv = in ? items[s] : 0;
            const bool ok = in && (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
            const int urow = ok ? cu : 0, irow = ok ? ids.ibase + cv : 0;
            float x[XQ];
            const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)(g < 2 ? urow : irow) * W + G + (g & 1) * XQ);
#pragma unroll
            for (int k4 = 0; k4 < XQ / 4; ++k4) {
                const float4 v = xs[k4];
                x[4 * k4] = ok ? v.x : 0.f, x[4 * k4 + 1] = ok ? v.y : 0.f;
                x[4 * k4 + 2] = ok ? v.z : 0.f, x[4 * k4 + 3] = ok ? v.w : 0.f;
            }
#pragma unroll
            for (int t = 0; t < B1; ++t) h[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            float a[2][B1];
            ldsv<B1>(wl + (XQ * g) * S::S1 + li * B1, a[0]);
#pragma unroll
            for (int q = 0; q < XQ; ++q) {
                if (q + 1 < XQ) ldsv<B1>(wl + (XQ * g + q + 1) * S::S1 + li * B1, a[(q + 1) & 1]);
#pragma unroll
                for (int t = 0; t < B1; ++t) h[t] = mfma16(a[q & 1][t], x[q], h[t]);
            }
            if (in) {
                float4* xo = reinterpret_cast<float4*>(x0 + s * L0 + XQ * g);
#pragma unroll
                for (int k4 = 0; k4 < XQ / 4; ++k4)
                    xo[k4] = make_float4(x[4 * k4], x[4 * k4 + 1], x[4 * k4 + 2], x[4 * k4 + 3]);
                store_h1(s, h);
            }
        }
    };
    Unit A, B;
    if (u0 < nunits) load(u0, A);
    for (int64_t u = u0; u < nunits; u += 2 * ustride) {
        const bool hb = u + ustride < nunits;
        if (hb) load(u + ustride, B);
        process(u, A);
        if (u + 2 * ustride < nunits) load(u + 2 * ustride, A);
        if (hb) process(u + ustride, B);
    }
}

// FOLD (2, 4, 8; 0 none): user-row folding (ncf_internal.h fold_of) — the user-side gradient rows of
// a group of FOLD samples that share the head's user are summed in fixed order into the head's row
// (its contribution c = 2 hd) and the other samples' user rows are not written (the index skips
// them: folded_user); a sample whose user is not its head's keeps its own row
template <class S, int NW, int FOLD>
__global__ __launch_bounds__(64 * NW, 1) void k_lay_l1b(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                    int wo_off, const int32_t* __restrict__ users,
                                                    const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                    const float* __restrict__ dzo, const float* __restrict__ g1,
                                                    float* __restrict__ gs) {
    constexpr int L1 = S::L1, G = S::G, W = S::W, B1 = S::B1, GQ = S::GQ, B0 = S::B0, D0 = S::D0;
    extern __shared__ __attribute__((aligned(16))) float wl[];
    load_w1<S, 64 * NW>(wl, mlp);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    const int64_t nunits = (n + 15) / 16, ustride = (int64_t)gridDim.x * NW;
    const float* wg = mlp + wo_off;  // output kernel, GMF part first

    struct Unit {
        float gv[B1][4];  // G1 features 16 t + 4 lq + r of sample li
    };
    auto load = [&](int64_t u, Unit& U) {
        const int64_t s = u * 16 + li;
        const float* gr = g1 + (s < n ? s : 0) * L1 + 4 * g;
#pragma unroll
        for (int t = 0; t < B1; ++t) {
            const float4 v = *reinterpret_cast<const float4*>(gr + 16 * t);
            U.gv[t][0] = v.x, U.gv[t][1] = v.y, U.gv[t][2] = v.z, U.gv[t][3] = v.w;
        }
    };
    auto process = [&](int64_t u, Unit& U) {
        const int64_t s = u * 16 + li;
        const bool in = s < n;
        int cu = 0, cv = 0;
        if (in) cu = users[s], cv = items[s];
        const bool ok = in && (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
        // folding: this sample's user is its group head's (lane li & ~(FOLD - 1) of the same lane group)
        const bool fmatch = FOLD > 1 && in && cu == __shfl(cu, lane & ~(FOLD > 1 ? FOLD - 1 : 0), 64);
        const bool fhead = FOLD <= 1 || (li & (FOLD > 1 ? FOLD - 1 : 0)) == 0;
        const bool uwrite = in && (!fmatch || fhead);   // this sample's user row is a contribution
        auto fold4 = [&](float4 v) {
            if constexpr (FOLD > 1) {
                const float4 sm = make_float4(fold_sum<(FOLD > 1 ? FOLD : 2)>(fmatch ? v.x : 0.f),
                                              fold_sum<(FOLD > 1 ? FOLD : 2)>(fmatch ? v.y : 0.f),
                                              fold_sum<(FOLD > 1 ? FOLD : 2)>(fmatch ? v.z : 0.f),
                                              fold_sum<(FOLD > 1 ? FOLD : 2)>(fmatch ? v.w : 0.f));
                return fmatch ? sm : v;
            } else {
                return v;
            }
        };
        // the GMF part's operands go out now, under the dX MFMAs
        float4 pu[GQ / 4], pi[GQ / 4], pw[GQ / 4];
        float d = 0.f;
        {
            const float4* gu = reinterpret_cast<const float4*>(emb + (size_t)(ok ? cu : 0) * W + GQ * g);
            const float4* gi = reinterpret_cast<const float4*>(emb + (size_t)(ok ? ids.ibase + cv : 0) * W + GQ * g);
            const float4* w4 = reinterpret_cast<const float4*>(wg + GQ * g);
#pragma unroll
            for (int k = 0; k < GQ / 4; ++k) pu[k] = gu[k], pi[k] = gi[k], pw[k] = w4[k];
            d = ok ? dzo[s] : 0.f;
        }
        float* ur = gs + (size_t)(2 * s) * W;      // user-row contribution c = 2s
        float* ir = gs + (size_t)(2 * s + 1) * W;  // item-row contribution c = 2s + 1
        // dX = W1 G1: block ti holds input features 16 ti + 4 lq + r of sample li; k-step (t, r)
        // takes G1 feature 16 t + 4 lq + r (one LDS read gives the B1 steps of one r)
        // (blocks two at a time: the whole block loop unrolled hoists every LDS read and spills)
#pragma unroll 2
        for (int ti = NCF_DIAG_DHALF ? B0 / 2 : 0; ti < B0; ++ti) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            float a[2][B1];
            ldsv<B1>(wl + (16 * ti + li) * S::S1 + (4 * g) * B1, a[0]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (r + 1 < 4) ldsv<B1>(wl + (16 * ti + li) * S::S1 + (4 * g + r + 1) * B1, a[(r + 1) & 1]);
#pragma unroll
                for (int t = 0; t < B1; ++t) acc = mfma16(a[r & 1][t], U.gv[t][r], acc);
            }
            const int f0 = 16 * ti + 4 * g;
            const bool user = 16 * ti < D0;   // uniform: ti is
            float4 dv = make_float4(acc[0], acc[1], acc[2], acc[3]);
            if (user) dv = fold4(dv);
            if (user ? uwrite : in) {
                float* dst = (user ? ur : ir) + G + (user ? f0 : f0 - D0);
                *reinterpret_cast<float4*>(dst) = dv;
            }
        }
        // GMF part: dz w_gmf * the other side's GMF vector (zero rows for a masked sample)
#pragma unroll
        for (int k = 0; k < GQ / 4; ++k) {
            const float4 p = pu[k], q = pi[k], w = pw[k];
            const float4 zu = fold4(ok ? make_float4(d * w.x * q.x, d * w.y * q.y, d * w.z * q.z, d * w.w * q.w)
                                       : make_float4(0.f, 0.f, 0.f, 0.f));
            const float4 zi = ok ? make_float4(d * w.x * p.x, d * w.y * p.y, d * w.z * p.z, d * w.w * p.w)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
            if (uwrite) reinterpret_cast<float4*>(ur + GQ * g)[k] = zu;
            if (in) reinterpret_cast<float4*>(ir + GQ * g)[k] = zi;
        }
    };
    const int64_t u0 = (int64_t)blockIdx.x * NW + wv;
    Unit A, B;
    if (u0 < nunits) load(u0, A);
    for (int64_t u = u0; u < nunits; u += 2 * ustride) {
        const bool hb = u + ustride < nunits;
        if (hb) load(u + ustride, B);
        process(u, A);
        if (u + 2 * ustride < nunits) load(u + 2 * ustride, A);
        if (hb) process(u + ustride, B);
    }
}

// waves per workgroup (4 or 8), measured at config D (profiles/r03_d): the forward 87.8 us with 4
// (two units' loads in flight per wave) vs 98.7 with 8; the backward 80.6 with 4 vs 70.4 with 8
#ifndef NCF_L1F_WAVES
#define NCF_L1F_WAVES 4
#endif
#ifndef NCF_L1B_WAVES
#define NCF_L1B_WAVES 8
#endif

// dW1 = X0^T G1 over one batch chunk per workgroup (the slab of the k_lay_mid workgroup of the same
// chunk: slab c already holds its other parameters), on fp32 MFMA: it replaces the strided-batched
// rocBLAS GEMM (profiles/r03_q2/tl_D.txt: 53.6 us of the 276 us forward/backward).  The L0 x L1
// result is (L0 / 16) x (L1 / 16) 16 x 16 tiles; wave w owns the X0-feature tiles XT w .. XT w +
// XT - 1 against every G1-feature tile, accumulated over the chunk's samples in order.  A 16-sample
// unit of X0 and G1 rows is staged in LDS (rows padded by 4 floats: the four lane groups' rows fall
// on different banks), double-buffered: the workgroup's float4 loads of unit u + 1 are in flight
// while unit u's MFMAs run, one barrier per unit.  k-step j of a unit gives lane group lq sample
// 4 j + lq and lane li feature li of a tile (A = X0[s][16 x + li], B = G1[s][16 y + li]).  Tile
// element (lane 16 lq + c, register r) is dW1 row 16 x + 4 lq + r (input feature), column 16 y + c
// (output feature): Keras' [in][out] kernel.
// the sum of FOLD consecutive rows (stride sg) at p, pairwise in fold_sum's order
template <int FOLD>
__device__ __forceinline__ float group_sum_rows(const float* p, int sg) {
    if constexpr (FOLD == 2) {
        return p[0] + p[sg];
    } else if constexpr (FOLD == 4) {
        return (p[0] + p[sg]) + (p[2 * sg] + p[3 * sg]);
    } else {
        return ((p[0] + p[sg]) + (p[2 * sg] + p[3 * sg])) + ((p[4 * sg] + p[5 * sg]) + (p[6 * sg] + p[7 * sg]));
    }
}

// waves per SIMD the dW1 kernel is compiled for (4: two workgroups per CU, the group form then
// spills a few registers; 3: one workgroup per CU, no spill) — measured in profiles/r06_ab
#ifndef NCF_DW1_WPE
#define NCF_DW1_WPE 4
#endif
constexpr int kDw1Waves = 8;
constexpr int kDw1Split = 2;    // workgroups per chunk (each takes 1 / kDw1Split of the G1 features)
constexpr int kDw1Depth = 3;    // LDS unit buffers: units u + 1, u + 2 in flight while u computes
template <int L0, int L1>
constexpr size_t dw1_lds() {
    return (size_t)kDw1Depth * (16 * (L0 + 16) + 16 * (L1 / kDw1Split + 16)) * 4;
}
// FOLD (2, 4, 8; 0 none, the group-user form with k_lay_l1f_gu): the user-feature waves (the first
// half) contract a unit over its groups instead of its samples — x_u of the group head (its X0 row:
// the group's rows are the head's) against the group's G1 sum — one k-step per four groups instead
// of one per four samples; a unit with a sample whose user is not its head's, or a masked sample,
// runs the per-sample k-steps (k_lay_l1f_gu wrote its whole X0 rows; in the others only the heads')
template <int L0, int L1, int FOLD>
__global__ __launch_bounds__(64 * kDw1Waves) __attribute__((amdgpu_waves_per_eu(NCF_DW1_WPE))) void k_lay_dw1(const float* __restrict__ x0,
                                                             const float* __restrict__ g1, int64_t n, int chunk,
                                                             float* __restrict__ slabs, int64_t P,
                                                             const int32_t* __restrict__ users,
                                                             const int32_t* __restrict__ items, IdSpace ids) {
    constexpr int LY = L1 / kDw1Split;                      // G1 features of this workgroup
    constexpr int XT = L0 / 16 / kDw1Waves, YT = LY / 16;
    constexpr int NT = 64 * kDw1Waves;
    // LDS row strides (floats): 16 banks apart, so the four lane groups' ds_read_b32 (16
    // consecutive floats each, rows 4 k + lq) fall on disjoint banks
    constexpr int SX = L0 + 16, SG = LY + 16;
    constexpr int BUF = 16 * SX + 16 * SG;                  // one unit's X0 and G1 rows
    constexpr int QX = 16 * L0 / 4, QG = 16 * LY / 4;       // float4s per unit
    constexpr int NQ = (QX + QG + NT - 1) / NT;             // float4s per thread per unit
    static_assert(L0 % (16 * kDw1Waves) == 0 && LY % 16 == 0, "dW1 tiles per wave");
    extern __shared__ __attribute__((aligned(16))) float lds[];   // [kDw1Depth * BUF]
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, lq = lane >> 4;
    const int chunk_id = (int)blockIdx.x / kDw1Split, ysplit = (int)blockIdx.x % kDw1Split;
    const int64_t s0 = (int64_t)chunk_id * chunk;
    const int64_t s1 = s0 + chunk < n ? s0 + chunk : n;
    const int nu = (int)((s1 - s0 + 15) / 16);
    const float* g1y = g1 + LY * ysplit;
    // FOLD: bit u of bad: unit u holds a masked sample or one whose user is not its head's
    constexpr int NGU = FOLD > 1 ? 16 / FOLD : 16;
    __shared__ unsigned bad[8];
    // the group sums of G1 of the next unit (two buffers by unit parity), computed by the whole
    // workgroup one unit ahead (at the end of the unit before, whose barrier made the rows visible)
    __shared__ float gsum[2][NGU * SG];
    if constexpr (FOLD > 1) {
        if (threadIdx.x < 8) bad[threadIdx.x] = nu > 256 ? ~0u : 0u;
        __syncthreads();
        for (int64_t s = s0 + threadIdx.x; s < s1; s += NT) {
            const int cu = users[s], cv = items[s];
            const int hu = users[s - (s - s0) % FOLD];
            const bool ok = (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
            const int u = (int)((s - s0) >> 4);
            if ((!ok || cu != hu) && u < 256) atomicOr(&bad[u >> 5], 1u << (u & 31));
        }
        __syncthreads();
    }
    f32x4 acc[XT][YT];
#pragma unroll
    for (int x = 0; x < XT; ++x)
#pragma unroll
        for (int y = 0; y < YT; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    // thread's float4 q of a unit: q < QX: X0 row q / (L0 / 4), column 4 (q % (L0 / 4)); else G1
    // the thread's float4s of a unit (q = tid + NT j): X0 row q / (L0 / 4) for q < QX, else G1;
    // ext-vector registers, filled and drained by macros (no arrays behind references: they would
    // live in scratch)
    f32x4 v0[NQ], v1[NQ];
#define NCF_DW1_FETCH(U, VV)                                                                           \
    _Pragma("unroll") for (int j = 0; j < NQ; ++j) {                                                   \
        const int q = (int)threadIdx.x + NT * j;                                                       \
        const bool isx = q < QX;                                                                       \
        const int r = isx ? q / (L0 / 4) : (q - QX) / (LY / 4);                                        \
        const int c = isx ? q % (L0 / 4) : (q - QX) % (LY / 4);                                        \
        const int64_t s = s0 + 16 * (int64_t)(U) + r;                                                  \
        const bool ok = (U) < nu && s < s1 && q < QX + QG;                                             \
        const f32x4* src = isx ? reinterpret_cast<const f32x4*>(x0 + s * L0) + c                       \
                               : reinterpret_cast<const f32x4*>(g1y + s * L1) + c;                     \
        VV[j] = ok ? *src : f32x4{0.f, 0.f, 0.f, 0.f};                                                 \
    }
#define NCF_DW1_STASH(VV, B)                                                                           \
    _Pragma("unroll") for (int j = 0; j < NQ; ++j) {                                                   \
        const int q = (int)threadIdx.x + NT * j;                                                       \
        const bool isx = q < QX;                                                                       \
        const int r = isx ? q / (L0 / 4) : (q - QX) / (LY / 4);                                        \
        const int c = isx ? q % (L0 / 4) : (q - QX) % (LY / 4);                                        \
        float* dst = isx ? (B) + r * SX + 4 * c : (B) + 16 * SX + r * SG + 4 * c;                      \
        if (q < QX + QG) *reinterpret_cast<f32x4*>(dst) = VV[j];                                       \
    }
    // FOLD, unit U of the group form: its group sums (row gi of gsum[U & 1]: G1 of the group's FOLD
    // rows summed pairwise) — unit U's rows are in LDS once the barrier before U - 1 has passed
#define NCF_DW1_GSUM(U)                                                                                \
    if (FOLD > 1 && (U) < nu && !((bad[(U) >> 5] >> ((U) & 31)) & 1u)) {                               \
        const float* gb = lds + ((U) % kDw1Depth) * BUF + 16 * SX;                                     \
        for (int e = threadIdx.x; e < NGU * LY; e += NT) {                                             \
            const int gi = e / LY, c = e % LY;                                                         \
            gsum[(U) & 1][gi * SG + c] = group_sum_rows<(FOLD > 1 ? FOLD : 2)>(gb + gi * (FOLD > 1 ? FOLD : 2) * SG + c, SG); \
        }                                                                                              \
    }
    // prologue: units 0 and 1 staged, unit 2 in registers
    NCF_DW1_FETCH(0, v0);
    NCF_DW1_FETCH(1, v1);
    NCF_DW1_STASH(v0, lds);
    NCF_DW1_STASH(v1, lds + BUF);
    NCF_DW1_FETCH(2, v0);
    __syncthreads();   // unit 0's rows, for its group sums
    NCF_DW1_GSUM(0);
    // one unit (a macro, not a lambda: the accumulators must stay in registers): unit u + 3's loads
    // go out into NXT (in flight under units u and u + 1), unit u's MFMAs, then unit u + 2 (held in
    // CUR since the previous unit) into the buffer unit u - 1 used
#define NCF_DW1_UNIT(U, CUR, NXT)                                                                      \
    {                                                                                                  \
        const int u_ = (U);                                                                            \
        NCF_DW1_FETCH(u_ + 3, NXT);                                                                    \
        __syncthreads();                                                                               \
        const float* base = lds + (u_ % kDw1Depth) * BUF;                                              \
        const float* bx = base + 16 * XT * wv + li;                                                    \
        const float* bg = base + 16 * SX + li;                                                         \
        if (FOLD > 1 && wv < kDw1Waves / 2 && !((bad[u_ >> 5] >> (u_ & 31)) & 1u)) {                   \
            _Pragma("unroll") for (int k2 = 0; k2 < (NGU + 3) / 4; ++k2) {                             \
                const int gi = 4 * k2 + lq, hr = gi * (FOLD > 1 ? FOLD : 1);                           \
                const bool gv = gi < NGU;                                                              \
                float a[XT], b[YT];                                                                    \
                _Pragma("unroll") for (int x = 0; x < XT; ++x) a[x] = gv ? bx[hr * SX + 16 * x] : 0.f; \
                _Pragma("unroll") for (int y = 0; y < YT; ++y) b[y] = gv ? gsum[u_ & 1][gi * SG + 16 * y + li] : 0.f; \
                _Pragma("unroll") for (int x = 0; x < XT; ++x)                                         \
                _Pragma("unroll") for (int y = 0; y < YT; ++y) acc[x][y] = mfma16(a[x], b[y], acc[x][y]); \
            }                                                                                          \
        } else {                                                                                       \
        _Pragma("unroll") for (int k = 0; k < 4; ++k) {                                                \
            if (NCF_DIAG_DHALF && wv < kDw1Waves / 2) break;                                           \
            const int row = 4 * k + lq;                                                                \
            float a[XT], b[YT];                                                                        \
            _Pragma("unroll") for (int x = 0; x < XT; ++x) a[x] = bx[row * SX + 16 * x];               \
            _Pragma("unroll") for (int y = 0; y < YT; ++y) b[y] = bg[row * SG + 16 * y];               \
            _Pragma("unroll") for (int x = 0; x < XT; ++x)                                             \
            _Pragma("unroll") for (int y = 0; y < YT; ++y) acc[x][y] = mfma16(a[x], b[y], acc[x][y]);  \
        }                                                                                              \
        }                                                                                              \
        if (u_ + 2 < nu) { NCF_DW1_STASH(CUR, lds + ((u_ + 2) % kDw1Depth) * BUF); }                  \
        NCF_DW1_GSUM(u_ + 1);                                                                          \
    }
    for (int u = 0; u < nu; u += 2) {   // two units per trip: the register sets alternate statically
        NCF_DW1_UNIT(u, v0, v1);
        if (u + 1 < nu) NCF_DW1_UNIT(u + 1, v1, v0);
    }
#undef NCF_DW1_UNIT
#undef NCF_DW1_FETCH
#undef NCF_DW1_STASH
#undef NCF_DW1_GSUM
    float* slab = slabs + (int64_t)chunk_id * P + LY * ysplit;
#pragma unroll
    for (int x = 0; x < XT; ++x)
#pragma unroll
        for (int y = 0; y < YT; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                slab[(int64_t)(16 * (XT * wv + x) + 4 * lq + r) * L1 + 16 * y + li] = acc[x][y][r];
}

using L1ShapeD = L1Shape<256, 128, 128>;  // config D

template <class S>
bool l1matches(const ncf_shape_t& s) {
    return s.num_layers >= 2 && s.layers[0] == S::L0 && s.layers[1] == S::L1 && s.gmf_dim == S::G &&
           s.gmf_stride == S::G && s.du == S::D0 && s.di == S::D0 && s.row_width == S::W && s.layer_off[1] == 0;
}

template <class S, int NW>
int grid_of(int64_t n) {
    const int64_t wgs = ((n + 15) / 16 + NW - 1) / NW;
    return (int)(wgs < 256 ? (wgs < 1 ? 1 : wgs) : 256);
}

template <class S>
hipError_t configure(const void* k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)S::LDS);
}

}  // namespace

bool layer1_supported(const ncf_shape_t& s) { return l1matches<L1ShapeD>(s); }

hipError_t launch_layer1_fwd(const ncf_shape_t& s, const float* emb, const float* mlp, const int32_t* users,
                             const int32_t* items, int64_t n, IdSpace ids, float* x0, float* gmf, float* h1,
                             hipStream_t st, int fold, float* gpart) {
    using S = L1ShapeD;
    if (!l1matches<S>(s)) return hipErrorInvalidValue;
    static bool cfg = false;
    if (!cfg) {
        if (hipError_t e = configure<S>((const void*)k_lay_l1f<S, NCF_L1F_WAVES, true>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1f<S, NCF_L1F_WAVES, false>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1f_gu<S, NCF_L1F_WAVES, 2>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1f_gu<S, NCF_L1F_WAVES, 4>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1f_gu<S, NCF_L1F_WAVES, 8>)) return e;
        cfg = true;
    }
    if (NCF_LAYERED_GU && !gmf && gpart && (fold == 2 || fold == 4 || fold == 8)) {
#define NCF_L1F_GU(F)                                                                                          \
    launch(k_lay_l1f_gu<S, NCF_L1F_WAVES, F>, grid_of<S, NCF_L1F_WAVES>(n), 64 * NCF_L1F_WAVES, S::LDS, st, emb, mlp, \
           users, items, n, ids, x0, h1, gpart)
        if (fold == 2) NCF_L1F_GU(2);
        else if (fold == 4) NCF_L1F_GU(4);
        else NCF_L1F_GU(8);
#undef NCF_L1F_GU
        return hipGetLastError();
    }
    if (gmf)
        launch(k_lay_l1f<S, NCF_L1F_WAVES, true>, grid_of<S, NCF_L1F_WAVES>(n), 64 * NCF_L1F_WAVES, S::LDS, st, emb, mlp,
               users, items, n, ids, x0, gmf, h1);
    else
        launch(k_lay_l1f<S, NCF_L1F_WAVES, false>, grid_of<S, NCF_L1F_WAVES>(n), 64 * NCF_L1F_WAVES, S::LDS, st, emb,
               mlp, users, items, n, ids, x0, gmf, h1);
    return hipGetLastError();
}

hipError_t launch_layer1_dw(const ncf_shape_t& s, const float* x0, const float* g1, int64_t n, int64_t chunk,
                            int nchunks, float* slabs, hipStream_t st, int fold, const int32_t* users,
                            const int32_t* items, IdSpace ids) {
    using S = L1ShapeD;
    if (!l1matches<S>(s) || chunk <= 0 || nchunks <= 0 || chunk % 16 != 0) return hipErrorInvalidValue;
    static bool cfg = false;
    if (!cfg) {
        for (const void* f : {(const void*)k_lay_dw1<S::L0, S::L1, 0>, (const void*)k_lay_dw1<S::L0, S::L1, 2>,
                              (const void*)k_lay_dw1<S::L0, S::L1, 4>, (const void*)k_lay_dw1<S::L0, S::L1, 8>})
            if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)dw1_lds<S::L0, S::L1>()))
                return e;
        cfg = true;
    }
    const bool gu = NCF_LAYERED_GU && users && items && (fold == 2 || fold == 4 || fold == 8);
#define NCF_DW1_LAUNCH(F)                                                                                     \
    launch(k_lay_dw1<S::L0, S::L1, F>, nchunks * kDw1Split, 64 * kDw1Waves, dw1_lds<S::L0, S::L1>(), st, x0, g1, n, \
           (int)chunk, slabs, (int64_t)s.mlp_params, users, items, ids)
    if (gu && fold == 2) NCF_DW1_LAUNCH(2);
    else if (gu && fold == 4) NCF_DW1_LAUNCH(4);
    else if (gu && fold == 8) NCF_DW1_LAUNCH(8);
    else NCF_DW1_LAUNCH(0);
#undef NCF_DW1_LAUNCH
    return hipGetLastError();
}

hipError_t launch_layer1_bwd(const ncf_shape_t& s, const float* emb, const float* mlp, const int32_t* users,
                             const int32_t* items, int64_t n, IdSpace ids, const float* dzo, const float* g1,
                             float* gs, hipStream_t st, int fold) {
    using S = L1ShapeD;
    if (!l1matches<S>(s) || (fold > 1 && fold != 2 && fold != 4 && fold != 8)) return hipErrorInvalidValue;
    static bool cfg = false;
    if (!cfg) {
        if (hipError_t e = configure<S>((const void*)k_lay_l1b<S, NCF_L1B_WAVES, 0>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1b<S, NCF_L1B_WAVES, 2>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1b<S, NCF_L1B_WAVES, 4>)) return e;
        if (hipError_t e = configure<S>((const void*)k_lay_l1b<S, NCF_L1B_WAVES, 8>)) return e;
        cfg = true;
    }
#define NCF_L1B_LAUNCH(F)                                                                                   \
    launch(k_lay_l1b<S, NCF_L1B_WAVES, F>, grid_of<S, NCF_L1B_WAVES>(n), 64 * NCF_L1B_WAVES, S::LDS, st, emb, mlp, \
           s.layer_off[0], users, items, n, ids, dzo, g1, gs)
    if (fold == 2) NCF_L1B_LAUNCH(2);
    else if (fold == 4) NCF_L1B_LAUNCH(4);
    else if (fold == 8) NCF_L1B_LAUNCH(8);
    else NCF_L1B_LAUNCH(0);
#undef NCF_L1B_LAUNCH
    return hipGetLastError();
}

}  // namespace ncf
