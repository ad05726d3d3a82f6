// Sample-unit fused NeuMF forward + backward on CDNA4 fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// One 256-thread workgroup (4 waves) per CU, persistent over UNITS of 32 samples.  The tile
// kernel (ncf_fused.hip) gives each wave its own 32 samples and the whole per-sample chain; here
// the 4 waves share one unit and split every layer's OUTPUT features between them.  Activations
// live in LDS as [feature][sample] with row stride 36 floats, which is bank-conflict-free for all
// three 16x16x4 operand patterns used below (B = act[k][s] with k on the lane group, A =
// act[k][s] with k on the lane, and the accumulator write-back).  A layer is one barrier-
// separated phase of independent 16x16 MFMA chains: with 16-row output blocks a 64-wide layer
// over 32 samples is 8 chains, so no wave ever reduces another wave's partial sums.
//
//   forward:  H1 = relu(W1^T X + b1), H2, H3 (A = W_l[k][o] from LDS, B = the activation)
//   output:   z = wo . [u_gmf * i_gmf | H3] + bo, Keras-clipped BCE, dz = (p - y) / B
//   backward: G3 = dz wo ⊙ relu'(H3), G2 = (W3 G3) ⊙ relu'(H2), G1 = (W2 G2) ⊙ relu'(H1),
//             dX = W1 G1 (A = W_l[k][o] with k on the lane)   -> per-sample gradient rows gs
//   weights:  dW_l += H_{l-1} G_l^T over the unit's samples (K = 32: 8 MFMA steps per tile),
//             tiles owned by one wave each and kept in accumulators across units
//
// A unit's critical path is about a quarter of a 128-sample tile's, so at 8192 samples (256
// units) every CU works and the launch is ~4x shorter than the tile kernel's 64 workgroups; the
// flops per sample are the same.  Outputs are those of k_fb_fused (probs, gs rows with the same
// user-row folding, one dense-gradient slab, one BCE / hit / dcg partial per workgroup), so the
// index, update and reduction launches do not care which kernel ran.  Every sum has a fixed
// order: results are bitwise reproducible.  Reference semantics: movierec/model.py:154-214.

#include <cmath>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// LDS row stride of a weight matrix with `lout` (padded) columns: conflict-free both as the
// forward A operand (lanes: 16 consecutive columns x 4 rows) and as the backward A operand
// (lanes: 16 consecutive rows x 4 columns), for ds_read_b32's 32-lane halves.
constexpr int wstride(int lout) { return lout <= 16 ? 18 : lout <= 32 ? 36 : lout <= 64 ? 82 : 146; }

template <int L0_, int L1_, int L2_, int L3_, int G_>
struct UShape {
    static constexpr int L0 = L0_, L1 = L1_, L2 = L2_, L3 = L3_, G = G_;
    static_assert(L0 % 16 == 0 && L1 % 16 == 0 && L2 % 16 == 0 && L3 % 8 == 0 && L3 <= 16 && G % 8 == 0,
                  "unit-kernel shapes");
    static constexpr int D0 = L0 / 2, W = G + D0;
    static constexpr int B0 = L0 / 16, B1 = L1 / 16, B2 = L2 / 16, B3 = 1, P3 = 16;
    // flat dense-parameter offsets (include/movierec_ncf.h layout)
    static constexpr int OW1 = 0, OB1 = L0 * L1, OW2 = OB1 + L1, OB2 = OW2 + L1 * L2, OW3 = OB2 + L2,
                         OB3 = OW3 + L2 * L3, OWO = OB3 + L3, OBO = OWO + G + L3, P = OBO + 1;
    // LDS: dense parameters (zero-padded to 16-column blocks), then the unit's activations
    static constexpr int LW1 = wstride(L1), LW2 = wstride(L2), LW3 = wstride(P3);
    static constexpr int SW1 = 0, SW2 = SW1 + L0 * LW1, SW3 = SW2 + L1 * LW2, SB1 = SW3 + L2 * LW3,
                         SB2 = SB1 + L1, SB3 = SB2 + L2, SWO = SB3 + P3, SBO = SWO + G + P3,
                         WLDS = (SBO + 1 + 3) / 4 * 4;
    static constexpr int LA = 36;  // activation row stride (floats)
    static constexpr int RX = 0, RH1 = RX + L0, RH2 = RH1 + L1, RH3 = RH2 + L2, RG1 = RH3 + P3, RG2 = RG1 + L1,
                         RG3 = RG2 + L2, RN = RG3 + P3;
    static constexpr int XP = L0 / 8;  // MLP-input floats gathered per thread (8 threads per sample)
    static constexpr int GP = G / 8;   // GMF floats per thread
    static_assert(XP % 4 == 0, "float4 gather");
    static constexpr int NBIAS = L1 + L2 + L3;
    static_assert(NBIAS <= 128, "bias rows: one per thread of waves 2-3");
    static constexpr size_t LDS_BYTES = (size_t)(WLDS + RN * LA + 8 * 32 + 32 + 32) * 4;
    static_assert(LDS_BYTES <= 163840, "LDS budget");
};

// A phase's Bo 16-row output blocks x 2 sample blocks over the 4 waves: Bo % 4 == 0 — wave w
// takes blocks w, w+4, ... and both sample blocks (the A operand is read once for both);
// Bo == 2 — one (block, sample block) pair per wave; Bo == 1 — waves 0-1, one sample block each.
template <int Bo>
struct OutSplit {
    static_assert(Bo == 1 || Bo == 2 || Bo % 4 == 0, "output blocks");
    static constexpr int NA = Bo % 4 == 0 ? Bo / 4 : 1;
    static constexpr int NB = Bo % 4 == 0 ? 2 : 1;
    __device__ static bool active(int w) { return Bo != 1 || w < 2; }
    __device__ static int ob(int w, int a) { return Bo % 4 == 0 ? w + 4 * a : Bo == 2 ? (w >> 1) : 0; }
    __device__ static int cb(int w, int b) { return Bo % 4 == 0 ? b : (w & 1); }
};

// Weight-gradient tiles: Bi input blocks x Bo output blocks, each owned by one wave.
template <int Bi, int Bo>
struct DwSplit {
    static constexpr bool BYI = Bi % 4 == 0;                    // input blocks w, w+4, ... x all outputs
    static constexpr bool HALF = !BYI && Bi == 2 && Bo % 2 == 0;  // input block w&1 x half the outputs
    static constexpr bool QUART = !BYI && Bi == 1 && Bo % 4 == 0;
    static constexpr int NA = BYI ? Bi / 4 : 1;
    static constexpr int NB = BYI ? Bo : HALF ? Bo / 2 : QUART ? Bo / 4 : Bo;
    // the rest: Bi == 2 (odd Bo) on waves 0-1, Bi == 1 on wave 2 (waves 0-1 may hold dW3 tiles)
    __device__ static bool active(int w) { return BYI || HALF || QUART || (Bi == 2 ? w < 2 : w == 2); }
    __device__ static int kb(int w, int a) { return BYI ? w + 4 * a : Bi == 2 ? (w & 1) : 0; }
    __device__ static int ob(int w, int b) { return BYI ? b : HALF ? (w >> 1) * NB + b : QUART ? w * NB + b : b; }
};

// acc[a][b] += sum over NS steps of A(a, t) x B(b, t): NA x NB independent 16x16 chains, the
// operands of the next 4 steps read (LDS) while the current 4 steps' MFMAs issue.
template <int NS, int NA, int NB, class FA, class FB>
__device__ __forceinline__ void mma_grid(f32x4 (&acc)[NA][NB], FA fa, FB fb) {
    constexpr int CH = NS < 4 ? NS : 4;
    static_assert(NS % CH == 0, "steps");
    float a[2][CH][NA], b[2][CH][NB];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
#pragma unroll
        for (int i = 0; i < NA; ++i) a[0][e][i] = fa(i, e);
#pragma unroll
        for (int i = 0; i < NB; ++i) b[0][e][i] = fb(i, e);
    }
#pragma unroll
    for (int c = 0; c < NS / CH; ++c) {
        if (c + 1 < NS / CH) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
#pragma unroll
                for (int i = 0; i < NA; ++i) a[(c + 1) & 1][e][i] = fa(i, CH * (c + 1) + e);
#pragma unroll
                for (int i = 0; i < NB; ++i) b[(c + 1) & 1][e][i] = fb(i, CH * (c + 1) + e);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < CH; ++e)
#pragma unroll
            for (int ia = 0; ia < NA; ++ia)
#pragma unroll
                for (int ib = 0; ib < NB; ++ib) acc[ia][ib] = mfma16(a[c & 1][e][ia], b[c & 1][e][ib], acc[ia][ib]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// x summed over the FOLD consecutive lanes of its group (FOLD 2, 4, 8; all lanes active)
template <int FOLD>
__device__ __forceinline__ float fold_sum(float x) {
    static_assert(FOLD == 2 || FOLD == 4 || FOLD == 8, "fold width");
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    if constexpr (FOLD >= 4)
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    if constexpr (FOLD >= 8) x += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x1F | (4 << 10)));
    return x;
}

__device__ __forceinline__ float wave_half_sum(float x) {
#pragma unroll
    for (int m = 16; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

// forward layer phase: out[o][s] = relu(sum_k W[k][o] in[k][s] + b[o]) (NS = K / 4 steps)
template <int Bo, int NS, int LW, int LA>
__device__ __forceinline__ void fwd_phase(const float* __restrict__ wt, const float* __restrict__ bias, int lout,
                                          const float* __restrict__ in, float* __restrict__ out, int w, int li,
                                          int lq) {
    using A = OutSplit<Bo>;
    if (!A::active(w)) return;
    f32x4 acc[A::NA][A::NB];
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma_grid<NS, A::NA, A::NB>(
        acc, [&](int a, int t) { return wt[(4 * t + lq) * LW + 16 * A::ob(w, a) + li]; },
        [&](int b, int t) { return in[(4 * t + lq) * LA + 16 * A::cb(w, b) + li]; });
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * A::ob(w, i) + 4 * lq + r;
                out[row * LA + 16 * A::cb(w, k) + li] = row < lout ? fmaxf(acc[i][k][r] + bias[row], 0.f) : 0.f;
            }
}

// backward data phase: gin[k][s] = (hin[k][s] > 0) ? sum_o W[k][o] gout[o][s] : 0
template <int Bo, int NS, int LW, int LA>
__device__ __forceinline__ void bwd_phase(const float* __restrict__ wt, const float* __restrict__ gout,
                                          const float* __restrict__ hin, float* __restrict__ gin, int w, int li,
                                          int lq) {
    using A = OutSplit<Bo>;
    if (!A::active(w)) return;
    f32x4 acc[A::NA][A::NB];
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma_grid<NS, A::NA, A::NB>(
        acc, [&](int a, int t) { return wt[(16 * A::ob(w, a) + li) * LW + 4 * t + lq]; },
        [&](int b, int t) { return gout[(4 * t + lq) * LA + 16 * A::cb(w, b) + li]; });
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = (16 * A::ob(w, i) + 4 * lq + r) * LA + 16 * A::cb(w, k) + li;
                gin[o] = hin[o] > 0.f ? acc[i][k][r] : 0.f;
            }
}

// weight-gradient phase: acc[a][b] += in[kb-block][s] x g[ob-block][s] over the unit's 32 samples
template <int Bi, int Bo, int LA, class ACC>
__device__ __forceinline__ void dw_phase(ACC& acc, const float* __restrict__ in, const float* __restrict__ g, int w, int li,
                                         int lq) {
    using D = DwSplit<Bi, Bo>;
    if (!D::active(w)) return;
    mma_grid<8, D::NA, D::NB>(
        acc, [&](int a, int t) { return in[(16 * D::kb(w, a) + li) * LA + 4 * t + lq]; },
        [&](int b, int t) { return g[(16 * D::ob(w, b) + li) * LA + 4 * t + lq]; });
}

template <int Bi, int Bo, class ACC>
__device__ __forceinline__ void dw_store(const ACC& acc, float* __restrict__ dst, int lin, int lout, int w, int li, int lq) {
    using D = DwSplit<Bi, Bo>;
    if (!D::active(w)) return;
#pragma unroll
    for (int a = 0; a < D::NA; ++a)
#pragma unroll
        for (int b = 0; b < D::NB; ++b) {
            const int col = 16 * D::ob(w, b) + li;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * D::kb(w, a) + 4 * lq + r;
                if (row < lin && col < lout) dst[row * lout + col] = acc[a][b][r];
            }
        }
}

// Phase timestamps (lane 0 of every wave, first two units of every workgroup): a profiling
// build (-DNCF_UNIT_TIMING) only; read with ncf_debug_unit_timing (tools/unit_timing.py).
#ifdef NCF_UNIT_TIMING
__device__ unsigned long long g_unit_t[256 * 2 * 4 * 20];
#define NCF_UT(ph)                                                                                  \
    do {                                                                                            \
        if (lane == 0 && blockIdx.x < 256 && itl < 2)                                               \
            g_unit_t[((blockIdx.x * 2 + itl) * 4 + w) * 20 + (ph)] = __builtin_readcyclecounter(); \
    } while (0)
#else
#define NCF_UT(ph) ((void)0)
#endif

template <class S, int FOLD>
__global__ __launch_bounds__(kBlock, 1) void k_fb_unit(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                       const int32_t* __restrict__ users,
                                                       const int32_t* __restrict__ items,
                                                       const float* __restrict__ labels, int64_t n, IdSpace ids,
                                                       float inv_batch, float* __restrict__ probs,
                                                       float* __restrict__ gs, float* __restrict__ slabs,
                                                       float* __restrict__ part_bce, int group, int topk,
                                                       float* __restrict__ part_hit, float* __restrict__ part_dcg) {
    constexpr int L0 = S::L0, L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, D0 = S::D0, W = S::W, LA = S::LA;
    constexpr int XP = S::XP, GP = S::GP, GPA = GP > 0 ? GP : 1;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wl = lds;
    float* act = lds + S::WLDS;                 // [RN][LA]
    float* zpart = act + S::RN * LA;            // [8][32] GMF partial dots
    float* dzb = zpart + 256;                   // [32] dz of the unit's samples
    int* su = reinterpret_cast<int*>(dzb + 32);  // [32] their user ids (-1: past n)

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;  // 16x16x4 operand coordinates
    const int sj = lane & 31, p = tid >> 5;    // gather / GMF / output role: sample sj, part p
    const float eps = 1e-7f, hi_clip = 1.0f - eps;
    const bool metrics = part_hit != nullptr;

    // dense parameters -> LDS (padding zeroed first: the L3 < 16 columns are read as zeros)
    for (int e = tid; e < S::WLDS; e += kBlock) wl[e] = 0.f;
    __syncthreads();
    for (int e = tid; e < L0 * L1; e += kBlock) wl[S::SW1 + (e / L1) * S::LW1 + e % L1] = mlp[S::OW1 + e];
    for (int e = tid; e < L1 * L2; e += kBlock) wl[S::SW2 + (e / L2) * S::LW2 + e % L2] = mlp[S::OW2 + e];
    for (int e = tid; e < L2 * L3; e += kBlock) wl[S::SW3 + (e / L3) * S::LW3 + e % L3] = mlp[S::OW3 + e];
    for (int e = tid; e < L1; e += kBlock) wl[S::SB1 + e] = mlp[S::OB1 + e];
    for (int e = tid; e < L2; e += kBlock) wl[S::SB2 + e] = mlp[S::OB2 + e];
    for (int e = tid; e < L3; e += kBlock) wl[S::SB3 + e] = mlp[S::OB3 + e];
    for (int e = tid; e < G; e += kBlock) wl[S::SWO + e] = mlp[S::OWO + e];
    for (int e = tid; e < L3; e += kBlock) wl[S::SWO + G + e] = mlp[S::OWO + G + e];
    if (tid == 0) wl[S::SBO] = mlp[S::OBO];
    __syncthreads();

    using S1 = DwSplit<S::B0, S::B1>;
    using S2 = DwSplit<S::B1, S::B2>;
    using S3 = DwSplit<S::B2, S::B3>;
    f32x4 dw1[S1::NA][S1::NB], dw2[S2::NA][S2::NB], dw3[S3::NA][S3::NB];
#pragma unroll
    for (int a = 0; a < S1::NA; ++a)
#pragma unroll
        for (int b = 0; b < S1::NB; ++b) dw1[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < S2::NA; ++a)
#pragma unroll
        for (int b = 0; b < S2::NB; ++b) dw2[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < S3::NA; ++a)
#pragma unroll
        for (int b = 0; b < S3::NB; ++b) dw3[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    float acc_gmf[GPA], acc_h3[2];
#pragma unroll
    for (int e = 0; e < GPA; ++e) acc_gmf[e] = 0.f;
    acc_h3[0] = acc_h3[1] = 0.f;
    float acc_bias = 0.f, acc_bce = 0.f, acc_dbo = 0.f, acc_hit = 0.f, acc_dcg = 0.f;

    const int64_t nunits = (n + 31) / 32;
    int itl = -1;
    for (int64_t un = blockIdx.x; un < nunits; un += gridDim.x) {
        ++itl;
        NCF_UT(0);
        const int64_t s0 = un * 32;
        // ---- gather: thread (sj, p) brings part p of its sample's MLP input (parts 0-3: the user
        // half, 4-7: the item half) and part p of both GMF slices.  Masked samples read row 0 (a
        // valid address) and get dz = 0: they contribute nothing.
        const int64_t si = s0 + sj;
        const bool inb = si < n;
        int u = 0, v = 0;
        float y = 0.f;
        if (inb) {
            u = users[si];
            v = items[si];
            y = labels[si];
        }
        const bool ok = inb && (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
        const int urow = ok ? u : 0, irow = ok ? ids.ibase + v : 0;
        {
            const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)(p < 4 ? urow : irow) * W + G + (p & 3) * XP);
            float4 xv[XP / 4];
#pragma unroll
            for (int q = 0; q < XP / 4; ++q) xv[q] = xs[q];
#pragma unroll
            for (int q = 0; q < XP / 4; ++q) {
                float* dst = act + (S::RX + p * XP + 4 * q) * LA + sj;
                dst[0] = xv[q].x;
                dst[LA] = xv[q].y;
                dst[2 * LA] = xv[q].z;
                dst[3 * LA] = xv[q].w;
            }
        }
        float ug[GPA], ig[GPA];
        if constexpr (G > 0) {
            const float* us = emb + (size_t)urow * W + p * GP;
            const float* is = emb + (size_t)irow * W + p * GP;
            if constexpr (GP % 4 == 0) {
#pragma unroll
                for (int q = 0; q < GP / 4; ++q) {
                    const float4 a = reinterpret_cast<const float4*>(us)[q];
                    const float4 b = reinterpret_cast<const float4*>(is)[q];
                    ug[4 * q] = a.x, ug[4 * q + 1] = a.y, ug[4 * q + 2] = a.z, ug[4 * q + 3] = a.w;
                    ig[4 * q] = b.x, ig[4 * q + 1] = b.y, ig[4 * q + 2] = b.z, ig[4 * q + 3] = b.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < GP; ++e) {
                    ug[e] = us[e];
                    ig[e] = is[e];
                }
            }
            float zg = 0.f;
#pragma unroll
            for (int e = 0; e < GP; ++e) zg += wl[S::SWO + p * GP + e] * (ug[e] * ig[e]);
            zpart[p * 32 + sj] = zg;
        }
        if (p == 0) su[sj] = inb ? u : -1;
        NCF_UT(1);
        __syncthreads();
        NCF_UT(2);

        // ---- forward
        fwd_phase<S::B1, L0 / 4, S::LW1, LA>(wl + S::SW1, wl + S::SB1, L1, act + S::RX * LA, act + S::RH1 * LA, w,
                                             li, lq);
        NCF_UT(3);
        __syncthreads();
        NCF_UT(4);
        fwd_phase<S::B2, L1 / 4, S::LW2, LA>(wl + S::SW2, wl + S::SB2, L2, act + S::RH1 * LA, act + S::RH2 * LA, w,
                                             li, lq);
        NCF_UT(5);
        __syncthreads();
        NCF_UT(6);
        fwd_phase<S::B3, L2 / 4, S::LW3, LA>(wl + S::SW3, wl + S::SB3, L3, act + S::RH2 * LA, act + S::RH3 * LA, w,
                                             li, lq);
        NCF_UT(7);
        __syncthreads();
        NCF_UT(8);

        // ---- output, BCE, dz, hr/dcg (wave 0: lane half h sums every other H3 row)
        if (w == 0) {
            const int h = lane >> 5;
            float zp = 0.f;
#pragma unroll
            for (int f = h; f < L3; f += 2) zp += wl[S::SWO + G + f] * act[(S::RH3 + f) * LA + sj];
            float z = (zp + __shfl_xor(zp, 32, 64));
            if constexpr (G > 0) {
                float zg = 0.f;
#pragma unroll
                for (int q = 0; q < 8; ++q) zg += zpart[q * 32 + sj];
                z += zg;
            }
            z += wl[S::SBO];
            const float pr = 1.0f / (1.0f + expf(-z));
            float dz = 0.f, bce = 0.f;
            if (ok) {
                const float pc = fminf(fmaxf(pr, eps), hi_clip);
                const float logit = logf(pc / (1.0f - pc));
                bce = fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
                dz = (pr >= eps && pr <= hi_clip) ? (pr - y) * inv_batch : 0.0f;
            }
            if (h == 0) {
                if (inb) probs[si] = ok ? pr : __int_as_float(0x7fc00000);
                dzb[sj] = dz;
                acc_bce += bce;
                acc_dbo += dz;
            }
            // RankLayer + _get_hits_per_user (model.py:344-455): label = first max of y;
            // position = #(p > p_lab) + #(earlier ties)
            if (metrics) {
                const int e = sj % group;
                const int base = 32 * h + sj - e;
                int lab = 0;
                float best = __shfl(y, base, 64);
                for (int q = 1; q < group; ++q) {
                    const float yq = __shfl(y, base + q, 64);
                    if (yq > best) {
                        best = yq;
                        lab = q;
                    }
                }
                const float pl = __shfl(pr, base + lab, 64);
                int pos = 0;
                for (int q = 0; q < group; ++q) {
                    const float pq = __shfl(pr, base + q, 64);
                    pos += (pq > pl) || (pq == pl && q < lab);
                }
                if (h == 0 && e == 0 && inb) {
                    const float hit = pos < topk ? 1.f : 0.f;
                    acc_hit += hit;
                    acc_dcg += hit * (logf(2.0f) / logf((float)pos + 2.0f));
                }
            }
        }
        NCF_UT(9);
        __syncthreads();
        NCF_UT(10);

        // ---- G3 and the output-kernel gradient of H3 (element slots e = tid, tid + 256)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q, f = e >> 5, s = e & 31;
            const float h3 = act[(S::RH3 + f) * LA + s];
            const float dz = dzb[s];
            act[(S::RG3 + f) * LA + s] = (f < L3 && h3 > 0.f) ? dz * wl[S::SWO + G + f] : 0.f;
            acc_h3[q] += dz * h3;
        }
        // ---- GMF backward: thread (sj, p), features [p GP, (p+1) GP) of its sample
        const int fm = FOLD > 1 ? FOLD - 1 : 0;
        if constexpr (G > 0) {
            const float dz = dzb[sj];
            const bool fmatch = FOLD > 1 && inb && su[sj] == su[sj & ~fm];
            const bool fhead = (sj & fm) == 0;
            float gu[GP], gi[GP];
#pragma unroll
            for (int e = 0; e < GP; ++e) {
                const float wo = wl[S::SWO + p * GP + e];
                gu[e] = dz * wo * ig[e];
                gi[e] = dz * wo * ug[e];
                acc_gmf[e] += dz * (ug[e] * ig[e]);
            }
            if constexpr (FOLD > 1) {
#pragma unroll
                for (int e = 0; e < GP; ++e) {
                    const float sm = fold_sum<FOLD>(fmatch ? gu[e] : 0.f);
                    if (fhead) gu[e] = sm;
                }
            }
            // masked samples (dz = 0) write zero rows: the index may count their other, valid id
            float* gur = gs + (size_t)(2 * si) * W + p * GP;
            float* gir = gur + W;
            if (inb && (fhead || !fmatch)) {
                if constexpr (GP % 4 == 0) {
#pragma unroll
                    for (int q = 0; q < GP / 4; ++q)
                        st_stream(reinterpret_cast<float4*>(gur) + q,
                                  make_float4(gu[4 * q], gu[4 * q + 1], gu[4 * q + 2], gu[4 * q + 3]));
                } else {
#pragma unroll
                    for (int e = 0; e < GP; ++e) gur[e] = gu[e];
                }
            }
            if (inb) {
                if constexpr (GP % 4 == 0) {
#pragma unroll
                    for (int q = 0; q < GP / 4; ++q)
                        st_stream(reinterpret_cast<float4*>(gir) + q,
                                  make_float4(gi[4 * q], gi[4 * q + 1], gi[4 * q + 2], gi[4 * q + 3]));
                } else {
#pragma unroll
                    for (int e = 0; e < GP; ++e) gir[e] = gi[e];
                }
            }
        }
        NCF_UT(11);
        __syncthreads();
        NCF_UT(12);

        // ---- backward data chain
        bwd_phase<S::B2, S::P3 / 4, S::LW3, LA>(wl + S::SW3, act + S::RG3 * LA, act + S::RH2 * LA, act + S::RG2 * LA,
                                                w, li, lq);
        NCF_UT(13);
        __syncthreads();
        NCF_UT(14);
        bwd_phase<S::B1, L2 / 4, S::LW2, LA>(wl + S::SW2, act + S::RG2 * LA, act + S::RH1 * LA, act + S::RG1 * LA, w,
                                             li, lq);
        NCF_UT(15);
        __syncthreads();
        NCF_UT(16);
        // dX = W1 G1 -> the per-sample gradient rows (user half folded like the GMF part)
        {
            using A = OutSplit<S::B0>;
            f32x4 acc[A::NA][A::NB];
#pragma unroll
            for (int i = 0; i < A::NA; ++i)
#pragma unroll
                for (int k = 0; k < A::NB; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
            mma_grid<L1 / 4, A::NA, A::NB>(
                acc, [&](int a, int t) { return wl[S::SW1 + (16 * A::ob(w, a) + li) * S::LW1 + 4 * t + lq]; },
                [&](int b, int t) { return act[(S::RG1 + 4 * t + lq) * LA + 16 * A::cb(w, b) + li]; });
#pragma unroll
            for (int k = 0; k < A::NB; ++k) {
                const int s = 16 * A::cb(w, k) + li;
                const int64_t sg = s0 + s;
                const bool sinb = sg < n;
                const bool fmatch = FOLD > 1 && sinb && su[s] == su[s & ~fm];
                const bool fhead = (s & fm) == 0;
                float* gur = gs + (size_t)(2 * sg) * W + G;
#pragma unroll
                for (int i = 0; i < A::NA; ++i) {
                    const int f0 = 16 * A::ob(w, i) + 4 * lq;
                    f32x4 d = acc[i][k];
                    if constexpr (FOLD > 1) {
                        if (16 * A::ob(w, i) < D0) {  // uniform per wave: user-half block
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float sm = fold_sum<FOLD>(fmatch ? d[r] : 0.f);
                                if (fhead) d[r] = sm;
                            }
                        }
                    }
                    const bool user = f0 < D0;
                    if (sinb && (!user || fhead || !fmatch))
                        st_stream(reinterpret_cast<float4*>(user ? gur + f0 : gur + W + (f0 - D0)),
                                  make_float4(d[0], d[1], d[2], d[3]));
                }
            }
        }
        NCF_UT(19);
        // ---- weight gradients (operands in LDS) and bias rows
        dw_phase<S::B0, S::B1, LA>(dw1, act + S::RX * LA, act + S::RG1 * LA, w, li, lq);
        dw_phase<S::B1, S::B2, LA>(dw2, act + S::RH1 * LA, act + S::RG2 * LA, w, li, lq);
        dw_phase<S::B2, S::B3, LA>(dw3, act + S::RH2 * LA, act + S::RG3 * LA, w, li, lq);
        if (tid >= 128 && tid - 128 < S::NBIAS) {
            const int br = tid - 128;
            const int rr = br < L1 ? S::RG1 + br : br < L1 + L2 ? S::RG2 + (br - L1) : S::RG3 + (br - L1 - L2);
            const float* row = act + rr * LA;
            float sacc = 0.f;
#pragma unroll
            for (int c = 0; c < 32; ++c) sacc += row[c];
            acc_bias += sacc;
        }
        NCF_UT(17);
        __syncthreads();
        NCF_UT(18);
    }

    // ---- epilogue: this workgroup's dense-gradient slab and BCE / metric partials
    float* slab = slabs + (size_t)blockIdx.x * S::P;
    dw_store<S::B0, S::B1>(dw1, slab + S::OW1, L0, L1, w, li, lq);
    dw_store<S::B1, S::B2>(dw2, slab + S::OW2, L1, L2, w, li, lq);
    dw_store<S::B2, S::B3>(dw3, slab + S::OW3, L2, L3, w, li, lq);
    if (tid >= 128 && tid - 128 < S::NBIAS) {
        const int br = tid - 128;
        if (br < L1) slab[S::OB1 + br] = acc_bias;
        else if (br < L1 + L2) slab[S::OB2 + (br - L1)] = acc_bias;
        else slab[S::OB3 + (br - L1 - L2)] = acc_bias;
    }
    // output kernel: GMF entries (thread (sj, p): features p GP + e) and H3 entries (slot q:
    // feature p + 8q), each summed over the 32 samples of a wave half
    if constexpr (G > 0) {
#pragma unroll
        for (int e = 0; e < GP; ++e) {
            const float v = wave_half_sum(acc_gmf[e]);
            if (sj == 0) slab[S::OWO + p * GP + e] = v;
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const float v = wave_half_sum(acc_h3[q]);
        const int f = p + 8 * q;
        if (sj == 0 && f < L3) slab[S::OWO + G + f] = v;
    }
    if (w == 0) {
        float dbo = acc_dbo, bce = acc_bce, hit = acc_hit, dcg = acc_dcg;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            dbo += __shfl_xor(dbo, m, 64);
            bce += __shfl_xor(bce, m, 64);
            hit += __shfl_xor(hit, m, 64);
            dcg += __shfl_xor(dcg, m, 64);
        }
        if (lane == 0) {
            slab[S::OBO] = dbo;
            part_bce[blockIdx.x] = bce;
            if (metrics) {
                part_hit[blockIdx.x] = hit;
                part_dcg[blockIdx.x] = dcg;
            }
        }
    }
}

using UShapeC = UShape<128, 64, 32, 16, 64>;  // ml-20m NeuMF (config C)
using UShapeB = UShape<64, 32, 16, 8, 8>;     // ml-1m NeuMF (config B)
using UShapeR = UShape<64, 32, 16, 8, 0>;     // reference trainer default (MLP-only)
using UShapeC0 = UShape<128, 64, 32, 16, 0>;

template <class S>
bool umatches(const ncf_shape_t& s) {
    return s.num_layers == 4 && s.layers[0] == S::L0 && s.layers[1] == S::L1 && s.layers[2] == S::L2 &&
           s.layers[3] == S::L3 && s.gmf_dim == S::G && s.row_width == S::W && s.gmf_stride == S::G;
}

template <class S>
hipError_t launch_unit_one(const WsLayout& L, void* ws, const float* emb, const float* mlp, const int32_t* users,
                           const int32_t* items, const float* labels, int64_t n, float inv_batch, IdSpace ids,
                           int group, int topk, int* nslab, int* nbce, int* nmet, hipStream_t st, int fold) {
    static bool configured = false;  // one-time attribute set per shape (idempotent)
    if (!configured) {
        for (const void* k : {(const void*)k_fb_unit<S, 0>, (const void*)k_fb_unit<S, 2>,
                              (const void*)k_fb_unit<S, 4>, (const void*)k_fb_unit<S, 8>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)S::LDS_BYTES);
            if (e != hipSuccess) return e;
        }
        configured = true;
    }
    const int64_t nunits = (n + 31) / 32;
    int grid = (int)(nunits < 256 ? nunits : 256);
    if (grid < 1) grid = 1;
    const bool in_kernel = group > 0 && group <= 32 && 32 % group == 0;
    auto go = [&](auto kern) {
        launch(kern, grid, kBlock, S::LDS_BYTES, st, emb, mlp, users, items, labels, n, ids, inv_batch,
               at<float>(ws, L.probs), at<float>(ws, L.gs), at<float>(ws, L.slabs), at<float>(ws, L.part_bce), group,
               topk, in_kernel ? at<float>(ws, L.part_hit) : nullptr, in_kernel ? at<float>(ws, L.part_dcg) : nullptr);
    };
    switch (fold) {
        case 0: go(k_fb_unit<S, 0>); break;
        case 2: go(k_fb_unit<S, 2>); break;
        case 4: go(k_fb_unit<S, 4>); break;
        case 8: go(k_fb_unit<S, 8>); break;
        default: return hipErrorInvalidValue;
    }
    *nslab = grid;
    *nbce = grid;
    *nmet = in_kernel ? grid : 0;
    return hipGetLastError();
}

}  // namespace

#ifdef NCF_UNIT_TIMING
extern "C" int ncf_debug_unit_timing(unsigned long long* out, size_t count) {
    size_t m = count < sizeof(g_unit_t) / 8 ? count : sizeof(g_unit_t) / 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_unit_t), m * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif

bool unit_supported(const ncf_shape_t& s) {
    return umatches<UShapeC>(s) || umatches<UShapeB>(s) || umatches<UShapeR>(s) || umatches<UShapeC0>(s);
}

hipError_t launch_fb_unit(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                          const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                          float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                          hipStream_t st, int fold) {
    if (fold != 0 && (fold < 2 || fold > 8 || (fold & (fold - 1)) != 0 || n % fold != 0)) return hipErrorInvalidValue;
#define NCF_TRY(SH)                                                                                                  \
    if (umatches<SH>(s))                                                                                             \
    return launch_unit_one<SH>(L, ws, emb, mlp, users, items, labels, n, inv_batch, ids, group, topk, nslab, nbce, \
                               nmet, st, fold)
    NCF_TRY(UShapeC);
    NCF_TRY(UShapeB);
    NCF_TRY(UShapeR);
    NCF_TRY(UShapeC0);
#undef NCF_TRY
    return hipErrorInvalidValue;
}

}  // namespace ncf
