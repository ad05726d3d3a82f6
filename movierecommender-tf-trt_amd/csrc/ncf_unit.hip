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

template <int L0_, int L1_, int L2_, int L3_, int G_, int U_, int NG_>
struct UShape {
    static constexpr int L0 = L0_, L1 = L1_, L2 = L2_, L3 = L3_, G = G_, U = U_;
    // NG unit groups of 4 waves per workgroup, each on its own unit (2: two waves per SIMD, the
    // dense parameters in LDS once for both)
    static constexpr int NG = NG_, NT = 256 * NG_;
    static_assert(L0 % 16 == 0 && L1 % 16 == 0 && L2 % 16 == 0 && L3 % 8 == 0 && L3 <= 16 && G % 8 == 0,
                  "unit-kernel shapes");
    static_assert(U == 32 || U == 64, "unit size");
    static constexpr int D0 = L0 / 2, W = G + D0;
    static constexpr int B0 = L0 / 16, B1 = L1 / 16, B2 = L2 / 16, B3 = 1, P3 = 16;
    static constexpr int NC = U / 16;  // 16-sample column blocks of a unit
    static constexpr int NQ = U / 32;  // 32-sample halves (each its own [row][36] buffer)
    // flat dense-parameter offsets (include/movierec_ncf.h layout)
    static constexpr int OW1 = 0, OB1 = L0 * L1, OW2 = OB1 + L1, OB2 = OW2 + L1 * L2, OW3 = OB2 + L2,
                         OB3 = OW3 + L2 * L3, OWO = OB3 + L3, OBO = OWO + G + L3, P = OBO + 1;
    // LDS: dense parameters (zero-padded to 16-column blocks), then the unit's activations
    static constexpr int LW1 = wstride(L1), LW2 = wstride(L2), LW3 = wstride(P3);
    static constexpr int SW1 = 0, SW2 = SW1 + L0 * LW1, SW3 = SW2 + L1 * LW2, SB1 = SW3 + L2 * LW3,
                         SB2 = SB1 + L1, SB3 = SB2 + L2, SWO = SB3 + P3, SBO = SWO + G + P3,
                         WLDS = (SBO + 1 + 3) / 4 * 4;
    static constexpr int LA = 36;  // activation row stride (floats) of a 32-sample half
    // (H3 never leaves registers: layer 3, the output and G3 share one phase)
    static constexpr int RX = 0, RH1 = RX + L0, RH2 = RH1 + L1, RG1 = RH2 + L2, RG2 = RG1 + L1, RG3 = RG2 + L2,
                         RN = RG3 + P3;
    static constexpr int HS = RN * LA;  // floats per half
    static constexpr int XP = L0 / 8;   // MLP-input floats gathered per thread and sample (8 threads per sample)
    static constexpr int GP = G / 8;    // GMF floats per thread and sample
    static_assert(XP % 4 == 0, "float4 gather");
    static constexpr int NBIAS = L1 + L2 + L3;
    static_assert(NBIAS <= 128, "bias rows: one per lane of roles 0-1");
    static constexpr int GREG = NQ * HS + 8 * U + 5 * U;  // floats of one group's unit buffers
    static constexpr size_t LDS_BYTES = (size_t)(WLDS + NG * GREG) * 4;
    static_assert(LDS_BYTES <= 163840, "LDS budget");
};

// element (row, sample 32 half + c) of the activation buffers: 32-sample halves, [row][LA] each.
// `half` is always known at compile time or wave-uniform at the call sites, so an operand read
// is one ds_read with an immediate offset from a per-lane base.
template <class S>
__device__ __forceinline__ int aidx(int half, int row, int c) {
    return half * S::HS + row * S::LA + c;
}
// sample column of 16-column block cb, lane li
template <class S>
__device__ __forceinline__ int cidx(int row, int cb, int li) {
    return aidx<S>(cb >> 1, row, 16 * (cb & 1) + li);
}

// A phase's Bo 16-row output blocks x NC sample blocks over the 4 waves: Bo % 4 == 0 — wave w
// takes blocks w, w+4, ... and every sample block (the A operand is read once for all);
// Bo == 2 — one block, half the sample blocks per wave; Bo == 1 — the sample blocks split.
template <int Bo, int NC>
struct OutSplit {
    static_assert(Bo == 1 || Bo == 2 || Bo % 4 == 0, "output blocks");
    static constexpr int NA = Bo % 4 == 0 ? Bo / 4 : 1;
    static constexpr int NB = Bo % 4 == 0 ? NC : Bo == 2 ? NC / 2 : (NC >= 4 ? NC / 4 : 1);
    __device__ static bool active(int w) { return Bo != 1 || NC >= 4 || w < 2; }
    __device__ static int ob(int w, int a) { return Bo % 4 == 0 ? w + 4 * a : Bo == 2 ? (w >> 1) : 0; }
    __device__ static int cb(int w, int b) {
        return Bo % 4 == 0 ? b : Bo == 2 ? (w & 1) * NB + b : (NC >= 4 ? w * NB + b : (w & 1));
    }
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

// acc[a][b] += sum over the K steps of A(a, k) x B(b, k): NA x NB independent 16x16 chains.
// The operand functions take (block, kc, kr) with k = kc + kr: kc known at compile time, kr the
// lane's offset (lq for the fp32 16x16x4 form, 4 lq for bf16 16x16x16), so an LDS operand is a
// read at an immediate offset from a per-lane base.
//
// fp32 (v_mfma_f32_16x16x4_f32): lane (li, lq) supplies k = 4 t + lq.  The operands of the next CH
// steps are read while the current CH steps' MFMAs issue; CH keeps a chunk's reads within the 15
// that lgkmcnt can count (more would force a full drain per chunk).
template <int K, int NA, int NB, class FA, class FB>
__device__ __forceinline__ void mma_grid(f32x4 (&acc)[NA][NB], FA fa, FB fb, int lq) {
    constexpr int NS = K / 4;
    constexpr int CHM = 15 / (NA + NB) >= 4 ? 4 : 15 / (NA + NB) >= 2 ? 2 : 1;
    constexpr int CH = NS < CHM ? NS : CHM;
    static_assert(K % 4 == 0 && NS % CH == 0, "steps");
    float a[2][CH][NA], b[2][CH][NB];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
#pragma unroll
        for (int i = 0; i < NA; ++i) a[0][e][i] = fa(i, 4 * e, lq);
#pragma unroll
        for (int i = 0; i < NB; ++i) b[0][e][i] = fb(i, 4 * e, lq);
    }
#pragma unroll
    for (int c = 0; c < NS / CH; ++c) {
        if (c + 1 < NS / CH) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
#pragma unroll
                for (int i = 0; i < NA; ++i) a[(c + 1) & 1][e][i] = fa(i, 4 * (CH * (c + 1) + e), lq);
#pragma unroll
                for (int i = 0; i < NB; ++i) b[(c + 1) & 1][e][i] = fb(i, 4 * (CH * (c + 1) + e), lq);
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

// bf16 operands, fp32 accumulation (v_mfma_f32_16x16x16_bf16): lane (li, lq) supplies
// k = 16 t + 4 lq + j, j = 0..3, rounded to bf16 (RNE, v_cvt_pk_bf16_f32) as they are read.
// The next step's operands are read while the current step's MFMAs issue.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int K, int NA, int NB, class FA, class FB>
__device__ __forceinline__ void mma_grid_bf(f32x4 (&acc)[NA][NB], FA fa, FB fb, int lq) {
    constexpr int NS = K / 16;
    static_assert(K % 16 == 0, "bf16 steps cover 16 k");
    s16x4 a[2][NA], b[2][NB];
    auto load = [&](int t, s16x4 (&aa)[NA], s16x4 (&bb)[NB]) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const bf16x4 v = {(__bf16)fa(i, 16 * t, 4 * lq), (__bf16)fa(i, 16 * t + 1, 4 * lq),
                              (__bf16)fa(i, 16 * t + 2, 4 * lq), (__bf16)fa(i, 16 * t + 3, 4 * lq)};
            aa[i] = __builtin_bit_cast(s16x4, v);
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const bf16x4 v = {(__bf16)fb(i, 16 * t, 4 * lq), (__bf16)fb(i, 16 * t + 1, 4 * lq),
                              (__bf16)fb(i, 16 * t + 2, 4 * lq), (__bf16)fb(i, 16 * t + 3, 4 * lq)};
            bb[i] = __builtin_bit_cast(s16x4, v);
        }
    };
    load(0, a[0], b[0]);
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        if (t + 1 < NS) load(t + 1, a[(t + 1) & 1], b[(t + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ia = 0; ia < NA; ++ia)
#pragma unroll
            for (int ib = 0; ib < NB; ++ib)
                acc[ia][ib] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[t & 1][ia], b[t & 1][ib], acc[ia][ib], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <bool BF, int K, int NA, int NB, class FA, class FB>
__device__ __forceinline__ void mma(f32x4 (&acc)[NA][NB], FA fa, FB fb, int lq) {
    if constexpr (BF) mma_grid_bf<K, NA, NB>(acc, fa, fb, lq);
    else mma_grid<K, NA, NB>(acc, fa, fb, lq);
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
template <class S, bool BF, int Bo, int K, int LW>
__device__ __forceinline__ void fwd_phase(const float* __restrict__ wt, const float* __restrict__ bias, int lout,
                                          const float* __restrict__ act, int rin, int rout, float* __restrict__ actw,
                                          int w, int li, int lq) {
    using A = OutSplit<Bo, S::NC>;
    if (!A::active(w)) return;
    f32x4 acc[A::NA][A::NB];
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma<BF, K, A::NA, A::NB>(
        acc, [&](int a, int kc, int kr) { return wt[(kc + kr) * LW + 16 * A::ob(w, a) + li]; },
        [&](int b, int kc, int kr) { return act[cidx<S>(rin + kc + kr, A::cb(w, b), li)]; }, lq);
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * A::ob(w, i) + 4 * lq + r;
                actw[cidx<S>(rout + row, A::cb(w, k), li)] =
                    row < lout ? fmaxf(acc[i][k][r] + bias[row], 0.f) : 0.f;
            }
}

// backward data phase: gin[k][s] = (hin[k][s] > 0) ? sum_o W[k][o] gout[o][s] : 0
template <class S, bool BF, int Bo, int K, int LW>
__device__ __forceinline__ void bwd_phase(const float* __restrict__ wt, const float* __restrict__ act, int rgout,
                                          int rhin, int rgin, float* __restrict__ actw, int w, int li, int lq) {
    using A = OutSplit<Bo, S::NC>;
    if (!A::active(w)) return;
    f32x4 acc[A::NA][A::NB];
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma<BF, K, A::NA, A::NB>(
        acc, [&](int a, int kc, int kr) { return wt[(16 * A::ob(w, a) + li) * LW + kc + kr]; },
        [&](int b, int kc, int kr) { return act[cidx<S>(rgout + kc + kr, A::cb(w, b), li)]; }, lq);
#pragma unroll
    for (int i = 0; i < A::NA; ++i)
#pragma unroll
        for (int k = 0; k < A::NB; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * A::ob(w, i) + 4 * lq + r, cb = A::cb(w, k);
                actw[cidx<S>(rgin + row, cb, li)] = act[cidx<S>(rhin + row, cb, li)] > 0.f ? acc[i][k][r] : 0.f;
            }
}

// weight-gradient phase: acc[a][b] += in[kb-block][s] x g[ob-block][s] over the unit's samples
template <class S, bool BF, int Bi, int Bo, class ACC>
__device__ __forceinline__ void dw_phase(ACC& acc, const float* __restrict__ act, int rin, int rg, int w, int li,
                                         int lq) {
    using D = DwSplit<Bi, Bo>;
    if (!D::active(w)) return;
    // K = the unit's samples, k = kc + kr: 32-sample half kc >> 5 (the lane offset never carries)
    mma<BF, S::U, D::NA, D::NB>(
        acc,
        [&](int a, int kc, int kr) { return act[aidx<S>(kc >> 5, rin + 16 * D::kb(w, a) + li, (kc & 31) + kr)]; },
        [&](int b, int kc, int kr) { return act[aidx<S>(kc >> 5, rg + 16 * D::ob(w, b) + li, (kc & 31) + kr)]; }, lq);
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
        if (lane == 0 && gq == 0 && blockIdx.x < 256 && itl < 2)                                    \
            g_unit_t[((blockIdx.x * 2 + itl) * 4 + w) * 20 + (ph)] = __builtin_readcyclecounter(); \
    } while (0)
#else
#define NCF_UT(ph) ((void)0)
#endif

template <class S, int FOLD, bool BF>
__global__ __launch_bounds__(S::NT, 1) void k_fb_unit(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                       const int32_t* __restrict__ users,
                                                       const int32_t* __restrict__ items,
                                                       const float* __restrict__ labels, int64_t n, IdSpace ids,
                                                       float inv_batch, float* __restrict__ probs,
                                                       float* __restrict__ gs, float* __restrict__ slabs,
                                                       float* __restrict__ part_bce, int group, int topk,
                                                       float* __restrict__ part_hit, float* __restrict__ part_dcg,
                                                       const int32_t* __restrict__ ifold, int32_t* __restrict__ ferr,
                                                       FillArgs fa, int nunit_blocks) {
    constexpr int L0 = S::L0, L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, D0 = S::D0, W = S::W, U = S::U;
    // a batch counted and scanned ahead (fa.cnt) and a unit grid that leaves CUs idle: the
    // workgroups past the unit grid fill this batch's index there (fill_wave) — no fill launch
    if ((int)blockIdx.x >= nunit_blocks) {
        if (fa.cnt)
            fill_wave(fa, users, items, n, FOLD, ((int)blockIdx.x - nunit_blocks) * (S::NT / 64) + (int)(threadIdx.x >> 6),
                      ((int)gridDim.x - nunit_blocks) * (S::NT / 64));
        return;
    }
    // an index built by an earlier call (ncf_build_index / ncf_shard_plan) must fold as this kernel does
    if (ifold && blockIdx.x == 0 && threadIdx.x == 0 && *ifold != FOLD) atomicOr(ferr, kErrFold);
    constexpr int XP = S::XP, GP = S::GP, GPA = GP > 0 ? GP : 1, NQ = S::NQ;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wl = lds;
    const int gq = threadIdx.x >> 8;                 // this thread's unit group
    float* act = lds + S::WLDS + gq * S::GREG;       // NQ halves of [RN][LA]
    float* zpart = act + NQ * S::HS;                 // [8][U] GMF partial dots
    float* dzb = zpart + 8 * U;                      // [U] dz of the unit's samples
    int* su = reinterpret_cast<int*>(dzb + U);       // [U] their user ids (-1: past n)
    float* prb = dzb + 2 * U;                        // [U] their probabilities (metrics, BCE)
    float* yb = dzb + 3 * U;                         // [U] their labels
    int* okb = reinterpret_cast<int*>(dzb + 4 * U);  // [U] id check passed

    const int tid = threadIdx.x & 255, lane = tid & 63;
    // the wave's role in its group; group 1 rotates the roles by two so that the two waves
    // sharing a SIMD (waves i and i + 4) never both hold the output / metric / bias extras
    const int w = ((tid >> 6) + 2 * gq) & 3;
    const int li = lane & 15, lq = lane >> 4;  // 16x16x4 operand coordinates
    const int sj = lane & 31, p = tid >> 5;    // gather / GMF role: samples sj + 32 q, part p
    const float eps = 1e-7f, hi_clip = 1.0f - eps;
    const bool metrics = part_hit != nullptr;

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
    float acc_gmf[GPA], acc_h3[4];  // acc_h3: output-kernel rows 4 lq + r of this lane's H3 samples
#pragma unroll
    for (int e = 0; e < GPA; ++e) acc_gmf[e] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc_h3[e] = 0.f;
    float acc_bias[1] = {0.f};
    float acc_bce = 0.f, acc_dbo = 0.f, acc_hit = 0.f, acc_dcg = 0.f;

    // ---- gather: thread (sj, p) brings part p of the MLP input of samples sj + 32 q (parts 0-3:
    // the user half, 4-7: the item half) and part p of both GMF slices.  Masked samples read row
    // 0 (a valid address) and get dz = 0: they contribute nothing.  The ids run two units ahead
    // and the rows one unit ahead: the next unit's rows are in flight during this unit's dW phase.
    const int64_t nunits = (n + U - 1) / U;
    int cu[NQ], cv[NQ], nu[NQ], nv[NQ];
    float cy[NQ], ny[NQ];
    auto load_ids = [&](int64_t un, int (&u)[NQ], int (&v)[NQ], float (&y)[NQ]) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int64_t si = un * U + 32 * q + sj;
            u[q] = 0, v[q] = 0, y[q] = 0.f;
            if (un < nunits && si < n) {
                u[q] = users[si];
                v[q] = items[si];
                y[q] = labels[si];
            }
        }
    };
    float4 xv[NQ][XP / 4];
    float ug[NQ][GPA], ig[NQ][GPA];
    auto load_rows = [&](int64_t un) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const bool okr = un * U + 32 * q + sj < n && (unsigned)cu[q] < (unsigned)ids.ubound &&
                             (unsigned)cv[q] < (unsigned)ids.ibound;
            const int urow = okr ? cu[q] : 0, irow = okr ? ids.ibase + cv[q] : 0;
            const float4* xs =
                reinterpret_cast<const float4*>(emb + (size_t)(p < 4 ? urow : irow) * W + G + (p & 3) * XP);
#pragma unroll
            for (int k = 0; k < XP / 4; ++k) xv[q][k] = xs[k];
            if constexpr (G > 0) {
                const float* us = emb + (size_t)urow * W + p * GP;
                const float* is = emb + (size_t)irow * W + p * GP;
                if constexpr (GP % 4 == 0) {
#pragma unroll
                    for (int k = 0; k < GP / 4; ++k) {
                        const float4 a = reinterpret_cast<const float4*>(us)[k];
                        const float4 b = reinterpret_cast<const float4*>(is)[k];
                        ug[q][4 * k] = a.x, ug[q][4 * k + 1] = a.y, ug[q][4 * k + 2] = a.z, ug[q][4 * k + 3] = a.w;
                        ig[q][4 * k] = b.x, ig[q][4 * k + 1] = b.y, ig[q][4 * k + 2] = b.z, ig[q][4 * k + 3] = b.w;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < GP; ++e) {
                        ug[q][e] = us[e];
                        ig[q][e] = is[e];
                    }
                }
            }
        }
    };
    // units of group gq: u0 + r * ustride; every group runs the workgroup's round count (the
    // barriers are shared), a group past the end works on masked samples and adds nothing.  The
    // stride is the UNIT grid's (nunit_blocks), not gridDim.x: the fill workgroups appended past
    // it take no units, and counting them would skip units [grid, grid + nfill) of every round.
    const int64_t u0 = (int64_t)blockIdx.x * S::NG + gq, ustride = (int64_t)nunit_blocks * S::NG;
    const int64_t first = (int64_t)blockIdx.x * S::NG;
    const int64_t rounds = nunits > first ? (nunits - first + ustride - 1) / ustride : 0;
    // Prologue.  The first unit's ids, then every dense parameter (one b128 buffer load per 4
    // floats, all issued before any is used), are in flight while the LDS parameter block is
    // zeroed (the L3 < 16 columns are read as zeros); the first unit's rows follow the ids; then
    // the parameters go to LDS.  Every segment of the flat layout starts at a multiple of 4 floats.
    load_ids(u0, cu, cv, cy);
    static_assert(S::OB1 % 4 == 0 && S::OW2 % 4 == 0 && S::OB2 % 4 == 0 && S::OW3 % 4 == 0 && S::OB3 % 4 == 0 &&
                      S::OWO % 4 == 0 && S::OBO % 4 == 0,
                  "float4 parameter groups");
    constexpr int NV4 = S::OBO / 4, NVT = (NV4 + S::NT - 1) / S::NT;
    const __amdgpu_buffer_rsrc_t ml_rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)mlp, (short)0, (int)(S::P * 4), 0x00020000);
    f32x4 pv[NVT];
#pragma unroll
    for (int j = 0; j < NVT; ++j) {
        const int q = (int)threadIdx.x + S::NT * j;
        pv[j] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(ml_rsrc, q < NV4 ? (uint32_t)q * 16u : 0x80000000u, 0, 0));
    }
    const float pbo = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ml_rsrc, (uint32_t)S::OBO * 4u, 0, 0));
    for (int e = threadIdx.x; e < S::WLDS / 4; e += S::NT) reinterpret_cast<f32x4*>(wl)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    load_rows(u0);
    load_ids(u0 + ustride, nu, nv, ny);
#pragma unroll
    for (int j = 0; j < NVT; ++j) {
        const int q = (int)threadIdx.x + S::NT * j;
        if (q < NV4) {
            const int e0 = 4 * q;
            int d;  // LDS position of element e0 (its 3 successors follow it)
            if (e0 < S::OB1) {
                d = S::SW1 + (e0 / L1) * S::LW1 + e0 % L1;
            } else if (e0 < S::OW2) {
                d = S::SB1 + (e0 - S::OB1);
            } else if (e0 < S::OB2) {
                d = S::SW2 + ((e0 - S::OW2) / L2) * S::LW2 + (e0 - S::OW2) % L2;
            } else if (e0 < S::OW3) {
                d = S::SB2 + (e0 - S::OB2);
            } else if (e0 < S::OB3) {
                d = S::SW3 + ((e0 - S::OW3) / L3) * S::LW3 + (e0 - S::OW3) % L3;
            } else if (e0 < S::OWO) {
                d = S::SB3 + (e0 - S::OB3);
            } else {
                d = S::SWO + (e0 - S::OWO);  // [gmf | layer 3] output kernel
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) wl[d + k] = pv[j][k];
        }
    }
    if (threadIdx.x == 0) wl[S::SBO] = pbo;
    __syncthreads();

    const int fm = FOLD > 1 ? FOLD - 1 : 0;
    int itl = -1;
    for (int64_t r = 0; r < rounds; ++r) {
        const int64_t un = u0 + r * ustride;
        ++itl;
        NCF_UT(0);
        // lane coordinates re-derived opaquely every unit: keeps the compiler from hoisting the
        // hundreds of lane-dependent LDS addresses out of the loop (and spilling them)
        int lane_t = lane;
        asm volatile("" : "+v"(lane_t));
        const int li = lane_t & 15, lq = lane_t >> 4, sj = lane_t & 31;
        const int64_t s0 = un * U;
        bool inb[NQ], ok[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            inb[q] = s0 + 32 * q + sj < n;
            ok[q] = inb[q] && (unsigned)cu[q] < (unsigned)ids.ubound && (unsigned)cv[q] < (unsigned)ids.ibound;
#pragma unroll
            for (int k = 0; k < XP / 4; ++k) {
                float* dst = act + aidx<S>(q, S::RX + p * XP + 4 * k, sj);
                dst[0] = xv[q][k].x;
                dst[S::LA] = xv[q][k].y;
                dst[2 * S::LA] = xv[q][k].z;
                dst[3 * S::LA] = xv[q][k].w;
            }
            if constexpr (G > 0) {
                float zg = 0.f;
#pragma unroll
                for (int e = 0; e < GP; ++e) zg += wl[S::SWO + p * GP + e] * (ug[q][e] * ig[q][e]);
                zpart[p * U + 32 * q + sj] = zg;
            }
            if (p == 0) {
                su[32 * q + sj] = inb[q] ? cu[q] : -1;
                yb[32 * q + sj] = cy[q];
                okb[32 * q + sj] = ok[q] ? 1 : 0;
            }
        }
        NCF_UT(1);
        __syncthreads();
        NCF_UT(2);

        // ---- forward
        fwd_phase<S, BF, S::B1, L0, S::LW1>(wl + S::SW1, wl + S::SB1, L1, act, S::RX, S::RH1, act, w, li, lq);
        NCF_UT(3);
        __syncthreads();
        NCF_UT(4);
        fwd_phase<S, BF, S::B2, L1, S::LW2>(wl + S::SW2, wl + S::SB2, L2, act, S::RH1, S::RH2, act, w, li, lq);
        NCF_UT(5);
        __syncthreads();
        NCF_UT(6);
        // ---- layer 3, output, dz and G3 in one phase: the roles holding an H3 block keep it in
        // registers; z sums the block's 16 rows (4 per lane, then across the 4 lane groups)
        {
            using A = OutSplit<S::B3, S::NC>;
            if (A::active(w)) {
                f32x4 acc[1][A::NB];
#pragma unroll
                for (int k = 0; k < A::NB; ++k) acc[0][k] = f32x4{0.f, 0.f, 0.f, 0.f};
                mma<BF, L2, 1, A::NB>(
                    acc, [&](int, int kc, int kr) { return wl[S::SW3 + (kc + kr) * S::LW3 + li]; },
                    [&](int b, int kc, int kr) { return act[cidx<S>(S::RH2 + kc + kr, A::cb(w, b), li)]; }, lq);
#pragma unroll
                for (int k = 0; k < A::NB; ++k) {
                    const int cb = A::cb(w, k), s = 16 * cb + li;
                    float h[4], zp = 0.f;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int f = 4 * lq + r;
                        h[r] = f < L3 ? fmaxf(acc[0][k][r] + wl[S::SB3 + f], 0.f) : 0.f;
                        zp += wl[S::SWO + G + f] * h[r];
                    }
                    zp += __shfl_xor(zp, 16, 64);
                    zp += __shfl_xor(zp, 32, 64);
                    float z = zp;
                    if constexpr (G > 0) {
                        float zg = 0.f;
#pragma unroll
                        for (int q = 0; q < 8; ++q) zg += zpart[q * U + s];
                        z += zg;
                    }
                    z += wl[S::SBO];
                    const float pr = 1.0f / (1.0f + expf(-z));
                    const bool okv = okb[s] != 0;
                    const float dz = okv && pr >= eps && pr <= hi_clip ? (pr - yb[s]) * inv_batch : 0.0f;
                    if (lq == 0) {
                        if (s0 + s < n) probs[s0 + s] = okv ? pr : __int_as_float(0x7fc00000);
                        dzb[s] = dz;
                        prb[s] = pr;
                        acc_dbo += dz;
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int f = 4 * lq + r;
                        act[cidx<S>(S::RG3 + f, cb, li)] = (f < L3 && h[r] > 0.f) ? dz * wl[S::SWO + G + f] : 0.f;
                        acc_h3[r] += dz * h[r];
                    }
                }
            }
        }
        NCF_UT(7);
        __syncthreads();
        NCF_UT(8);

        // ---- GMF backward: thread (sj, p), features [p GP, (p+1) GP) of samples sj + 32 q
        if constexpr (G > 0) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int s = 32 * q + sj;
                const float dz = dzb[s];
                const bool fmatch = FOLD > 1 && inb[q] && su[s] == su[s & ~fm];
                const bool fhead = (s & fm) == 0;
                float gu[GP], gi[GP];
#pragma unroll
                for (int e = 0; e < GP; ++e) {
                    const float wo = wl[S::SWO + p * GP + e];
                    gu[e] = dz * wo * ig[q][e];
                    gi[e] = dz * wo * ug[q][e];
                    acc_gmf[e] += dz * (ug[q][e] * ig[q][e]);
                }
                if constexpr (FOLD > 1) {
#pragma unroll
                    for (int e = 0; e < GP; ++e) {
                        const float sm = fold_sum<FOLD>(fmatch ? gu[e] : 0.f);
                        if (fhead) gu[e] = sm;
                    }
                }
                // masked samples (dz = 0) write zero rows: the index may count their other, valid id
                float* gur = gs + (size_t)(2 * (s0 + s)) * W + p * GP;
                float* gir = gur + W;
                if (inb[q] && (fhead || !fmatch)) {
                    if constexpr (GP % 4 == 0) {
#pragma unroll
                        for (int k = 0; k < GP / 4; ++k)
                            st_stream(reinterpret_cast<float4*>(gur) + k,
                                      make_float4(gu[4 * k], gu[4 * k + 1], gu[4 * k + 2], gu[4 * k + 3]));
                    } else {
#pragma unroll
                        for (int e = 0; e < GP; ++e) gur[e] = gu[e];
                    }
                }
                if (inb[q]) {
                    if constexpr (GP % 4 == 0) {
#pragma unroll
                        for (int k = 0; k < GP / 4; ++k)
                            st_stream(reinterpret_cast<float4*>(gir) + k,
                                      make_float4(gi[4 * k], gi[4 * k + 1], gi[4 * k + 2], gi[4 * k + 3]));
                    } else {
#pragma unroll
                        for (int e = 0; e < GP; ++e) gir[e] = gi[e];
                    }
                }
            }
        }
        // ---- backward data chain (G2 shares the phase with the GMF backward)
        bwd_phase<S, BF, S::B2, S::P3, S::LW3>(wl + S::SW3, act, S::RG3, S::RH2, S::RG2, act, w, li, lq);
        NCF_UT(13);
        __syncthreads();
        NCF_UT(14);
        bwd_phase<S, BF, S::B1, L2, S::LW2>(wl + S::SW2, act, S::RG2, S::RH1, S::RG1, act, w, li, lq);
        NCF_UT(15);
        __syncthreads();
        NCF_UT(16);
        // dX = W1 G1 -> the per-sample gradient rows (user half folded like the GMF part)
        {
            using A = OutSplit<S::B0, S::NC>;
            f32x4 acc[A::NA][A::NB];
#pragma unroll
            for (int i = 0; i < A::NA; ++i)
#pragma unroll
                for (int k = 0; k < A::NB; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
            mma<BF, L1, A::NA, A::NB>(
                acc, [&](int a, int kc, int kr) { return wl[S::SW1 + (16 * A::ob(w, a) + li) * S::LW1 + kc + kr]; },
                [&](int b, int kc, int kr) { return act[cidx<S>(S::RG1 + kc + kr, A::cb(w, b), li)]; }, lq);
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
                        if (16 * A::ob(w, i) < D0) {  // uniform per wave: a user-half block
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
        // the next unit's rows (ids loaded a unit ago), and the ids of the one after
        {
            const int64_t un1 = un + ustride;
#pragma unroll
            for (int q = 0; q < NQ; ++q) cu[q] = nu[q], cv[q] = nv[q], cy[q] = ny[q];
            if (un1 < nunits) load_rows(un1);
            load_ids(un1 + ustride, nu, nv, ny);
        }
        // ---- weight gradients (operands in LDS); bias rows (wave 3); BCE + hr/dcg (wave 2)
        dw_phase<S, BF, S::B0, S::B1>(dw1, act, S::RX, S::RG1, w, li, lq);
        dw_phase<S, BF, S::B1, S::B2>(dw2, act, S::RH1, S::RG2, w, li, lq);
        dw_phase<S, BF, S::B2, S::B3>(dw3, act, S::RH2, S::RG3, w, li, lq);
        // extras beside the MFMA chains, one per role: bias rows 0-63 (role 0) and 64- (role 1),
        // hr/dcg (role 2), BCE (role 3)
        if (w < 2) {
            const int br = lane + 64 * w;
            if (br < S::NBIAS) {
                const int rr = br < L1 ? S::RG1 + br : br < L1 + L2 ? S::RG2 + (br - L1) : S::RG3 + (br - L1 - L2);
                float sacc = 0.f;
#pragma unroll
                for (int c = 0; c < U; ++c) sacc += act[aidx<S>(c >> 5, rr, c & 31)];
                acc_bias[0] += sacc;
            }
        }
        if (w == 3 && lane < U && okb[lane]) {
            // Keras BCE of the clipped probability (binary_crossentropy through the logit); a
            // masked sample adds nothing
            const float pc = fminf(fmaxf(prb[lane], eps), hi_clip);
            const float logit = logf(pc / (1.0f - pc));
            acc_bce += fmaxf(logit, 0.0f) - logit * yb[lane] + log1pf(expf(-fabsf(logit)));
        }
        // RankLayer + _get_hits_per_user (model.py:344-455): label = first max of y; position =
        // #(p > p_lab) + #(earlier ties)
        if (metrics && w == 2 && lane < U) {
            const int s = lane, e = s % group, base = s - e;
            int lab = 0;
            float best = yb[base];
            for (int q = 1; q < group; ++q) {
                const float yq = yb[base + q];
                if (yq > best) {
                    best = yq;
                    lab = q;
                }
            }
            const float pl = prb[base + lab];
            int pos = 0;
            for (int q = 0; q < group; ++q) {
                const float pq = prb[base + q];
                pos += (pq > pl) || (pq == pl && q < lab);
            }
            if (e == 0 && s0 + s < n) {
                const float hit = pos < topk ? 1.f : 0.f;
                acc_hit += hit;
                acc_dcg += hit * (logf(2.0f) / logf((float)pos + 2.0f));
            }
        }
        NCF_UT(17);
        __syncthreads();
        NCF_UT(18);
    }

    // ---- epilogue: this workgroup's dense-gradient slab and BCE / metric partials
    const int slot = blockIdx.x * S::NG + gq;  // this group's slab and partials
    float* slab = slabs + (size_t)slot * S::P;
    dw_store<S::B0, S::B1>(dw1, slab + S::OW1, L0, L1, w, li, lq);
    dw_store<S::B1, S::B2>(dw2, slab + S::OW2, L1, L2, w, li, lq);
    dw_store<S::B2, S::B3>(dw3, slab + S::OW3, L2, L3, w, li, lq);
    if (w < 2) {
        const int br = lane + 64 * w;
        if (br < L1) slab[S::OB1 + br] = acc_bias[0];
        else if (br < L1 + L2) slab[S::OB2 + (br - L1)] = acc_bias[0];
        else if (br < S::NBIAS) slab[S::OB3 + (br - L1 - L2)] = acc_bias[0];
    }
    // output kernel, GMF entries: thread (sj, p) holds features p GP + e of its samples, summed
    // over the 32 lanes of its wave half
    if constexpr (G > 0) {
#pragma unroll
        for (int e = 0; e < GP; ++e) {
            const float v = wave_half_sum(acc_gmf[e]);
            if (sj == 0) slab[S::OWO + p * GP + e] = v;
        }
    }
    // H3 output-kernel rows, output bias, BCE, hr, dcg: summed over each role's lanes, then over
    // the roles in role order through LDS (this group's GMF scratch: [role][20])
    {
        float* xr = zpart;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = acc_h3[r];
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) v[r] += __shfl_xor(v[r], m, 64);
        }
        float x[4] = {acc_dbo, acc_bce, acc_hit, acc_dcg};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) x[k] += __shfl_xor(x[k], m, 64);
        if (li == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) xr[w * 20 + 4 * lq + r] = v[r];
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) xr[w * 20 + 16 + k] = x[k];
        }
        __syncthreads();
        if (tid < 20) {
            float t = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) t += xr[r * 20 + tid];
            if (tid < L3) slab[S::OWO + G + tid] = t;
            else if (tid == 16) slab[S::OBO] = t;
            else if (tid == 17) part_bce[slot] = t;
            else if (tid == 18 && metrics) part_hit[slot] = t;
            else if (tid == 19 && metrics) part_dcg[slot] = t;
        }
    }
}

template <int U, int NG> using UShapeC = UShape<128, 64, 32, 16, 64, U, NG>;  // ml-20m NeuMF (config C)
template <int U, int NG> using UShapeB = UShape<64, 32, 16, 8, 8, U, NG>;     // ml-1m NeuMF (config B)
template <int U, int NG> using UShapeR = UShape<64, 32, 16, 8, 0, U, NG>;     // trainer default (MLP-only)
template <int U, int NG> using UShapeC0 = UShape<128, 64, 32, 16, 0, U, NG>;

template <class S>
bool umatches(const ncf_shape_t& s) {
    return s.num_layers == 4 && s.layers[0] == S::L0 && s.layers[1] == S::L1 && s.layers[2] == S::L2 &&
           s.layers[3] == S::L3 && s.gmf_dim == S::G && s.row_width == S::W && s.gmf_stride == S::G;
}

// fill workgroups of NT threads for one pass per wave (fill_wave: 256 keys, 128 contributions)
int unit_fill_blocks(int64_t r1, int64_t n, int nt) {
    const int64_t rows = (r1 + 255) / 256, contribs = (2 * n + 127) / 128;
    const int64_t waves = rows > contribs ? rows : contribs;
    return (int)((waves + nt / 64 - 1) / (nt / 64));
}

template <class S, bool BF>
hipError_t launch_unit_one(const WsLayout& L, void* ws, const float* emb, const float* mlp, const int32_t* users,
                           const int32_t* items, const float* labels, int64_t n, float inv_batch, IdSpace ids,
                           int group, int topk, int* nslab, int* nbce, int* nmet, hipStream_t st, int fold,
                           bool check_fold, const FillArgs* fill) {
    static bool configured = false;  // one-time attribute set per shape (idempotent)
    if (!configured) {
        for (const void* k : {(const void*)k_fb_unit<S, 0, BF>, (const void*)k_fb_unit<S, 2, BF>,
                              (const void*)k_fb_unit<S, 4, BF>, (const void*)k_fb_unit<S, 8, BF>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)S::LDS_BYTES);
            if (e != hipSuccess) return e;
        }
        configured = true;
    }
    const int64_t nunits = (n + S::U - 1) / S::U;
    const int64_t wgs = (nunits + S::NG - 1) / S::NG;
    int grid = (int)(wgs < 256 ? wgs : 256);
    if (grid < 1) grid = 1;
    const bool in_kernel = group > 0 && group <= 32 && 32 % group == 0;
    const int nfill = fill ? unit_fill_blocks(fill->r1, n, S::NT) : 0;
    if (fill && (check_fold || fill->nscan < 1 || fill->nscan > kMaxFillScan)) return hipErrorInvalidValue;
    const FillArgs fa = fill ? *fill : FillArgs{};
    auto go = [&](auto kern) {
        launch(kern, grid + nfill, S::NT, S::LDS_BYTES, st, emb, mlp, users, items, labels, n, ids, inv_batch,
               at<float>(ws, L.probs), at<float>(ws, L.gs), at<float>(ws, L.slabs), at<float>(ws, L.part_bce), group,
               topk, in_kernel ? at<float>(ws, L.part_hit) : nullptr, in_kernel ? at<float>(ws, L.part_dcg) : nullptr,
               check_fold ? at<const int32_t>(ws, L.ifold) : nullptr, at<int32_t>(ws, L.err), fa, grid);
    };
    switch (fold) {
        case 0: go(k_fb_unit<S, 0, BF>); break;
        case 2: go(k_fb_unit<S, 2, BF>); break;
        case 4: go(k_fb_unit<S, 4, BF>); break;
        case 8: go(k_fb_unit<S, 8, BF>); break;
        default: return hipErrorInvalidValue;
    }
    *nslab = grid * S::NG;
    *nbce = grid * S::NG;
    *nmet = in_kernel ? grid * S::NG : 0;
    return hipGetLastError();
}

// Schedule: one group of 32-sample units per workgroup while the units do not fill every CU
// twice over, then two groups per workgroup (two waves per SIMD, one unit each);
// NCF_UNIT_SCHED=1|2|64 forces one (64: one group of 64-sample units)
int unit_sched(int64_t n) {
    static const int forced = [] {
        const char* e = ncf::experiment_env("NCF_UNIT_SCHED");
        return e ? atoi(e) : 0;
    }();
    if (forced == 1 || forced == 2 || forced == 64) return forced;
    return n >= 256 * 32 * 2 ? 2 : 1;
}

}  // namespace

#ifdef NCF_UNIT_TIMING
extern "C" int ncf_debug_unit_timing(unsigned long long* out, size_t count) {
    size_t m = count < sizeof(g_unit_t) / 8 ? count : sizeof(g_unit_t) / 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_unit_t), m * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif

bool unit_supported(const ncf_shape_t& s) {
    return umatches<UShapeC<32, 1>>(s) || umatches<UShapeB<32, 1>>(s) || umatches<UShapeR<32, 1>>(s) ||
           umatches<UShapeC0<32, 1>>(s);
}

#ifndef NCF_UNIT_FILL_MAX_BLOCKS
#define NCF_UNIT_FILL_MAX_BLOCKS 1024  // unit + fill workgroups (a fill workgroup shares a CU with a unit one when the units take them all: C at 8,192 53.3 vs 56.3 us with a fill launch)
#endif
// the unit launch's grid leaves room for the fill workgroups on CUs it does not use (in-kernel fill)
bool unit_fill_fits(const ncf_shape_t& s, int64_t n, bool bf16, int64_t r1) {
    if (!unit_supported(s)) return false;
    const int sched = bf16 ? 1 : unit_sched(n);
    const int ng = sched == 2 ? 2 : 1, nt = 256 * ng;
    const int64_t units = (n + (sched == 64 ? 63 : 31)) / (sched == 64 ? 64 : 32);
    const int64_t wgs = (units + ng - 1) / ng;
    return wgs + unit_fill_blocks(r1, n, nt) <= NCF_UNIT_FILL_MAX_BLOCKS;
}

hipError_t launch_fb_unit(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                          const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                          float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                          hipStream_t st, int fold, bool bf16, bool check_fold, const FillArgs* fill) {
    if (fold != 0 && (fold < 2 || fold > 8 || (fold & (fold - 1)) != 0 || n % fold != 0)) return hipErrorInvalidValue;
    const int sched = unit_sched(n);
    // bf16 operands: one 32-sample unit group per workgroup at every size (config B's path)
#define NCF_ARGS \
    L, ws, emb, mlp, users, items, labels, n, inv_batch, ids, group, topk, nslab, nbce, nmet, st, fold, check_fold, fill
#define NCF_TRY(SH)                                                                                           \
    if (umatches<SH<32, 1>>(s))                                                                               \
        return bf16 ? launch_unit_one<SH<32, 1>, true>(NCF_ARGS)                                              \
                    : sched == 2 ? launch_unit_one<SH<32, 2>, false>(NCF_ARGS)                                \
                                 : sched == 64 ? launch_unit_one<SH<64, 1>, false>(NCF_ARGS)                  \
                                               : launch_unit_one<SH<32, 1>, false>(NCF_ARGS);
    NCF_TRY(UShapeC)
    NCF_TRY(UShapeB)
    NCF_TRY(UShapeR)
    NCF_TRY(UShapeC0)
#undef NCF_TRY
#undef NCF_ARGS
    return hipErrorInvalidValue;
}

}  // namespace ncf
