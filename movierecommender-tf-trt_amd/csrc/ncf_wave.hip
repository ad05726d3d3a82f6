// Wave-chain fused NeuMF forward + backward on CDNA4 fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// One 256-thread workgroup (4 waves, one per SIMD) per CU; every wave works ALONE on its own
// 16-sample units, so the per-unit loop has no workgroup barrier at all.  The unit kernel
// (ncf_unit.hip) splits each layer's output features over 4 waves and pays 7 barriers and the
// imbalance of the narrow layers per 32 samples; here each wave runs the whole chain:
//
//   forward:  H1 = relu(W1^T X + b1), H2, H3 as 16x16 MFMA tiles [feature][sample] — the output
//             registers of one layer ARE the B operand of the next (the k order of a layer's
//             contraction is free, so k-step (tile t, register r) takes feature 16 t + 4 lq + r
//             from lane group lq), no LDS round trip between layers
//   output:   z = wo . [u_gmf * i_gmf | H3] + bo (in-lane partial sums + two cross-group adds),
//             Keras-clipped BCE, dz = (p - y) / B
//   backward: G3 = dz wo ⊙ relu'(H3); G2 = (W3 G3) ⊙ relu'(H2); G1 = (W2 G2) ⊙ relu'(H1);
//             dX = W1 G1 -> per-sample gradient rows gs (users folded as in the unit kernel)
//   weights:  dW_l += H_{l-1} G_l^T over the unit's 16 samples (K = 16: 4 MFMA steps per tile).
//             The contraction runs over samples, so the wave writes X, H1, H2, G1, G2, G3
//             transposed ([sample][feature]) into its own LDS buffers and reads them back in the
//             operand layout; every dW tile of the model lives in this wave's accumulators
//             (168 registers at config C — one wave per SIMD has 512).
//
// Dense weights sit in LDS once per workgroup in an operand-friendly layout: column c of a
// matrix with NB 16-column blocks is stored at position (c mod 16) NB + c / 16, so one
// ds_read_b32/b64/b128 returns the A operands of all NB output tiles of a forward k-step, or NB
// k-steps of the backward contraction.  Per 16-sample unit a wave issues 504 MFMAs (config C)
// and ~134 LDS reads.  The next unit's MLP input is loaded into the registers layer 1 has just
// consumed; a unit's GMF slices are loaded as it starts (first needed after layer 3).
//
// Epilogue: each wave reduces its per-lane bias / output-kernel / loss sums over its 16 sample
// lanes, the four waves' contributions are added in LDS in a fixed order ((w0 + w2) + (w1 + w3))
// and the workgroup writes one dense-gradient slab and one BCE / hit / dcg partial — the outputs
// of k_fb_unit, so the index, update and reduction launches do not care which kernel ran.
// Bitwise reproducible.  Reference semantics: movierec/model.py:154-214.

#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "ncf_adam.h"
#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// NB contiguous floats from / to LDS as one (or two, NB = 8) ds_read / ds_write
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
        const f32x2 x = *reinterpret_cast<const f32x2*>(p);
        o[0] = x[0], o[1] = x[1];
    } else {
        static_assert(NB == 1, "vector width");
        o[0] = p[0];
    }
}
template <int NB>
__device__ __forceinline__ void stsv(float* p, const float (&v)[NB]) {
    if constexpr (NB == 4) {
        *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    } else if constexpr (NB == 2) {
        *reinterpret_cast<f32x2*>(p) = f32x2{v[0], v[1]};
    } else {
        static_assert(NB == 1, "vector width");
        p[0] = v[0];
    }
}

template <int L0_, int L1_, int L2_, int L3_, int G_>
struct WShape {
    static constexpr int L0 = L0_, L1 = L1_, L2 = L2_, L3 = L3_, G = G_;
    static constexpr int D0 = L0 / 2, W = G + D0;
    static constexpr int B0 = L0 / 16, B1 = L1 / 16, B2 = L2 / 16;
    static_assert(L0 % 64 == 0 && L1 % 16 == 0 && L2 % 16 == 0 && L3 <= 16 && L3 % 4 == 0 && G % 4 == 0,
                  "wave-kernel shapes");
    static_assert((B0 == 4 || B0 == 8) && (B1 == 1 || B1 == 2 || B1 == 4) && (B2 == 1 || B2 == 2 || B2 == 4),
                  "16-column blocks per layer");
    static constexpr int XQ = L0 / 4;  // MLP-input floats per lane: features XQ lq + q of sample li
    static constexpr int GQ = G / 4;   // GMF floats per lane: dims GQ lq + e
    // flat dense-parameter offsets (include/movierec_ncf.h layout)
    static constexpr int OW1 = 0, OB1 = L0 * L1, OW2 = OB1 + L1, OB2 = OW2 + L1 * L2, OW3 = OB2 + L2,
                         OB3 = OW3 + L2 * L3, OWO = OB3 + L3, OBO = OWO + G + L3, P = OBO + 1;
    // LDS: weights [in][pos] with row strides 16 NB + 4 (bank-conflict-free for the forward
    // reads, at most 2-way for the backward ones under MI355X_MICROARCH.md's LDS model); layer 3
    // padded to 16 output columns (zeros)
    static constexpr int S1 = 16 * B1 + 4, S2 = 16 * B2 + 4, S3 = 20;
    static constexpr int SW1 = 0, SW2 = SW1 + L0 * S1, SW3 = SW2 + L1 * S2, SB1 = SW3 + L2 * S3,
                         SB2 = SB1 + L1, SB3 = SB2 + L2, SWO = SB3 + 16, SBO = SWO + G + 16,
                         WLDS = (SBO + 1 + 3) / 4 * 4;
    // per-wave transposed buffers [sample][pos], pos = (f mod 16) NT + f / 16, row stride ts(NT)
    static constexpr int ts(int nt) { return nt == 8 ? 132 : 16 * nt; }
    static constexpr int TX = 0, TH1 = TX + 16 * ts(B0), TG1 = TH1 + 16 * ts(B1), TH2 = TG1 + 16 * ts(B1),
                         TG2 = TH2 + 16 * ts(B2), TG3 = TG2 + 16 * ts(B2), WREG = TG3 + 16 * 16;
    static constexpr size_t LDS_BYTES = (size_t)(WLDS + 4 * WREG) * 4;
    static_assert(LDS_BYTES <= 163840, "LDS budget");
    // split form (k_fb_wave<..., true>): no X^T buffer (the weight-gradient wave loads X from the
    // table), two buffers per chain wave (the unit being written, the unit being contracted)
    static constexpr int XSZ = 16 * ts(B0), WREG2 = WREG - XSZ;
    static constexpr size_t LDS_BYTES2 = (size_t)(WLDS + 8 * WREG2) * 4;
    static constexpr bool SPLIT_OK = LDS_BYTES2 <= 163840 && WLDS >= XSZ;
    // the prologue moves the flat parameters as float4 groups: no group straddles two segments,
    // and the contiguous segments land on 16-byte-aligned LDS positions
    static_assert(OB1 % 4 == 0 && OW2 % 4 == 0 && OB2 % 4 == 0 && OW3 % 4 == 0 && OB3 % 4 == 0 && OWO % 4 == 0 &&
                      OBO % 4 == 0 && SW3 % 4 == 0 && S3 % 4 == 0 && SB1 % 4 == 0 && SB2 % 4 == 0 && SB3 % 4 == 0 &&
                      SWO % 4 == 0,
                  "float4 parameter groups");
    // epilogue: one reduction row per wave, holding half of its NT dW tiles at a time in the
    // accumulator layout ([tile][lane][4], one ds_write_b128 per tile and lane) followed by the
    // bias / output-kernel / loss entries
    static constexpr int NT1 = B0 * B1, NT2 = B1 * B2, NT = NT1 + NT2 + B2, NTH = (NT + 1) / 2;
    static constexpr int RB1 = NTH * 256, RB2 = RB1 + L1, RB3 = RB2 + L2, RWO = RB3 + L3, RBO = RWO + G + L3,
                         RX = RBO + 1, PR = (RX + 3 + 3) / 4 * 4;
    static_assert((size_t)4 * PR * 4 <= LDS_BYTES, "epilogue rows");
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Operand registers of one pipelined step
template <int N>
struct Ops {
    float v[N];
};
template <int M, int N>
struct Ops2 {
    float v[M][N];
};
template <int B0, int B1, int B2>
struct DwOps {
    float x[B0], g1[B1], h1[B1], g2[B2], h2[B2], g3;
};

// NSTEP steps of LDS operand reads + MFMAs with the reads PD steps ahead (a ring of PD operand
// sets): step s issues its MFMAs, then the reads of step s + PD into the set it just used.  The
// scheduling barriers keep that order (a single wave per SIMD has no other wave to hide a read
// behind), and lgkmcnt counts the reads each step waits for.
template <int NSTEP, int PD, class OPS, class LD, class MM>
__device__ __forceinline__ void pipe(LD ld, MM mm) {
    OPS ring[PD];
#pragma unroll
    for (int s = 0; s < PD && s < NSTEP; ++s) ld(s, ring[s]);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
        __builtin_amdgcn_sched_barrier(0);
        mm(s, ring[s % PD]);
        if (s + PD < NSTEP) ld(s + PD, ring[s % PD]);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// x summed over the FOLD consecutive sample lanes of its group (FOLD 2, 4, 8; all lanes active)
template <int FOLD>
__device__ __forceinline__ float fold_sum(float x) {
    static_assert(FOLD == 2 || FOLD == 4 || FOLD == 8, "fold width");
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    if constexpr (FOLD >= 4)
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    if constexpr (FOLD >= 8) x += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x1F | (4 << 10)));
    return x;
}

// sum over the 16 sample lanes of a lane group (DPP row rotations: full-rate VALU; each lane
// associates differently, the callers read lane li == 0)
__device__ __forceinline__ float row_sum(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));  // row_ror:8
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));  // row_ror:4
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));  // row_ror:2
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));  // row_ror:1
    return x;
}

// sum over the 4 lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48): gfx950's permlane swaps (VALU),
// every lane gets (g0 + g1) + (g2 + g3)
__device__ __forceinline__ float group_allsum(float x) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// element q of this lane's group of FOLD consecutive lanes (DPP quad permutes for FOLD 2, 4;
// q is a compile-time constant at every call site, the switch folds away)
template <int CTRL>
__device__ __forceinline__ int dpp_mov(int x) {
    return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
}
template <int FOLD, class T>
__device__ __forceinline__ T grp_bcast(T x, int q, int lane) {
    static_assert(sizeof(T) == 4, "32-bit values");
    const int v = __builtin_bit_cast(int, x);
    if constexpr (FOLD == 4) {
        switch (q) {
            case 0: return __builtin_bit_cast(T, dpp_mov<0x00>(v));  // quad_perm [0,0,0,0]
            case 1: return __builtin_bit_cast(T, dpp_mov<0x55>(v));  // [1,1,1,1]
            case 2: return __builtin_bit_cast(T, dpp_mov<0xAA>(v));  // [2,2,2,2]
            default: return __builtin_bit_cast(T, dpp_mov<0xFF>(v)); // [3,3,3,3]
        }
    } else if constexpr (FOLD == 2) {
        return q == 0 ? __builtin_bit_cast(T, dpp_mov<0xA0>(v))   // [0,0,2,2]
                      : __builtin_bit_cast(T, dpp_mov<0xF5>(v));  // [1,1,3,3]
    } else {
        return __shfl(x, (lane & ~(FOLD - 1)) + q, 64);
    }
}

// Span stamps (g_wave_s, 16 per wave): 0/1 entry (s_memrealtime / cycles), 2 weights in LDS,
// 3 + k start of the wave's unit k (k < 8), 11 loop done, 14 epilogue's first barrier passed,
// 15 the four waves' sums in LDS, 12 end (cycles), 13 end (s_memrealtime).
#ifdef NCF_WAVE_TIMING
__device__ unsigned long long g_wave_t[256 * 4 * 2 * 10];
__device__ unsigned long long g_wave_s[256 * 4 * 16];
#define NCF_WT(it, ph)                                                                                 \
    do {                                                                                               \
        if (lane == 0 && blockIdx.x < 256 && (it) < 2)                                                 \
            g_wave_t[((blockIdx.x * 4 + wv) * 2 + (it)) * 10 + (ph)] = __builtin_readcyclecounter(); \
        if (lane == 0 && blockIdx.x < 256 && (ph) == 0 && (it) < 8)                                    \
            g_wave_s[(blockIdx.x * 4 + wv) * 16 + 3 + (it)] = __builtin_readcyclecounter();            \
    } while (0)
#define NCF_WS(slot, v)                                                                                \
    do {                                                                                               \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 256 && threadIdx.x < 256) g_wave_s[blockIdx.x * 64 + (threadIdx.x >> 6) * 16 + (slot)] = (v); \
    } while (0)
#else
#define NCF_WT(it, ph) ((void)0)
#define NCF_WS(slot, v) ((void)0)
#endif

// SPLIT: 8 waves, two per SIMD.  Waves 0-3 run the chain of their units as above except the
// weight gradients; wave 4 + p (the same SIMD as chain wave p) contracts chain wave p's units into
// the dW accumulators: it reads G1, H1, G2, H2, G3 from the transposed buffers the chain wave
// wrote (two per chain wave, by unit parity) and X from the table rows (lane li: features
// B0 li .. B0 li + B0 - 1 of sample 4 q + lq, so dW1 tile a's row i is feature B0 i + a).  One
// workgroup barrier per unit hands a unit over: barrier k follows chain unit k and precedes its
// contraction, so barrier k + 1 also frees unit k's buffers for unit k + 2.  The chain's phases
// that issue no MFMA now have the weight-gradient wave's 168 MFMAs per unit beside them on the
// same SIMD.  Same MFMAs on the same operands in the same order as the one-wave form: bitwise.
// 1 (the default): the epilogue's tile rows transposed in LDS and the slab written 16 bytes per lane
// (reduce_tiles); 0: the round-2 epilogue (4-byte slab stores), for A/B
#ifndef NCF_EPI_WIDE
#define NCF_EPI_WIDE 1
#endif
#ifndef NCF_PRIO_P0
#define NCF_PRIO_P0 1
#endif
#ifndef NCF_SPLIT_PRIO
#define NCF_SPLIT_PRIO 1
#endif
// experiment switches (wrong results, timing only): NCF_SPLIT_NODW 1 = the weight-gradient waves
// skip their contraction; NCF_SPLIT_NOSYNC 1 = also no per-unit barrier
#ifndef NCF_SPLIT_NODW
#define NCF_SPLIT_NODW 0
#endif
#ifndef NCF_SPLIT_NOSYNC
#define NCF_SPLIT_NOSYNC 0
#endif
// 1: a weight-gradient wave contracts unit k while its chain wave runs unit k + 1 past layer 1
// (two barriers per unit); 0 (the default): right after unit k (one barrier, beside the chain's
// layer 1).  Measured at config C (profiles/r03_b): 0 53.0-53.3 us, 1 54.4-55.3, the one-wave
// form 55.0-55.2; phase stamps of 1 show the chain's MFMA-free output and G3 sections growing by
// the partner's MFMA time (a SIMD's VALU / MFMA issue is shared, MI355X_MICROARCH.md "Two waves
// per SIMD" item 3)
#ifndef NCF_SPLIT_LATE
#define NCF_SPLIT_LATE 0
#endif
// 1: the split form's weight-gradient wave also computes dX = W1 G1 and writes the gradient rows'
// MLP parts (from the transposed G1 the chain wave hands over anyway), taking 128 MFMAs per unit
// off the chain; 0 (the default): the chain wave computes dX.  Measured at config C (round 4,
// profiles/r04_i/ab, same session): 58.6 us with 1 against 54.4-54.9 us with 0 — the two waves of a
// SIMD share its issue (MI355X_MICROARCH.md "Two waves per SIMD"), and the partner wave then needs
// more than the 256 registers two waves per SIMD leave it (a few spills)
#ifndef NCF_SPLIT_DX
#define NCF_SPLIT_DX 0
#endif
// timing diagnostic (wrong results): 1 = the chain runs layer 1 and dX over half of the MLP input
// (the MFMAs a per-group user half would leave per unit)
// 1 (the default): with user-row folding (FOLD 2, 4, 8) the split form's chain computes the user
// half of layer 1 and of dX once per group instead of once per sample (see k_fb_wave)
#ifndef NCF_GROUP_USER
#define NCF_GROUP_USER 1
#endif
#if NCF_GROUP_USER && NCF_SPLIT_LATE
#error "the late contraction is not written for the group-user form: build it with NCF_GROUP_USER=0"
#endif
#if NCF_GROUP_USER && NCF_SPLIT_DX
#error "NCF_SPLIT_DX computes dX per sample on the weight-gradient wave: build it with NCF_GROUP_USER=0"
#endif
// timing diagnostics (wrong results): NCF_DIAG_NOP0 1 skips the group-user form's phase 0 (its
// loads of P_u stay), NCF_DIAG_NOPN 1 skips phase N on both waves
#ifndef NCF_DIAG_NOP0
#define NCF_DIAG_NOP0 0
#endif
#ifndef NCF_DIAG_NOPN
#define NCF_DIAG_NOPN 0
#endif
#ifndef NCF_DIAG_HALFL1
#define NCF_DIAG_HALFL1 0
#endif
template <class S, int FOLD, bool MET, bool SPLIT = false>
__global__ __launch_bounds__(SPLIT ? 512 : 256, 1) void k_fb_wave(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                     const int32_t* __restrict__ users,
                                                     const int32_t* __restrict__ items,
                                                     const float* __restrict__ labels, int64_t n, IdSpace ids,
                                                     float inv_batch, float* __restrict__ probs,
                                                     float* __restrict__ gs, float* __restrict__ slabs,
                                                     float* __restrict__ part_bce, int group, int topk,
                                                     float* __restrict__ part_hit, float* __restrict__ part_dcg,
                                                     const int32_t* __restrict__ ifold, int32_t* __restrict__ ferr,
                                                     float* __restrict__ gpart, FillArgs fa) {
    constexpr int L0 = S::L0, L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, D0 = S::D0, W = S::W;
    constexpr int B0 = S::B0, B1 = S::B1, B2 = S::B2, XQ = S::XQ, GQ = S::GQ, GQA = GQ > 0 ? GQ : 1;
    // Group-user form (GU: split form, FOLD > 1).  The reference's batches are groups of FOLD
    // samples sharing one user (data_pipeline.py:141), and layer 1 is linear in the user half of
    // its input: W1^T [x_u; x_i] = W1_u^T x_u + W1_i^T x_i, and the folded user row's dX is
    // sum_s W1_u g1_s = W1_u (sum_s g1_s).  So the chain computes P_u = W1_u^T x_u once per group
    // (16 groups, one MFMA tile, per FOLD units: phase 0) into gpart, starts each sample's layer-1
    // accumulators from its group's P_u and runs only the item half per unit, writes each group's
    // sum of G1 over the samples that share the head's user to gpart, and after its units computes
    // W1_u (sum g1) for 16 groups per tile (phase N) into the head samples' user rows.  Per 16-sample
    // unit that is 2 x 64 MFMAs less on the chain at config C, for 2 x 64 per FOLD units.  A sample
    // whose user differs from its group head's (any batch is accepted) takes its own user half in a
    // per-unit branch that only such units enter.  Same sums, reassociated: within fp32 rounding of
    // the per-sample form, checked against the oracle like it.
    constexpr bool GU = SPLIT && FOLD > 1 && NCF_GROUP_USER;
    constexpr int XH = XQ / 2;                // per lane: D0 / 4 features of one half of the input
    constexpr int XN = GU ? XH : XQ;          // MLP-input floats per lane in the unit loop
    constexpr int NGU = FOLD > 1 ? 16 / FOLD : 16;  // groups per unit
    constexpr int T0 = S::ts(B0), T1 = S::ts(B1), T2 = S::ts(B2);
    NCF_WS(0, __builtin_amdgcn_s_memrealtime());
    NCF_WS(1, __builtin_readcyclecounter());
    // an index built by an earlier call (ncf_build_index / ncf_shard_plan) must fold as this kernel does
    if (ifold && blockIdx.x == 0 && threadIdx.x == 0 && *ifold != FOLD) atomicOr(ferr, kErrFold);
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wl = lds;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int pw = wv & 3;                     // the chain (split: chain / weight-gradient pair) index
    const bool dwave = SPLIT && wv >= 4;       // split: the weight-gradient wave of pair pw
    static_assert(!SPLIT || S::SPLIT_OK, "split form: LDS budget");
    // split: chain wave pw's buffer for units of parity `par` (its TX offset is never used)
    auto tbuf = [&](int par) {
        return SPLIT ? lds + S::WLDS + (pw * 2 + par) * S::WREG2 - S::XSZ : lds + S::WLDS + wv * S::WREG;
    };
    float* tb = tbuf(0);
    const float eps = 1e-7f, hi_clip = 1.0f - eps;
    static_assert(!MET || FOLD > 1, "in-kernel metrics for groups of FOLD samples");

    const int li = lane & 15, g = lane >> 4;  // sample lane, lane group (the MFMA k index)
    const int64_t nunits = (n + 15) / 16;
    const int64_t ustride = (int64_t)gridDim.x * 4;
    int64_t un = (int64_t)blockIdx.x * 4 + pw;
    // split: units (barriers) of this workgroup = those of its chain wave 0, the one with the most
    const int64_t nit = SPLIT ? (nunits - (int64_t)blockIdx.x * 4 + ustride - 1) / ustride : 0;

    // ids run two units ahead, rows one unit ahead.  A masked sample (past n or an id outside the
    // table) reads row 0 (a valid address) and gets dz = 0: it contributes nothing.
    // (buffer loads: a lane past n reads 0 without a branch)
    const uint32_t nbytes = (uint32_t)(n * 4);
    const __amdgpu_buffer_rsrc_t us_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)users, (short)0, (int)nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t it_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)items, (short)0, (int)nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t lb_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)labels, (short)0, (int)nbytes, 0x00020000);
    auto load_ids = [&](int64_t u, int& cu, int& cv, float& cy) {
        const int64_t si = u * 16 + li;
        const uint32_t off = si < n ? (uint32_t)si * 4u : 0x80000000u;
        cu = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, off, 0, 0);
        cv = (int)__builtin_amdgcn_raw_buffer_load_b32(it_rsrc, off, 0, 0);
        cy = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(lb_rsrc, off, 0, 0));
    };
    auto rows_of = [&](int64_t u, int cu, int cv, int& urow, int& irow) {
        const bool okr = u * 16 + li < n && (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
        urow = okr ? cu : 0;
        irow = okr ? ids.ibase + cv : 0;
    };
    constexpr uint32_t kDrop = 0x80000000u;
    constexpr unsigned kVmcnt0 = 0x0F70;  // s_waitcnt vmcnt(0), expcnt / lgkmcnt unconstrained
    float xr[XN], gu[GQA], gi[GQA];
    // GU: gpart = P_u [n / FOLD][L1] (rows 16 t + 4 lq .. + 3 of a group at 16 t + 4 lq), then the
    // groups' G1 sums [n / FOLD][L1] at gpart + (n / 2) L1
    const int64_t ngrp = FOLD > 1 ? n / (FOLD > 1 ? FOLD : 1) : 0;
    const __amdgpu_buffer_rsrc_t pu_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(gpart, (short)0, (int)(uint32_t)(ngrp * L1 * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t sgr_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(gpart + (n / 2) * L1, (short)0, (int)(uint32_t)(ngrp * L1 * 4), 0x00020000);
    f32x4 pun[B1];  // GU: the unit's layer-1 accumulators as its groups' P_u left them
    auto load_pu = [&](int64_t u) {
        if constexpr (GU) {
            const int64_t si = u * 16 + li;
            const uint32_t off = si < n ? (uint32_t)(((si / FOLD) * L1 + 4 * g) * 4) : kDrop;
#pragma unroll
            for (int t = 0; t < B1; ++t)
                pun[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pu_rsrc, off + 64u * t, 0, 0));
        }
    };
    auto load_x = [&](int64_t u, int cu, int cv) {
        int urow, irow;
        rows_of(u, cu, cv, urow, irow);
        if constexpr (GU) {
            // the item half only: lane group lq holds item features XH lq .. + XH - 1
            const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)irow * W + G + g * XH);
#pragma unroll
            for (int k = 0; k < XH / 4; ++k) {
                const float4 v = xs[k];
                xr[4 * k] = v.x, xr[4 * k + 1] = v.y, xr[4 * k + 2] = v.z, xr[4 * k + 3] = v.w;
            }
        } else {
            const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)(g < 2 ? urow : irow) * W + G + (g & 1) * XQ);
#pragma unroll
            for (int k = 0; k < XQ / 4; ++k) {
                const float4 v = xs[k];
                xr[4 * k] = v.x, xr[4 * k + 1] = v.y, xr[4 * k + 2] = v.z, xr[4 * k + 3] = v.w;
            }
        }
    };
    auto load_g = [&](int64_t u, int cu, int cv) {
        if constexpr (G > 0) {
            int urow, irow;
            rows_of(u, cu, cv, urow, irow);
            const float* us = emb + (size_t)urow * W + g * GQ;
            const float* is = emb + (size_t)irow * W + g * GQ;
            if constexpr (GQ % 4 == 0) {
#pragma unroll
                for (int k = 0; k < GQ / 4; ++k) {
                    const float4 a = reinterpret_cast<const float4*>(us)[k];
                    const float4 b = reinterpret_cast<const float4*>(is)[k];
                    gu[4 * k] = a.x, gu[4 * k + 1] = a.y, gu[4 * k + 2] = a.z, gu[4 * k + 3] = a.w;
                    gi[4 * k] = b.x, gi[4 * k + 1] = b.y, gi[4 * k + 2] = b.z, gi[4 * k + 3] = b.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < GQ; ++e) gu[e] = us[e], gi[e] = is[e];
            }
        }
    };
    int cu, cv, nu, nv;
    float cy, ny;

    // Prologue.  The first unit's ids, then every dense parameter (one b128 buffer load per 4
    // floats, all issued before any is used), are in flight while the operand layout's padding is
    // zeroed; the first unit's MLP input follows the ids; then the parameters go to LDS.  Every
    // segment of the flat layout starts at a multiple of 4 floats, so a float4 never straddles two.
    // (split: the chain waves load the parameters; the weight-gradient waves only pass the barriers)
    constexpr int NV4 = S::OBO / 4, NVT = (NV4 + 255) / 256;
    const __amdgpu_buffer_rsrc_t ml_rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)mlp, (short)0, (int)(S::P * 4), 0x00020000);
    f32x4 pv[NVT];
    float pbo = 0.f;
    // GU: phase-0 tile tau's column li is group li % NGU of the wave's unit tau FOLD + li / NGU
    const int64_t un0 = un;
    const int64_t nown = un0 < nunits ? (nunits - un0 + ustride - 1) / ustride : 0;
    auto tile_head = [&](int64_t tau, int64_t& hs) {
        const int64_t k = tau * FOLD + li / NGU;
        hs = (un0 + k * ustride) * 16 + (li % NGU) * FOLD;
        return k < nown && hs < n;
    };
    float xu[GU ? XH : 1];
    auto load_xu = [&](int hu, bool hv) {  // the head's user half: features XH lq .. + XH - 1
        const int row = hv && (unsigned)hu < (unsigned)ids.ubound ? hu : 0;
        const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)row * W + G + g * XH);
#pragma unroll
        for (int k = 0; k < (GU ? XH / 4 : 0); ++k) {
            const float4 v = xs[k];
            xu[4 * k] = v.x, xu[4 * k + 1] = v.y, xu[4 * k + 2] = v.z, xu[4 * k + 3] = v.w;
        }
    };
    int64_t hs0 = 0;
    bool hv0 = false;
    int hu0 = 0;
    if (!dwave) {
        load_ids(un, cu, cv, cy);
        if constexpr (GU) {
            hv0 = tile_head(0, hs0);
            hu0 = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, hv0 ? (uint32_t)hs0 * 4u : kDrop, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < NVT; ++j) {
            const int q = (int)threadIdx.x + 256 * j;
            pv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ml_rsrc, q < NV4 ? (uint32_t)q * 16u : kDrop, 0, 0));
        }
        pbo = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ml_rsrc, (uint32_t)S::OBO * 4u, 0, 0));
        for (int e = threadIdx.x; e < S::WLDS / 4; e += 256) reinterpret_cast<f32x4*>(wl)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    if (!dwave) {
        load_x(un, cu, cv);
        if constexpr (GU) load_xu(hu0, hv0);
        load_ids(un + ustride, nu, nv, ny);
    }
    // float4 group at flat offset e0 -> its LDS operand-layout positions
    auto put4 = [&](int e0, const f32x4& v) {
        if (e0 < S::OB1) {
            const int i = e0 / L1, c0 = e0 % L1, base = S::SW1 + i * S::S1 + (c0 & 15) * B1 + (c0 >> 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) wl[base + k * B1] = v[k];
        } else if (e0 < S::OW2) {
            *reinterpret_cast<f32x4*>(wl + S::SB1 + (e0 - S::OB1)) = v;
        } else if (e0 < S::OB2) {
            const int e = e0 - S::OW2, i = e / L2, c0 = e % L2, base = S::SW2 + i * S::S2 + (c0 & 15) * B2 + (c0 >> 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) wl[base + k * B2] = v[k];
        } else if (e0 < S::OW3) {
            *reinterpret_cast<f32x4*>(wl + S::SB2 + (e0 - S::OB2)) = v;
        } else if (e0 < S::OB3) {
            const int e = e0 - S::OW3;
            *reinterpret_cast<f32x4*>(wl + S::SW3 + (e / L3) * S::S3 + e % L3) = v;
        } else if (e0 < S::OWO) {
            *reinterpret_cast<f32x4*>(wl + S::SB3 + (e0 - S::OB3)) = v;
        } else {
            *reinterpret_cast<f32x4*>(wl + S::SWO + (e0 - S::OWO)) = v;  // [gmf | layer 3] output kernel
        }
    };
    if (!dwave) {
#pragma unroll
        for (int j = 0; j < NVT; ++j) {
            const int q = (int)threadIdx.x + 256 * j;
            if (q < NV4) put4(4 * q, pv[j]);
        }
        if (threadIdx.x == 0) wl[S::SBO] = pbo;
    }
    __syncthreads();
    NCF_WS(2, __builtin_readcyclecounter());
    // split, a batch counted and scanned ahead (fa.cnt): the weight-gradient waves, idle until the
    // chain hands over its first unit, build this batch's index (the fill; the lists unsorted, the
    // touched-row update after this launch orders them) — the step's fill launch and list sort
    // launch disappear.
    if constexpr (SPLIT) {
        if (dwave && fa.cnt)
            fill_wave(fa, users, items, n, FOLD, (int)blockIdx.x * 4 + pw, (int)gridDim.x * 4);
#if NCF_SPLIT_PRIO && NCF_PRIO_P0
        // the chain waves' phase 0 and first unit ahead of their partners' fill in the SIMD's issue
        if (!dwave) __builtin_amdgcn_s_setprio(1);
#endif
    }
    // GU phase 0: P_u = W1_u^T x_u of every group of this chain wave's units, one 16-group tile per
    // FOLD units (k-step q takes user feature XH lq + q), into gpart
    if constexpr (GU) {
        if (!dwave) {
            const int64_t ntile = NCF_DIAG_NOP0 ? 0 : (nown + FOLD - 1) / FOLD;
            for (int64_t tau = 0; tau < ntile; ++tau) {
                int64_t hs = hs0;
                bool hv = hv0;
                if (tau > 0) {
                    hv = tile_head(tau, hs);
                    load_xu((int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, hv ? (uint32_t)hs * 4u : kDrop, 0, 0), hv);
                }
                f32x4 acc[B1];
#pragma unroll
                for (int t = 0; t < B1; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
                pipe<XH, 4, Ops<B1>>(
                    [&](int q, Ops<B1>& o) { ldsv<B1>(wl + S::SW1 + (XH * g + q) * S::S1 + li * B1, o.v); },
                    [&](int q, const Ops<B1>& o) {
#pragma unroll
                        for (int t = 0; t < B1; ++t) acc[t] = mfma16(o.v[t], xu[q], acc[t]);
                    });
                const uint32_t off = hv ? (uint32_t)(((hs / FOLD) * L1 + 4 * g) * 4) : kDrop;
#pragma unroll
                for (int t = 0; t < B1; ++t)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[t]), pu_rsrc,
                                                           off == kDrop ? kDrop : off + 64u * t, 0, 0);
            }
            // the P_u rows are read back by other lanes of this wave: wait for the stores (a
            // workgroup-scope fence emits no vmcnt wait on gfx950, nor does __syncthreads)
            __builtin_amdgcn_s_waitcnt(kVmcnt0);
            load_pu(un);
        }
    }

    // ---- epilogue pieces shared by both forms: row w (one per chain / pair) holds half of the dW
    // tiles at a time in the accumulator layout ([tile][lane][4]) followed by the bias /
    // output-kernel / loss entries; the rows are added in a fixed order ((w0 + w2) + (w1 + w3))
    constexpr int NTHR = SPLIT ? 512 : 256;
    float* slab = slabs + (size_t)blockIdx.x * S::P;
    const float* R0 = lds;
    const float* R1 = lds + S::PR;
    const float* R2 = lds + 2 * S::PR;
    const float* R3 = lds + 3 * S::PR;
    float* R = lds + pw * S::PR;
    static_assert((size_t)4 * S::PR * 4 <= (SPLIT ? S::LDS_BYTES2 : S::LDS_BYTES), "epilogue rows");
    // tile element (lane gq * 16 + c, register r) is row 16 a + 4 gq + r (split dW1: row
    // B0 (4 gq + r) + a), column 16 b + c of its matrix
#if NCF_EPI_WIDE
    // Wide form: a tile sits in its row as [4 gq + r][c] (put_tile: four ds_write_b32 per lane, 2-way
    // at most), so thread q of a reduction round reads 4 consecutive columns of tile row (q & 63) / 4
    // (b128, the wave's 256 contiguous floats: conflict-free) and writes them with ONE 16-byte store
    // (buffer store: a slab starts at blockIdx.x * P floats, 4-byte aligned) — a quarter of the
    // end-of-kernel store instructions, which set that tail (MI355X_MICROARCH.md, epilogue store tail)
    const __amdgpu_buffer_rsrc_t slab_rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, (int)(S::P * 4), 0x00020000);
    auto put_tile = [&](float* Rt, const f32x4& v) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Rt[(4 * g + r) * 16 + li] = v[r];
    };
    auto reduce_tiles = [&](int t0, int t1) {
        for (int q = threadIdx.x; q < (t1 - t0) * 64; q += NTHR) {
            const int tl = q >> 6, tr = (q & 63) >> 2, cq = q & 3;
            auto at4 = [&](const float* row) { return *reinterpret_cast<const f32x4*>(row + tl * 256 + 4 * (q & 63)); };
            const f32x4 x = (at4(R0) + at4(R2)) + (at4(R1) + at4(R3));
            const int t = t0 + tl;  // uniform per wave
            int off;
            bool keep = true;
            if (t < S::NT1) {
                int row;
                if constexpr (GU) {
                    const int a = t / B1;
                    row = (a < B0 / 2 ? 0 : D0) + a % (B0 / 2) + tr * (B0 / 2);
                } else if constexpr (SPLIT) {
                    row = t / B1 + tr * B0;
                } else {
                    row = 16 * (t / B1) + tr;
                }
                off = S::OW1 + row * L1 + 16 * (t % B1) + 4 * cq;
            } else if (t < S::NT1 + S::NT2) {
                off = S::OW2 + (16 * ((t - S::NT1) / B2) + tr) * L2 + 16 * ((t - S::NT1) % B2) + 4 * cq;
            } else {
                off = S::OW3 + (16 * (t - S::NT1 - S::NT2) + tr) * L3 + 4 * cq;
                keep = 4 * cq < L3;
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), slab_rsrc,
                                                   keep ? (uint32_t)off * 4u : kDrop, 0, 0);
        }
    };
#else
    auto put_tile = [&](float* Rt, const f32x4& v) { *reinterpret_cast<f32x4*>(Rt + lane * 4) = v; };
    auto reduce_tiles = [&](int t0, int t1) {
        for (int q = threadIdx.x; q < (t1 - t0) * 64; q += NTHR) {
            auto at4 = [&](const float* row) { return *reinterpret_cast<const f32x4*>(row + 4 * q); };
            const f32x4 x = (at4(R0) + at4(R2)) + (at4(R1) + at4(R3));
            const int t = t0 + (q >> 6);  // uniform per wave
            int base, ld, rs = 1;
            bool keep = true;
            if (t < S::NT1) {
                if constexpr (GU) {
                    // tile a < B0 / 2: user feature (B0 / 2) row + a; else item feature D0 + (B0 / 2) row + a - B0 / 2
                    const int a = t / B1;
                    base = S::OW1 + ((a < B0 / 2 ? 0 : D0) + a % (B0 / 2)) * L1 + 16 * (t % B1) + li, ld = L1,
                    rs = B0 / 2;
                } else if constexpr (SPLIT) {
                    base = S::OW1 + (t / B1) * L1 + 16 * (t % B1) + li, ld = L1, rs = B0;
                } else {
                    base = S::OW1 + 16 * (t / B1) * L1 + 16 * (t % B1) + li, ld = L1;
                }
            } else if (t < S::NT1 + S::NT2) {
                base = S::OW2 + 16 * ((t - S::NT1) / B2) * L2 + 16 * ((t - S::NT1) % B2) + li, ld = L2;
            } else {
                base = S::OW3 + 16 * (t - S::NT1 - S::NT2) * L3 + li, ld = L3;
                keep = li < L3;
            }
            if (keep) {
#pragma unroll
                for (int r = 0; r < 4; ++r) slab[base + (4 * g + r) * rs * ld] = x[r];
            }
        }
    };
#endif
    // biases, output kernel, output bias: back to back in the rows (RB1 .. RBO), segment by
    // segment in the flat layout; the loss / hit / dcg partials
    auto reduce_rest = [&]() {
        for (int e = threadIdx.x; e <= S::RBO - S::RB1; e += NTHR) {
            const int d = e < L1 ? S::OB1 + e
                          : e < L1 + L2 ? S::OB2 + (e - L1)
                          : e < L1 + L2 + L3 ? S::OB3 + (e - L1 - L2)
                                             : S::OWO + (e - L1 - L2 - L3);
            slab[d] = (R0[S::RB1 + e] + R2[S::RB1 + e]) + (R1[S::RB1 + e] + R3[S::RB1 + e]);
        }
        if (threadIdx.x == 0) {
            part_bce[blockIdx.x] = (R0[S::RX] + R2[S::RX]) + (R1[S::RX] + R3[S::RX]);
            if constexpr (MET) {
                part_hit[blockIdx.x] = (R0[S::RX + 1] + R2[S::RX + 1]) + (R1[S::RX + 1] + R3[S::RX + 1]);
                part_dcg[blockIdx.x] = (R0[S::RX + 2] + R2[S::RX + 2]) + (R1[S::RX + 2] + R3[S::RX + 2]);
            }
        }
    };

    const int fm = FOLD > 1 ? FOLD - 1 : 0;
    // stores through buffer resources: a lane whose sample is past n (or whose user row is folded
    // into its group head) gets an offset past the buffer (kDrop) and the hardware drops the
    // store, so the unit body has no branches and the scheduler sees it as one block
    const __amdgpu_buffer_rsrc_t gs_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(gs, (short)0, (int)(uint32_t)(2 * n * W * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t pr_rsrc = __builtin_amdgcn_make_buffer_rsrc(probs, (short)0, (int)(uint32_t)(n * 4), 0x00020000);
    auto st4 = [&](uint32_t off, float a, float b, float c, float d) {
        const f32x4 v = {a, b, c, d};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), gs_rsrc, off, 0, 0);
    };
    // dX = W1 G1 of one 16-sample unit into the gradient rows' MLP parts: block ti holds input
    // features 16 ti + 4 lq .. + 3 of sample li (user half folded into the group head like the
    // GMF part); two blocks' chains interleaved, k-step (t, r) takes G1 feature 16 t + 4 lq + r
    // (tile pairs [TP0, TP1): B0 / 4 pairs of user tiles, then the item ones; FU: fold the user rows)
    auto dx_rows = [&](const float (&g1)[B1][4], uint32_t urow_off, uint32_t irow_off, bool fmatch, bool fhead,
                       auto tp0c, auto tp1c, auto fuc) {
        constexpr int TP0 = decltype(tp0c)::value, TP1 = decltype(tp1c)::value;
        constexpr bool FU = decltype(fuc)::value;
#pragma unroll
        for (int tp = NCF_DIAG_HALFL1 ? B0 / 4 : TP0; tp < TP1; ++tp) {
            f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            pipe<4, 2, Ops2<2, B1>>(
                [&](int r, Ops2<2, B1>& o) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        ldsv<B1>(wl + S::SW1 + (16 * (2 * tp + j) + li) * S::S1 + (4 * g + r) * B1, o.v[j]);
                },
                [&](int r, const Ops2<2, B1>& o) {
#pragma unroll
                    for (int t = 0; t < B1; ++t)
#pragma unroll
                        for (int j = 0; j < 2; ++j) acc[j] = mfma16(o.v[j][t], g1[t][r], acc[j]);
                });
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int ti = 2 * tp + j;
                const int f0 = 16 * ti + 4 * g;
                const bool user = 16 * ti < D0;  // compile time: D0 is a multiple of 16
                f32x4 d = acc[j];
                if constexpr (FOLD > 1 && FU) {
                    if (user) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float sm = fold_sum<FOLD>(fmatch ? d[r] : 0.f);
                            d[r] = fhead ? sm : d[r];
                        }
                    }
                }
                const uint32_t base = user ? urow_off : irow_off;
                st4(base == kDrop ? kDrop : base + (G + (user ? f0 : f0 - D0)) * 4, d[0], d[1], d[2], d[3]);
            }
        }
    };
    using ic0 = std::integral_constant<int, 0>;
    using icU = std::integral_constant<int, B0 / 4>;
    using icA = std::integral_constant<int, B0 / 2>;

    if constexpr (SPLIT) {
        if (dwave) {
            // ---- the weight-gradient wave of pair pw
            f32x4 dw1[B0][B1], dw2[B1][B2], dw3[B2];
#pragma unroll
            for (int a = 0; a < B0; ++a)
#pragma unroll
                for (int b = 0; b < B1; ++b) dw1[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int a = 0; a < B1; ++a)
#pragma unroll
                for (int b = 0; b < B2; ++b) dw2[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int a = 0; a < B2; ++a) dw3[a] = f32x4{0.f, 0.f, 0.f, 0.f};
            float ab1[B1], ab2[B2], ab3 = 0.f;
#pragma unroll
            for (int t = 0; t < B1; ++t) ab1[t] = 0.f;
#pragma unroll
            for (int t = 0; t < B2; ++t) ab2[t] = 0.f;
            // X operands of k-step q (sample 4 q + lq, MLP-input features B0 li .. + B0 - 1: lanes
            // li < 8 the user half, else the item half) in slot q & 1: steps 0 and 1 are loaded
            // before the unit's barrier, steps 2 and 3 once the MFMAs of steps 0 and 1 have read
            // their slot.  A masked sample reads the chain's row 0 (its G rows are zero).
            // GU: the unit contracts the item half only (lane li: item features HB li .. + HB - 1, dW1
            // tiles HB + a); the user half is contracted per group after the units (phase N)
            constexpr int HB = B0 / 2;
            constexpr int XW = GU ? HB : B0;
            float xq[2][XW];
            // XW floats of table row `row` from MLP-input float f0 of the row's MLP half into the local
            // array dst (a macro: an array handed to a lambda by reference would live in scratch)
#define NCF_LD_HALF(dst, row, f0)                                                                      \
    do {                                                                                               \
        const float* xs_ = emb + (size_t)(row) * W + G + (f0);                                         \
        if constexpr (XW % 4 == 0) {                                                                   \
            _Pragma("unroll") for (int k_ = 0; k_ < XW / 4; ++k_) {                                     \
                const float4 v_ = reinterpret_cast<const float4*>(xs_)[k_];                            \
                dst[4 * k_] = v_.x, dst[4 * k_ + 1] = v_.y, dst[4 * k_ + 2] = v_.z, dst[4 * k_ + 3] = v_.w; \
            }                                                                                          \
        } else {                                                                                       \
            _Pragma("unroll") for (int k_ = 0; k_ < XW / 2; ++k_) {                                     \
                const float2 v_ = reinterpret_cast<const float2*>(xs_)[k_];                            \
                dst[2 * k_] = v_.x, dst[2 * k_ + 1] = v_.y;                                            \
            }                                                                                          \
        }                                                                                              \
    } while (0)
            auto load_xq = [&](int64_t u, int q) {
                const int64_t si = u * 16 + 4 * q + g;
                const uint32_t off = si < n ? (uint32_t)si * 4u : kDrop;
                const int xu = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, off, 0, 0);
                const int xv = (int)__builtin_amdgcn_raw_buffer_load_b32(it_rsrc, off, 0, 0);
                const bool okr = si < n && (unsigned)xu < (unsigned)ids.ubound && (unsigned)xv < (unsigned)ids.ibound;
                const int row = GU ? (okr ? ids.ibase + xv : 0) : (okr ? (li < 8 ? xu : ids.ibase + xv) : 0);
                const float* xs = emb + (size_t)row * W + G + (GU ? li * HB : (li & 7) * B0);
                if constexpr (XW % 4 == 0) {
#pragma unroll
                    for (int k = 0; k < XW / 4; ++k) {
                        const float4 v = reinterpret_cast<const float4*>(xs)[k];
                        xq[q & 1][4 * k] = v.x, xq[q & 1][4 * k + 1] = v.y, xq[q & 1][4 * k + 2] = v.z,
                                     xq[q & 1][4 * k + 3] = v.w;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < XW / 2; ++k) {
                        const float2 v = reinterpret_cast<const float2*>(xs)[k];
                        xq[q & 1][2 * k] = v.x, xq[q & 1][2 * k + 1] = v.y;
                    }
                }
            };
            // GU, a unit with samples whose user is not their group head's: their user half per sample
            // (k-step q: sample 4 q + lq, G1 zero for the other samples, whose user half is the group's)
            auto contract_mixed = [&](int64_t u, int par) {
                const float* tq = tbuf(par);
#pragma unroll 1
                for (int q = 0; q < 4; ++q) {
                    const int64_t si = u * 16 + 4 * q + g;
                    const uint32_t off = si < n ? (uint32_t)si * 4u : kDrop;
                    const int xu = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, off, 0, 0);
                    const int xv = (int)__builtin_amdgcn_raw_buffer_load_b32(it_rsrc, off, 0, 0);
                    const int hu = (int)__builtin_amdgcn_raw_buffer_load_b32(
                        us_rsrc, si < n ? (uint32_t)(si & ~(int64_t)(FOLD - 1)) * 4u : kDrop, 0, 0);
                    const bool okr = si < n && (unsigned)xu < (unsigned)ids.ubound && (unsigned)xv < (unsigned)ids.ibound;
                    const bool mism = si < n && xu != hu;
                    float g1v[B1], xo[XW];
                    NCF_LD_HALF(xo, okr ? xu : 0, li * HB);
                    ldsv<B1>(tq + S::TG1 + (4 * q + g) * T1 + li * B1, g1v);
#pragma unroll
                    for (int b = 0; b < B1; ++b) g1v[b] = mism ? g1v[b] : 0.f;
#pragma unroll
                    for (int a = 0; a < HB; ++a)
#pragma unroll
                        for (int b = 0; b < B1; ++b) dw1[a][b] = mfma16(xo[a], g1v[b], dw1[a][b]);
                }
            };
            // unit u's contraction from chain buffer `par`
            auto contract = [&](int64_t u, int par) {
                const float* tq = tbuf(par);
                pipe<4, 1, DwOps<1, B1, B2>>(
                    [&](int q, DwOps<1, B1, B2>& o) {
                        const int srow = 4 * q + g;
                        ldsv<B1>(tq + S::TG1 + srow * T1 + li * B1, o.g1);
                        ldsv<B1>(tq + S::TH1 + srow * T1 + li * B1, o.h1);
                        ldsv<B2>(tq + S::TG2 + srow * T2 + li * B2, o.g2);
                        ldsv<B2>(tq + S::TH2 + srow * T2 + li * B2, o.h2);
                        o.g3 = tq[S::TG3 + srow * 16 + li];
                    },
                    [&](int q, const DwOps<1, B1, B2>& o) {
#pragma unroll
                        for (int a = 0; a < XW; ++a)
#pragma unroll
                            for (int b = 0; b < B1; ++b)
                                dw1[GU ? HB + a : a][b] = mfma16(xq[q & 1][a], o.g1[b], dw1[GU ? HB + a : a][b]);
#pragma unroll
                        for (int a = 0; a < B1; ++a)
#pragma unroll
                            for (int b = 0; b < B2; ++b) dw2[a][b] = mfma16(o.h1[a], o.g2[b], dw2[a][b]);
#pragma unroll
                        for (int a = 0; a < B2; ++a) dw3[a] = mfma16(o.h2[a], o.g3, dw3[a]);
#pragma unroll
                        for (int b = 0; b < B1; ++b) ab1[b] += o.g1[b];
#pragma unroll
                        for (int b = 0; b < B2; ++b) ab2[b] += o.g2[b];
                        ab3 += o.g3;
                        if (q < 2) load_xq(u, q + 2);
                    });
            };
            // GU: the user ids of phase N's first tile, loaded now (one memory round trip less
            // at the kernel's tail)
            int phu[4] = {0, 0, 0, 0};
            if constexpr (GU) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = 4 * q + g;
                    const int64_t hs = (un0 + (int64_t)(c / NGU) * ustride) * 16 + (c % NGU) * FOLD;
                    const bool hv = c / NGU < nown && hs < n;
                    phu[q] = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, hv ? (uint32_t)hs * 4u : kDrop, 0, 0);
                }
            }
            if constexpr (NCF_SPLIT_LATE) {
                // unit it - 1 is contracted between barriers A(it) (the chain's layer 1 of unit it
                // done) and B(it): beside the chain's sections that issue few MFMAs, not beside its
                // layer 1
                int64_t uprev = nunits;  // none
                for (int64_t it = 0; it < nit; ++it, un += ustride) {
                    const bool havep = uprev < nunits;
                    if (havep) {  // in flight while the chain runs layer 1
                        load_xq(uprev, 0);
                        load_xq(uprev, 1);
                    }
                    if (!NCF_SPLIT_NOSYNC) __syncthreads();  // A(it)
                    if (havep && !NCF_SPLIT_NODW) contract(uprev, (int)((it - 1) & 1));
                    if (!NCF_SPLIT_NOSYNC) __syncthreads();  // B(it): unit it's buffers written
                    uprev = un;
                }
                if (uprev < nunits && !NCF_SPLIT_NODW) {
                    load_xq(uprev, 0);
                    load_xq(uprev, 1);
                    contract(uprev, (int)((nit - 1) & 1));
                }
            } else {
                for (int64_t it = 0; it < nit; ++it, un += ustride) {
                    const bool have = un < nunits;
                    int xu = 0;
                    bool mixed = false;
                    if (have) {  // in flight while the chain finishes the unit
                        load_xq(un, 0);
                        load_xq(un, 1);
                        if constexpr (GU) {
                            // sample li's user against its group head's
                            const int64_t si = un * 16 + li;
                            const int su = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, si < n ? (uint32_t)si * 4u : kDrop, 0, 0);
                            const int hu = (int)__builtin_amdgcn_raw_buffer_load_b32(
                                us_rsrc, si < n ? (uint32_t)(si & ~(int64_t)(FOLD - 1)) * 4u : kDrop, 0, 0);
                            mixed = __ballot(si < n && su != hu) != 0;
                        }
                        if constexpr (NCF_SPLIT_DX) {
                            // sample li's user id: the dX rows' offsets and folding
                            const int64_t si = un * 16 + li;
                            xu = (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, si < n ? (uint32_t)si * 4u : kDrop,
                                                                          0, 0);
                        }
                    }
                    if (!NCF_SPLIT_NOSYNC) __syncthreads();  // barrier it: chain wave pw wrote unit it's buffers
                    if (have && !NCF_SPLIT_NODW) {
                        // the contraction first: its X operands (loaded before the barrier) are dead
                        // once it is done, which leaves dX the registers its chains need
                        contract(un, (int)(it & 1));
                        if constexpr (GU) {
                            if (mixed) contract_mixed(un, (int)(it & 1));
                        }
                        if constexpr (NCF_SPLIT_DX) {
                            // the chain's G1 (transposed buffer row li: feature 16 t + 4 lq + r at
                            // position (4 lq + r) B1 + t), read with each k-step's W1 operands (the
                            // 168 accumulators leave no room to hold all of it), and the row offsets
                            // the chain uses
                            const float* tq = tbuf((int)(it & 1));
                            const int64_t sg = un * 16 + li;
                            const bool inb = sg < n;
                            const int su = inb ? xu : -1;
                            const bool fmatch = FOLD > 1 && inb && su == grp_bcast<(FOLD > 1 ? FOLD : 2)>(su, 0, lane);
                            const bool fhead = (li & fm) == 0;
                            const uint32_t urow_off = inb && (fhead || !fmatch) ? (uint32_t)(2 * sg * W) * 4u : kDrop;
                            const uint32_t irow_off = inb ? (uint32_t)((2 * sg + 1) * W) * 4u : kDrop;
#pragma unroll
                            for (int tp = 0; tp < B0 / 2; ++tp) {
                                f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
                                pipe<4, 2, Ops2<3, B1>>(
                                    [&](int r, Ops2<3, B1>& o) {
#pragma unroll
                                        for (int j = 0; j < 2; ++j)
                                            ldsv<B1>(wl + S::SW1 + (16 * (2 * tp + j) + li) * S::S1 + (4 * g + r) * B1,
                                                     o.v[j]);
                                        ldsv<B1>(tq + S::TG1 + li * T1 + (4 * g + r) * B1, o.v[2]);
                                    },
                                    [&](int r, const Ops2<3, B1>& o) {
#pragma unroll
                                        for (int t = 0; t < B1; ++t)
#pragma unroll
                                            for (int j = 0; j < 2; ++j) acc[j] = mfma16(o.v[j][t], o.v[2][t], acc[j]);
                                    });
#pragma unroll
                                for (int j = 0; j < 2; ++j) {
                                    const int ti = 2 * tp + j;
                                    const int f0 = 16 * ti + 4 * g;
                                    const bool user = 16 * ti < D0;
                                    f32x4 d = acc[j];
                                    if constexpr (FOLD > 1) {
                                        if (user) {
#pragma unroll
                                            for (int r = 0; r < 4; ++r) {
                                                const float sm = fold_sum<FOLD>(fmatch ? d[r] : 0.f);
                                                d[r] = fhead ? sm : d[r];
                                            }
                                        }
                                    }
                                    const uint32_t base = user ? urow_off : irow_off;
                                    st4(base == kDrop ? kDrop : base + (G + (user ? f0 : f0 - D0)) * 4, d[0], d[1], d[2],
                                        d[3]);
                                }
                            }
                        }
                    }
                }
            }
            if constexpr (GU) {
                // phase N: dW1's user half, sum over groups of x_u (sum g1)^T, 16 groups per tile
                // (k-step q: column 4 q + lq of chain wave pw's phase-0 tile); the chain wave waited
                // for its group-sum stores before the last unit barrier, so this runs beside the
                // chain wave's own phase N
                const int64_t ntile = NCF_DIAG_NOPN ? 0 : (nown + FOLD - 1) / FOLD;
                for (int64_t tau = 0; tau < ntile; ++tau) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int c = 4 * q + g;
                        const int64_t k = tau * FOLD + c / NGU;
                        const int64_t hs = (un0 + k * ustride) * 16 + (c % NGU) * FOLD;
                        const bool hv = k < nown && hs < n;
                        const int hu = tau == 0 ? phu[q]
                                                : (int)__builtin_amdgcn_raw_buffer_load_b32(us_rsrc, hv ? (uint32_t)hs * 4u : kDrop, 0, 0);
                        float s1[B1], xo[XW];
                        NCF_LD_HALF(xo, hv && (unsigned)hu < (unsigned)ids.ubound ? hu : 0, li * HB);
                        const uint32_t off = hv ? (uint32_t)(((hs / FOLD) * L1 + li) * 4) : kDrop;
#pragma unroll
                        for (int b = 0; b < B1; ++b)
                            s1[b] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(sgr_rsrc, off == kDrop ? kDrop : off + 64u * b, 0, 0));
#pragma unroll
                        for (int a = 0; a < HB; ++a)
#pragma unroll
                            for (int b = 0; b < B1; ++b) dw1[a][b] = mfma16(xo[a], s1[b], dw1[a][b]);
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < B1; ++t) ab1[t] = group_allsum(ab1[t]);
#pragma unroll
            for (int t = 0; t < B2; ++t) ab2[t] = group_allsum(ab2[t]);
            ab3 = group_allsum(ab3);
            auto put_tiles = [&](int t0, int t1) {
#pragma unroll
                for (int a = 0; a < B0; ++a)
#pragma unroll
                    for (int b = 0; b < B1; ++b) {
                        const int t = a * B1 + b;
                        if (t >= t0 && t < t1) put_tile(R + (t - t0) * 256, dw1[a][b]);
                    }
#pragma unroll
                for (int a = 0; a < B1; ++a)
#pragma unroll
                    for (int b = 0; b < B2; ++b) {
                        const int t = S::NT1 + a * B2 + b;
                        if (t >= t0 && t < t1) put_tile(R + (t - t0) * 256, dw2[a][b]);
                    }
#pragma unroll
                for (int a = 0; a < B2; ++a) {
                    const int t = S::NT1 + S::NT2 + a;
                    if (t >= t0 && t < t1) put_tile(R + (t - t0) * 256, dw3[a]);
                }
            };
            __syncthreads();  // every wave is done with the weights and the buffers
#undef NCF_LD_HALF
            if (g == 0) {
#pragma unroll
                for (int t = 0; t < B1; ++t) R[S::RB1 + 16 * t + li] = ab1[t];
#pragma unroll
                for (int t = 0; t < B2; ++t) R[S::RB2 + 16 * t + li] = ab2[t];
                if (li < L3) R[S::RB3 + li] = ab3;
            }
            put_tiles(0, S::NTH);
            __syncthreads();
            reduce_tiles(0, S::NTH);
            reduce_rest();
            __syncthreads();  // the first round's rows are read before the second overwrites them
            put_tiles(S::NTH, S::NT);
            __syncthreads();
            reduce_tiles(S::NTH, S::NT);
            return;
        }
    }

    f32x4 dw1[B0][B1], dw2[B1][B2], dw3[B2];
#pragma unroll
    for (int a = 0; a < B0; ++a)
#pragma unroll
        for (int b = 0; b < B1; ++b) dw1[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < B1; ++a)
#pragma unroll
        for (int b = 0; b < B2; ++b) dw2[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < B2; ++a) dw3[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    // bias gradients: summed from the dW phase's G operands (lane: output feature 16 t + li,
    // samples 4 q + lq), so a layer costs one register per 16-column block
    float ab1[B1], ab2[B2], ab3 = 0.f, ah3[4], agmf[GQA];
#pragma unroll
    for (int t = 0; t < B1; ++t) ab1[t] = 0.f;
#pragma unroll
    for (int t = 0; t < B2; ++t) ab2[t] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) ah3[r] = 0.f;
#pragma unroll
    for (int e = 0; e < GQA; ++e) agmf[e] = 0.f;
    float acc_bce = 0.f, acc_dbo = 0.f, acc_hit = 0.f, acc_dcg = 0.f;

    NCF_WT(0, 8);
#if NCF_SPLIT_PRIO
    if constexpr (SPLIT) __builtin_amdgcn_s_setprio(1);  // the chain wave's serial sections first
#endif
    int itw = -1;
    // split: one pass per barrier of the workgroup (a chain wave past its last unit only passes
    // the barrier)
    for (int64_t it = 0; SPLIT ? it < nit : un < nunits; ++it, un += ustride) {
      if (SPLIT && un >= nunits) {
        // GU: this wave's group sums have landed before the last barrier (its partner reads them
        // right after the loop)
        if constexpr (GU) if (it + 1 == nit) __builtin_amdgcn_s_waitcnt(kVmcnt0);
        if (!NCF_SPLIT_NOSYNC) {
            if (NCF_SPLIT_LATE) __syncthreads();
            __syncthreads();
        }
        continue;
      }
      if constexpr (SPLIT) tb = tbuf((int)(it & 1));
      {
        ++itw;
        NCF_WT(itw, 0);
        const int64_t s0 = un * 16, sg = s0 + li, un1 = un + ustride;
        int tu, tv;
        float ty;
        load_ids(un1 + ustride, tu, tv, ty);  // ids two units ahead, consumed at this unit's end
        load_g(un, cu, cv);                    // this unit's GMF slices, first used by the output
        const bool inb = sg < n;
        const bool ok = inb && (unsigned)cu < (unsigned)ids.ubound && (unsigned)cv < (unsigned)ids.ibound;
        // user rows of a fold group summed into its head sample (fmatch: this sample's user is the head's)
        const int su = inb ? cu : -1;
        const bool fmatch = FOLD > 1 && inb && su == grp_bcast<(FOLD > 1 ? FOLD : 2)>(su, 0, lane);
        const bool fhead = (li & fm) == 0;
        // byte offsets of this sample's user / item gradient rows (or dropped)
        const uint32_t urow_off = inb && (fhead || !fmatch) ? (uint32_t)(2 * sg * W) * 4u : kDrop;
        const uint32_t irow_off = inb ? (uint32_t)((2 * sg + 1) * W) * 4u : kDrop;

        // ---- X^T for dW1 (row li: features XQ lq + q), then layer 1: k-step q takes feature
        // XQ lq + q from lane group lq (A: W1 row XQ lq + q, all B1 output blocks in one read)
        if constexpr (!SPLIT) {
#pragma unroll
            for (int q = 0; q < XQ; ++q)
                tb[S::TX + li * T0 + (XQ / 16) * g + (q & 15) * B0 + (q >> 4)] = xr[q];
        }
        f32x4 h1[B1];
        if constexpr (GU) {
            // the group's P_u, then the item half (k-step q: item feature XH lq + q)
#pragma unroll
            for (int t = 0; t < B1; ++t) h1[t] = pun[t];
            if (__ballot(inb && !fmatch)) {
                // a sample whose user is not its head's: its own user half (units of such batches only)
                int urow, irow;
                rows_of(un, cu, cv, urow, irow);
                const float4* xs = reinterpret_cast<const float4*>(emb + (size_t)urow * W + G + g * XH);
                float xo[XH];
#pragma unroll
                for (int k = 0; k < XH / 4; ++k) {
                    const float4 v = xs[k];
                    xo[4 * k] = v.x, xo[4 * k + 1] = v.y, xo[4 * k + 2] = v.z, xo[4 * k + 3] = v.w;
                }
                f32x4 a2[B1];
#pragma unroll
                for (int t = 0; t < B1; ++t) a2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
                pipe<XH, 4, Ops<B1>>(
                    [&](int q, Ops<B1>& o) { ldsv<B1>(wl + S::SW1 + (XH * g + q) * S::S1 + li * B1, o.v); },
                    [&](int q, const Ops<B1>& o) {
#pragma unroll
                        for (int t = 0; t < B1; ++t) a2[t] = mfma16(o.v[t], xo[q], a2[t]);
                    });
                if (inb && !fmatch) {
#pragma unroll
                    for (int t = 0; t < B1; ++t) h1[t] = a2[t];
                }
            }
            pipe<XH, 4, Ops<B1>>(
                [&](int q, Ops<B1>& o) { ldsv<B1>(wl + S::SW1 + (D0 + XH * g + q) * S::S1 + li * B1, o.v); },
                [&](int q, const Ops<B1>& o) {
#pragma unroll
                    for (int t = 0; t < B1; ++t) h1[t] = mfma16(o.v[t], xr[q], h1[t]);
                });
        } else {
#pragma unroll
            for (int t = 0; t < B1; ++t) h1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            pipe<NCF_DIAG_HALFL1 ? XQ / 2 : XQ, 4, Ops<B1>>(
                [&](int q, Ops<B1>& o) { ldsv<B1>(wl + S::SW1 + (XQ * g + q) * S::S1 + li * B1, o.v); },
                [&](int q, const Ops<B1>& o) {
#pragma unroll
                    for (int t = 0; t < B1; ++t) h1[t] = mfma16(o.v[t], xr[q], h1[t]);
                });
        }

#pragma unroll
        for (int t = 0; t < B1; ++t) {
            float b[4];
            ldsv<4>(wl + S::SB1 + 16 * t + 4 * g, b);
#pragma unroll
            for (int r = 0; r < 4; ++r) h1[t][r] = fmaxf(h1[t][r] + b[r], 0.f);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v[B1];
#pragma unroll
            for (int t = 0; t < B1; ++t) v[t] = h1[t][r];
            stsv<B1>(tb + S::TH1 + li * T1 + (4 * g + r) * B1, v);
        }

        // split, late contraction: barrier A (the weight-gradient wave starts on the previous unit)
        if constexpr (SPLIT) if (NCF_SPLIT_LATE && !NCF_SPLIT_NOSYNC) __syncthreads();
        NCF_WT(itw, 1);
        // ---- layer 2: k-step (t, r) takes H1 feature 16 t + 4 lq + r (this lane's register)
        f32x4 h2[B2];
#pragma unroll
        for (int t = 0; t < B2; ++t) h2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        pipe<4 * B1, 4, Ops<B2>>(
            [&](int k, Ops<B2>& o) { ldsv<B2>(wl + S::SW2 + (16 * (k >> 2) + 4 * g + (k & 3)) * S::S2 + li * B2, o.v); },
            [&](int k, const Ops<B2>& o) {
#pragma unroll
                for (int t2 = 0; t2 < B2; ++t2) h2[t2] = mfma16(o.v[t2], h1[k >> 2][k & 3], h2[t2]);
            });
#pragma unroll
        for (int t = 0; t < B2; ++t) {
            float b[4];
            ldsv<4>(wl + S::SB2 + 16 * t + 4 * g, b);
#pragma unroll
            for (int r = 0; r < 4; ++r) h2[t][r] = fmaxf(h2[t][r] + b[r], 0.f);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v[B2];
#pragma unroll
            for (int t = 0; t < B2; ++t) v[t] = h2[t][r];
            stsv<B2>(tb + S::TH2 + li * T2 + (4 * g + r) * B2, v);
        }

        // ---- layer 3 (one 16-row block, padded): two accumulation chains, then added
        f32x4 h3c[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        pipe<4 * B2, 4, Ops<1>>(
            [&](int k, Ops<1>& o) { o.v[0] = wl[S::SW3 + (16 * (k >> 2) + 4 * g + (k & 3)) * S::S3 + li]; },
            [&](int k, const Ops<1>& o) { h3c[k & 1] = mfma16(o.v[0], h2[k >> 2][k & 3], h3c[k & 1]); });
        float h3[4], wo3[4];
        {
            float b[4];
            ldsv<4>(wl + S::SB3 + 4 * g, b);
            ldsv<4>(wl + S::SWO + G + 4 * g, wo3);
#pragma unroll
            for (int r = 0; r < 4; ++r) h3[r] = fmaxf(h3c[0][r] + h3c[1][r] + b[r], 0.f);
        }

        NCF_WT(itw, 2);
        // ---- output: this lane's 4 H3 features and GQ GMF dims, then the 4 lane groups
        float wg[GQA];
        float zp = 0.f;
        if constexpr (G > 0) {
            // the GMF slices are first used here: without this fence the compiler hoists their
            // products next to the loads (issued after layer 1) and the unit waits for them there
#pragma unroll
            for (int e = 0; e < GQ; ++e) asm volatile("" : "+v"(gu[e]), "+v"(gi[e]));
        }
        // the next unit's MLP input into the registers layer 1 has consumed (issued after the
        // fence above, whose wait covers every load before it)
        if (un1 < nunits) {
            load_x(un1, nu, nv);
            load_pu(un1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) zp += wo3[r] * h3[r];
        if constexpr (G > 0) {
            if constexpr (GQ % 4 == 0) {
#pragma unroll
                for (int k = 0; k < GQ / 4; ++k) {
                    float v[4];
                    ldsv<4>(wl + S::SWO + GQ * g + 4 * k, v);
#pragma unroll
                    for (int i = 0; i < 4; ++i) wg[4 * k + i] = v[i];
                }
            } else {
#pragma unroll
                for (int e = 0; e < GQ; ++e) wg[e] = wl[S::SWO + GQ * g + e];
            }
#pragma unroll
            for (int e = 0; e < GQ; ++e) zp += wg[e] * (gu[e] * gi[e]);
        }
        const float z = group_allsum(zp) + wl[S::SBO];
        // v_exp_f32 / v_rcp_f32 (about 1 ulp each): the probability stays within ~1e-7 of the
        // correctly rounded sigmoid, far inside the 2e-6 the tests hold it to
        const float pr = __builtin_amdgcn_rcpf(1.0f + __expf(-z));
        const float dz = ok && pr >= eps && pr <= hi_clip ? (pr - cy) * inv_batch : 0.0f;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ok ? pr : __int_as_float(0x7fc00000)), pr_rsrc,
                                              g == 0 && inb ? (uint32_t)sg * 4u : kDrop, 0, 0);
        {
            // Keras BCE of the clipped probability: binary_crossentropy through the logit,
            // max(l, 0) - l y + log(1 + e^-|l|) with l = log(pc / (1 - pc)), equals
            // -y log(pc) - (1 - y) log(1 - pc) (v_log_f32, ~1 ulp); one lane group counts each
            // sample, a masked one adds nothing
            const float pc = fminf(fmaxf(pr, eps), hi_clip);
            const float bce = -(cy * __logf(pc) + (1.0f - cy) * __logf(1.0f - pc));
            acc_bce += g == 0 && ok ? bce : 0.f;
            acc_dbo += g == 0 ? dz : 0.f;
        }
        // RankLayer + _get_hits_per_user (model.py:344-455) for groups of FOLD samples (the
        // launch asks for it when group == FOLD): label = first max of y; position =
        // #(p > p_lab) + #(earlier ties)
        if constexpr (MET) {
            const int e = li & fm;
            int lab = 0;
            float best = grp_bcast<FOLD>(cy, 0, lane), pq[FOLD];
#pragma unroll
            for (int q = 1; q < FOLD; ++q) {
                const float yq = grp_bcast<FOLD>(cy, q, lane);
                lab = yq > best ? q : lab;
                best = fmaxf(best, yq);
            }
#pragma unroll
            for (int q = 0; q < FOLD; ++q) pq[q] = grp_bcast<FOLD>(pr, q, lane);
            float pl = pq[0];
#pragma unroll
            for (int q = 1; q < FOLD; ++q) pl = lab == q ? pq[q] : pl;
            int pos = 0;
#pragma unroll
            for (int q = 0; q < FOLD; ++q) pos += (pq[q] > pl) || (pq[q] == pl && q < lab);
            const float hit = g == 0 && e == 0 && inb && pos < topk ? 1.f : 0.f;
            acc_hit += hit;
            acc_dcg += hit * (0.69314718f * __builtin_amdgcn_rcpf(__logf((float)pos + 2.0f)));
        }

        NCF_WT(itw, 3);
        // ---- G3 (registers; padded features have h3 = 0 -> 0) and its transposed copy
        float g3[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            g3[r] = h3[r] > 0.f ? dz * wo3[r] : 0.f;
            ah3[r] += dz * h3[r];
        }
        stsv<4>(tb + S::TG3 + li * 16 + 4 * g, g3);

        // ---- GMF backward; user rows of a fold group summed into its head sample
        if constexpr (G > 0) {
            float gug[GQ], gig[GQ];
#pragma unroll
            for (int e = 0; e < GQ; ++e) {
                gug[e] = dz * wg[e] * gi[e];
                gig[e] = dz * wg[e] * gu[e];
                agmf[e] += dz * (gu[e] * gi[e]);
            }
            if constexpr (FOLD > 1) {
#pragma unroll
                for (int e = 0; e < GQ; ++e) {
                    const float sm = fold_sum<FOLD>(fmatch ? gug[e] : 0.f);
                    gug[e] = fhead ? sm : gug[e];
                }
            }
            // masked samples (dz = 0) write zero rows: the index may count their other, valid id
            if constexpr (GQ % 4 == 0) {
#pragma unroll
                for (int k = 0; k < GQ / 4; ++k) {
                    st4(urow_off == kDrop ? kDrop : urow_off + (GQ * g + 4 * k) * 4, gug[4 * k], gug[4 * k + 1],
                        gug[4 * k + 2], gug[4 * k + 3]);
                    st4(irow_off == kDrop ? kDrop : irow_off + (GQ * g + 4 * k) * 4, gig[4 * k], gig[4 * k + 1],
                        gig[4 * k + 2], gig[4 * k + 3]);
                }
            } else {
#pragma unroll
                for (int e = 0; e < GQ; ++e) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(gug[e]), gs_rsrc,
                                                          urow_off == kDrop ? kDrop : urow_off + (GQ * g + e) * 4, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(gig[e]), gs_rsrc,
                                                          irow_off == kDrop ? kDrop : irow_off + (GQ * g + e) * 4, 0, 0);
                }
            }
        }

        NCF_WT(itw, 4);
        // ---- G2 = (W3 G3) ⊙ relu'(H2): k-step r takes G3 feature 4 lq + r; one b128 read gives
        // the 4 steps' A operands (W3 row 16 ti + li, columns 4 lq .. 4 lq + 3).  relu' of H2 and
        // H1 from the transposed copies: their registers are free after layer 3
        float g2[B2][4];
        {
            float hv[4][B2], a[B2][4];
#pragma unroll
            for (int r = 0; r < 4; ++r) ldsv<B2>(tb + S::TH2 + li * T2 + (4 * g + r) * B2, hv[r]);
#pragma unroll
            for (int ti = 0; ti < B2; ++ti) ldsv<4>(wl + S::SW3 + (16 * ti + li) * S::S3 + 4 * g, a[ti]);
            f32x4 acc[B2];
#pragma unroll
            for (int ti = 0; ti < B2; ++ti) acc[ti] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ti = 0; ti < B2; ++ti) acc[ti] = mfma16(a[ti][r], g3[r], acc[ti]);
#pragma unroll
            for (int ti = 0; ti < B2; ++ti)
#pragma unroll
                for (int r = 0; r < 4; ++r) g2[ti][r] = hv[r][ti] > 0.f ? acc[ti][r] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v[B2];
#pragma unroll
            for (int t = 0; t < B2; ++t) v[t] = g2[t][r];
            stsv<B2>(tb + S::TG2 + li * T2 + (4 * g + r) * B2, v);
        }

        // ---- G1 = (W2 G2) ⊙ relu'(H1): k-step (t, r) takes G2 feature 16 t + 4 lq + r; the B1
        // output blocks' chains interleaved
        float g1[B1][4];
        {
            f32x4 acc[B1];
#pragma unroll
            for (int ti = 0; ti < B1; ++ti) acc[ti] = f32x4{0.f, 0.f, 0.f, 0.f};
            pipe<4, 2, Ops2<B1, B2>>(
                [&](int r, Ops2<B1, B2>& o) {
#pragma unroll
                    for (int ti = 0; ti < B1; ++ti)
                        ldsv<B2>(wl + S::SW2 + (16 * ti + li) * S::S2 + (4 * g + r) * B2, o.v[ti]);
                },
                [&](int r, const Ops2<B1, B2>& o) {
#pragma unroll
                    for (int t = 0; t < B2; ++t)
#pragma unroll
                        for (int ti = 0; ti < B1; ++ti) acc[ti] = mfma16(o.v[ti][t], g2[t][r], acc[ti]);
                });
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float hv[B1];
                ldsv<B1>(tb + S::TH1 + li * T1 + (4 * g + r) * B1, hv);
#pragma unroll
                for (int ti = 0; ti < B1; ++ti) g1[ti][r] = hv[ti] > 0.f ? acc[ti][r] : 0.f;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v[B1];
#pragma unroll
            for (int t = 0; t < B1; ++t) v[t] = g1[t][r];
            stsv<B1>(tb + S::TG1 + li * T1 + (4 * g + r) * B1, v);
        }

        NCF_WT(itw, 5);
        // ---- dX = W1 G1 -> the per-sample gradient rows (split form: the weight-gradient wave's)
        if constexpr (GU) {
            // the group's G1 summed over the samples that share the head's user, for phase N; the
            // item half here; a sample whose user is not its head's: its own user row here too
            {
                const uint32_t off = inb && fhead ? (uint32_t)(((sg / FOLD) * L1 + 4 * g) * 4) : kDrop;
#pragma unroll
                for (int t = 0; t < B1; ++t) {
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = fold_sum<FOLD>(fmatch ? g1[t][r] : 0.f);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), sgr_rsrc,
                                                           off == kDrop ? kDrop : off + 64u * t, 0, 0);
                }
            }
            dx_rows(g1, kDrop, irow_off, fmatch, fhead, icU{}, icA{}, std::false_type{});
            if (__ballot(inb && !fmatch))
                dx_rows(g1, inb && !fmatch ? (uint32_t)(2 * sg * W) * 4u : kDrop, kDrop, fmatch, fhead, ic0{}, icU{},
                        std::false_type{});
        } else if constexpr (!SPLIT || !NCF_SPLIT_DX || NCF_SPLIT_LATE) {
            dx_rows(g1, urow_off, irow_off, fmatch, fhead, ic0{}, icA{}, std::true_type{});
        }

        // ---- weight gradients over the unit's 16 samples: k-step q takes sample 4 q + lq
        NCF_WT(itw, 6);
        if constexpr (!SPLIT) pipe<4, 2, DwOps<B0, B1, B2>>(
            [&](int q, DwOps<B0, B1, B2>& o) {
                const int srow = 4 * q + g;
                ldsv<B0>(tb + S::TX + srow * T0 + li * B0, o.x);
                ldsv<B1>(tb + S::TG1 + srow * T1 + li * B1, o.g1);
                ldsv<B1>(tb + S::TH1 + srow * T1 + li * B1, o.h1);
                ldsv<B2>(tb + S::TG2 + srow * T2 + li * B2, o.g2);
                ldsv<B2>(tb + S::TH2 + srow * T2 + li * B2, o.h2);
                o.g3 = tb[S::TG3 + srow * 16 + li];
            },
            [&](int, const DwOps<B0, B1, B2>& o) {
#pragma unroll
                for (int a = 0; a < B0; ++a)
#pragma unroll
                    for (int b = 0; b < B1; ++b) dw1[a][b] = mfma16(o.x[a], o.g1[b], dw1[a][b]);
#pragma unroll
                for (int a = 0; a < B1; ++a)
#pragma unroll
                    for (int b = 0; b < B2; ++b) dw2[a][b] = mfma16(o.h1[a], o.g2[b], dw2[a][b]);
#pragma unroll
                for (int a = 0; a < B2; ++a) dw3[a] = mfma16(o.h2[a], o.g3, dw3[a]);
#pragma unroll
                for (int b = 0; b < B1; ++b) ab1[b] += o.g1[b];
#pragma unroll
                for (int b = 0; b < B2; ++b) ab2[b] += o.g2[b];
                ab3 += o.g3;
            });

        // rotate the ids: the loop-carried registers take values loaded a whole unit ago (a load
        // issued here and carried into the next iteration got copied between registers at once,
        // a memory round trip per unit spent waiting)
        cu = nu, cv = nv, cy = ny;
        nu = tu, nv = tv, ny = ty;
        NCF_WT(itw, 7);
      }
      if constexpr (GU) if (it + 1 == nit) __builtin_amdgcn_s_waitcnt(kVmcnt0);  // as above
      if constexpr (SPLIT) if (!NCF_SPLIT_NOSYNC) __syncthreads();  // hand the unit to the weight-gradient wave
    }
#if NCF_SPLIT_PRIO
    if constexpr (SPLIT) __builtin_amdgcn_s_setprio(0);
#endif

    // ---- GU phase N: the folded user rows' MLP part, W1_u (sum g1), 16 groups per tile
    if constexpr (GU) {
        // the group sums were stored by this wave's lanes and waited for before the last barrier
        const int64_t ntile = NCF_DIAG_NOPN ? 0 : (nown + FOLD - 1) / FOLD;
        for (int64_t tau = 0; tau < ntile; ++tau) {
            int64_t hs;
            const bool hv = tile_head(tau, hs);
            const uint32_t off = hv ? (uint32_t)(((hs / FOLD) * L1 + 4 * g) * 4) : kDrop;
            float s1[B1][4];
#pragma unroll
            for (int t = 0; t < B1; ++t) {
                const f32x4 v = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(sgr_rsrc, off == kDrop ? kDrop : off + 64u * t, 0, 0));
#pragma unroll
                for (int r = 0; r < 4; ++r) s1[t][r] = v[r];
            }
            dx_rows(s1, hv ? (uint32_t)(2 * hs * W) * 4u : kDrop, kDrop, true, true, ic0{}, icU{}, std::false_type{});
        }
    }
    // ---- epilogue: per-lane sums over the 16 sample lanes, then the four waves in LDS
    NCF_WS(11, __builtin_readcyclecounter());
#pragma unroll
    for (int r = 0; r < 4; ++r) ah3[r] = row_sum(ah3[r]);
    if constexpr (!SPLIT) {
        // bias sums: over the 4 lane groups (samples 4 q + lq)
#pragma unroll
        for (int t = 0; t < B1; ++t) ab1[t] = group_allsum(ab1[t]);
#pragma unroll
        for (int t = 0; t < B2; ++t) ab2[t] = group_allsum(ab2[t]);
        ab3 = group_allsum(ab3);
    }
#pragma unroll
    for (int e = 0; e < GQ; ++e) agmf[e] = row_sum(agmf[e]);
    acc_dbo = group_allsum(row_sum(acc_dbo));
    acc_bce = group_allsum(row_sum(acc_bce));
    acc_hit = group_allsum(row_sum(acc_hit));
    acc_dcg = group_allsum(row_sum(acc_dcg));
    __syncthreads();  // every wave is done with the weights and its buffers
    NCF_WS(14, __builtin_readcyclecounter());
    // every dW tile of this wave with its tile number (one-wave form)
    auto for_tiles = [&](auto f) {
#pragma unroll
        for (int a = 0; a < B0; ++a)
#pragma unroll
            for (int b = 0; b < B1; ++b) f(a * B1 + b, dw1[a][b]);
#pragma unroll
        for (int a = 0; a < B1; ++a)
#pragma unroll
            for (int b = 0; b < B2; ++b) f(S::NT1 + a * B2 + b, dw2[a][b]);
#pragma unroll
        for (int a = 0; a < B2; ++a) f(S::NT1 + S::NT2 + a, dw3[a]);
    };
    if constexpr (!SPLIT) {
        if (g == 0) {
#pragma unroll
            for (int t = 0; t < B1; ++t) R[S::RB1 + 16 * t + li] = ab1[t];
#pragma unroll
            for (int t = 0; t < B2; ++t) R[S::RB2 + 16 * t + li] = ab2[t];
            if (li < L3) R[S::RB3 + li] = ab3;
        }
    }
    if (li == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (4 * g + r < L3) R[S::RWO + G + 4 * g + r] = ah3[r];
#pragma unroll
        for (int e = 0; e < GQ; ++e) R[S::RWO + GQ * g + e] = agmf[e];
    }
    if (lane == 0) {
        R[S::RBO] = acc_dbo;
        R[S::RX] = acc_bce;
        R[S::RX + 1] = acc_hit;
        R[S::RX + 2] = acc_dcg;
    }
    // Two rounds of half the tiles: every wave (split: every weight-gradient wave) puts its tiles
    // in its own row straight from the accumulators, then all threads add the four rows in a fixed
    // order, slab = (w0 + w2) + (w1 + w3), and write the flat slab
    auto put_tiles = [&](int t0, int t1) {
        if constexpr (!SPLIT)
            for_tiles([&](int t, f32x4& v) {
                if (t >= t0 && t < t1) put_tile(R + (t - t0) * 256, v);
            });
    };
    put_tiles(0, S::NTH);
    __syncthreads();
    reduce_tiles(0, S::NTH);
    reduce_rest();
    NCF_WS(15, __builtin_readcyclecounter());
    __syncthreads();  // the first round's rows are read before the second overwrites them
    put_tiles(S::NTH, S::NT);
    __syncthreads();
    reduce_tiles(S::NTH, S::NT);
    NCF_WT(0, 9);
    NCF_WS(12, __builtin_readcyclecounter());
    NCF_WS(13, __builtin_amdgcn_s_memrealtime());
}

using WShapeC = WShape<128, 64, 32, 16, 64>;  // ml-20m NeuMF (config C)
using WShapeB = WShape<64, 32, 16, 8, 8>;     // ml-1m NeuMF (config B)
using WShapeR = WShape<64, 32, 16, 8, 0>;     // trainer default (MLP-only)
using WShapeC0 = WShape<128, 64, 32, 16, 0>;

template <class S>
bool wmatches(const ncf_shape_t& s) {
    return s.num_layers == 4 && s.layers[0] == S::L0 && s.layers[1] == S::L1 && s.layers[2] == S::L2 &&
           s.layers[3] == S::L3 && s.gmf_dim == S::G && s.row_width == S::W && s.gmf_stride == S::G;
}

// NCF_WAVE_SPLIT (environment, read once): 0 forces the one-wave form on shapes the split form fits
static bool split_enabled() {
    static const int on = [] {
        const char* e = ncf::experiment_env("NCF_WAVE_SPLIT");
        return e && *e ? atoi(e) : 1;
    }();
    return on != 0;
}

template <class S, bool SPLIT>
hipError_t launch_wave_form(const WsLayout& L, void* ws, const float* emb, const float* mlp, const int32_t* users,
                            const int32_t* items, const float* labels, int64_t n, float inv_batch, IdSpace ids,
                            int group, int topk, int* nslab, int* nbce, int* nmet, hipStream_t st, int fold,
                            bool check_fold, const FillArgs* fill) {
    constexpr size_t lds = SPLIT ? S::LDS_BYTES2 : S::LDS_BYTES;
    if (fill && !SPLIT) return hipErrorInvalidValue;
    const FillArgs fa = fill ? *fill : FillArgs{};
    static bool configured = false;  // one-time attribute set per shape and form (idempotent)
    if (!configured) {
        for (const void* k : {(const void*)k_fb_wave<S, 0, false, SPLIT>, (const void*)k_fb_wave<S, 2, false, SPLIT>,
                              (const void*)k_fb_wave<S, 4, false, SPLIT>, (const void*)k_fb_wave<S, 8, false, SPLIT>,
                              (const void*)k_fb_wave<S, 2, true, SPLIT>, (const void*)k_fb_wave<S, 4, true, SPLIT>,
                              (const void*)k_fb_wave<S, 8, true, SPLIT>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        configured = true;
    }
    const int64_t nunits = (n + 15) / 16;
    const int64_t wgs = (nunits + 3) / 4;
    int grid = (int)(wgs < 256 ? wgs : 256);
    if (grid < 1) grid = 1;
    // hr/dcg in the kernel when the metric groups are the fold groups (group 2, 4, 8); other
    // groups get the separate metrics launch
    const bool in_kernel = fold > 1 && group == fold;
    auto go = [&](auto kern) {
        launch(kern, grid, SPLIT ? 512 : 256, lds, st, emb, mlp, users, items, labels, n, ids, inv_batch,
               at<float>(ws, L.probs), at<float>(ws, L.gs), at<float>(ws, L.slabs), at<float>(ws, L.part_bce), group,
               topk, at<float>(ws, L.part_hit), at<float>(ws, L.part_dcg),
               check_fold ? at<const int32_t>(ws, L.ifold) : nullptr, at<int32_t>(ws, L.err), at<float>(ws, L.act), fa);
    };
    switch (fold * 2 + (in_kernel ? 1 : 0)) {
        case 0: go(k_fb_wave<S, 0, false, SPLIT>); break;
        case 4: go(k_fb_wave<S, 2, false, SPLIT>); break;
        case 8: go(k_fb_wave<S, 4, false, SPLIT>); break;
        case 16: go(k_fb_wave<S, 8, false, SPLIT>); break;
        case 5: go(k_fb_wave<S, 2, true, SPLIT>); break;
        case 9: go(k_fb_wave<S, 4, true, SPLIT>); break;
        case 17: go(k_fb_wave<S, 8, true, SPLIT>); break;
        default: return hipErrorInvalidValue;
    }
    *nslab = grid;
    *nbce = grid;
    *nmet = in_kernel ? grid : 0;
    return hipGetLastError();
}

template <class S>
hipError_t launch_wave_one(const WsLayout& L, void* ws, const float* emb, const float* mlp, const int32_t* users,
                           const int32_t* items, const float* labels, int64_t n, float inv_batch, IdSpace ids,
                           int group, int topk, int* nslab, int* nbce, int* nmet, hipStream_t st, int fold,
                           bool check_fold, bool one_wave, const FillArgs* fill) {
    if constexpr (S::SPLIT_OK) {
        if (split_enabled() && !one_wave)
            return launch_wave_form<S, true>(L, ws, emb, mlp, users, items, labels, n, inv_batch, ids, group, topk,
                                             nslab, nbce, nmet, st, fold, check_fold, fill);
    }
    if (fill) return hipErrorInvalidValue;  // the fill needs the split form's weight-gradient waves
    return launch_wave_form<S, false>(L, ws, emb, mlp, users, items, labels, n, inv_batch, ids, group, topk, nslab,
                                      nbce, nmet, st, fold, check_fold, nullptr);
}

}  // namespace

#ifdef NCF_WAVE_TIMING
extern "C" int ncf_debug_wave_timing(unsigned long long* out, size_t count) {
    size_t m = count < sizeof(g_wave_t) / 8 ? count : sizeof(g_wave_t) / 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), m * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
extern "C" int ncf_debug_wave_spans(unsigned long long* out, size_t count) {
    size_t m = count < sizeof(g_wave_s) / 8 ? count : sizeof(g_wave_s) / 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_s), m * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif

bool wave_supported(const ncf_shape_t& s) {
    return wmatches<WShapeC>(s) || wmatches<WShapeB>(s) || wmatches<WShapeR>(s) || wmatches<WShapeC0>(s);
}

bool wave_fill_supported(const ncf_shape_t& s) {
    auto ok = [](bool split_ok) { return split_ok && split_enabled(); };
    return (wmatches<WShapeC>(s) && ok(WShapeC::SPLIT_OK)) || (wmatches<WShapeB>(s) && ok(WShapeB::SPLIT_OK)) ||
           (wmatches<WShapeR>(s) && ok(WShapeR::SPLIT_OK)) || (wmatches<WShapeC0>(s) && ok(WShapeC0::SPLIT_OK));
}

hipError_t launch_fb_wave(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                          const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                          float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                          hipStream_t st, int fold, bool check_fold, bool one_wave, const FillArgs* fill) {
    if (fold != 0 && (fold < 2 || fold > 8 || (fold & (fold - 1)) != 0 || n % fold != 0)) return hipErrorInvalidValue;
    if (fill && (fill->nscan > kMaxFillScan || fill->nscan < 1)) return hipErrorInvalidValue;
#define NCF_ARGS \
    L, ws, emb, mlp, users, items, labels, n, inv_batch, ids, group, topk, nslab, nbce, nmet, st, fold, check_fold, \
        one_wave, fill
    if (wmatches<WShapeC>(s)) return launch_wave_one<WShapeC>(NCF_ARGS);
    if (wmatches<WShapeB>(s)) return launch_wave_one<WShapeB>(NCF_ARGS);
    if (wmatches<WShapeR>(s)) return launch_wave_one<WShapeR>(NCF_ARGS);
    if (wmatches<WShapeC0>(s)) return launch_wave_one<WShapeC0>(NCF_ARGS);
#undef NCF_ARGS
    return hipErrorInvalidValue;
}

}  // namespace ncf
