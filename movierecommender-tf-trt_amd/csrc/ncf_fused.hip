// Fused NeuMF forward + backward on CDNA4 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One 256-thread workgroup (4 waves) per CU, persistent over 128-sample tiles.
// Each wave owns a 32-sample block and runs the whole per-sample chain in
// registers, "feature-major": every activation tile is the 32x32 MFMA D layout
// with the SAMPLE on the lane (j = lane&31) and 16 FEATURE rows in registers
// (row(r, h) = (r&3) + 8(r>>2) + 4h, h = lane>>5).  Because the next layer's
// B operand wants exactly [k = feature][j = sample] with k taken from the lane
// half and the step, a D tile feeds the next MFMA chain register-for-register:
// step s uses B = D[s] and A = W[row(s,h)][out] — no LDS round trip between
// layers (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's
// operand").  Forward:   H1 = relu(W1^T X + b1), H2, H3 (A from W_l [in][out])
// Backward (data):      G3 = dz w_out ⊙ relu'(H3), G2 = (W3 G3) ⊙ relu'(H2),
//                       G1 = (W2 G2) ⊙ relu'(H1), dX = W1 G1  (A from W_l^T)
// The layer-1 B operand X comes straight from the gathered embedding rows:
// the user half of the lanes holds its sample's user MLP vector, the item half
// the item vector (K order h*D0 + s), so the gather needs no concatenation.
//
// Weight gradients reduce over samples (K = samples), which is transposed with
// respect to the D layout: each wave stages H1, H2, G1, G2, G3 of its block
// into LDS ([feature][sample], stride 33: conflict-free), then the 4 waves
// split the dW tiles of the 128-sample tile (A = H_{l-1}[in][sample] from
// LDS — or, for dW1, the embedding rows again from L2 —, B = G_l[out][sample]
// from LDS) and keep them in MFMA accumulators across tiles.  Bias gradients
// are LDS row sums; output-layer gradients are lane transpose-reductions.
// Every sum runs in a fixed order: results are bitwise reproducible.
//
// Outputs match the generic kernel: probs, per-sample embedding gradient rows
// gs[2i] (user) / gs[2i+1] (item), one dense-gradient slab per workgroup and
// one BCE partial per workgroup.  Reference semantics: movierec/model.py:154-214.
// With user-row folding (fold > 1, ncf_internal.h fold_of) the user rows of a
// group's samples that share the head's user are summed across their lanes
// (fixed butterfly order) and only the head writes gs[2 head]: a batch of
// (1 positive + negs) per user writes one user row per group instead of fold.

#include <cmath>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// feature row held in accumulator register r by lane half h
__device__ __forceinline__ constexpr int drow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }

template <int L0_, int L1_, int L2_, int L3_, int G_>
struct FShape {
    static constexpr int L0 = L0_, L1 = L1_, L2 = L2_, L3 = L3_, G = G_;
    static constexpr int D0 = L0 / 2;
    static constexpr int W = G + D0;
    static constexpr int NT0 = cdiv(L0, 32), NT1 = cdiv(L1, 32), NT2 = cdiv(L2, 32), NT3 = cdiv(L3, 32);
    // flat dense-parameter offsets (include/movierec_ncf.h layout)
    static constexpr int OW1 = 0, OB1 = L0 * L1, OW2 = OB1 + L1, OB2 = OW2 + L1 * L2, OW3 = OB2 + L2,
                         OB3 = OW3 + L2 * L3, OWO = OB3 + L3, OBO = OWO + G + L3, P = OBO + 1;
    // LDS copy of the dense parameters: kernels row-major [in][out] with rows padded to out+1
    // floats, so the forward A operand (W[k][out], consecutive out) and the backward A operand
    // (W[in][k], consecutive in: stride out+1, odd) are both bank-conflict-free ds_read_b32
    static constexpr int LW1 = L1 + 1, LW2 = L2 + 1, LW3 = L3 + 1;
    static constexpr int SW1 = 0, SW2 = SW1 + L0 * LW1, SW3 = SW2 + L1 * LW2, SB1 = SW3 + L2 * LW3,
                         SB2 = SB1 + L1, SB3 = SB2 + L2, SWO = SB3 + L3, SBO = SWO + G + L3,
                         WLDS = (SBO + 1 + 3) / 4 * 4;
    // LDS staging rows per 32-sample block (G3 only has L3 real rows)
    static constexpr int RH1 = 0, RH2 = RH1 + 32 * NT1, RG1 = RH2 + 32 * NT2, RG2 = RG1 + 32 * NT1,
                         RG3 = RG2 + 32 * NT2, RB = RG3 + L3;
    static constexpr int LS = 33;
    // MFMA steps of a chain whose K runs over the (NT-tile, 16-register) rows of an
    // activation with L real features: full tiles take 16 steps, a partial last tile
    // only the steps whose rows (8 per 4 steps) reach below L
    static constexpr int nsteps(int L) { return 16 * (cdiv(L, 32) - 1) + (4 * cdiv(L - 32 * (cdiv(L, 32) - 1), 8) < 16 ? 4 * cdiv(L - 32 * (cdiv(L, 32) - 1), 8) : 16); }
    static constexpr int NS1 = nsteps(L1), NS2 = nsteps(L2), NS3 = nsteps(L3);
    static constexpr int NDW1 = NT0 * NT1, NDW2 = NT1 * NT2, NDW3 = NT2 * NT3, NDW = NDW1 + NDW2 + NDW3;
    static constexpr int MAXT = cdiv(NDW, 4);
    // weight-gradient tile t (0..NDW-1, dW1 tiles t = ti*NT1 + to first) of slot m of wave w:
    // when the dW1 tiles split evenly into per-wave input-feature groups (NT0 % 4 == 0), wave w
    // takes the NT1 output tiles of groups ti = w, w+4, ... back to back (the second chain
    // re-reads the gathered rows the first one just pulled into L2), then dW2/dW3 tiles go to
    // waves 3, 2, 1, 0, ...; otherwise round-robin t = w + 4m.  -1: no tile.
    static constexpr int NSLOT1 = (NT0 % 4 == 0) ? (NT0 / 4) * NT1 : 0;
    __device__ static constexpr int dw_tile(int w, int m) {
        if (NSLOT1 == 0) return w + 4 * m < NDW ? w + 4 * m : -1;
        if (m < NSLOT1) return (w + 4 * (m / NT1)) * NT1 + m % NT1;
        const int u = 4 * (m - NSLOT1) + (3 - w);
        return u < NDW - NDW1 ? NDW1 + u : -1;
    }
    static constexpr int GH = G / 2;                     // GMF features per lane half
    static constexpr int GCH = GH >= 16 ? 16 : GH;       // reduction chunk (bounds register pressure)
    static constexpr int NGC = GH >= 16 ? GH / 16 : (GH > 0 ? 1 : 0);
    static constexpr int XCH = G + L3 + 4;               // per-wave exchange floats
    static constexpr size_t LDS_BYTES = (size_t)(4 * RB * LS + WLDS) * 4 + 256 * 4 + (size_t)4 * XCH * 4;
    static_assert(LDS_BYTES <= 163840, "LDS budget");
};

// Sum x[0..V) over the 32 lanes of each wave half (V a power of two <= 32).
// Lane l ends with the total of element (l & 31) >> (5 - log2 V).
template <int V>
__device__ __forceinline__ float half_transpose_reduce(float* x, int lane) {
    constexpr int P = ilog2(V);
#pragma unroll
    for (int st = 0; st < P; ++st) {
        const int m = 16 >> st;
        const int c = V >> st;
        const bool hi = (lane & m) != 0;
#pragma unroll
        for (int v = 0; v < c / 2; ++v) {
            // opaque copies: selecting between two array elements would otherwise be folded into
            // one lane-dependent index into x[] (a c-way v_cndmask chain per element)
            float a = x[v], b = x[v + c / 2];
            asm volatile("" : "+v"(a), "+v"(b));
            const float send = hi ? a : b;
            const float keep = hi ? b : a;
            x[v] = keep + __shfl_xor(send, m, 64);
        }
    }
    float r = x[0];
#pragma unroll
    for (int m = 16 >> P; m >= 1; m >>= 1) r += __shfl_xor(r, m, 64);
    return r;
}

#ifndef NCF_DW1_SHARED
#define NCF_DW1_SHARED 1
#endif
#ifndef NCF_DW1_CH
#define NCF_DW1_CH 8
#endif
#ifndef NCF_SCHED_BARRIER
#define NCF_SCHED_BARRIER 1
#endif
#if NCF_SCHED_BARRIER
#define NCF_SB() __builtin_amdgcn_sched_barrier(0)
#else
#define NCF_SB() ((void)0)
#endif

// acc += sum_t A(t) x B(t) over NS MFMA steps.  A(t) (an LDS/global read) is
// double-buffered CH steps ahead; B(t) is a register (activation tile element).
template <int NS, int CH, class FA, class FB>
__device__ __forceinline__ f32x16 mchain(f32x16 acc, FA fa, FB fb) {
    static_assert(NS % CH == 0, "chain length must be a multiple of the chunk");
    float ab[2][CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) ab[0][e] = fa(e);
#pragma unroll
    for (int c = 0; c < NS / CH; ++c) {
        if (c + 1 < NS / CH) {
#pragma unroll
            for (int e = 0; e < CH; ++e) ab[(c + 1) & 1][e] = fa((c + 1) * CH + e);
        }
        NCF_SB();
#pragma unroll
        for (int e = 0; e < CH; ++e) acc = mfma32(ab[c & 1][e], fb(c * CH + e), acc);
        NCF_SB();
    }
    return acc;
}

// Same with both operands read from memory and double-buffered.
template <int NS, int CH, class FA, class FB>
__device__ __forceinline__ f32x16 mchain2(f32x16 acc, FA fa, FB fb) {
    static_assert(NS % CH == 0, "chain length must be a multiple of the chunk");
    float ab[2][CH], bb[2][CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
        ab[0][e] = fa(e);
        bb[0][e] = fb(e);
    }
#pragma unroll
    for (int c = 0; c < NS / CH; ++c) {
        if (c + 1 < NS / CH) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                ab[(c + 1) & 1][e] = fa((c + 1) * CH + e);
                bb[(c + 1) & 1][e] = fb((c + 1) * CH + e);
            }
        }
        NCF_SB();
#pragma unroll
        for (int e = 0; e < CH; ++e) acc = mfma32(ab[c & 1][e], bb[c & 1][e], acc);
        NCF_SB();
    }
    return acc;
}

// x summed over the FOLD consecutive lanes of its lane group (FOLD = 2, 4 or 8; all lanes
// active): xor butterfly, the quad steps as DPP adds, the third on ds_swizzle (within 32 lanes).
// Every lane of the group ends with the same value.
template <int FOLD>
__device__ __forceinline__ float fold_sum(float x) {
    static_assert(FOLD == 2 || FOLD == 4 || FOLD == 8, "fold width");
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    if constexpr (FOLD >= 4)
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    if constexpr (FOLD >= 8) x += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x1F | (4 << 10)));
    return x;
}

// Phase timestamps of waves 0 and 3 (lane 0) for the first two tiles of every workgroup:
// a profiling build (-DNCF_FUSED_TIMING) only; read with ncf_debug_fused_timing.
#ifdef NCF_FUSED_TIMING
__device__ unsigned long long g_fused_t[256 * 2 * 2 * 16];
#define NCF_T(ph)                                                                                    \
    do {                                                                                             \
        if (lane == 0 && (w == 0 || w == 3) && blockIdx.x < 256 && itl < 2)                          \
            g_fused_t[((blockIdx.x * 2 + itl) * 2 + (w == 3)) * 16 + (ph)] = __builtin_readcyclecounter(); \
    } while (0)
#else
#define NCF_T(ph) ((void)0)
#endif

template <class S, int FOLD>
__global__ __launch_bounds__(kBlock, 1) void k_fb_fused(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                        const int32_t* __restrict__ users,
                                                        const int32_t* __restrict__ items,
                                                        const float* __restrict__ labels, int64_t n, IdSpace ids,
                                                        float inv_batch, float* __restrict__ probs,
                                                        float* __restrict__ gs, float* __restrict__ slabs,
                                                        float* __restrict__ part_bce, int group, int topk,
                                                        float* __restrict__ part_hit, float* __restrict__ part_dcg) {
    constexpr int L0 = S::L0, L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, D0 = S::D0, W = S::W, LS = S::LS;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wl = lds;                                      // dense parameters (WLDS floats)
    float* stg = lds + S::WLDS;                           // [4][RB][LS]
    int* srow = reinterpret_cast<int*>(stg + 4 * S::RB * LS);  // [2][128] table rows (-1 = masked)
    float* xch = reinterpret_cast<float*>(srow + 256);    // [4][XCH]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 31, h = lane >> 5;
    const float eps = 1e-7f, hi_clip = 1.0f - eps;

    f32x16 dwacc[S::MAXT];
#pragma unroll
    for (int m = 0; m < S::MAXT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) dwacc[m][r] = 0.f;
    // bias-gradient rows (L1 + L2 + L3 of them): when the dW tiles leave wave 0 one tile short
    // (3 dW2/dW3 tiles after the dW1 groups, config C) wave 0 sums them all, NBR rows per lane;
    // otherwise thread tid sums row tid.  Same per-row order either way.
    constexpr int NB = L1 + L2 + L3;
    constexpr bool BW0 = S::NSLOT1 > 0 && (S::NDW - S::NDW1) % 4 != 0;
    constexpr int NBR = BW0 ? cdiv(NB, 64) : 1;
    float acc_bias[NBR];
#pragma unroll
    for (int q = 0; q < NBR; ++q) acc_bias[q] = 0.f;
    float acc_h3 = 0.f, acc_dbo = 0.f, acc_bce = 0.f, acc_hit = 0.f, acc_dcg = 0.f;
    const bool metrics = part_hit != nullptr;  // groups never straddle a 32-sample block (group | 32)
    // output-kernel gradients, accumulated per lane (its own samples) across tiles and reduced
    // across lanes once, in the epilogue: a per-tile transpose-reduction is a chain of 16
    // dependent cross-lane shuffles
    float acc_gmf_l[S::GH > 0 ? S::GH : 1];
#pragma unroll
    for (int c = 0; c < (S::GH > 0 ? S::GH : 1); ++c) acc_gmf_l[c] = 0.f;
    float acc_h3_l[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc_h3_l[r] = 0.f;

    // dense parameters → LDS (once per persistent workgroup).  W1 is most of them: all of this
    // thread's loads are issued before the first LDS store, so the L2 latency is paid once
    {
        constexpr int NW1 = (L0 * L1 + kBlock - 1) / kBlock;
        float w1r[NW1];
#pragma unroll
        for (int q = 0; q < NW1; ++q) {
            const int e = tid + q * kBlock;
            w1r[q] = e < L0 * L1 ? mlp[S::OW1 + e] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < NW1; ++q) {
            const int e = tid + q * kBlock;
            if (e < L0 * L1) wl[S::SW1 + (e / L1) * S::LW1 + e % L1] = w1r[q];
        }
    }
    for (int e = tid; e < L1 * L2; e += kBlock) wl[S::SW2 + (e / L2) * S::LW2 + e % L2] = mlp[S::OW2 + e];
    for (int e = tid; e < L2 * L3; e += kBlock) wl[S::SW3 + (e / L3) * S::LW3 + e % L3] = mlp[S::OW3 + e];
    for (int e = tid; e < L1; e += kBlock) wl[S::SB1 + e] = mlp[S::OB1 + e];
    for (int e = tid; e < L2; e += kBlock) wl[S::SB2 + e] = mlp[S::OB2 + e];
    for (int e = tid; e < L3; e += kBlock) wl[S::SB3 + e] = mlp[S::OB3 + e];
    for (int e = tid; e < G + L3 + 1; e += kBlock) wl[S::SWO + e] = mlp[S::OWO + e];
    __syncthreads();

    const int64_t niter = (n + 127) / 128;
    int itl = -1;
    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        // lane coordinates re-derived opaquely every tile: keeps the compiler from hoisting the
        // hundreds of lane-dependent LDS addresses out of the loop (and spilling them)
        int lane_t = lane;
        asm volatile("" : "+v"(lane_t));
        const int j = lane_t & 31, h = lane_t >> 5;
        ++itl;
        NCF_T(0);
        const int64_t si = it * 128 + 32 * w + j;
        const bool inb = si < n;
        int u = 0, v = 0;
        float y = 0.f;
        if (inb) {
            u = users[si];
            v = items[si];
            y = labels[si];
        }
        // Masked samples read row 0 (a valid address) and get dz = 0: they contribute nothing.
        const bool ok = inb && (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
        const int urow = ok ? u : 0, irow = ok ? ids.ibase + v : 0;
        // user-row folding: fmatch = this sample's user row joins its group head's sum; the head
        // writes the sum, a sample with another user (any batch stays exact) its own row
        constexpr int fm = FOLD > 1 ? FOLD - 1 : 0;
        const int uhead = FOLD > 1 ? __shfl(u, lane_t - (j & fm), 64) : u;
        const bool fmatch = FOLD > 1 && inb && u == uhead;
        const bool fhead = (j & fm) == 0;
        const bool ustore = inb && (fhead || !fmatch);
        if (h == 0) {
            srow[32 * w + j] = ok ? urow : -1;
            srow[128 + 32 * w + j] = ok ? irow : -1;
        }
        const float* eu = emb + (size_t)urow * W;
        const float* ei = emb + (size_t)irow * W;
        float* sb = stg + w * S::RB * LS;  // this wave's staging block

        // ---- bulk gather: this half's MLP vector and both GMF slices, all loads in flight at once
        float4 xv[D0 / 4];
        {
            const float4* src = reinterpret_cast<const float4*>((h ? ei : eu) + G);
#pragma unroll
            for (int q = 0; q < D0 / 4; ++q) xv[q] = src[q];
        }
        float zp = 0.f;
        const float4* us = reinterpret_cast<const float4*>(eu + h * S::GH);
        const float4* is = reinterpret_cast<const float4*>(ei + h * S::GH);
        if constexpr (G > 0) {
            float4 ua[S::GH / 4], ia[S::GH / 4];
#pragma unroll
            for (int q = 0; q < S::GH / 4; ++q) {
                ua[q] = us[q];
                ia[q] = is[q];
            }
            const float* wo = wl + S::SWO + h * S::GH;
#pragma unroll
            for (int q = 0; q < S::GH / 4; ++q)
                zp += wo[4 * q] * (ua[q].x * ia[q].x) + wo[4 * q + 1] * (ua[q].y * ia[q].y) +
                      wo[4 * q + 2] * (ua[q].z * ia[q].z) + wo[4 * q + 3] * (ua[q].w * ia[q].w);
        }

        NCF_T(1);
        // ---- forward chain.  Layer 1: B operand = this half's MLP vector (K order h*D0 + s),
        // A operand = W1[k][out] from LDS, double-buffered 4 steps ahead.  Each activation tile
        // is staged to LDS for the weight-gradient phase as soon as it exists; only its ReLU
        // mask (one bit per register) is kept for the backward chain.
        uint32_t m1[S::NT1], m2[S::NT2];
        f32x16 h1[S::NT1];
        {
            f32x16 acc[S::NT1];
#pragma unroll
            for (int to = 0; to < S::NT1; ++to) acc[to] = f32x16{};
            float ab[2][4][S::NT1];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int to = 0; to < S::NT1; ++to) {
                    const int oc = 32 * to + j;
                    ab[0][e][to] = oc < L1 ? wl[S::SW1 + (h * D0 + e) * S::LW1 + oc] : 0.f;
                }
#pragma unroll
            for (int c = 0; c < D0 / 4; ++c) {
                if (c + 1 < D0 / 4) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int to = 0; to < S::NT1; ++to) {
                            const int oc = 32 * to + j;
                            ab[(c + 1) & 1][e][to] =
                                oc < L1 ? wl[S::SW1 + (h * D0 + 4 * (c + 1) + e) * S::LW1 + oc] : 0.f;
                        }
                }
                NCF_SB();
                const float xs[4] = {xv[c].x, xv[c].y, xv[c].z, xv[c].w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int to = 0; to < S::NT1; ++to) acc[to] = mfma32(ab[c & 1][e][to], xs[e], acc[to]);
                NCF_SB();
            }
#pragma unroll
            for (int to = 0; to < S::NT1; ++to) {
                m1[to] = 0u;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int f = 32 * to + drow(r, h);
                    const float val = (f < L1) ? fmaxf(acc[to][r] + wl[S::SB1 + f], 0.f) : 0.f;
                    h1[to][r] = val;
                    m1[to] |= (val > 0.f ? 1u : 0u) << r;
                    sb[(S::RH1 + f) * LS + j] = val;
                }
            }
        }
        NCF_T(2);
        // GMF slices again for the backward (L2-resident by now; in flight during layers 2-3)
        float4 ua[S::GH / 4 > 0 ? S::GH / 4 : 1], ia[S::GH / 4 > 0 ? S::GH / 4 : 1];
        if constexpr (G > 0) {
#pragma unroll
            for (int q = 0; q < S::GH / 4; ++q) {
                ua[q] = us[q];
                ia[q] = is[q];
            }
        }
        f32x16 h2[S::NT2];
#pragma unroll
        for (int to = 0; to < S::NT2; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS1, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L2 && k < L1) ? wl[S::SW2 + k * S::LW2 + oc] : 0.f;
                },
                [&](int t) { return h1[t / 16][t % 16]; });
            m2[to] = 0u;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * to + drow(r, h);
                const float val = (f < L2) ? fmaxf(acc[r] + wl[S::SB2 + f], 0.f) : 0.f;
                h2[to][r] = val;
                m2[to] |= (val > 0.f ? 1u : 0u) << r;
                sb[(S::RH2 + f) * LS + j] = val;
            }
        }
        f32x16 h3[S::NT3];
#pragma unroll
        for (int to = 0; to < S::NT3; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS2, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L3 && k < L2) ? wl[S::SW3 + k * S::LW3 + oc] : 0.f;
                },
                [&](int t) { return h2[t / 16][t % 16]; });
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * to + drow(r, h);
                h3[to][r] = (f < L3) ? fmaxf(acc[r] + wl[S::SB3 + f], 0.f) : 0.f;
            }
        }
        NCF_T(3);
        // ---- output, BCE, dz (both halves compute the same sample's values)
#pragma unroll
        for (int t = 0; t < S::NT3; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * t + drow(r, h);
                if (f < L3) zp += wl[S::SWO + G + f] * h3[t][r];
            }
        const float z = (zp + __shfl_xor(zp, 32, 64)) + wl[S::SBO];
        const float p = 1.0f / (1.0f + expf(-z));
        float dz = 0.f, bce = 0.f;
        if (ok) {
            const float pc = fminf(fmaxf(p, eps), hi_clip);
            const float logit = logf(pc / (1.0f - pc));
            bce = fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
            dz = (p >= eps && p <= hi_clip) ? (p - y) * inv_batch : 0.0f;
        }
        if (h == 0) {
            if (inb) probs[si] = ok ? p : __int_as_float(0x7fc00000);
            acc_bce += bce;
            acc_dbo += dz;
        }
        // ---- hr@k / dcg@k of the user groups in this block (RankLayer + _get_hits_per_user,
        // model.py:344-455): label = first max of y; position = #(p > p_lab) + #(earlier ties)
        if (metrics) {
            const int e = j % group;
            const int base = 32 * h + j - e;
            int lab = 0;
            float best = __shfl(y, base, 64);
            for (int q = 1; q < group; ++q) {
                const float yq = __shfl(y, base + q, 64);
                if (yq > best) { best = yq; lab = q; }
            }
            const float pl = __shfl(p, base + lab, 64);
            int pos = 0;
            for (int q = 0; q < group; ++q) {
                const float pq = __shfl(p, base + q, 64);
                pos += (pq > pl) || (pq == pl && q < lab);
            }
            if (h == 0 && e == 0 && inb) {
                const float hit = pos < topk ? 1.f : 0.f;
                acc_hit += hit;
                acc_dcg += hit * (logf(2.0f) / logf((float)pos + 2.0f));
            }
        }
        NCF_T(4);
        float* gu = gs + (size_t)(2 * si) * W;  // user contribution row
        float* gi = gu + W;                     // item contribution row

        // ---- GMF backward: embedding grads + output-kernel grads (transpose-reduced)
        if constexpr (G > 0) {
            const float* wo = wl + S::SWO + h * S::GH;
#pragma unroll
            for (int c = 0; c < S::NGC; ++c) {
                float contrib[S::GCH];
#pragma unroll
                for (int q = 0; q < S::GCH / 4; ++q) {
                    const int f = c * S::GCH + 4 * q;
                    const float4 a = ua[f / 4], b = ia[f / 4];
                    contrib[4 * q] = dz * (a.x * b.x);
                    contrib[4 * q + 1] = dz * (a.y * b.y);
                    contrib[4 * q + 2] = dz * (a.z * b.z);
                    contrib[4 * q + 3] = dz * (a.w * b.w);
                    float4 gu4 = make_float4(dz * wo[f] * b.x, dz * wo[f + 1] * b.y, dz * wo[f + 2] * b.z,
                                             dz * wo[f + 3] * b.w);
                    if constexpr (FOLD > 1) {
                        const float4 s = make_float4(fold_sum<FOLD>(fmatch ? gu4.x : 0.f),
                                                     fold_sum<FOLD>(fmatch ? gu4.y : 0.f),
                                                     fold_sum<FOLD>(fmatch ? gu4.z : 0.f),
                                                     fold_sum<FOLD>(fmatch ? gu4.w : 0.f));
                        if (fhead) gu4 = s;
                    }
                    // masked samples (dz = 0) write zero rows: the index may count their other, valid id
                    if (ustore) st_stream(reinterpret_cast<float4*>(gu + h * S::GH + f), gu4);
                    if (inb) {
                        const float4 gi4 = make_float4(dz * wo[f] * a.x, dz * wo[f + 1] * a.y, dz * wo[f + 2] * a.z,
                                                       dz * wo[f + 3] * a.w);
                        st_stream(reinterpret_cast<float4*>(gi + h * S::GH + f), gi4);
                    }
                }
#pragma unroll
                for (int q = 0; q < S::GCH; ++q) acc_gmf_l[c * S::GCH + q] += contrib[q];
            }
        }
        NCF_T(5);
        // ---- output-kernel grads of the MLP features, and G3
        f32x16 g3[S::NT3];
#pragma unroll
        for (int t = 0; t < S::NT3; ++t) {
            float contrib[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * t + drow(r, h);
                contrib[r] = dz * h3[t][r];
                const float g = (f < L3 && h3[t][r] > 0.f) ? dz * wl[S::SWO + G + f] : 0.f;
                g3[t][r] = g;
                if (f < L3) sb[(S::RG3 + f) * LS + j] = g;
            }
            if (t == 0) {  // NT3 == 1 for the supported shapes
#pragma unroll
                for (int r = 0; r < 16; ++r) acc_h3_l[r] += contrib[r];
            }
        }
        // ---- backward data chain (A = W_l[in][out] read along `in`: row stride out+1)
        f32x16 g2[S::NT2];
#pragma unroll
        for (int to = 0; to < S::NT2; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS3, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L2 && k < L3) ? wl[S::SW3 + oc * S::LW3 + k] : 0.f;
                },
                [&](int t) { return g3[t / 16][t % 16]; });
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float g = ((m2[to] >> r) & 1u) ? acc[r] : 0.f;
                g2[to][r] = g;
                sb[(S::RG2 + 32 * to + drow(r, h)) * LS + j] = g;
            }
        }
        NCF_T(6);
        f32x16 g1[S::NT1];
#pragma unroll
        for (int to = 0; to < S::NT1; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS2, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L1 && k < L2) ? wl[S::SW2 + oc * S::LW2 + k] : 0.f;
                },
                [&](int t) { return g2[t / 16][t % 16]; });
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float g = ((m1[to] >> r) & 1u) ? acc[r] : 0.f;
                g1[to][r] = g;
                sb[(S::RG1 + 32 * to + drow(r, h)) * LS + j] = g;
            }
        }
        NCF_T(7);
#pragma unroll
        for (int to = 0; to < S::NT0; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS1, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L0 && k < L1) ? wl[S::SW1 + oc * S::LW1 + k] : 0.f;
                },
                [&](int t) { return g1[t / 16][t % 16]; });
            f32x16 dx = acc;
            if constexpr (FOLD > 1) if (32 * to < D0) {  // user-half rows: folded like the GMF part
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float s = fold_sum<FOLD>(fmatch ? acc[r] : 0.f);
                    if (fhead && 32 * to + drow(r, h) < D0) dx[r] = s;
                }
            }
            // masked samples (dz = 0) write zero rows: the index may count their other, valid id
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int f = 32 * to + 8 * q + 4 * h;  // rows drow(4q..4q+3, h) are f..f+3
                if (f < L0 && (f < D0 ? ustore : inb)) {
                    float* dst = (f < D0) ? gu + G + f : gi + G + (f - D0);
                    st_stream(reinterpret_cast<float4*>(dst),
                              make_float4(dx[4 * q], dx[4 * q + 1], dx[4 * q + 2], dx[4 * q + 3]));
                }
            }
        }
        NCF_T(8);
        __syncthreads();
        NCF_T(9);

        // ---- weight gradients: wave w owns tiles dw_tile(w, m) (K = 128 samples, 64 MFMA
        // steps per tile; both operands double-buffered one chunk ahead)
#if NCF_DW1_SHARED
        // the NT1 output tiles of an input-feature group in one chain: each gathered-row value
        // (the A operand, re-read from L2/HBM) is fetched once for all of them
        if constexpr (S::NSLOT1 > 0) {
#pragma unroll
            for (int g = 0; g < S::NSLOT1 / S::NT1; ++g) {
                const int ti = w + 4 * g;
                const int fi = 32 * ti + j;
                const int side = fi < D0 ? 0 : 128;
                const int col = G + (fi < D0 ? fi : fi - D0);
                const bool aok = fi < L0;
                // Unconditional loads, unmasked: a masked sample (row -1) reads row 0, but its G1
                // column (the B operand) is exactly zero; lanes past L0 feed only dW1 rows that are
                // never written.  (A load under a branch, or a select on its value right after the
                // load, makes the compiler wait for all outstanding loads before the next chunk.)
                const int colc = aok ? col : 0;
                auto lda = [&](int tt) {
                    const int row = srow[side + 32 * (tt >> 4) + 2 * (tt & 15) + h];
                    return emb[(size_t)(row < 0 ? 0 : row) * W + colc];
                };
                auto ldb = [&](int tt, int o) {
                    const int fo = 32 * o + j;
                    return fo < L1 ? stg[(tt >> 4) * S::RB * LS + (S::RG1 + fo) * LS + 2 * (tt & 15) + h] : 0.f;
                };
                constexpr int CH = NCF_DW1_CH;
                float ab[2][CH], bb[2][CH][S::NT1];
#pragma unroll
                for (int e = 0; e < CH; ++e) {
                    ab[0][e] = lda(e);
#pragma unroll
                    for (int o = 0; o < S::NT1; ++o) bb[0][e][o] = ldb(e, o);
                }
#pragma unroll
                for (int c = 0; c < 64 / CH; ++c) {
                    if (c + 1 < 64 / CH) {
#pragma unroll
                        for (int e = 0; e < CH; ++e) {
                            ab[(c + 1) & 1][e] = lda(CH * (c + 1) + e);
#pragma unroll
                            for (int o = 0; o < S::NT1; ++o) bb[(c + 1) & 1][e][o] = ldb(CH * (c + 1) + e, o);
                        }
                    }
                    NCF_SB();
#pragma unroll
                    for (int e = 0; e < CH; ++e)
#pragma unroll
                        for (int o = 0; o < S::NT1; ++o)
                            dwacc[g * S::NT1 + o] = mfma32(ab[c & 1][e], bb[c & 1][e][o], dwacc[g * S::NT1 + o]);
                    NCF_SB();
                }
            }
        }
#endif
#pragma unroll
        for (int m = 0; m < S::MAXT; ++m) {
            const int t = S::dw_tile(w, m);
            if (t < 0) continue;
#if NCF_DW1_SHARED
            if (m < S::NSLOT1) continue;
#endif
            int layer, ti, to;
            if (t < S::NDW1) { layer = 1; ti = t / S::NT1; to = t % S::NT1; }
            else if (t < S::NDW1 + S::NDW2) { layer = 2; ti = (t - S::NDW1) / S::NT2; to = (t - S::NDW1) % S::NT2; }
            else { layer = 3; ti = (t - S::NDW1 - S::NDW2) / S::NT3; to = (t - S::NDW1 - S::NDW2) % S::NT3; }
            const int fi = 32 * ti + j;  // A row (input feature) supplied by this lane
            const int fo = 32 * to + j;  // B column (output feature) supplied by this lane
            const int lout = layer == 1 ? L1 : layer == 2 ? L2 : L3;
            const int brow = (layer == 1 ? S::RG1 : layer == 2 ? S::RG2 : S::RG3) + fo;
            const bool bok = fo < lout;
            // B(t): G_l[fo][sample] of block t/16, column 2(t%16)+h
            auto fb = [&](int tt) {
                return bok ? stg[(tt >> 4) * S::RB * LS + brow * LS + 2 * (tt & 15) + h] : 0.f;
            };
            if (layer == 1) {
                const int side = fi < D0 ? 0 : 128;
                const int col = G + (fi < D0 ? fi : fi - D0);
                const bool aok = fi < L0;
                const int colc = aok ? col : 0;  // see the shared chain above: no masks needed
                dwacc[m] = mchain2<64, NCF_DW1_CH>(dwacc[m],
                                           [&](int tt) {
                                               const int row = srow[side + 32 * (tt >> 4) + 2 * (tt & 15) + h];
                                               return emb[(size_t)(row < 0 ? 0 : row) * W + colc];
                                           },
                                           fb);
            } else {
                const int arow = (layer == 2 ? S::RH1 : S::RH2) + fi;
                dwacc[m] = mchain2<64, 8>(
                    dwacc[m], [&](int tt) { return stg[(tt >> 4) * S::RB * LS + arow * LS + 2 * (tt & 15) + h]; },
                    fb);
            }
        }
        NCF_T(10);
        // ---- bias gradients: one G row per thread, summed over the 128 samples
#pragma unroll
        for (int q = 0; q < NBR; ++q) {
            const int br = BW0 ? (tid & 63) + 64 * q : tid;
            if ((!BW0 || w == 0) && br < NB) {
                const int rr = br < L1 ? S::RG1 + br : br < L1 + L2 ? S::RG2 + (br - L1) : S::RG3 + (br - L1 - L2);
                float sacc = 0.f;
                for (int b = 0; b < 4; ++b) {
                    const float* bb = stg + b * S::RB * LS + rr * LS;
#pragma unroll
                    for (int c = 0; c < 32; ++c) sacc += bb[c];
                }
                acc_bias[q] += sacc;
            }
        }
        NCF_T(11);
        __syncthreads();
        NCF_T(12);
    }

    // ---- epilogue: this workgroup's dense-gradient slab and BCE partial
    float* slab = slabs + (size_t)blockIdx.x * S::P;
#pragma unroll
    for (int m = 0; m < S::MAXT; ++m) {
        const int t = S::dw_tile(w, m);
        if (t < 0) continue;
        int off, lin, lout, ti, to;
        if (t < S::NDW1) { off = S::OW1; lin = L0; lout = L1; ti = t / S::NT1; to = t % S::NT1; }
        else if (t < S::NDW1 + S::NDW2) {
            off = S::OW2; lin = L1; lout = L2; ti = (t - S::NDW1) / S::NT2; to = (t - S::NDW1) % S::NT2;
        } else {
            off = S::OW3; lin = L2; lout = L3; ti = (t - S::NDW1 - S::NDW2) / S::NT3;
            to = (t - S::NDW1 - S::NDW2) % S::NT3;
        }
        const int oc = 32 * to + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ir = 32 * ti + drow(r, h);
            if (ir < lin && oc < lout) slab[off + ir * lout + oc] = dwacc[m][r];
        }
    }
#pragma unroll
    for (int q = 0; q < NBR; ++q) {
        const int br = BW0 ? (tid & 63) + 64 * q : tid;
        if (!BW0 || w == 0) {
            if (br < L1) slab[S::OB1 + br] = acc_bias[q];
            else if (br < L1 + L2) slab[S::OB2 + (br - L1)] = acc_bias[q];
            else if (br < NB) slab[S::OB3 + (br - L1 - L2)] = acc_bias[q];
        }
    }

    // output layer: reduce the per-lane partials across each wave half, then combine the 4
    // waves in fixed order through LDS
    float acc_gmf[S::NGC > 0 ? S::NGC : 1];
    if constexpr (G > 0) {
#pragma unroll
        for (int c = 0; c < S::NGC; ++c) acc_gmf[c] = half_transpose_reduce<S::GCH>(acc_gmf_l + c * S::GCH, lane);
    }
    acc_h3 = half_transpose_reduce<16>(acc_h3_l, lane);
    float* xw = xch + w * S::XCH;
    if constexpr (G > 0) {
#pragma unroll
        for (int c = 0; c < S::NGC; ++c) {
            constexpr int sh = 5 - ilog2(S::GCH);
            if ((j & ((1 << sh) - 1)) == 0) xw[h * S::GH + c * S::GCH + (j >> sh)] = acc_gmf[c];
        }
    }
    if ((j & 1) == 0) {
        const int f = drow(j >> 1, h);
        if (f < L3) xw[G + f] = acc_h3;
    }
    float dbo = acc_dbo, bce = acc_bce, hit = acc_hit, dcg = acc_dcg;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        dbo += __shfl_xor(dbo, m, 64);
        bce += __shfl_xor(bce, m, 64);
        hit += __shfl_xor(hit, m, 64);
        dcg += __shfl_xor(dcg, m, 64);
    }
    if (lane == 0) {
        xw[G + L3] = dbo;
        xw[G + L3 + 1] = bce;
        xw[G + L3 + 2] = hit;
        xw[G + L3 + 3] = dcg;
    }
    __syncthreads();
    if (tid < G + L3 + 1) {
        const float v = (xch[tid] + xch[S::XCH + tid]) + (xch[2 * S::XCH + tid] + xch[3 * S::XCH + tid]);
        slab[S::OWO + tid] = v;  // G + L3 kernel entries, then the bias at OBO = OWO + G + L3
    }
    if (tid < 3) {
        const int o = G + L3 + 1 + tid;
        const float v = (xch[o] + xch[S::XCH + o]) + (xch[2 * S::XCH + o] + xch[3 * S::XCH + o]);
        if (tid == 0) part_bce[blockIdx.x] = v;
        else if (metrics) (tid == 1 ? part_hit : part_dcg)[blockIdx.x] = v;
    }
}

// ---------------------------------------------------------------------------
// Forward only (ncf_predict / ncf_evaluate: Model.predict_on_batch output[0], the validation
// pass of fit_generator, model.py:184-194, 329-333): the forward chain of k_fb_fused with no
// staging, no masks and no backward.  LDS holds the dense weights only (WLDS floats), so two
// workgroups share a CU; 128-sample tiles, persistent grid.  With labels: one Keras-BCE partial
// per workgroup (fixed order: wave sums, then the 4 waves in order).

template <class S>
__global__ __launch_bounds__(kBlock, 2) void k_fwd_fused(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                         const int32_t* __restrict__ users,
                                                         const int32_t* __restrict__ items,
                                                         const float* __restrict__ labels, int64_t n, IdSpace ids,
                                                         float* __restrict__ probs, float* __restrict__ part_bce) {
    constexpr int L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, D0 = S::D0, W = S::W;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wl = lds;
    __shared__ float red[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float eps = 1e-7f, hi_clip = 1.0f - eps;
    // dense parameters -> LDS: every float4 group of the flat layout loaded first (one b128 buffer
    // load each, all in flight together; every segment starts at a multiple of 4 floats), then
    // stored element by element into the padded rows
    static_assert(S::OB1 % 4 == 0 && S::OW2 % 4 == 0 && S::OB2 % 4 == 0 && S::OW3 % 4 == 0 && S::OB3 % 4 == 0 &&
                      S::OWO % 4 == 0 && S::OBO % 4 == 0,
                  "float4 parameter groups");
    {
        constexpr int NV4 = S::OBO / 4, NVT = (NV4 + kBlock - 1) / kBlock;
        const __amdgpu_buffer_rsrc_t ml_rsrc =
            __builtin_amdgcn_make_buffer_rsrc((void*)mlp, (short)0, (int)(S::P * 4), 0x00020000);
        typedef float f4v __attribute__((ext_vector_type(4)));
        f4v pv[NVT];
#pragma unroll
        for (int j = 0; j < NVT; ++j) {
            const int q = tid + kBlock * j;
            pv[j] = __builtin_bit_cast(
                f4v, __builtin_amdgcn_raw_buffer_load_b128(ml_rsrc, q < NV4 ? (uint32_t)q * 16u : 0x80000000u, 0, 0));
        }
        const float pbo = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ml_rsrc, (uint32_t)S::OBO * 4u, 0, 0));
#pragma unroll
        for (int j = 0; j < NVT; ++j) {
            const int q = tid + kBlock * j;
            if (q < NV4) {
                const int e0 = 4 * q;
                int d;  // LDS position of element e0 (its 3 successors follow it in the same row)
                if (e0 < S::OB1) d = S::SW1 + (e0 / L1) * S::LW1 + e0 % L1;
                else if (e0 < S::OW2) d = S::SB1 + (e0 - S::OB1);
                else if (e0 < S::OB2) d = S::SW2 + ((e0 - S::OW2) / L2) * S::LW2 + (e0 - S::OW2) % L2;
                else if (e0 < S::OW3) d = S::SB2 + (e0 - S::OB2);
                else if (e0 < S::OB3) d = S::SW3 + ((e0 - S::OW3) / L3) * S::LW3 + (e0 - S::OW3) % L3;
                else if (e0 < S::OWO) d = S::SB3 + (e0 - S::OB3);
                else d = S::SWO + (e0 - S::OWO);
#pragma unroll
                for (int k = 0; k < 4; ++k) wl[d + k] = pv[j][k];
            }
        }
        if (tid == 0) wl[S::SWO + G + L3] = pbo;
    }
    __syncthreads();

    float acc_bce = 0.f;
    const int64_t niter = (n + 127) / 128;
    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        int lane_t = lane;
        asm volatile("" : "+v"(lane_t));
        const int j = lane_t & 31, h = lane_t >> 5;
        const int64_t si = it * 128 + 32 * w + j;
        const bool inb = si < n;
        int u = 0, v = 0;
        if (inb) {
            u = users[si];
            v = items[si];
        }
        const bool ok = inb && (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
        const float* eu = emb + (size_t)(ok ? u : 0) * W;
        const float* ei = emb + (size_t)(ok ? ids.ibase + v : 0) * W;
        float4 xv[D0 / 4];
        {
            const float4* src = reinterpret_cast<const float4*>((h ? ei : eu) + G);
#pragma unroll
            for (int q = 0; q < D0 / 4; ++q) xv[q] = src[q];
        }
        float zp = 0.f;
        if constexpr (G > 0) {
            const float4* us = reinterpret_cast<const float4*>(eu + h * S::GH);
            const float4* is = reinterpret_cast<const float4*>(ei + h * S::GH);
            const float* wo = wl + S::SWO + h * S::GH;
#pragma unroll
            for (int q = 0; q < S::GH / 4; ++q) {
                const float4 a = us[q], b = is[q];
                zp += wo[4 * q] * (a.x * b.x) + wo[4 * q + 1] * (a.y * b.y) + wo[4 * q + 2] * (a.z * b.z) +
                      wo[4 * q + 3] * (a.w * b.w);
            }
        }
        // layer 1 (A = W1[k][out] from LDS, B = the gathered MLP vector, K order h*D0 + s)
        f32x16 h1[S::NT1];
        {
            f32x16 acc[S::NT1];
#pragma unroll
            for (int to = 0; to < S::NT1; ++to) acc[to] = f32x16{};
            float ab[2][4][S::NT1];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int to = 0; to < S::NT1; ++to) {
                    const int oc = 32 * to + j;
                    ab[0][e][to] = oc < L1 ? wl[S::SW1 + (h * D0 + e) * S::LW1 + oc] : 0.f;
                }
#pragma unroll
            for (int c = 0; c < D0 / 4; ++c) {
                if (c + 1 < D0 / 4) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int to = 0; to < S::NT1; ++to) {
                            const int oc = 32 * to + j;
                            ab[(c + 1) & 1][e][to] =
                                oc < L1 ? wl[S::SW1 + (h * D0 + 4 * (c + 1) + e) * S::LW1 + oc] : 0.f;
                        }
                }
                NCF_SB();
                const float xs[4] = {xv[c].x, xv[c].y, xv[c].z, xv[c].w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int to = 0; to < S::NT1; ++to) acc[to] = mfma32(ab[c & 1][e][to], xs[e], acc[to]);
                NCF_SB();
            }
#pragma unroll
            for (int to = 0; to < S::NT1; ++to)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int f = 32 * to + drow(r, h);
                    h1[to][r] = (f < L1) ? fmaxf(acc[to][r] + wl[S::SB1 + f], 0.f) : 0.f;
                }
        }
        f32x16 h2[S::NT2];
#pragma unroll
        for (int to = 0; to < S::NT2; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS1, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L2 && k < L1) ? wl[S::SW2 + k * S::LW2 + oc] : 0.f;
                },
                [&](int t) { return h1[t / 16][t % 16]; });
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * to + drow(r, h);
                h2[to][r] = (f < L2) ? fmaxf(acc[r] + wl[S::SB2 + f], 0.f) : 0.f;
            }
        }
#pragma unroll
        for (int to = 0; to < S::NT3; ++to) {
            const int oc = 32 * to + j;
            const f32x16 acc = mchain<S::NS2, 4>(
                f32x16{},
                [&](int t) {
                    const int k = 32 * (t / 16) + drow(t % 16, h);
                    return (oc < L3 && k < L2) ? wl[S::SW3 + k * S::LW3 + oc] : 0.f;
                },
                [&](int t) { return h2[t / 16][t % 16]; });
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * to + drow(r, h);
                if (f < L3) zp += wl[S::SWO + G + f] * fmaxf(acc[r] + wl[S::SB3 + f], 0.f);
            }
        }
        const float z = (zp + __shfl_xor(zp, 32, 64)) + wl[S::SBO];
        const float p = 1.0f / (1.0f + expf(-z));
        if (h == 0 && inb) {
            probs[si] = ok ? p : __int_as_float(0x7fc00000);
            if (labels && ok) {
                const float y = labels[si];
                const float pc = fminf(fmaxf(p, eps), hi_clip);
                const float logit = logf(pc / (1.0f - pc));
                acc_bce += fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
            }
        }
    }
    if (part_bce) {
        const float b = block_sum_256(acc_bce, red);
        if (tid == 0) part_bce[blockIdx.x] = b;
    }
}

// ---------------------------------------------------------------------------

using ShapeC = FShape<128, 64, 32, 16, 64>;   // ml-20m NeuMF (config C)
using ShapeB = FShape<64, 32, 16, 8, 8>;      // ml-1m NeuMF (config B)
using ShapeR = FShape<64, 32, 16, 8, 0>;      // reference trainer default (MLP-only)
using ShapeC0 = FShape<128, 64, 32, 16, 0>;

template <class S>
static bool matches(const ncf_shape_t& s) {
    return s.num_layers == 4 && s.layers[0] == S::L0 && s.layers[1] == S::L1 && s.layers[2] == S::L2 &&
           s.layers[3] == S::L3 && s.gmf_dim == S::G && s.row_width == S::W && s.gmf_stride == S::G;
}

bool fused_supported(const ncf_shape_t& s) {
    return matches<ShapeC>(s) || matches<ShapeB>(s) || matches<ShapeR>(s) || matches<ShapeC0>(s);
}

template <class S>
static hipError_t launch_one(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                             const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                             float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                             hipStream_t st, int fold) {
    static bool configured = false;
    if (!configured) {
        for (const void* k : {(const void*)k_fb_fused<S, 0>, (const void*)k_fb_fused<S, 2>,
                              (const void*)k_fb_fused<S, 4>, (const void*)k_fb_fused<S, 8>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)S::LDS_BYTES);
            if (e != hipSuccess) return e;
        }
        configured = true;
    }
    const int64_t niter = (n + 127) / 128;
    int grid = (int)(niter < 256 ? niter : 256);
    if (grid > kMaxSlabs) grid = kMaxSlabs;
    const bool in_kernel = group > 0 && group <= 32 && 32 % group == 0;
    auto go = [&](auto kern) {
        launch(kern, grid, kBlock, S::LDS_BYTES, st, emb, mlp, users, items, labels, n, ids, inv_batch,
               at<float>(ws, L.probs), at<float>(ws, L.gs), at<float>(ws, L.slabs), at<float>(ws, L.part_bce), group,
               topk, in_kernel ? at<float>(ws, L.part_hit) : nullptr, in_kernel ? at<float>(ws, L.part_dcg) : nullptr);
    };
    switch (fold) {
        case 0: go(k_fb_fused<S, 0>); break;
        case 2: go(k_fb_fused<S, 2>); break;
        case 4: go(k_fb_fused<S, 4>); break;
        case 8: go(k_fb_fused<S, 8>); break;
        default: return hipErrorInvalidValue;
    }
    *nslab = grid;
    *nbce = grid;
    *nmet = in_kernel ? grid : 0;
    return hipGetLastError();
}

hipError_t launch_fb_fused(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                           const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                           float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                           hipStream_t st, int fold) {
    // the lanes of a fold group are consecutive samples of one 32-sample block
    if (fold != 0 && (fold < 2 || fold > 8 || (fold & (fold - 1)) != 0 || n % fold != 0)) return hipErrorInvalidValue;
#define NCF_TRY(SH)                                                                                             \
    if (matches<SH>(s))                                                                                         \
    return launch_one<SH>(s, L, ws, emb, mlp, users, items, labels, n, inv_batch, ids, group, topk, nslab, nbce, \
                          nmet, st, fold)
    NCF_TRY(ShapeC);
    NCF_TRY(ShapeB);
    NCF_TRY(ShapeR);
    NCF_TRY(ShapeC0);
#undef NCF_TRY
    return hipErrorNotSupported;
}

template <class S>
static hipError_t launch_fwd_one(const float* emb, const float* mlp, const int32_t* users, const int32_t* items,
                                 const float* labels, int64_t n, IdSpace ids, float* probs, float* part_bce,
                                 int* nbce, hipStream_t st) {
    const int64_t niter = (n + 127) / 128;
    int grid = (int)(niter < 512 ? niter : 512);  // two workgroups per CU, persistent
    if (grid > kMaxSlabs) grid = kMaxSlabs;
    launch(k_fwd_fused<S>, grid, kBlock, (size_t)S::WLDS * 4, st, emb, mlp, users, items, labels, n, ids, probs,
           labels ? part_bce : nullptr);
    *nbce = labels ? grid : 0;
    return hipGetLastError();
}

hipError_t launch_fwd_fused(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                            const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                            float* probs, IdSpace ids, int* nbce, hipStream_t st) {
    float* part = at<float>(ws, L.part_bce);
#define NCF_TRY(SH) \
    if (matches<SH>(s)) return launch_fwd_one<SH>(emb, mlp, users, items, labels, n, ids, probs, part, nbce, st)
    NCF_TRY(ShapeC);
    NCF_TRY(ShapeB);
    NCF_TRY(ShapeR);
    NCF_TRY(ShapeC0);
#undef NCF_TRY
    return hipErrorNotSupported;
}

}  // namespace ncf

#ifdef NCF_FUSED_TIMING
extern "C" int ncf_debug_fused_timing(unsigned long long* out, size_t count) {
    size_t n = count < sizeof(ncf::g_fused_t) / 8 ? count : sizeof(ncf::g_fused_t) / 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(ncf::g_fused_t), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif
