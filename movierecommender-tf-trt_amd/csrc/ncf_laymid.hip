// The layers after the first of the layer-by-layer path (config D: 128 -> 64 -> 32 -> output,
// GMF 128) fused into one hand-written fp32 MFMA kernel.
//
// rocBLAS ran them as six GEMMs plus bias/ReLU, output/BCE, G_{n-1}, ReLU-mask and six GEMV passes
// over the batch (profiles/r03_d: ~255 us of the 0.49 ms forward/backward per 65,536-sample step),
// every activation and gradient through HBM.  Here W2 (32 KB), W3 (8 KB) and the output layer sit
// in LDS once per workgroup in the wave kernel's operand layout (ncf_wave.hip) and each wave runs
// its own 16-sample units through the whole middle of the chain, the activations in registers:
//
//   in:   H1 = relu(W1^T x + b1) [n x 128] (k_lay_l1f's output) and the two rows' GMF vectors
//   fwd:  H2 = relu(W2^T H1 + b2), H3 = relu(W3^T H2 + b3) as 16 x 16 tiles [feature][sample]
//         (a layer's output registers are the next layer's B operand), z = w_out . [GMF | H3] +
//         b_out, Keras-clipped BCE, dz = (p - y) / B (model.py:175-188, 213-214)
//   bwd:  G3 = dz w3 * relu'(H3); G2 = (W3 G3) * relu'(H2); G1 = (W2 G2) * relu'(H1) -> HBM (for
//         k_lay_l1b and the dW1 GEMM); dz -> HBM (k_lay_l1b's GMF part)
//   dW:   dW2 += H1^T G2, dW3 += H2^T G3 over the unit's samples (K = 16: the wave writes H1, H2,
//         G2, G3 transposed into its own LDS buffers and reads them back as operands), bias and
//         output-layer sums and db1 = sum of G1; per workgroup one slab of these parameters (the
//         dW1 region of the slab is the rocBLAS chunk GEMM's: one chunk per workgroup)
//
// Same outputs as the replaced launches (probs, dz, G1, BCE partials, the slabs' parameters after
// layer 1), fixed summation order, no atomics.

#include <cmath>
#include <cstdlib>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
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
    } else {
        static_assert(NB == 2, "vector width");
        const f32x2 x = *reinterpret_cast<const f32x2*>(p);
        o[0] = x[0], o[1] = x[1];
    }
}
template <int NB>
__device__ __forceinline__ void stsv(float* p, const float (&v)[NB]) {
    if constexpr (NB == 8) {
        *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else if constexpr (NB == 4) {
        *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
        static_assert(NB == 2, "vector width");
        *reinterpret_cast<f32x2*>(p) = f32x2{v[0], v[1]};
    }
}

// sum over the 16 sample lanes of a lane group (DPP row rotations); every lane gets the sum
__device__ __forceinline__ float row_sum(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));
    return x;
}
// sum over the 4 lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48), (g0 + g1) + (g2 + g3) in every lane
__device__ __forceinline__ float group_allsum(float x) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <int L1_, int L2_, int L3_, int G_>
struct MShape {
    static constexpr int L1 = L1_, L2 = L2_, L3 = L3_, G = G_;
    static constexpr int B1 = L1 / 16, B2 = L2 / 16, B3 = L3 / 16, GQ = G / 4;
    static_assert(B1 == 8 && B2 == 4 && B3 == 2 && G % 16 == 0, "middle-layer shape (config D)");
    // weights [in][pos], pos = (c mod 16) NB + c / 16, row strides 16 NB + 4
    static constexpr int S2 = 16 * B2 + 4, S3 = 16 * B3 + 4;
    static constexpr int SW2 = 0, SW3 = SW2 + L1 * S2, SB2 = SW3 + L2 * S3, SB3 = SB2 + L2, SWO = SB3 + L3,
                         SBO = SWO + G + L3, WLDS = (SBO + 1 + 3) / 4 * 4;
    // per-wave transposed buffers [sample][pos]
    static constexpr int T1 = 132, T2 = 16 * B2, T3 = 16 * B3;
    static constexpr int TH1 = 0, TH2 = TH1 + 16 * T1, TG2 = TH2 + 16 * T2, TG3 = TG2 + 16 * T2, WREG = TG3 + 16 * T3;
    static constexpr size_t LDS_BYTES = (size_t)(WLDS + 4 * WREG) * 4;
    static_assert(LDS_BYTES <= 163840, "LDS budget");
    // epilogue rows: NTR tiles at a time in the accumulator layout, then the sums
    static constexpr int NT2 = B1 * B2, NT = NT2 + B2 * B3, NTR = (NT + 1) / 2;
    static constexpr int RB2 = NTR * 256, RB3 = RB2 + L2, RWO = RB3 + L3, RBO = RWO + G + L3, RX = RBO + 1,
                         RB1 = RX + 1, PR = (RB1 + L1 + 3) / 4 * 4;
    static_assert((size_t)4 * PR * 4 <= LDS_BYTES, "epilogue rows");
};

struct MidArgs {
    const float* mlp;
    int off2, off3, offo;  // flat offsets of the hidden_2 / hidden_3 / output kernels
    int b1off;             // flat offset of b1
    const float* h1;
    const float* emb;  // the GMF vectors of the two rows (row width W)
    int W;
    const float* labels;
    const int32_t* users;
    const int32_t* items;
    int64_t n;
    IdSpace ids;
    float inv_batch;
    float* probs;
    float* dzo;
    float* g1;
    float* slabs;
    int P;
    float* part_bce;
};

// FWD: forward only (ncf_predict / ncf_evaluate): probabilities and, labels given, the BCE partial
// of the workgroup; no gradients
template <class S, bool FWD>
__global__ __launch_bounds__(256, 1) void k_lay_mid(MidArgs a) {
    constexpr int L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, B1 = S::B1, B2 = S::B2, B3 = S::B3, GQ = S::GQ;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wl = lds;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    float* tb = lds + S::WLDS + wv * S::WREG;
    const float eps = 1e-7f, hi_clip = 1.0f - eps;

    // ---- prologue: W2, W3 (operand layout), b2, b3, output kernel + bias into LDS; the loads of
    // each thread in one batch before its stores
    {
        constexpr int N2 = L1 * L2 / 4, N3 = L2 * L3 / 4, NV2 = (N2 + 255) / 256, NV3 = (N3 + 255) / 256;
        const float4* w2 = reinterpret_cast<const float4*>(a.mlp + a.off2);
        const float4* w3 = reinterpret_cast<const float4*>(a.mlp + a.off3);
        float4 v2[NV2], v3[NV3];
#pragma unroll
        for (int j = 0; j < NV2; ++j) {
            const int e = threadIdx.x + 256 * j;
            v2[j] = e < N2 ? w2[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < NV3; ++j) {
            const int e = threadIdx.x + 256 * j;
            v3[j] = e < N3 ? w3[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const float b2v = threadIdx.x < L2 ? a.mlp[a.off2 + L1 * L2 + threadIdx.x] : 0.f;
        const float b3v = threadIdx.x < L3 ? a.mlp[a.off3 + L2 * L3 + threadIdx.x] : 0.f;
        const float wov = threadIdx.x < G + L3 + 1 ? a.mlp[a.offo + threadIdx.x] : 0.f;
#pragma unroll
        for (int j = 0; j < NV2; ++j) {
            const int e = threadIdx.x + 256 * j;
            if (e < N2) {
                const int i = (4 * e) / L2, c0 = (4 * e) % L2;
                float* row = wl + S::SW2 + i * S::S2;
                row[((c0 + 0) & 15) * B2 + ((c0 + 0) >> 4)] = v2[j].x;
                row[((c0 + 1) & 15) * B2 + ((c0 + 1) >> 4)] = v2[j].y;
                row[((c0 + 2) & 15) * B2 + ((c0 + 2) >> 4)] = v2[j].z;
                row[((c0 + 3) & 15) * B2 + ((c0 + 3) >> 4)] = v2[j].w;
            }
        }
#pragma unroll
        for (int j = 0; j < NV3; ++j) {
            const int e = threadIdx.x + 256 * j;
            if (e < N3) {
                const int i = (4 * e) / L3, c0 = (4 * e) % L3;
                float* row = wl + S::SW3 + i * S::S3;
                row[((c0 + 0) & 15) * B3 + ((c0 + 0) >> 4)] = v3[j].x;
                row[((c0 + 1) & 15) * B3 + ((c0 + 1) >> 4)] = v3[j].y;
                row[((c0 + 2) & 15) * B3 + ((c0 + 2) >> 4)] = v3[j].z;
                row[((c0 + 3) & 15) * B3 + ((c0 + 3) >> 4)] = v3[j].w;
            }
        }
        if (threadIdx.x < L2) wl[S::SB2 + threadIdx.x] = b2v;
        if (threadIdx.x < L3) wl[S::SB3 + threadIdx.x] = b3v;
        if (threadIdx.x < G + L3 + 1) wl[S::SWO + threadIdx.x] = wov;  // [gmf | H3] kernel, then b_out
        __syncthreads();
    }

    // accumulators over the wave's units
    f32x4 dw2[B1][B2], dw3[B2][B3];
#pragma unroll
    for (int x = 0; x < B1; ++x)
#pragma unroll
        for (int y = 0; y < B2; ++y) dw2[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int x = 0; x < B2; ++x)
#pragma unroll
        for (int y = 0; y < B3; ++y) dw3[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ab1[B1][4], ab2[B2], ab3[B3], ah3[B3][4], agmf[GQ];
#pragma unroll
    for (int x = 0; x < B1; ++x)
#pragma unroll
        for (int r = 0; r < 4; ++r) ab1[x][r] = 0.f;
#pragma unroll
    for (int x = 0; x < B2; ++x) ab2[x] = 0.f;
#pragma unroll
    for (int x = 0; x < B3; ++x) {
        ab3[x] = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) ah3[x][r] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < GQ; ++e) agmf[e] = 0.f;
    float acc_bce = 0.f, acc_dbo = 0.f;
    float wo3[B3][4], b3r[B3][4], b2r[B2][4];
#pragma unroll
    for (int t = 0; t < B3; ++t) {
        ldsv<4>(wl + S::SWO + G + 16 * t + 4 * g, wo3[t]);
        ldsv<4>(wl + S::SB3 + 16 * t + 4 * g, b3r[t]);
    }
#pragma unroll
    for (int t = 0; t < B2; ++t) ldsv<4>(wl + S::SB2 + 16 * t + 4 * g, b2r[t]);
    const float bo = wl[S::SBO];

    const int64_t nunits = (a.n + 15) / 16, ustride = (int64_t)gridDim.x * 4;
    for (int64_t u = (int64_t)blockIdx.x * 4 + wv; u < nunits; u += ustride) {
        const int64_t s = u * 16 + li;
        const bool in = s < a.n;
        const int64_t sr = in ? s : 0;
        // ---- inputs: H1 (lane: features 16 t + 4 lq + r of sample li), the GMF product, the ids
        float h1[B1][4], gm[GQ];
        {
            const float* hr = a.h1 + sr * L1 + 4 * g;
#pragma unroll
            for (int t = 0; t < B1; ++t) {
                const float4 v = *reinterpret_cast<const float4*>(hr + 16 * t);
                h1[t][0] = v.x, h1[t][1] = v.y, h1[t][2] = v.z, h1[t][3] = v.w;
            }
        }
        const int cu = in ? a.users[s] : 0, cv = in ? a.items[s] : 0;
        const float y = in && a.labels ? a.labels[s] : 0.f;
        const bool ok = in && (unsigned)cu < (unsigned)a.ids.ubound && (unsigned)cv < (unsigned)a.ids.ibound;
        {
            // the GMF product of the two rows (dims GQ lq .. GQ lq + GQ - 1; zero for a masked sample)
            const float4* gu = reinterpret_cast<const float4*>(a.emb + (size_t)(ok ? cu : 0) * a.W + GQ * g);
            const float4* gi = reinterpret_cast<const float4*>(a.emb + (size_t)(ok ? a.ids.ibase + cv : 0) * a.W + GQ * g);
#pragma unroll
            for (int k = 0; k < GQ / 4; ++k) {
                const float4 p = gu[k], q = gi[k];
                gm[4 * k] = ok ? p.x * q.x : 0.f, gm[4 * k + 1] = ok ? p.y * q.y : 0.f;
                gm[4 * k + 2] = ok ? p.z * q.z : 0.f, gm[4 * k + 3] = ok ? p.w * q.w : 0.f;
            }
        }
        // H1^T for dW2
#pragma unroll
        for (int r = 0; r < 4 && !FWD; ++r) {
            float v[B1];
#pragma unroll
            for (int t = 0; t < B1; ++t) v[t] = h1[t][r];
            stsv<B1>(tb + S::TH1 + li * S::T1 + (4 * g + r) * B1, v);
        }
        // ---- layer 2: k-step (t, r) takes H1 feature 16 t + 4 lq + r (this lane's register)
        f32x4 h2[B2];
#pragma unroll
        for (int t = 0; t < B2; ++t) h2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4 * B1; ++k) {
            float w[B2];
            ldsv<B2>(wl + S::SW2 + (16 * (k >> 2) + 4 * g + (k & 3)) * S::S2 + li * B2, w);
#pragma unroll
            for (int t = 0; t < B2; ++t) h2[t] = mfma16(w[t], h1[k >> 2][k & 3], h2[t]);
        }
#pragma unroll
        for (int t = 0; t < B2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) h2[t][r] = fmaxf(h2[t][r] + b2r[t][r], 0.f);
#pragma unroll
        for (int r = 0; r < 4 && !FWD; ++r) {
            float v[B2];
#pragma unroll
            for (int t = 0; t < B2; ++t) v[t] = h2[t][r];
            stsv<B2>(tb + S::TH2 + li * S::T2 + (4 * g + r) * B2, v);
        }
        // ---- layer 3
        f32x4 h3[B3];
#pragma unroll
        for (int t = 0; t < B3; ++t) h3[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4 * B2; ++k) {
            float w[B3];
            ldsv<B3>(wl + S::SW3 + (16 * (k >> 2) + 4 * g + (k & 3)) * S::S3 + li * B3, w);
#pragma unroll
            for (int t = 0; t < B3; ++t) h3[t] = mfma16(w[t], h2[k >> 2][k & 3], h3[t]);
        }
#pragma unroll
        for (int t = 0; t < B3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) h3[t][r] = fmaxf(h3[t][r] + b3r[t][r], 0.f);
        // ---- output: this lane's H3 features and GMF dims, then the 4 lane groups
        float zp = 0.f;
#pragma unroll
        for (int t = 0; t < B3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) zp += wo3[t][r] * h3[t][r];
#pragma unroll
        for (int e = 0; e < GQ; ++e) zp += wl[S::SWO + GQ * g + e] * gm[e];
        const float z = group_allsum(zp) + bo;
        const float p = 1.0f / (1.0f + expf(-z));
        const float dz = ok && p >= eps && p <= hi_clip ? (p - y) * a.inv_batch : 0.0f;
        if (g == 0 && in) {
            a.probs[s] = ok ? p : __int_as_float(0x7fc00000);
            if constexpr (!FWD) a.dzo[s] = dz;
        }
        {
            const float pc = fminf(fmaxf(p, eps), hi_clip);
            const float logit = logf(pc / (1.0f - pc));
            const float bce = fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
            acc_bce += g == 0 && ok ? bce : 0.f;
            acc_dbo += g == 0 ? dz : 0.f;
        }
        if constexpr (FWD) continue;
#pragma unroll
        for (int e = 0; e < GQ; ++e) agmf[e] += dz * gm[e];
        // ---- G3 (registers) and its transposed copy
        float g3[B3][4];
#pragma unroll
        for (int t = 0; t < B3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                g3[t][r] = h3[t][r] > 0.f ? dz * wo3[t][r] : 0.f;
                ah3[t][r] += dz * h3[t][r];
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v[B3];
#pragma unroll
            for (int t = 0; t < B3; ++t) v[t] = g3[t][r];
            stsv<B3>(tb + S::TG3 + li * S::T3 + (4 * g + r) * B3, v);
        }
        // ---- G2 = (W3 G3) * relu'(H2): block ob holds features 16 ob + 4 lq + r; k-step (t, r)
        // takes G3 feature 16 t + 4 lq + r (one read gives the B3 steps of one r)
        float g2[B2][4];
#pragma unroll
        for (int ob = 0; ob < B2; ++ob) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float w[B3];
                ldsv<B3>(wl + S::SW3 + (16 * ob + li) * S::S3 + (4 * g + r) * B3, w);
#pragma unroll
                for (int t = 0; t < B3; ++t) acc = mfma16(w[t], g3[t][r], acc);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) g2[ob][r] = h2[ob][r] > 0.f ? acc[r] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v[B2];
#pragma unroll
            for (int t = 0; t < B2; ++t) v[t] = g2[t][r];
            stsv<B2>(tb + S::TG2 + li * S::T2 + (4 * g + r) * B2, v);
        }
        // ---- G1 = (W2 G2) * relu'(H1) -> HBM (row-major [n][L1]), and its sum for db1
#pragma unroll
        for (int ob = 0; ob < B1; ++ob) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float w[B2];
                ldsv<B2>(wl + S::SW2 + (16 * ob + li) * S::S2 + (4 * g + r) * B2, w);
#pragma unroll
                for (int t = 0; t < B2; ++t) acc = mfma16(w[t], g2[t][r], acc);
            }
            float4 o;
            o.x = h1[ob][0] > 0.f ? acc[0] : 0.f;
            o.y = h1[ob][1] > 0.f ? acc[1] : 0.f;
            o.z = h1[ob][2] > 0.f ? acc[2] : 0.f;
            o.w = h1[ob][3] > 0.f ? acc[3] : 0.f;
            if (in) *reinterpret_cast<float4*>(a.g1 + s * L1 + 16 * ob + 4 * g) = o;
            // db1 = sum of G1 over the samples (a sample past n has dz = 0: zero G1)
            ab1[ob][0] += o.x, ab1[ob][1] += o.y, ab1[ob][2] += o.z, ab1[ob][3] += o.w;
        }
        // ---- dW2 += H1^T G2, dW3 += H2^T G3 over the unit's samples: k-step q takes sample 4 q + lq
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int srow = 4 * q + g;
            float x1[B1], x2[B2], y2[B2], y3[B3];
            ldsv<B1>(tb + S::TH1 + srow * S::T1 + li * B1, x1);
            ldsv<B2>(tb + S::TH2 + srow * S::T2 + li * B2, x2);
            ldsv<B2>(tb + S::TG2 + srow * S::T2 + li * B2, y2);
            ldsv<B3>(tb + S::TG3 + srow * S::T3 + li * B3, y3);
#pragma unroll
            for (int x = 0; x < B1; ++x)
#pragma unroll
                for (int yy = 0; yy < B2; ++yy) dw2[x][yy] = mfma16(x1[x], y2[yy], dw2[x][yy]);
#pragma unroll
            for (int x = 0; x < B2; ++x)
#pragma unroll
                for (int yy = 0; yy < B3; ++yy) dw3[x][yy] = mfma16(x2[x], y3[yy], dw3[x][yy]);
#pragma unroll
            for (int yy = 0; yy < B2; ++yy) ab2[yy] += y2[yy];
#pragma unroll
            for (int yy = 0; yy < B3; ++yy) ab3[yy] += y3[yy];
        }
    }

    if constexpr (FWD) {
        // the workgroup's BCE partial, the four waves summed as the training epilogue sums them
        acc_bce = group_allsum(row_sum(acc_bce));
        __syncthreads();
        if (lane == 0) lds[wv] = acc_bce;
        __syncthreads();
        if (threadIdx.x == 0 && a.labels) a.part_bce[blockIdx.x] = (lds[0] + lds[2]) + (lds[1] + lds[3]);
        return;
    }
    // ---- epilogue: per-lane sums, then the four waves' contributions in LDS, one slab per workgroup
#pragma unroll
    for (int t = 0; t < B2; ++t) ab2[t] = group_allsum(ab2[t]);
#pragma unroll
    for (int t = 0; t < B3; ++t) {
        ab3[t] = group_allsum(ab3[t]);
#pragma unroll
        for (int r = 0; r < 4; ++r) ah3[t][r] = row_sum(ah3[t][r]);
    }
#pragma unroll
    for (int e = 0; e < GQ; ++e) agmf[e] = row_sum(agmf[e]);
#pragma unroll
    for (int x = 0; x < B1; ++x)
#pragma unroll
        for (int r = 0; r < 4; ++r) ab1[x][r] = row_sum(ab1[x][r]);
    acc_dbo = group_allsum(row_sum(acc_dbo));
    acc_bce = group_allsum(row_sum(acc_bce));
    __syncthreads();  // every wave is done with the weights and its buffers
    float* R = lds + wv * S::PR;
    if (g == 0) {
#pragma unroll
        for (int t = 0; t < B2; ++t) R[S::RB2 + 16 * t + li] = ab2[t];
#pragma unroll
        for (int t = 0; t < B3; ++t) R[S::RB3 + 16 * t + li] = ab3[t];
    }
    if (li == 0) {
#pragma unroll
        for (int t = 0; t < B3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) R[S::RWO + G + 16 * t + 4 * g + r] = ah3[t][r];
#pragma unroll
        for (int e = 0; e < GQ; ++e) R[S::RWO + GQ * g + e] = agmf[e];
    }
    if (li == 0) {
#pragma unroll
        for (int x = 0; x < B1; ++x)
#pragma unroll
            for (int r = 0; r < 4; ++r) R[S::RB1 + 16 * x + 4 * g + r] = ab1[x][r];
    }
    if (lane == 0) {
        R[S::RBO] = acc_dbo;
        R[S::RX] = acc_bce;
    }
    float* slab = a.slabs + (size_t)blockIdx.x * a.P;
    const float* R0 = lds;
    const float* R1 = lds + S::PR;
    const float* R2 = lds + 2 * S::PR;
    const float* R3 = lds + 3 * S::PR;
    auto put = [&](int t0, int t1) {
#pragma unroll
        for (int x = 0; x < B1; ++x)
#pragma unroll
            for (int yy = 0; yy < B2; ++yy) {
                const int t = x * B2 + yy;
                if (t >= t0 && t < t1) *reinterpret_cast<f32x4*>(R + (t - t0) * 256 + lane * 4) = dw2[x][yy];
            }
#pragma unroll
        for (int x = 0; x < B2; ++x)
#pragma unroll
            for (int yy = 0; yy < B3; ++yy) {
                const int t = S::NT2 + x * B3 + yy;
                if (t >= t0 && t < t1) *reinterpret_cast<f32x4*>(R + (t - t0) * 256 + lane * 4) = dw3[x][yy];
            }
    };
    // tile element (lane gq * 16 + c, register r) is row 16 x + 4 gq + r, column 16 y + c
    auto reduce = [&](int t0, int t1) {
        for (int q = threadIdx.x; q < (t1 - t0) * 64; q += 256) {
            auto at4 = [&](const float* row) { return *reinterpret_cast<const f32x4*>(row + 4 * q); };
            const f32x4 v = (at4(R0) + at4(R2)) + (at4(R1) + at4(R3));
            const int t = t0 + (q >> 6);
            int base, ld;
            if (t < S::NT2) {
                base = a.off2 + 16 * (t / B2) * L2 + 16 * (t % B2) + li, ld = L2;
            } else {
                base = a.off3 + 16 * ((t - S::NT2) / B3) * L3 + 16 * ((t - S::NT2) % B3) + li, ld = L3;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) slab[base + (4 * g + r) * ld] = v[r];
        }
    };
    put(0, S::NTR);
    __syncthreads();
    reduce(0, S::NTR);
    for (int e = threadIdx.x; e <= S::RBO - S::RB2; e += 256) {
        const int d = e < L2 ? a.off2 + L1 * L2 + e
                      : e < L2 + L3 ? a.off3 + L2 * L3 + (e - L2)
                                    : a.offo + (e - L2 - L3);
        slab[d] = (R0[S::RB2 + e] + R2[S::RB2 + e]) + (R1[S::RB2 + e] + R3[S::RB2 + e]);
    }
    if (threadIdx.x == 0) a.part_bce[blockIdx.x] = (R0[S::RX] + R2[S::RX]) + (R1[S::RX] + R3[S::RX]);
    for (int e = threadIdx.x; e < L1; e += 256)  // db1 (flat: after the hidden_1 kernel at offset 0)
        slab[a.b1off + e] = (R0[S::RB1 + e] + R2[S::RB1 + e]) + (R1[S::RB1 + e] + R3[S::RB1 + e]);
    __syncthreads();
    put(S::NTR, S::NT);
    __syncthreads();
    reduce(S::NTR, S::NT);
}

using MShapeD = MShape<128, 64, 32, 128>;  // config D after layer 1

}  // namespace

bool laymid_supported(const ncf_shape_t& s) {
    using S = MShapeD;
    return s.num_layers == 4 && s.layers[1] == S::L1 && s.layers[2] == S::L2 && s.layers[3] == S::L3 &&
           s.gmf_dim == S::G && s.gmf_stride == S::G && layer1_supported(s);
}

hipError_t launch_laymid(const ncf_shape_t& s, const float* mlp, const float* h1, const float* emb,
                         const float* labels, const int32_t* users, const int32_t* items, int64_t n, IdSpace ids,
                         float inv_batch, float* probs, float* dzo, float* g1, float* slabs, float* part_bce,
                         int grid, hipStream_t st) {
    using S = MShapeD;
    const bool fwd = dzo == nullptr;
    if (!laymid_supported(s) || grid < 1 || grid > kMaxSlabs || (!fwd && (!labels || !g1 || !slabs)))
        return hipErrorInvalidValue;
    static bool cfg = false;
    if (!cfg) {
        for (const void* k : {(const void*)k_lay_mid<S, false>, (const void*)k_lay_mid<S, true>})
            if (hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)S::LDS_BYTES))
                return e;
        cfg = true;
    }
    MidArgs a{mlp, s.layer_off[2], s.layer_off[3], s.layer_off[0], s.layer_off[1] + s.layers[0] * s.layers[1], h1, emb,
              s.row_width, labels, users, items, n, ids, inv_batch, probs, dzo, g1, slabs, s.mlp_params, part_bce};
    launch(fwd ? k_lay_mid<S, true> : k_lay_mid<S, false>, grid, 256, S::LDS_BYTES, st, a);
    return hipGetLastError();
}

}  // namespace ncf
