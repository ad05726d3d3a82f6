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
    // transposed kernels [out][in]
    static constexpr int T1 = 0, T2 = L0 * L1, T3 = T2 + L1 * L2, TP = T3 + L2 * L3;
    // LDS staging rows per 32-sample block
    static constexpr int RH1 = 0, RH2 = RH1 + 32 * NT1, RG1 = RH2 + 32 * NT2, RG2 = RG1 + 32 * NT1,
                         RG3 = RG2 + 32 * NT2, RB = RG3 + 32 * NT3;
    static constexpr int LS = 33;
    static constexpr int NDW1 = NT0 * NT1, NDW2 = NT1 * NT2, NDW3 = NT2 * NT3, NDW = NDW1 + NDW2 + NDW3;
    static constexpr int MAXT = cdiv(NDW, 4);
    static constexpr int GH = G / 2;                     // GMF features per lane half
    static constexpr int GCH = GH >= 16 ? 16 : GH;       // reduction chunk (bounds register pressure)
    static constexpr int NGC = GH >= 16 ? GH / 16 : (GH > 0 ? 1 : 0);
    static constexpr int XCH = G + L3 + 2;               // per-wave exchange floats
    static constexpr size_t LDS_BYTES = (size_t)(4 * RB * LS) * 4 + 256 * 4 + (size_t)4 * XCH * 4;
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
            const float send = hi ? x[v] : x[v + c / 2];
            const float keep = hi ? x[v + c / 2] : x[v];
            x[v] = keep + __shfl_xor(send, m, 64);
        }
    }
    float r = x[0];
#pragma unroll
    for (int m = 16 >> P; m >= 1; m >>= 1) r += __shfl_xor(r, m, 64);
    return r;
}

// W_l^T for the backward chains (A operand rows must be contiguous in `in`).
__global__ __launch_bounds__(kBlock) void k_transpose_kernels(const float* __restrict__ mlp, float* __restrict__ wt,
                                                              int l0, int l1, int l2, int l3) {
    const int dims[4] = {l0, l1, l2, l3};
    int src = 0, dst = 0;
    for (int l = 1; l <= 3; ++l) {
        const int lin = dims[l - 1], lout = dims[l];
        for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < lin * lout; e += gridDim.x * blockDim.x) {
            const int i = e / lout, o = e - i * lout;
            wt[dst + o * lin + i] = mlp[src + e];
        }
        src += lin * lout + lout;
        dst += lin * lout;
    }
}

template <class S>
__global__ __launch_bounds__(kBlock, 1) void k_fb_fused(const float* __restrict__ emb, const float* __restrict__ mlp_in,
                                                        const float* __restrict__ wt_in,
                                                        const int32_t* __restrict__ users,
                                                        const int32_t* __restrict__ items,
                                                        const float* __restrict__ labels, int64_t n, int U, int I,
                                                        float inv_batch, float* __restrict__ probs,
                                                        float* __restrict__ gs, float* __restrict__ slabs,
                                                        float* __restrict__ part_bce) {
    constexpr int L0 = S::L0, L1 = S::L1, L2 = S::L2, L3 = S::L3, G = S::G, D0 = S::D0, W = S::W, LS = S::LS;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* stg = lds;                                     // [4][RB][LS]
    int* srow = reinterpret_cast<int*>(lds + 4 * S::RB * LS);  // [2][128] table rows (-1 = masked)
    float* xch = reinterpret_cast<float*>(srow + 256);    // [4][XCH]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 31, h = lane >> 5;
    const float eps = 1e-7f, hi_clip = 1.0f - eps;

    f32x16 dwacc[S::MAXT];
#pragma unroll
    for (int m = 0; m < S::MAXT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) dwacc[m][r] = 0.f;
    float acc_bias = 0.f, acc_h3 = 0.f, acc_dbo = 0.f, acc_bce = 0.f;
    float acc_gmf[S::NGC > 0 ? S::NGC : 1];
#pragma unroll
    for (int c = 0; c < (S::NGC > 0 ? S::NGC : 1); ++c) acc_gmf[c] = 0.f;

    const int64_t niter = (n + 127) / 128;
    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        // Opaque per-iteration copies of the weight pointers: without them LICM hoists every
        // (loop-invariant) weight load out of the tile loop and the kernel spills.
        const float* mlp = mlp_in;
        const float* wt = wt_in;
        asm volatile("" : "+s"(mlp), "+s"(wt));

        const int64_t si = it * 128 + 32 * w + j;
        bool ok = false;
        int urow = 0, irow = 0;
        float y = 0.f;
        if (si < n) {
            const int u = users[si], v = items[si];
            ok = (unsigned)u < (unsigned)U && (unsigned)v < (unsigned)I;
            if (ok) { urow = u; irow = U + v; }
            y = labels[si];
        }
        if (h == 0) {
            srow[32 * w + j] = ok ? urow : -1;
            srow[128 + 32 * w + j] = ok ? irow : -1;
        }
        const float* eu = emb + (size_t)urow * W;
        const float* ei = emb + (size_t)irow * W;
        float* sb = stg + w * S::RB * LS;  // this wave's staging block

        // ---- GMF forward partial over this half's features
        float zp = 0.f;
        if constexpr (G > 0) {
            const float4* ug = reinterpret_cast<const float4*>(eu + h * S::GH);
            const float4* ig = reinterpret_cast<const float4*>(ei + h * S::GH);
            const float* wo = mlp + S::OWO + h * S::GH;
#pragma unroll 2
            for (int q = 0; q < S::GH / 4; ++q) {
                if (ok) {
                    const float4 a = ug[q], b = ig[q];
                    zp += wo[4 * q] * (a.x * b.x) + wo[4 * q + 1] * (a.y * b.y) + wo[4 * q + 2] * (a.z * b.z) +
                          wo[4 * q + 3] * (a.w * b.w);
                }
            }
        }

        // ---- forward chain.  Layer 1: the lane half h supplies its sample's user (h=0) or
        // item (h=1) MLP vector as the B operand, K order h*D0 + s; the row is streamed in
        // float4 chunks straight from the gathered embedding row.  Each activation tile is
        // staged to LDS for the weight-gradient phase as soon as it exists, and only its
        // ReLU mask (one bit per register) is kept for the backward chain.
        uint32_t m1[S::NT1], m2[S::NT2];
        f32x16 h1[S::NT1];
        {
            f32x16 acc[S::NT1];
#pragma unroll
            for (int to = 0; to < S::NT1; ++to) acc[to] = f32x16{};
            const float4* xsrc = reinterpret_cast<const float4*>((h ? ei : eu) + G);
#pragma unroll 2
            for (int q = 0; q < D0 / 4; ++q) {
                const float4 xv = ok ? xsrc[q] : make_float4(0.f, 0.f, 0.f, 0.f);
                const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = h * D0 + 4 * q + e;
#pragma unroll
                    for (int to = 0; to < S::NT1; ++to) {
                        const int oc = 32 * to + j;
                        const float a = (oc < L1) ? mlp[S::OW1 + k * L1 + oc] : 0.f;
                        acc[to] = mfma32(a, xs[e], acc[to]);
                    }
                }
            }
#pragma unroll
            for (int to = 0; to < S::NT1; ++to) {
                m1[to] = 0u;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int f = 32 * to + drow(r, h);
                    const float v = (f < L1) ? fmaxf(acc[to][r] + mlp[S::OB1 + f], 0.f) : 0.f;
                    h1[to][r] = v;
                    m1[to] |= (v > 0.f ? 1u : 0u) << r;
                    sb[(S::RH1 + f) * LS + j] = v;
                }
            }
        }
        f32x16 h2[S::NT2];
#pragma unroll
        for (int to = 0; to < S::NT2; ++to) {
            f32x16 acc = {};
            const int oc = 32 * to + j;
#pragma unroll
            for (int ti = 0; ti < S::NT1; ++ti)
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    const int k = 32 * ti + drow(s, h);
                    const float a = (oc < L2 && k < L1) ? mlp[S::OW2 + k * L2 + oc] : 0.f;
                    acc = mfma32(a, h1[ti][s], acc);
                }
            m2[to] = 0u;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * to + drow(r, h);
                const float v = (f < L2) ? fmaxf(acc[r] + mlp[S::OB2 + f], 0.f) : 0.f;
                h2[to][r] = v;
                m2[to] |= (v > 0.f ? 1u : 0u) << r;
                sb[(S::RH2 + f) * LS + j] = v;
            }
        }
        f32x16 h3[S::NT3];
#pragma unroll
        for (int to = 0; to < S::NT3; ++to) {
            f32x16 acc = {};
            const int oc = 32 * to + j;
#pragma unroll
            for (int ti = 0; ti < S::NT2; ++ti)
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    const int k = 32 * ti + drow(s, h);
                    const float a = (oc < L3 && k < L2) ? mlp[S::OW3 + k * L3 + oc] : 0.f;
                    acc = mfma32(a, h2[ti][s], acc);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * to + drow(r, h);
                h3[to][r] = (f < L3) ? fmaxf(acc[r] + mlp[S::OB3 + f], 0.f) : 0.f;
            }
        }
        // ---- output, BCE, dz (both halves compute the same sample's values)
#pragma unroll
        for (int t = 0; t < S::NT3; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * t + drow(r, h);
                if (f < L3) zp += mlp[S::OWO + G + f] * h3[t][r];
            }
        const float z = (zp + __shfl_xor(zp, 32, 64)) + mlp[S::OBO];
        const float p = 1.0f / (1.0f + expf(-z));
        float dz = 0.f, bce = 0.f;
        if (ok) {
            const float pc = fminf(fmaxf(p, eps), hi_clip);
            const float logit = logf(pc / (1.0f - pc));
            bce = fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
            dz = (p >= eps && p <= hi_clip) ? (p - y) * inv_batch : 0.0f;
        }
        if (h == 0) {
            if (si < n) probs[si] = ok ? p : __int_as_float(0x7fc00000);
            acc_bce += bce;
            acc_dbo += dz;
        }
        float* gu = gs + (size_t)(2 * si) * W;  // user contribution row
        float* gi = gu + W;                     // item contribution row

        // ---- GMF backward: embedding grads + output-kernel grads (transpose-reduced)
        if constexpr (G > 0) {
            const float* ug = eu + h * S::GH;
            const float* ig = ei + h * S::GH;
            const float* wo = mlp + S::OWO + h * S::GH;
#pragma unroll
            for (int c = 0; c < S::NGC; ++c) {
                __builtin_amdgcn_sched_barrier(0);
                float contrib[S::GCH];
#pragma unroll
                for (int q = 0; q < S::GCH / 4; ++q) {
                    const int f = c * S::GCH + 4 * q;
                    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
                    if (ok) {
                        a = *reinterpret_cast<const float4*>(ug + f);
                        b = *reinterpret_cast<const float4*>(ig + f);
                    }
                    contrib[4 * q] = dz * (a.x * b.x);
                    contrib[4 * q + 1] = dz * (a.y * b.y);
                    contrib[4 * q + 2] = dz * (a.z * b.z);
                    contrib[4 * q + 3] = dz * (a.w * b.w);
                    if (ok) {
                        const float4 gu4 = make_float4(dz * wo[f] * b.x, dz * wo[f + 1] * b.y, dz * wo[f + 2] * b.z,
                                                       dz * wo[f + 3] * b.w);
                        const float4 gi4 = make_float4(dz * wo[f] * a.x, dz * wo[f + 1] * a.y, dz * wo[f + 2] * a.z,
                                                       dz * wo[f + 3] * a.w);
                        *reinterpret_cast<float4*>(gu + h * S::GH + f) = gu4;
                        *reinterpret_cast<float4*>(gi + h * S::GH + f) = gi4;
                    }
                }
                acc_gmf[c] += half_transpose_reduce<S::GCH>(contrib, lane);
            }
        }
        // ---- output-kernel grads of the MLP features, and G3
        f32x16 g3[S::NT3];
#pragma unroll
        for (int t = 0; t < S::NT3; ++t) {
            float contrib[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * t + drow(r, h);
                contrib[r] = dz * h3[t][r];
                const float g = (f < L3 && h3[t][r] > 0.f) ? dz * mlp[S::OWO + G + f] : 0.f;
                g3[t][r] = g;
                sb[(S::RG3 + f) * LS + j] = g;
            }
            const float red = half_transpose_reduce<16>(contrib, lane);
            if (t == 0) acc_h3 += red;  // NT3 == 1 for the supported shapes
        }
        // ---- backward data chain
        f32x16 g2[S::NT2];
#pragma unroll
        for (int to = 0; to < S::NT2; ++to) {
            f32x16 acc = {};
            const int oc = 32 * to + j;
#pragma unroll
            for (int ti = 0; ti < S::NT3; ++ti)
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    if (32 * ti + 8 * (s >> 2) >= L3) continue;  // whole step beyond L3 (both halves)
                    const int k = 32 * ti + drow(s, h);
                    const float a = (oc < L2 && k < L3) ? wt[S::T3 + k * L2 + oc] : 0.f;
                    acc = mfma32(a, g3[ti][s], acc);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float g = ((m2[to] >> r) & 1u) ? acc[r] : 0.f;
                g2[to][r] = g;
                sb[(S::RG2 + 32 * to + drow(r, h)) * LS + j] = g;
            }
        }
        f32x16 g1[S::NT1];
#pragma unroll
        for (int to = 0; to < S::NT1; ++to) {
            f32x16 acc = {};
            const int oc = 32 * to + j;
#pragma unroll
            for (int ti = 0; ti < S::NT2; ++ti)
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    if (32 * ti + 8 * (s >> 2) >= L2) continue;
                    const int k = 32 * ti + drow(s, h);
                    const float a = (oc < L1 && k < L2) ? wt[S::T2 + k * L1 + oc] : 0.f;
                    acc = mfma32(a, g2[ti][s], acc);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float g = ((m1[to] >> r) & 1u) ? acc[r] : 0.f;
                g1[to][r] = g;
                sb[(S::RG1 + 32 * to + drow(r, h)) * LS + j] = g;
            }
        }
#pragma unroll
        for (int to = 0; to < S::NT0; ++to) {
            f32x16 acc = {};
            const int oc = 32 * to + j;
#pragma unroll
            for (int ti = 0; ti < S::NT1; ++ti)
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    if (32 * ti + 8 * (s >> 2) >= L1) continue;
                    const int k = 32 * ti + drow(s, h);
                    const float a = (oc < L0 && k < L1) ? wt[S::T1 + k * L0 + oc] : 0.f;
                    acc = mfma32(a, g1[ti][s], acc);
                }
            if (ok) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int f = 32 * to + 8 * q + 4 * h;  // rows drow(4q..4q+3, h) are f..f+3
                    if (f < L0) {
                        float* dst = (f < D0) ? gu + G + f : gi + G + (f - D0);
                        *reinterpret_cast<float4*>(dst) =
                            make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                    }
                }
            }
        }
        __syncthreads();

        // ---- weight gradients: wave w owns tiles w, w+4, w+8, ... (K = 128 samples)
#pragma unroll
        for (int m = 0; m < S::MAXT; ++m) {
            const int t = w + 4 * m;
            if (t >= S::NDW) break;
            int layer, ti, to;
            if (t < S::NDW1) { layer = 1; ti = t / S::NT1; to = t % S::NT1; }
            else if (t < S::NDW1 + S::NDW2) { layer = 2; ti = (t - S::NDW1) / S::NT2; to = (t - S::NDW1) % S::NT2; }
            else { layer = 3; ti = (t - S::NDW1 - S::NDW2) / S::NT3; to = (t - S::NDW1 - S::NDW2) % S::NT3; }
            const int fi = 32 * ti + j;  // A row (input feature) supplied by this lane
            const int fo = 32 * to + j;  // B column (output feature) supplied by this lane
            const int arow = layer == 2 ? S::RH1 + fi : S::RH2 + fi;
            const int brow = (layer == 1 ? S::RG1 : layer == 2 ? S::RG2 : S::RG3) + fo;
            const int lin = layer == 1 ? L0 : layer == 2 ? L1 : L2;
            f32x16 acc = dwacc[m];
            for (int b = 0; b < 4; ++b) {
                const float* bb = stg + b * S::RB * LS;
                if (layer == 1) {
                    const int side = fi < D0 ? 0 : 128;
                    const int col = G + (fi < D0 ? fi : fi - D0);
#pragma unroll 4
                    for (int s = 0; s < 16; ++s) {
                        const int c = 2 * s + h;
                        const int row = srow[side + 32 * b + c];
                        const float a = (row >= 0 && fi < lin) ? emb[(size_t)row * W + col] : 0.f;
                        acc = mfma32(a, bb[brow * LS + c], acc);
                    }
                } else {
#pragma unroll 4
                    for (int s = 0; s < 16; ++s) {
                        const int c = 2 * s + h;
                        acc = mfma32(bb[arow * LS + c], bb[brow * LS + c], acc);
                    }
                }
            }
            dwacc[m] = acc;
        }
        // ---- bias gradients: one G row per thread, summed over the 128 samples
        if (tid < L1 + L2 + L3) {
            const int rr = tid < L1 ? S::RG1 + tid : tid < L1 + L2 ? S::RG2 + (tid - L1) : S::RG3 + (tid - L1 - L2);
            float sacc = 0.f;
            for (int b = 0; b < 4; ++b) {
                const float* bb = stg + b * S::RB * LS + rr * LS;
#pragma unroll
                for (int c = 0; c < 32; ++c) sacc += bb[c];
            }
            acc_bias += sacc;
        }
        __syncthreads();
    }

    // ---- epilogue: this workgroup's dense-gradient slab and BCE partial
    const float* mlp = mlp_in;
    float* slab = slabs + (size_t)blockIdx.x * S::P;
#pragma unroll
    for (int m = 0; m < S::MAXT; ++m) {
        const int t = w + 4 * m;
        if (t >= S::NDW) break;
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
    if (tid < L1) slab[S::OB1 + tid] = acc_bias;
    else if (tid < L1 + L2) slab[S::OB2 + (tid - L1)] = acc_bias;
    else if (tid < L1 + L2 + L3) slab[S::OB3 + (tid - L1 - L2)] = acc_bias;

    // output layer: combine the 4 waves in fixed order through LDS
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
    float dbo = acc_dbo, bce = acc_bce;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        dbo += __shfl_xor(dbo, m, 64);
        bce += __shfl_xor(bce, m, 64);
    }
    if (lane == 0) {
        xw[G + L3] = dbo;
        xw[G + L3 + 1] = bce;
    }
    __syncthreads();
    if (tid < G + L3 + 1) {
        const float v = (xch[tid] + xch[S::XCH + tid]) + (xch[2 * S::XCH + tid] + xch[3 * S::XCH + tid]);
        slab[S::OWO + tid] = v;  // G + L3 kernel entries, then the bias at OBO = OWO + G + L3
    }
    if (tid == 0) {
        const int o = G + L3 + 1;
        part_bce[blockIdx.x] = (xch[o] + xch[S::XCH + o]) + (xch[2 * S::XCH + o] + xch[3 * S::XCH + o]);
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
                             float inv_batch, int* nslab, int* nbce, hipStream_t st) {
    static bool configured = false;
    if (!configured) {
        hipError_t e = hipFuncSetAttribute((const void*)k_fb_fused<S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)S::LDS_BYTES);
        if (e != hipSuccess) return e;
        configured = true;
    }
    float* wt = at<float>(ws, L.wt);
    k_transpose_kernels<<<16, kBlock, 0, st>>>(mlp, wt, S::L0, S::L1, S::L2, S::L3);
    const int64_t niter = (n + 127) / 128;
    int grid = (int)(niter < 256 ? niter : 256);
    if (grid > kMaxSlabs) grid = kMaxSlabs;
    k_fb_fused<S><<<grid, kBlock, S::LDS_BYTES, st>>>(emb, mlp, wt, users, items, labels, n, s.num_users,
                                                      s.num_items, inv_batch, at<float>(ws, L.probs),
                                                      at<float>(ws, L.gs), at<float>(ws, L.slabs),
                                                      at<float>(ws, L.part_bce));
    *nslab = grid;
    *nbce = grid;
    return hipGetLastError();
}

hipError_t launch_fb_fused(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                           const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                           float inv_batch, int* nslab, int* nbce, hipStream_t st) {
#define NCF_TRY(SH) \
    if (matches<SH>(s)) return launch_one<SH>(s, L, ws, emb, mlp, users, items, labels, n, inv_batch, nslab, nbce, st)
    NCF_TRY(ShapeC);
    NCF_TRY(ShapeB);
    NCF_TRY(ShapeR);
    NCF_TRY(ShapeC0);
#undef NCF_TRY
    return hipErrorNotSupported;
}

}  // namespace ncf
