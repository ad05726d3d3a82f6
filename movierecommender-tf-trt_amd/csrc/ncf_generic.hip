// Generic (any shape) forward / backward of the NCF/NeuMF hot path.
//
// One thread per sample, runtime layer sizes, fp32 FMA chains, dense weights
// staged in LDS when they fit.  This is the correctness path for shapes the
// fused MFMA kernel (ncf_fused.hip) does not cover (e.g. the reference's
// test model layers_sizes=[6,4]); it keeps per-sample activations in a
// workspace so the dense-layer weight gradients can be reduced in a second,
// deterministic kernel (k_dw_generic).
//
// Per sample i (reference movierec/model.py:154-194 + NeuMF GMF branch):
//   h0 = [E_u_mlp[u], E_i_mlp[v]]                    (model.py:161-172)
//   h_l = relu(h_{l-1} W_l + b_l), l = 1..n-1         (model.py:175-181)
//   f = [E_u_gmf[u] * E_i_gmf[v], h_{n-1}]           (NeuMF; empty GMF = reference)
//   p = sigmoid(f . w_out + b_out)                    (model.py:184-188)
// BCE (Keras clip→logit→sigmoid xent, model.py:214), dz = (p-y)/B where the
// clip is inactive; backward writes the two per-sample embedding gradient rows
// (user row c=2i, item row c=2i+1) in the table's row layout.

#include <cmath>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

struct GenShape {
    int n;             // num_layers
    int L[NCF_MAX_LAYERS];
    int U, I, IB, G, G4, W, du, di, P, F;  // U / I: id bounds, IB: row of item 0
    int off[NCF_MAX_LAYERS];      // [l>=1] hidden kernel offset, [0] output kernel offset
    int act_off[NCF_MAX_LAYERS];  // h_l offset inside an activation row
    int gmf_off;                  // gmf product offset inside an activation row
    int A;                        // activation row width
    int dz_off[NCF_MAX_LAYERS];   // dz_l offset (l>=1) inside a dz row
    int D;                        // dz row width (last entry = output dz)
};

static GenShape make_gen_shape(const ncf_shape_t& s, IdSpace ids) {
    GenShape g{};
    g.n = s.num_layers;
    for (int l = 0; l < s.num_layers; ++l) g.L[l] = s.layers[l];
    g.U = ids.ubound;
    g.I = ids.ibound;
    g.IB = ids.ibase;
    g.G = s.gmf_dim;
    g.G4 = s.gmf_stride;
    g.W = s.row_width;
    g.du = s.du;
    g.di = s.di;
    g.P = s.mlp_params;
    g.F = s.out_features;
    for (int l = 0; l < NCF_MAX_LAYERS; ++l) g.off[l] = s.layer_off[l];
    int a = 0;
    for (int l = 0; l < s.num_layers; ++l) { g.act_off[l] = a; a += s.layers[l]; }
    g.gmf_off = a;
    g.A = a + s.gmf_dim;
    int d = 0;
    for (int l = 1; l < s.num_layers; ++l) { g.dz_off[l] = d; d += s.layers[l]; }
    g.D = d + 1;
    return g;
}

constexpr int kLdsWeightsMax = 12288;  // floats (48 KB) of dense weights staged in LDS

template <bool TRAIN>
__global__ __launch_bounds__(kBlock) void k_fb_generic(GenShape S, const float* __restrict__ emb,
                                                       const float* __restrict__ mlp,
                                                       const int32_t* __restrict__ users,
                                                       const int32_t* __restrict__ items,
                                                       const float* __restrict__ labels, int64_t n, float inv_batch,
                                                       float* __restrict__ probs, float* __restrict__ act,
                                                       float* __restrict__ dzb, float* __restrict__ gs,
                                                       float* __restrict__ part_bce, int use_lds) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];
    __shared__ float red[4];
    const float* Wt = mlp;
    if (use_lds) {
        for (int j = threadIdx.x; j < S.P; j += kBlock) wsh[j] = mlp[j];
        __syncthreads();
        Wt = wsh;
    }
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    float bce = 0.0f;
    if (i < n) {
        const int u = users[i];
        const int v = items[i];
        const bool ok = (unsigned)u < (unsigned)S.U && (unsigned)v < (unsigned)S.I;
        float* a = act + (size_t)i * S.A;
        const float* eu = emb + (size_t)u * S.W;
        const float* ei = emb + ((size_t)S.IB + (size_t)v) * S.W;
        const float* wo = Wt + S.off[0];
        float p;
        if (ok) {
            for (int k = 0; k < S.du; ++k) a[k] = eu[S.G4 + k];
            for (int k = 0; k < S.di; ++k) a[S.du + k] = ei[S.G4 + k];
            for (int l = 1; l < S.n; ++l) {
                const int lin = S.L[l - 1], lout = S.L[l];
                const float* Wl = Wt + S.off[l];
                const float* bl = Wl + lin * lout;
                const float* in = a + S.act_off[l - 1];
                float* out = a + S.act_off[l];
                for (int o = 0; o < lout; ++o) {
                    float z = 0.0f;
                    for (int k = 0; k < lin; ++k) z += in[k] * Wl[k * lout + o];
                    z += bl[o];
                    out[o] = fmaxf(z, 0.0f);
                }
            }
            float z = 0.0f;
            for (int f = 0; f < S.G; ++f) {
                const float gm = eu[f] * ei[f];
                a[S.gmf_off + f] = gm;
                z += gm * wo[f];
            }
            if (S.n > 0) {  // n == 0: GMF-only model
                const float* hl = a + S.act_off[S.n - 1];
                for (int o = 0; o < S.L[S.n - 1]; ++o) z += hl[o] * wo[S.G + o];
            }
            z += wo[S.F];
            p = 1.0f / (1.0f + expf(-z));
        } else {
            p = __int_as_float(0x7fc00000);
            for (int k = 0; k < S.A; ++k) a[k] = 0.0f;
        }
        if (probs) probs[i] = p;
        float dzo = 0.0f;
        if (labels && ok) {
            const float y = labels[i];
            const float eps = 1e-7f;
            const float hi = 1.0f - eps;
            const float pc = fminf(fmaxf(p, eps), hi);
            const float logit = logf(pc / (1.0f - pc));
            bce = fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
            dzo = (p >= eps && p <= hi) ? (p - y) * inv_batch : 0.0f;
        }
        if (TRAIN) {
            float* d = dzb + (size_t)i * S.D;
            float* gu = gs + (size_t)(2 * i) * S.W;
            float* gi = gu + S.W;
            d[S.D - 1] = dzo;
            for (int f = 0; f < S.G4; ++f) {
                gu[f] = (ok && f < S.G) ? dzo * wo[f] * ei[f] : 0.0f;
                gi[f] = (ok && f < S.G) ? dzo * wo[f] * eu[f] : 0.0f;
            }
            for (int k = S.du; k < S.W - S.G4; ++k) gu[S.G4 + k] = 0.0f;
            for (int k = S.di; k < S.W - S.G4; ++k) gi[S.G4 + k] = 0.0f;
            if (S.n >= 2) {
                float* dh = d + S.dz_off[S.n - 1];
                for (int o = 0; o < S.L[S.n - 1]; ++o) dh[o] = dzo * wo[S.G + o];
                for (int l = S.n - 1; l >= 1; --l) {
                    const int lin = S.L[l - 1], lout = S.L[l];
                    float* dzl = d + S.dz_off[l];
                    const float* hl = a + S.act_off[l];
                    for (int o = 0; o < lout; ++o) dzl[o] = hl[o] > 0.0f ? dzl[o] : 0.0f;
                    const float* Wl = Wt + S.off[l];
                    for (int k = 0; k < lin; ++k) {
                        float s = 0.0f;
                        for (int o = 0; o < lout; ++o) s += dzl[o] * Wl[k * lout + o];
                        if (l >= 2)
                            d[S.dz_off[l - 1] + k] = s;
                        else if (k < S.du)
                            gu[S.G4 + k] = s;
                        else
                            gi[S.G4 + k - S.du] = s;
                    }
                }
            } else if (S.n == 1) {
                for (int k = 0; k < S.L[0]; ++k) {
                    const float s = dzo * wo[S.G + k];
                    if (k < S.du) gu[S.G4 + k] = s;
                    else gi[S.G4 + k - S.du] = s;
                }
            }
        }
    }
    if (part_bce) {  // uniform across the block
        bce = block_sum_256(bce, red);
        if (threadIdx.x == 0) part_bce[blockIdx.x] = bce;
    }
}

// Dense-layer weight gradients: slab[s][p] = sum over the samples of chunk s
// (fixed ascending order) of in_i[k] * dz_i[o] (kernels) or dz_i[o] (biases).
__global__ __launch_bounds__(kBlock) void k_dw_generic(GenShape S, const float* __restrict__ act,
                                                       const float* __restrict__ dzb, int64_t n, int64_t chunk,
                                                       float* __restrict__ slabs) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= S.P) return;
    const int64_t i0 = (int64_t)blockIdx.y * chunk;
    const int64_t i1 = min(n, i0 + chunk);
    int ain = -1, dcol;  // activation column (or -1 for bias), dz column
    bool found = false;
    for (int l = 1; l < S.n && !found; ++l) {
        const int lin = S.L[l - 1], lout = S.L[l];
        const int q = p - S.off[l];
        if (q >= 0 && q < lin * lout) {
            ain = S.act_off[l - 1] + q / lout;
            dcol = S.dz_off[l] + q % lout;
            found = true;
        } else if (q >= lin * lout && q < lin * lout + lout) {
            ain = -1;
            dcol = S.dz_off[l] + (q - lin * lout);
            found = true;
        }
    }
    if (!found) {
        const int q = p - S.off[0];
        dcol = S.D - 1;
        if (q < S.F)
            ain = (q < S.G || S.n == 0) ? S.gmf_off + q : S.act_off[S.n - 1] + (q - S.G);
        else
            ain = -1;
    }
    float acc = 0.0f;
    if (ain >= 0) {
        for (int64_t i = i0; i < i1; ++i) acc += act[(size_t)i * S.A + ain] * dzb[(size_t)i * S.D + dcol];
    } else {
        for (int64_t i = i0; i < i1; ++i) acc += dzb[(size_t)i * S.D + dcol];
    }
    slabs[(size_t)blockIdx.y * S.P + p] = acc;
}

hipError_t launch_fb_generic(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                             const float* mlp, const int32_t* users, const int32_t* items,
                             const float* labels, int64_t n, float inv_batch, IdSpace ids, int* nslab, int* nbce,
                             hipStream_t st) {
    const GenShape S = make_gen_shape(s, ids);
    const int use_lds = s.mlp_params <= kLdsWeightsMax ? 1 : 0;
    const int grid = (int)((n + kBlock - 1) / kBlock);
    launch(k_fb_generic<true>, grid, kBlock, use_lds ? (size_t)s.mlp_params * 4 : 0, st, 
        S, emb, mlp, users, items, labels, n, inv_batch, at<float>(ws, L.probs), at<float>(ws, L.act),
        at<float>(ws, L.dz), at<float>(ws, L.gs), at<float>(ws, L.part_bce), use_lds);
    *nbce = grid;
    int64_t chunk = 1024;
    int64_t ns = (n + chunk - 1) / chunk;
    if (ns > kMaxSlabs) {
        chunk = (n + kMaxSlabs - 1) / kMaxSlabs;
        ns = (n + chunk - 1) / chunk;
    }
    dim3 g2((s.mlp_params + kBlock - 1) / kBlock, (unsigned)ns);
    launch(k_dw_generic, g2, kBlock, 0, st, S, at<float>(ws, L.act), at<float>(ws, L.dz), n, chunk,
                                        at<float>(ws, L.slabs));
    *nslab = (int)ns;
    return hipGetLastError();
}

hipError_t launch_predict_generic(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                                  const float* mlp, const int32_t* users, const int32_t* items,
                                  const float* labels, int64_t n, float* probs, IdSpace ids, int* nbce,
                                  hipStream_t st) {
    const GenShape S = make_gen_shape(s, ids);
    const int use_lds = s.mlp_params <= kLdsWeightsMax ? 1 : 0;
    const int grid = (int)((n + kBlock - 1) / kBlock);
    launch(k_fb_generic<false>, grid, kBlock, use_lds ? (size_t)s.mlp_params * 4 : 0, st, 
        S, emb, mlp, users, items, labels, n, 0.0f, probs, at<float>(ws, L.act), nullptr, nullptr,
        labels ? at<float>(ws, L.part_bce) : nullptr, use_lds);
    *nbce = labels ? grid : 0;
    return hipGetLastError();
}

}  // namespace ncf
