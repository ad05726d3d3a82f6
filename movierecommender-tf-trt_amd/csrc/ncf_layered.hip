// Layer-by-layer forward / backward for shapes whose dense weights do not fit the fused
// kernel's LDS budget (config D: MLP [256,128,64,32] + GMF 128, 174 KB of weights).
//
// The fused kernel (ncf_fused.hip) keeps every weight in LDS and every activation in
// registers; past ~45 KB of weights that stops fitting.  Here the batch is processed one
// layer at a time, each dense layer a plain fp32 GEMM over the whole batch (rocBLAS,
// MFMA-backed on gfx950, atomics off so every sum runs in a fixed order), with the gather,
// bias+ReLU, output/BCE, ReLU-mask and gradient-row scatter as small HBM-bound kernels:
//
//   k_lay_gather(4)  X0 = [E_u_mlp | E_i_mlp], GMF = E_u_gmf * E_i_gmf     (model.py:161-172)
//   sgemm + k_bias_relu   X_l = relu(X_{l-1} W_l + b_l)                     (model.py:175-181)
//   k_lay_out2 + k_lay_gl   p = sigmoid([GMF, X_{n-1}] w_out + b_out); Keras BCE, dz;
//                  G_{n-1} = dz w_mlp * relu'(X_{n-1})                     (model.py:184-188, 213-214)
//   sgemm          dW_l = X_{l-1}^T G_l;  sgemv: db_l, output-layer grads (one slab)
//   sgemm + k_relu_mask   G_{l-1} = (G_l W_l^T) * relu'(X_{l-1});  dX0 = G_1 W_1^T
//   k_lay_scatter(4)  per-sample gradient rows gs[2i] (user) / gs[2i+1] (item)
//
// The outputs are exactly those of the generic kernel (probs, gs, part_bce, one dense-gradient
// slab), so the index build, the optimizer sweeps and the data-parallel paths are shared.
// Activations live in the generic kernel's act / dz workspace regions, re-cut as one
// [batch x width] matrix per layer.

#include <cmath>
#include <cstdlib>

#include <rocblas/rocblas.h>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

namespace {

// one handle per host thread (and device); deliberately never destroyed, so no rocBLAS call runs
// from a thread-exit destructor after the HIP runtime has begun tearing down
struct BlasHandle {
    rocblas_handle h = nullptr;
    int device = -1;
};

hipError_t blas(hipStream_t st, rocblas_handle* out) {
    thread_local BlasHandle bh;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (!bh.h || bh.device != dev) {
        if (bh.h) rocblas_destroy_handle(bh.h);
        bh.h = nullptr;
        if (rocblas_create_handle(&bh.h) != rocblas_status_success) return hipErrorNotInitialized;
        // fixed-order reductions: no split-K kernels that combine partial sums with atomics
        rocblas_set_atomics_mode(bh.h, rocblas_atomics_not_allowed);
        bh.device = dev;
    }
    if (rocblas_set_stream(bh.h, st) != rocblas_status_success) return hipErrorInvalidValue;
    *out = bh.h;
    return hipSuccess;
}

inline hipError_t blas_err(rocblas_status s) { return s == rocblas_status_success ? hipSuccess : hipErrorLaunchFailure; }

}  // namespace

// X0[i][c] = MLP halves of the two rows, GMF[i][f] = E_u_gmf * E_i_gmf; zeros for masked samples.
__global__ __launch_bounds__(kBlock) void k_lay_gather(const float* __restrict__ emb, const int32_t* __restrict__ users,
                                                       const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                       int W, int G, int G4, int du, int di,
                                                       float* __restrict__ x0, float* __restrict__ gmf) {
    const int C = du + di + G;
    const int64_t total = n * C;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / C;
        const int c = (int)(e - i * C);
        const int u = users[i], v = items[i];
        const bool ok = (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
        const float* eu = emb + (size_t)(ok ? u : 0) * W;
        const float* ei = emb + (size_t)(ok ? ids.ibase + v : 0) * W;
        if (c < du) {
            x0[i * (du + di) + c] = ok ? eu[G4 + c] : 0.f;
        } else if (c < du + di) {
            x0[i * (du + di) + c] = ok ? ei[G4 + c - du] : 0.f;
        } else {
            const int f = c - du - di;
            gmf[i * G + f] = ok ? eu[f] * ei[f] : 0.f;
        }
    }
}

// float4 variant (du, di, G multiples of 4 and G == G4): one thread per float4 of the
// [X0 | GMF] row, the row id loaded once per float4 instead of once per float
__global__ __launch_bounds__(kBlock) void k_lay_gather4(const float4* __restrict__ emb,
                                                        const int32_t* __restrict__ users,
                                                        const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                        int W4, int G4q, int du4, int di4, float4* __restrict__ x0,
                                                        float4* __restrict__ gmf) {
    const int C = du4 + di4 + G4q;
    const int64_t total = n * C;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / C;
        const int c = (int)(e - i * C);
        const int u = users[i], v = items[i];
        const bool ok = (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
        const float4* eu = emb + (size_t)(ok ? u : 0) * W4;
        const float4* ei = emb + (size_t)(ok ? ids.ibase + v : 0) * W4;
        if (c < du4) {
            x0[i * (du4 + di4) + c] = ok ? eu[G4q + c] : zero;
        } else if (c < du4 + di4) {
            x0[i * (du4 + di4) + c] = ok ? ei[G4q + c - du4] : zero;
        } else {
            const int f = c - du4 - di4;
            const float4 a = eu[f], b = ei[f];
            gmf[i * G4q + f] = ok ? make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w) : zero;
        }
    }
}

// float4 variant of k_lay_scatter (same alignment conditions)
__global__ __launch_bounds__(kBlock) void k_lay_scatter4(const float4* __restrict__ emb, const float* __restrict__ mlp,
                                                         int wo_off, const int32_t* __restrict__ users,
                                                         const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                         int W4, int G4q, int du4, int di4,
                                                         const float* __restrict__ dzo,
                                                         const float4* __restrict__ dx0, float4* __restrict__ gs) {
    const int64_t total = n * 2 * W4;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rowc = e / W4;  // contribution 2i (user) / 2i+1 (item)
        const int q = (int)(e - rowc * W4);
        const int64_t i = rowc >> 1;
        const int side = (int)(rowc & 1);
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q < G4q) {
            const int u = users[i], v = items[i];
            const bool ok = (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
            if (ok) {
                const float4 o = emb[(size_t)(side ? u : ids.ibase + v) * W4 + q];  // the other side's GMF
                const float d = dzo[i];
                const float* w = mlp + wo_off + 4 * q;
                g = make_float4(d * w[0] * o.x, d * w[1] * o.y, d * w[2] * o.z, d * w[3] * o.w);
            }
        } else {
            const int k = q - G4q;
            if (side == 0 && k < du4) g = dx0[i * (du4 + di4) + k];
            else if (side == 1 && k < di4) g = dx0[i * (du4 + di4) + du4 + k];
        }
        gs[e] = g;
    }
}

__global__ __launch_bounds__(kBlock) void k_bias_relu(float* __restrict__ x, int64_t total, int lout,
                                                      const float* __restrict__ bias) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x)
        x[e] = fmaxf(x[e] + bias[e % lout], 0.f);
}

__global__ __launch_bounds__(kBlock) void k_relu_mask(float* __restrict__ g, const float* __restrict__ x,
                                                      int64_t total) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x)
        g[e] = x[e] > 0.f ? g[e] : 0.f;
}

// Output layer: one thread per sample, z = [GMF, X_{n-1}] w_out + b_out (float4 reads when both
// widths are multiples of 4), sigmoid, Keras BCE, dz; G_{n-1} elementwise in k_lay_gl.
template <bool VEC>
__global__ __launch_bounds__(kBlock) void k_lay_out2(const float* __restrict__ gmf, const float* __restrict__ xl,
                                                     const float* __restrict__ wo, int G, int Ll,
                                                     const int32_t* __restrict__ users,
                                                     const int32_t* __restrict__ items, IdSpace ids,
                                                     const float* __restrict__ labels, int64_t n, float inv_batch,
                                                     float* __restrict__ probs, float* __restrict__ dzo,
                                                     float* __restrict__ ones, float* __restrict__ part_bce) {
    __shared__ float red[4];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    float bce = 0.f;
    if (i < n) {
        const int u = users[i], v = items[i];
        const bool ok = (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
        float z = 0.f;
        if (VEC) {
            const float4* g4 = reinterpret_cast<const float4*>(gmf + i * G);
            const float4* x4 = reinterpret_cast<const float4*>(xl + i * Ll);
            for (int f = 0; f < G / 4; ++f) {
                const float4 a = g4[f];
                z += a.x * wo[4 * f] + a.y * wo[4 * f + 1] + a.z * wo[4 * f + 2] + a.w * wo[4 * f + 3];
            }
            for (int o = 0; o < Ll / 4; ++o) {
                const float4 a = x4[o];
                const float* w = wo + G + 4 * o;
                z += a.x * w[0] + a.y * w[1] + a.z * w[2] + a.w * w[3];
            }
        } else {
            for (int f = 0; f < G; ++f) z += gmf[i * G + f] * wo[f];
            for (int o = 0; o < Ll; ++o) z += xl[i * Ll + o] * wo[G + o];
        }
        z += wo[G + Ll];
        const float p = 1.0f / (1.0f + expf(-z));
        float d = 0.f;
        if (ok && labels) {   // forward only (ncf_predict): no labels, no loss
            const float y = labels[i];
            const float eps = 1e-7f, hi = 1.0f - eps;
            const float pc = fminf(fmaxf(p, eps), hi);
            const float logit = logf(pc / (1.0f - pc));
            bce = fmaxf(logit, 0.0f) - logit * y + log1pf(expf(-fabsf(logit)));
            d = (p >= eps && p <= hi) ? (p - y) * inv_batch : 0.0f;
        }
        probs[i] = ok ? p : __int_as_float(0x7fc00000);
        dzo[i] = d;
        ones[i] = 1.0f;
    }
    bce = block_sum_256(bce, red);
    if (threadIdx.x == 0) part_bce[blockIdx.x] = bce;
}

__global__ __launch_bounds__(kBlock) void k_lay_gl(const float* __restrict__ xl, const float* __restrict__ dzo,
                                                   const float* __restrict__ wmlp, int Ll, int64_t total,
                                                   float* __restrict__ gl) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / Ll;
        const int o = (int)(e - i * Ll);
        gl[e] = xl[e] > 0.f ? dzo[i] * wmlp[o] : 0.f;
    }
}

// gs[2i] = [dz w_gmf * E_i_gmf | dX0[:du] | 0-pad], gs[2i+1] = [dz w_gmf * E_u_gmf | dX0[du:] | 0-pad]
__global__ __launch_bounds__(kBlock) void k_lay_scatter(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                        int wo_off, const int32_t* __restrict__ users,
                                                        const int32_t* __restrict__ items, int64_t n, IdSpace ids,
                                                        int W, int G, int G4, int du, int di,
                                                        const float* __restrict__ dzo, const float* __restrict__ dx0,
                                                        float* __restrict__ gs) {
    const int64_t total = n * 2 * W;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rowc = e / W;  // contribution 2i (user) / 2i+1 (item)
        const int c = (int)(e - rowc * W);
        const int64_t i = rowc >> 1;
        const int side = (int)(rowc & 1);
        float g = 0.f;
        if (c < G4) {
            if (c < G) {
                const int u = users[i], v = items[i];
                const bool ok = (unsigned)u < (unsigned)ids.ubound && (unsigned)v < (unsigned)ids.ibound;
                if (ok) {
                    // the other side's GMF vector
                    const float* other = emb + (size_t)(side ? u : ids.ibase + v) * W;
                    g = dzo[i] * mlp[wo_off + c] * other[c];
                }
            }
        } else {
            const int k = c - G4;
            if (side == 0 && k < du) g = dx0[i * (du + di) + k];
            else if (side == 1 && k < di) g = dx0[i * (du + di) + du + k];
        }
        gs[e] = g;
    }
}

bool layered_supported(const ncf_shape_t& s) { return s.num_layers >= 2; }

static unsigned grid_for(int64_t total) {
    int64_t g = (total + kBlock - 1) / kBlock;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// Forward only (ncf_predict / ncf_evaluate on layered shapes): the gather, the dense layers as
// GEMMs + bias/ReLU, the output layer with (labels given) the Keras BCE partials, one per
// 256-sample block in part_bce (*nbce).  Same arithmetic as the forward half of
// launch_fb_layered, so evaluation matches training's forward.
hipError_t launch_predict_layered(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                                  const float* mlp, const int32_t* users, const int32_t* items, const float* labels,
                                  int64_t n, float* probs, IdSpace ids, int* nbce, hipStream_t st) {
    if (!layered_supported(s) || n > L.max_batch) return hipErrorInvalidValue;
    // (the rocBLAS handle only on the general-shape path below: none on config D's)
    rocblas_handle bh = nullptr;
    hipError_t e = hipSuccess;
    const int nl = s.num_layers, G = s.gmf_dim, G4 = s.gmf_stride, W = s.row_width;
    const int du = s.du, di = s.di, Ll = s.layers[nl - 1];
    float* act = at<float>(ws, L.act);
    float* X[NCF_MAX_LAYERS];
    int64_t o = 0;
    for (int l = 0; l < nl; ++l) { X[l] = act + o; o += (int64_t)L.max_batch * s.layers[l]; }
    float* gmf = act + o;
    float* dzo = at<float>(ws, L.dz);
    float* ones = at<float>(ws, L.ones);
    const float one = 1.0f, zero = 0.0f;
    const bool vec4 = du % 4 == 0 && di % 4 == 0 && G == G4 && W % 4 == 0;
    // layer 1 on hand-written MFMA with the gather fused (ncf_layer1.hip), where the shape has it
    const bool l1 = layer1_supported(s);
    if (l1 && laymid_supported(s)) {
        // config D: layers 2.., the output and the BCE partials in the middle kernel's forward-only
        // form (ncf_laymid.hip) — no vendor GEMM on the evaluation path either
        e = launch_layer1_fwd(s, emb, mlp, users, items, n, ids, X[0], nullptr, X[1], st);
        if (e != hipSuccess) return e;
        const int64_t units = (n + 15) / 16;
        const int grid = (int)(units >= 8 * 512 ? 512 : (units + 7) / 8);
        e = launch_laymid(s, mlp, X[1], emb, labels, users, items, n, ids, 1.0f, probs, nullptr, nullptr, nullptr,
                          at<float>(ws, L.part_bce), grid, st);
        *nbce = labels ? grid : 0;
        return e;
    }
    if (l1)
        e = launch_layer1_fwd(s, emb, mlp, users, items, n, ids, X[0], gmf, X[1], st);
    else if (vec4)
        launch(k_lay_gather4, grid_for(n * (du + di + G) / 4), kBlock, 0, st, (const float4*)emb, users, items, n, ids,
               W / 4, G / 4, du / 4, di / 4, (float4*)X[0], (float4*)gmf);
    else
        launch(k_lay_gather, grid_for(n * (du + di + G)), kBlock, 0, st, emb, users, items, n, ids, W, G, G4, du, di,
               X[0], gmf);
    if (e != hipSuccess) return e;
    e = blas(st, &bh);
    if (e != hipSuccess) return e;
    for (int l = l1 ? 2 : 1; l < nl; ++l) {
        const int lin = s.layers[l - 1], lout = s.layers[l];
        const float* Wl = mlp + s.layer_off[l];
        e = blas_err(rocblas_sgemm(bh, rocblas_operation_none, rocblas_operation_none, lout, (int)n, lin, &one, Wl,
                                   lout, X[l - 1], lin, &zero, X[l], lout));
        if (e != hipSuccess) return e;
        launch(k_bias_relu, grid_for(n * lout), kBlock, 0, st, X[l], n * lout, lout, Wl + (int64_t)lin * lout);
    }
    const unsigned gb = (unsigned)((n + kBlock - 1) / kBlock);
    const int wo_off = s.layer_off[0];
    if (G % 4 == 0 && Ll % 4 == 0)
        launch(k_lay_out2<true>, gb, kBlock, 0, st, (const float*)gmf, (const float*)X[nl - 1], mlp + wo_off, G, Ll,
               users, items, ids, labels, n, 1.0f, probs, dzo, ones, at<float>(ws, L.part_bce));
    else
        launch(k_lay_out2<false>, gb, kBlock, 0, st, (const float*)gmf, (const float*)X[nl - 1], mlp + wo_off, G, Ll,
               users, items, ids, labels, n, 1.0f, probs, dzo, ones, at<float>(ws, L.part_bce));
    *nbce = labels ? (int)gb : 0;
    return hipGetLastError();
}

constexpr int kLayeredSlabs = 64;  // batch chunks of the weight-gradient GEMMs (<= kMaxSlabs)

bool layered_all_mfma(const ncf_shape_t& s) { return layer1_supported(s) && laymid_supported(s); }


hipError_t launch_fb_layered(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                             const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                             float inv_batch, IdSpace ids, int* nslab, int* nbce, hipStream_t st) {
    if (!layered_supported(s) || n > L.max_batch) return hipErrorInvalidValue;
    // (the rocBLAS handle only on the general-shape path below: none on config D's)
    rocblas_handle bh = nullptr;
    hipError_t e = hipSuccess;
    const int nl = s.num_layers, G = s.gmf_dim, G4 = s.gmf_stride, W = s.row_width;
    const int du = s.du, di = s.di, Ll = s.layers[nl - 1];
    const int wo_off = s.layer_off[0];
    const int B = (int)n;
    // activation matrices X_l [n x L_l] back to back in `act`, then GMF [n x G]; gradients G_l
    // [n x L_l] (l >= 1) in `dz`, then dz_out [n]; a ones vector [n] for the column sums
    float* act = at<float>(ws, L.act);
    float* dzb = at<float>(ws, L.dz);
    float* X[NCF_MAX_LAYERS];
    float* Gd[NCF_MAX_LAYERS];
    int64_t o = 0;
    for (int l = 0; l < nl; ++l) { X[l] = act + o; o += (int64_t)L.max_batch * s.layers[l]; }
    float* gmf = act + o;
    o = 0;
    Gd[0] = nullptr;
    for (int l = 1; l < nl; ++l) { Gd[l] = dzb + o; o += (int64_t)L.max_batch * s.layers[l]; }
    float* dzo = dzb + o;
    float* ones = at<float>(ws, L.ones);
    float* slab = at<float>(ws, L.slabs);
    float* probs = at<float>(ws, L.probs);
    float* gs = at<float>(ws, L.gs);
    const float one = 1.0f, zero = 0.0f;

    // float4 paths when every part of the row is float4-aligned (config D); float otherwise
    const bool vec4 = du % 4 == 0 && di % 4 == 0 && G == G4 && W % 4 == 0;
    // layer 1 forward (with the gather) and its data gradient (with the gradient-row scatter) on
    // hand-written MFMA (ncf_layer1.hip), where the shape has them
    const bool l1 = layer1_supported(s);
    const bool mid = l1 && laymid_supported(s);  // the middle kernel forms the GMF product itself
    if (l1)
        e = launch_layer1_fwd(s, emb, mlp, users, items, n, ids, X[0], mid ? nullptr : gmf, X[1], st);
    else if (vec4)
        launch(k_lay_gather4, grid_for(n * (du + di + G) / 4), kBlock, 0, st, (const float4*)emb, users, items, n, ids,
               W / 4, G / 4, du / 4, di / 4, (float4*)X[0], (float4*)gmf);
    else
        launch(k_lay_gather, grid_for(n * (du + di + G)), kBlock, 0, st, emb, users, items, n, ids, W, G, G4, du, di,
               X[0], gmf);
    if (e != hipSuccess) return e;
    if (mid) {
        // layers 2.., output, BCE and the backward to G1 (+ db1) in one kernel (ncf_laymid.hip), one
        // workgroup per batch chunk of the dW1 GEMM: slab c = that workgroup's parameters other than
        // dW1 + chunk c's dW1
        int64_t chunk = 256;
        while ((n + chunk - 1) / chunk > 256) chunk *= 2;
        const int nfull = (int)(n / chunk), rem = (int)(n - (int64_t)nfull * chunk);
        const int nsl = nfull + (rem > 0 ? 1 : 0);
        e = launch_laymid(s, mlp, X[1], emb, labels, users, items, n, ids, inv_batch, probs, dzo, Gd[1], slab,
                          at<float>(ws, L.part_bce), nsl, st);
        if (e != hipSuccess) return e;
        // dW1 on hand-written MFMA (ncf_layer1.hip), one workgroup per chunk
        e = launch_layer1_dw(s, X[0], Gd[1], n, chunk, nsl, slab, st);
        if (e != hipSuccess) return e;
        e = launch_layer1_bwd(s, emb, mlp, users, items, n, ids, (const float*)dzo, (const float*)Gd[1], gs, st);
        if (e != hipSuccess) return e;
        *nbce = nsl;
        *nslab = nsl;
        return hipGetLastError();
    }
    e = blas(st, &bh);
    if (e != hipSuccess) return e;
    for (int l = l1 ? 2 : 1; l < nl; ++l) {
        const int lin = s.layers[l - 1], lout = s.layers[l];
        const float* Wl = mlp + s.layer_off[l];
        // X_l^T (lout x n) = W_l^T (lout x lin) * X_{l-1}^T (lin x n), column-major views of row-major data
        e = blas_err(rocblas_sgemm(bh, rocblas_operation_none, rocblas_operation_none, lout, B, lin, &one, Wl, lout,
                                   X[l - 1], lin, &zero, X[l], lout));
        if (e != hipSuccess) return e;
        launch(k_bias_relu, grid_for(n * lout), kBlock, 0, st, X[l], n * lout, lout, Wl + (int64_t)lin * lout);
    }
    const unsigned gb = (unsigned)((n + kBlock - 1) / kBlock);
    if (G % 4 == 0 && Ll % 4 == 0)
        launch(k_lay_out2<true>, gb, kBlock, 0, st, (const float*)gmf, (const float*)X[nl - 1], mlp + wo_off, G, Ll,
               users, items, ids, labels, n, inv_batch, probs, dzo, ones, at<float>(ws, L.part_bce));
    else
        launch(k_lay_out2<false>, gb, kBlock, 0, st, (const float*)gmf, (const float*)X[nl - 1], mlp + wo_off, G, Ll,
               users, items, ids, labels, n, inv_batch, probs, dzo, ones, at<float>(ws, L.part_bce));
    launch(k_lay_gl, grid_for(n * Ll), kBlock, 0, st, (const float*)X[nl - 1], (const float*)dzo, mlp + wo_off + G, Ll,
           n * Ll, Gd[nl - 1]);
    *nbce = (int)gb;
    // Gradients that reduce over the batch (dW_l, db_l, output layer) are computed per chunk of
    // `chunk` samples into slab s (split-K by hand: a GEMM with K = batch and a 128 x 256
    // output has too few tiles to fill 256 CUs, and rocBLAS' own split-K is atomic); the
    // existing slab reduction sums the nslab slabs in a fixed order.
    int64_t chunk = 1024;
    while ((n + chunk - 1) / chunk > kLayeredSlabs) chunk *= 2;
    const int nfull = (int)(n / chunk), rem = (int)(n - (int64_t)nfull * chunk);
    const int64_t P = s.mlp_params;
    // y[s] (len m, stride P between slabs) = A[s] (m x k col-major, k = chunk samples) * x[s]
    auto gemv_parts = [&](int m, const float* A, const float* x, float* y) -> hipError_t {
        if (nfull > 0) {
            hipError_t r = blas_err(rocblas_sgemv_strided_batched(
                bh, rocblas_operation_none, m, (int)chunk, &one, A, m, (rocblas_stride)chunk * m, x, 1,
                (rocblas_stride)chunk, &zero, y, 1, (rocblas_stride)P, nfull));
            if (r != hipSuccess) return r;
        }
        if (rem > 0)
            return blas_err(rocblas_sgemv(bh, rocblas_operation_none, m, rem, &one, A + (int64_t)nfull * chunk * m, m,
                                          x + (int64_t)nfull * chunk, 1, &zero, y + (int64_t)nfull * P, 1));
        return hipSuccess;
    };
    // output-layer gradients: [GMF | X_{n-1}]^T dz, bias sum(dz)
    if (G > 0) {
        e = gemv_parts(G, gmf, dzo, slab + wo_off);
        if (e != hipSuccess) return e;
    }
    e = gemv_parts(Ll, X[nl - 1], dzo, slab + wo_off + G);
    if (e != hipSuccess) return e;
    e = gemv_parts(1, dzo, ones, slab + wo_off + G + Ll);
    if (e != hipSuccess) return e;
    for (int l = nl - 1; l >= 1; --l) {
        const int lin = s.layers[l - 1], lout = s.layers[l];
        const float* Wl = mlp + s.layer_off[l];
        float* dWl = slab + s.layer_off[l];
        // dW_l^T (lout x lin) = G_l^T (lout x chunk) * X_{l-1} (chunk x lin), per chunk
        if (nfull > 0) {
            e = blas_err(rocblas_sgemm_strided_batched(
                bh, rocblas_operation_none, rocblas_operation_transpose, lout, lin, (int)chunk, &one, Gd[l], lout,
                (rocblas_stride)chunk * lout, X[l - 1], lin, (rocblas_stride)chunk * lin, &zero, dWl, lout,
                (rocblas_stride)P, nfull));
            if (e != hipSuccess) return e;
        }
        if (rem > 0) {
            e = blas_err(rocblas_sgemm(bh, rocblas_operation_none, rocblas_operation_transpose, lout, lin, rem, &one,
                                       Gd[l] + (int64_t)nfull * chunk * lout, lout,
                                       X[l - 1] + (int64_t)nfull * chunk * lin, lin, &zero, dWl + (int64_t)nfull * P,
                                       lout));
            if (e != hipSuccess) return e;
        }
        // db_l = G_l^T 1
        e = gemv_parts(lout, Gd[l], ones, dWl + (int64_t)lin * lout);
        if (e != hipSuccess) return e;
        // G_{l-1}^T (lin x n) = W_l (lin x lout) * G_l^T (lout x n); layer 0: dX0 overwrites X0
        // (hand-written layer 1: dX straight into the gradient rows, below)
        if (l == 1 && l1) break;
        float* dst = l >= 2 ? Gd[l - 1] : X[0];
        e = blas_err(rocblas_sgemm(bh, rocblas_operation_transpose, rocblas_operation_none, lin, B, lout, &one, Wl,
                                   lout, Gd[l], lout, &zero, dst, lin));
        if (e != hipSuccess) return e;
        if (l >= 2) launch(k_relu_mask, grid_for(n * lin), kBlock, 0, st, Gd[l - 1], (const float*)X[l - 1], n * lin);
    }
    if (l1) {
        e = launch_layer1_bwd(s, emb, mlp, users, items, n, ids, (const float*)dzo, (const float*)Gd[1], gs, st);
        if (e != hipSuccess) return e;
    } else if (vec4)
        launch(k_lay_scatter4, grid_for(n * 2 * W / 4), kBlock, 0, st, (const float4*)emb, mlp, wo_off, users, items, n,
               ids, W / 4, G / 4, du / 4, di / 4, (const float*)dzo, (const float4*)X[0], (float4*)gs);
    else
        launch(k_lay_scatter, grid_for(n * 2 * W), kBlock, 0, st, emb, mlp, wo_off, users, items, n, ids, W, G, G4, du,
               di, (const float*)dzo, (const float*)X[0], gs);
    *nslab = nfull + (rem > 0 ? 1 : 0);
    return hipGetLastError();
}

}  // namespace ncf
