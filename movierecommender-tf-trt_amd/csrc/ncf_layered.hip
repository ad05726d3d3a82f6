// Layer-by-layer forward / backward for shapes whose dense weights do not fit the fused
// kernel's LDS budget (config D: MLP [256,128,64,32] + GMF 128, 174 KB of weights).
//
// The fused kernels (ncf_wave.hip, ncf_unit.hip, ncf_fused.hip) keep every weight in LDS and
// every activation in registers; past ~45 KB of weights that stops fitting.  Here the batch goes
// through three hand-written fp32 MFMA kernels plus one for dW1, each weight matrix staged in LDS
// by the kernel that uses it:
//
//   k_lay_l1f  (ncf_layer1.hip)  gather + layer 1: X0 = [E_u_mlp | E_i_mlp], H1 = relu(X0 W1 + b1)
//                                 (model.py:161-181)
//   k_lay_mid  (ncf_laymid.hip)  layers 2.., output, sigmoid, Keras BCE, dz, back to G1; dW2.., the
//                                 biases and the output-layer gradients (model.py:175-188, 213-214)
//   k_lay_dw1  (ncf_layer1.hip)  dW1 = X0^T G1, one batch chunk per workgroup pair
//   k_lay_l1b  (ncf_layer1.hip)  dX0 = G1 W1^T straight into the per-sample gradient rows, with the
//                                 GMF part dz w_gmf * (the other side's GMF vector); a group's user
//                                 rows folded into its head's (user-row folding, as the fused kernels)
//
// The outputs are exactly those of the other forward/backward kernels (probs, gs, part_bce, one
// dense-gradient slab per batch chunk), so the index build, the optimizer sweeps and the data-
// parallel paths are shared.  Shapes that neither the fused nor these kernels hold run the
// per-sample generic kernel (ncf_generic.hip): there is no vendor-GEMM path in the library.

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

bool layered_supported(const ncf_shape_t& s) { return s.num_layers >= 2 && layer1_supported(s) && laymid_supported(s); }

bool layered_all_mfma(const ncf_shape_t& s) { return layered_supported(s); }

// Forward only (ncf_predict / ncf_evaluate on the layered shape): layer 1 with the gather, then
// layers 2.., the output and (labels given) the Keras BCE partials in the middle kernel's
// forward-only form, one partial per workgroup in part_bce (*nbce).  Same arithmetic as the
// forward half of launch_fb_layered, so evaluation matches training's forward.
hipError_t launch_predict_layered(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                                  const float* mlp, const int32_t* users, const int32_t* items, const float* labels,
                                  int64_t n, float* probs, IdSpace ids, int* nbce, hipStream_t st) {
    if (!layered_supported(s) || n > L.max_batch) return hipErrorInvalidValue;
    const int nl = s.num_layers;
    float* act = at<float>(ws, L.act);
    float* X[NCF_MAX_LAYERS];
    int64_t o = 0;
    for (int l = 0; l < nl; ++l) { X[l] = act + o; o += (int64_t)L.max_batch * s.layers[l]; }
    hipError_t e = launch_layer1_fwd(s, emb, mlp, users, items, n, ids, X[0], nullptr, X[1], st);
    if (e != hipSuccess) return e;
    const int64_t units = (n + 15) / 16;
    const int grid = (int)(units >= 8 * 512 ? 512 : (units + 7) / 8);
    e = launch_laymid(s, mlp, X[1], emb, labels, users, items, n, ids, 1.0f, probs, nullptr, nullptr, nullptr,
                      at<float>(ws, L.part_bce), grid, st);
    *nbce = labels ? grid : 0;
    return e;
}

hipError_t launch_fb_layered(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                             const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                             float inv_batch, IdSpace ids, int* nslab, int* nbce, hipStream_t st, int fold) {
    if (!layered_supported(s) || n > L.max_batch) return hipErrorInvalidValue;
    const int nl = s.num_layers;
    // activation matrices X_l [n x L_l] back to back in `act`; gradients G_l [n x L_l] (l >= 1) in
    // `dz`, then dz_out [n]
    float* act = at<float>(ws, L.act);
    float* dzb = at<float>(ws, L.dz);
    float* X[NCF_MAX_LAYERS];
    float* Gd[NCF_MAX_LAYERS];
    int64_t o = 0;
    for (int l = 0; l < nl; ++l) { X[l] = act + o; o += (int64_t)L.max_batch * s.layers[l]; }
    const int64_t xend = o;
    o = 0;
    Gd[0] = nullptr;
    for (int l = 1; l < nl; ++l) { Gd[l] = dzb + o; o += (int64_t)L.max_batch * s.layers[l]; }
    float* dzo = dzb + o;
    float* slab = at<float>(ws, L.slabs);
    float* probs = at<float>(ws, L.probs);
    float* gs = at<float>(ws, L.gs);
    // the group-user form's P_u rows ([n / fold][L1]) behind the activations (the region's last
    // gmf_dim columns per sample are unused on this path)
    const int64_t gfree = (int64_t)L.max_batch * L.act_w - xend;
    float* gpart = fold > 1 && gfree * fold >= (int64_t)L.max_batch * s.layers[1] ? act + xend : nullptr;
    // layer 1 forward with the gather (the middle kernel forms the GMF product itself)
    hipError_t e = launch_layer1_fwd(s, emb, mlp, users, items, n, ids, X[0], nullptr, X[1], st, fold, gpart);
    if (e != hipSuccess) return e;
    // layers 2.., output, BCE and the backward to G1 (+ db1) in one kernel, one workgroup per batch
    // chunk of dW1: slab c = that workgroup's parameters other than dW1 + chunk c's dW1
    int64_t chunk = 256;
    while ((n + chunk - 1) / chunk > 256) chunk *= 2;
    const int nfull = (int)(n / chunk), rem = (int)(n - (int64_t)nfull * chunk);
    const int nsl = nfull + (rem > 0 ? 1 : 0);
    e = launch_laymid(s, mlp, X[1], emb, labels, users, items, n, ids, inv_batch, probs, dzo, Gd[1], slab,
                      at<float>(ws, L.part_bce), nsl, st);
    if (e != hipSuccess) return e;
    // (the group form of dW1 needs the group form's X0: both follow gpart)
    e = launch_layer1_dw(s, X[0], Gd[1], n, chunk, nsl, slab, st, gpart ? fold : 0, users, items, ids);
    if (e != hipSuccess) return e;
    e = launch_layer1_bwd(s, emb, mlp, users, items, n, ids, (const float*)dzo, (const float*)Gd[1], gs, st, fold);
    if (e != hipSuccess) return e;
    *nbce = nsl;
    *nslab = nsl;
    return hipGetLastError();
}

}  // namespace ncf
