// Internal declarations shared by the HIP translation units of libmovierec_ncf.
// Not part of the ABI (see include/movierec_ncf.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "movierec_ncf.h"

namespace ncf {

constexpr int kBlock = 256;            // threads per workgroup for the streaming kernels
constexpr int kScanBlock = 2048;       // keys per block of the offset scan (8 per thread)
constexpr int kSmallSeg = 16;          // segments up to this length are sorted in registers
constexpr int kMaxSlabs = 1024;        // partial dense-gradient slabs (one per producing block)
constexpr int kSlabSplit = 16;         // first-level slab reduction fan-in groups
constexpr int kUpdateGrid = 2048;      // grid of the embedding-table sweep (fixed: deterministic partials)
constexpr int64_t kMaxBatch = 262144;  // heavy-segment bitmap must fit the LDS (2*B bits = 64 KB)

// Scalars every kernel of a step reads (device copy of hyper + derived).
struct StepScalars {
    int32_t t;       // optimizer iteration being applied (1-based)
    float lr_t;      // Adam bias-corrected lr (Keras v1 formula)
};

// Byte offsets of the workspace regions (host-computed, passed by value).
struct WsLayout {
    size_t cnt;       // int32[R+1]  persistent, all-zero between calls
    size_t heavy_n;   // int32       persistent
    size_t err;       // int32       persistent (sticky id-out-of-range flag)
    size_t persistent_end;
    size_t probs;     // float[B]
    size_t gs;        // float[2B * W] per-contribution gradient rows
    size_t list;      // int32[2B]   contributions grouped by table row (sorted inside a row)
    size_t offs_local;// int32[R+1]  per-2048-row local exclusive scan
    size_t offs;      // int32[R+1]  row -> first list slot
    size_t tot;       // int32[nscan]
    size_t heavy;     // int32[2B]
    size_t part_bce;  // float[kMaxSlabs]
    size_t part_hit;  // float[nmetric]
    size_t part_dcg;  // float[nmetric]
    size_t part_reg;  // float[kUpdateGrid + mlp blocks]
    size_t summary;   // float[NCF_NUM_SUMMARY]
    size_t slabs;     // float[kMaxSlabs * P]
    size_t mlp_grad;  // float[P] (reduced dense-layer gradient, single-device path)
    size_t slab_part; // float[kSlabSplit * P] first-level slab sums
    size_t act;       // float[B * A] generic kernel activations
    size_t dz;        // float[B * D] generic kernel pre-activation gradients
    size_t total;
    int64_t max_batch;
    int nscan;        // blocks of the offset scan
    int nmetric;      // max blocks of the metrics kernel
    int act_w;        // A
    int dz_w;         // D
};

WsLayout make_layout(const ncf_shape_t& s, int64_t max_batch);

template <typename T>
__host__ __device__ inline T* at(void* base, size_t off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}

// Launchers (return hipError_t of the launch). ------------------------------

// index build: contribution c = 2*i + side (0 user row, 1 item row) grouped by table row
hipError_t launch_index_build(const ncf_shape_t& s, const WsLayout& L, void* ws, const int32_t* users,
                              const int32_t* items, int64_t n, hipStream_t st);

// forward+backward, generic per-sample kernel: writes probs, gs rows, bce partials, dense slabs.
// returns number of slabs written in *nslab, bce partial count in *nbce
hipError_t launch_fb_generic(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                             const float* mlp, const int32_t* users, const int32_t* items,
                             const float* labels, int64_t n, float inv_batch, int* nslab, int* nbce,
                             hipStream_t st);
// forward only; with labels also writes per-block BCE partials (*nbce of them)
hipError_t launch_predict_generic(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                                  const float* mlp, const int32_t* users, const int32_t* items,
                                  const float* labels, int64_t n, float* probs, int* nbce, hipStream_t st);

// fused MFMA forward+backward (shapes with s.fast_path); same outputs as the generic kernel
// also computes the hr/dcg group metrics in-kernel when group divides 32 (*nmet = partial count, else 0)
hipError_t launch_fb_fused(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                           const float* mlp, const int32_t* users, const int32_t* items, const float* labels,
                           int64_t n, float inv_batch, int group, int topk, int* nslab, int* nbce, int* nmet,
                           hipStream_t st);
bool fused_supported(const ncf_shape_t& s);

// metrics / summaries
hipError_t launch_group_metrics(const float* probs, const float* labels, int64_t n_groups, int group, int k,
                                float* hit, float* dcg, float* part_hit, float* part_dcg, int* nparts,
                                hipStream_t st);
hipError_t launch_rank(const float* probs, int64_t n_groups, int group, int32_t* rank_idx, hipStream_t st);
hipError_t launch_summary(const WsLayout& L, void* ws, int nbce, int nmet, float n_groups, int nreg_emb,
                          int nreg_mlp, float* summary, hipStream_t st);

// updates
enum GradSource { kGradSparse = 0, kGradDense = 1 };
hipError_t launch_emb_update(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m, float* v,
                             const int32_t* step, const ncf_hyper_t& h, const float* dense_grad, int64_t rows,
                             hipStream_t st);
hipError_t launch_emb_grad_dense(const ncf_shape_t& s, const WsLayout& L, void* ws, float* out, hipStream_t st);
// mlp: reduce slabs (if nslab > 0) or read grad_in; optionally write grad_out; optionally update
hipError_t launch_mlp_update(const ncf_shape_t& s, const WsLayout& L, void* ws, float* mlp, float* m, float* v,
                             const int32_t* step, const ncf_hyper_t& h, int nslab, const float* grad_in,
                             float* grad_out, bool do_update, int* nreg, hipStream_t st, bool want_reg = false);
hipError_t launch_emb_reg(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, int64_t rows,
                          float lam, hipStream_t st);
hipError_t launch_stats(const WsLayout& L, void* ws, const float* summary, int nreg_emb, int nreg_mlp,
                        float inv_batch, double* stats, int32_t* step, bool bump_step, hipStream_t st);

}  // namespace ncf
