/*
 * movierec_ncf.h — C ABI of the MI355X-native NCF/NeuMF training hot path.
 *
 * This is the drop-in boundary below the Python mirror of the reference's
 * `movierec.model.MovierecModel` (see INTEGRATION.md for the ctypes binding).
 * The reference has no FFI of its own: its hot path is the Keras graph built
 * in movierec/model.py:135-215 and executed by Keras' training loop
 * (model.py:305-333).  Each entry point below names the reference behaviour it
 * replaces.
 *
 * Conventions
 *  - Every pointer argument that names device data is a caller-owned device
 *    pointer (allocated e.g. by PyTorch's caching allocator).  The library
 *    never allocates or frees device memory; scratch lives in a caller-provided
 *    workspace (ncf_workspace_size / ncf_workspace_init).
 *  - `stream` is a hipStream_t passed as void*; all work is enqueued on it, no
 *    call synchronises, so every call is hipGraph-capturable.
 *  - Return value: 0 = ok, NCF_EINVAL (-1) = invalid argument (the Python layer
 *    raises ValueError, like the reference's parameter checks model.py:77-112),
 *    NCF_EHIP (-2) = HIP error (RuntimeError).  The message is available from
 *    ncf_last_error() (thread-local).  No C++ exception crosses the ABI.
 *  - Process-wide state, all of it set once and idempotent: the kernels' dynamic-LDS
 *    attributes (set on first launch of each kernel variant), the NCF_* tuning knobs read from
 *    the environment on first use (NCF_SIDE_STREAM, NCF_FB_KERNEL, NCF_FOLD_USERS,
 *    NCF_UNIT_SCHED; experiments only), and the side streams of NCF_SIDE_STREAM (one per
 *    device, mutex-guarded).  Thread-local: the error text, the profiling events.  Calls on
 *    different workspaces may run concurrently from different threads.
 *  - Every kernel is hand-written HIP for gfx950; the library links no vendor BLAS.
 *
 * Device data layout (DESIGN.md §Data layout)
 *  - One combined embedding table `emb`: rows [0, num_users) are users, rows
 *    [num_users, num_users+num_items) are items; each row holds
 *    [gmf part (gmf_dim, padded to gmf_stride) | mlp part (du or di, padded)],
 *    `row_width` floats, 16-byte aligned rows.
 *  - `mlp`: flat fp32 vector of the dense parameters, Keras layouts:
 *    for l = 1..n-1: hidden_l kernel (layers[l-1] x layers[l], row-major) then
 *    hidden_l bias (layers[l]); then output kernel (out_features) and output
 *    bias (1).  out_features = gmf_dim + layers[n-1], ordered [gmf, mlp].
 */
#ifndef MOVIEREC_NCF_H
#define MOVIEREC_NCF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NCF_ABI_VERSION 11
#define NCF_MAX_LAYERS 8
#define NCF_EINVAL (-1)
#define NCF_EHIP (-2)

#define NCF_OPT_ADAM 0
#define NCF_OPT_SGD 1

/* stats accumulator layout (double[NCF_NUM_STATS], device) */
#define NCF_STAT_LOSS_SUM 0   /* sum over steps of batch loss (BCE mean + L2) */
#define NCF_STAT_HR_SUM 1     /* sum over steps of batch HR@k */
#define NCF_STAT_DCG_SUM 2    /* sum over steps of batch DCG@k */
#define NCF_STAT_STEPS 3      /* number of batches accumulated */
#define NCF_STAT_LAST_LOSS 4
#define NCF_STAT_LAST_HR 5
#define NCF_STAT_LAST_DCG 6
#define NCF_STAT_BCE_SUM 7    /* sum over steps of the batch BCE mean alone (Keras' output_loss) */
#define NCF_NUM_STATS 8

/* summary of one forward/backward (float[NCF_NUM_SUMMARY], device);
 * summed over ranks in data-parallel training */
#define NCF_SUM_BCE 0      /* sum over samples of per-sample BCE */
#define NCF_SUM_HIT 1      /* sum over groups of hit@k */
#define NCF_SUM_DCG 2      /* sum over groups of dcg@k */
#define NCF_SUM_GROUPS 3   /* number of groups */
#define NCF_SUM_REG 4      /* L2 loss of the current weights covered by this rank (forward_backward) */
#define NCF_NUM_SUMMARY 8

typedef struct ncf_shape {
    /* inputs (MovierecModel params: num_users, num_items, layers_sizes; gmf_dim = NeuMF extension) */
    int32_t num_users;
    int32_t num_items;
    int32_t num_layers;                 /* len(layers_sizes); 0 = GMF-only model (needs gmf_dim > 0) */
    int32_t gmf_dim;                    /* 0 = the reference's MLP-only model */
    int32_t layers[NCF_MAX_LAYERS];
    /* derived by ncf_shape_init */
    int32_t du, di;                     /* model.py:159-160 */
    int32_t gmf_stride;                 /* gmf_dim rounded up to 4 */
    int32_t row_width;                  /* floats per emb row */
    int64_t num_rows;                   /* num_users + num_items */
    int32_t out_features;               /* gmf_dim + layers[n-1] */
    int32_t mlp_params;                 /* length of the flat dense vector */
    int32_t layer_off[NCF_MAX_LAYERS];  /* [l] = offset of hidden_l kernel (l>=1); [0] = output kernel */
    int32_t fast_path;                  /* 1 if the fused MFMA kernel supports this shape */
    int32_t reserved[7];
} ncf_shape_t;

typedef struct ncf_model {
    float* emb;   /* num_rows x row_width */
    float* mlp;   /* mlp_params */
} ncf_model_t;

typedef struct ncf_optim {
    float* emb_m;
    float* emb_v;
    float* mlp_m;
    float* mlp_v;
    int32_t* step;   /* device: Keras `iterations` (optimizer steps taken so far) */
    /* Deferred exact decay (optional, NULL = sweep every row every step).  int32[num_rows]: the
     * optimizer steps row r has received.  ncf_train_step then updates only the batch's rows:
     * their missed zero-gradient steps are replayed (same arithmetic, so the result is bitwise
     * the dense sweep's) before the forward pass, then the step is applied to them.  Needs
     * layers_l2reg[0] == 0.  Every other entry point reads the table as stored: call
     * ncf_lazy_flush first.
     * row_step[r] == NCF_ROW_PRISTINE: row r's Adam moments are exactly +0 (a fresh table, or
     * rows set_optimizer_state found at zero).  Such a row is a fixed point of the zero-gradient
     * step (m = b1*0 + 0 = +0, v = +0, p -= (lr_t*0)/(sqrt(0)+eps) = p), so it is current at every
     * step: no replay, no flush traffic, and its first update reads p only.  Initialise row_step
     * to NCF_ROW_PRISTINE when the moments start at zero.
     * row_step[r] < 0 (set only by ncf_train_step_ahead's catch-up ahead, consumed by the next
     * step, ncf_lazy_flush or the stale-count gate): row r's p is current, its m and v are at step
     * -row_step[r] - 2 (the next update re-derives them).  Call ncf_lazy_flush before giving up a
     * counted-ahead batch (ncf_workspace_discard_counts). */
    int32_t* row_step;
} ncf_optim_t;

#define NCF_ROW_PRISTINE 0x7fffffff

typedef struct ncf_hyper {
    int32_t optimizer;                  /* NCF_OPT_ADAM / NCF_OPT_SGD (model.py:199-204) */
    float lr, beta_1, beta_2, epsilon;  /* epsilon: Keras K.epsilon() = 1e-7 */
    float l2[NCF_MAX_LAYERS];           /* layers_l2reg (model.py:163,168,178) */
    int32_t group;                      /* samples per user group (num_negs_per_pos + 1) */
    int32_t k;                          /* top-k of the hr/dcg metrics */
    float inv_batch;                    /* 1 / (global batch) for the BCE mean */
    int32_t force_generic;              /* 1: the generic per-sample kernel even if fast_path;
                                           2: the layer-by-layer MFMA path where the shape has it
                                           (config D's widths; the default there), else the
                                           generic kernel;
                                           3 / 4 / 5: (fast_path shapes) the 128-sample tile
                                           kernel / the sample-unit kernel (the default) / the
                                           wave-chain kernel (fp32 operands; else the unit one);
                                           6: the wave-chain kernel in its one-wave form (no
                                           separate weight-gradient waves) */
    int32_t index_ready;                /* 1: the contribution index of this call's batch was built
                                           beforehand by ncf_build_index (same ids, same ws): skip it;
                                           2: its contributions were counted and scanned by the
                                           previous ncf_train_step_ahead (same ids, same ws);
                                           3: its contributions were counted and scanned (and
                                           its own deferred rows caught up) by the previous
                                           ncf_user_dp_step[_split]; the step fills its index
                                           inside its forward/backward where it can */
    int32_t mlp_bf16;                   /* 1: the MLP tower's matrix products (forward, data and
                                           weight gradients) take bf16 operands with fp32
                                           accumulation; embeddings, GMF, loss, master weights
                                           and Adam stay fp32 (BASELINE config B; fast_path
                                           shapes, unit kernel only) */
    int32_t lazy_rows;                  /* deferred exact decay (optim->row_step) covers table rows
                                           [0, lazy_rows) only, 0 = every row; the rows past it are
                                           swept densely by the caller (the replicated item rows of
                                           user-partitioned data parallelism), and row_step needs
                                           lazy_rows entries */
    int32_t reserved[3];
} ncf_hyper_t;

int ncf_abi_version(void);

/* The forward/backward kernel a training call with n samples runs (for reporting). */
#define NCF_FB_GENERIC 0
#define NCF_FB_LAYERED 1        /* retired in ABI 11 (the rocBLAS layered path): never returned */
#define NCF_FB_TILE 2
#define NCF_FB_UNIT 3
#define NCF_FB_WAVE 4
#define NCF_FB_LAYERED_MFMA 5   /* the layer-by-layer path with every layer on hand-written MFMA (config D) */
int ncf_fb_kernel(const ncf_shape_t* shape, const ncf_hyper_t* hyper, int64_t n);
const char* ncf_last_error(void);

/* Provenance of the loaded library (ABI 11): a JSON object with the SHA-256 of the sources it was
 * compiled from (every .hip and .h source of csrc/ and this header, in name order, plus the
 * compiler flags), the -D defines of the build ("" for the product build), the offload arch and the ABI
 * version.  build.py recompiles whenever the hash of the tree differs from the one embedded. */
const char* ncf_build_info(void);

/* Validate the model dimensions and fill the derived fields.
 * Replaces the shape checks of MovierecModel.__init__ (model.py:73-80).  num_layers == 0 with
 * gmf_dim > 0 is the GMF-only model (BASELINE config A; an extension like the GMF branch):
 * p = sigmoid(w . (u_gmf * i_gmf) + b); `layers` may then be NULL. */
int ncf_shape_init(ncf_shape_t* shape, int32_t num_users, int32_t num_items, const int32_t* layers,
                   int32_t num_layers, int32_t gmf_dim);

/* Bytes of scratch needed for batches of up to max_batch samples. */
int ncf_workspace_size(const ncf_shape_t* shape, int64_t max_batch, size_t* bytes);
/* Zero the workspace's persistent region (call once after allocating it). */
int ncf_workspace_init(const ncf_shape_t* shape, int64_t max_batch, void* ws, size_t ws_bytes, void* stream);

/* Sticky error flags of the workspace's index builds, copied to flags (device int32) and cleared:
 *   NCF_WSERR_ID_RANGE     an index build met a user/item id outside the table (the kernels mask
 *                          such samples; the Python layer raises ValueError, like TF's gather)
 *   NCF_WSERR_STALE_COUNT  a batch passed with hyper->index_ready = 2 differed from the ids
 *                          ncf_train_step_ahead counted (their contents changed in between): the
 *                          index build wrote no slot outside its keys' ranges and cleared the
 *                          counters; with the in-kernel index (the single-table default) a step
 *                          whose changed ids reached a row that was not counted was dropped —
 *                          nothing of it applied, the state a consistent deferred-decay state —
 *                          and one whose changed ids only left counted rows short was applied
 *                          exactly on the ids passed (the unfilled list slots skipped); on the
 *                          other index paths that step's embedding gradient is wrong.
 *   NCF_WSERR_FOLD         an index built by an earlier call (ncf_build_index, ncf_shard_plan)
 *                          folds user rows differently than the step that used it (their hypers'
 *                          group / force_generic differ): that step's embedding gradient is wrong.
 * Nothing else in the library synchronises on them.  ncf_shard_workspace_flags reads the flags of
 * a row-sharded workspace (its layout depends on world).
 *
 * User-row folding: when the fused kernel runs and hyper->group is 2, 4 or 8, the user-row
 * gradients of a group's samples that share the group head's user (the reference's batches: one
 * positive + negs per user, data_pipeline.py:141) are summed inside the kernel and written once;
 * the index lists that one contribution.  Any batch stays exact (a sample with another user keeps
 * its own row); only the fp32 summation order of those rows changes. */
#define NCF_WSERR_ID_RANGE 1
#define NCF_WSERR_STALE_COUNT 4
#define NCF_WSERR_FOLD 8
int ncf_workspace_flags(const ncf_shape_t* shape, int64_t max_batch, void* ws, size_t ws_bytes, int32_t* flags,
                        void* stream);
int ncf_shard_workspace_flags(const ncf_shape_t* shape, int64_t max_batch, int32_t world, void* ws, size_t ws_bytes,
                              int32_t* flags, void* stream);
/* Drop the next batch's index counts that ncf_train_step_ahead took (the batch will not be
 * passed after all): clears the index counters only — the sticky error flags and the fold of the
 * last index build stay (ncf_workspace_init would clear them too).  Under deferred decay call
 * ncf_lazy_flush first: the counted batch's rows were caught up ahead with p only (row_step). */
int ncf_workspace_discard_counts(const ncf_shape_t* shape, int64_t max_batch, void* ws, size_t ws_bytes,
                                 void* stream);

/* Forward only: probs[n] = sigmoid output for (users[i], items[i]).
 * Replaces Model.predict_on_batch output[0] (model.py:184-194). */
int ncf_predict(const ncf_shape_t* shape, const ncf_model_t* model, const int32_t* users,
                const int32_t* items, int64_t n, float* probs, void* ws, size_t ws_bytes, void* stream);

/* RankLayer (model.py:344-352): per group of `group` consecutive probs, the
 * stable descending order (ties: lower index first). rank_idx[n_groups*group]. */
int ncf_rank(const float* probs, int64_t n_groups, int32_t group, int32_t* rank_idx, void* stream);

/* Per-group hit@k and dcg@k (model.py:361-455): label = argmax of the group's
 * labels, position = its place in the RankLayer order. hit/dcg[n_groups]. */
int ncf_group_metrics(const float* probs, const float* labels, int64_t n_groups, int32_t group, int32_t k,
                      float* hit, float* dcg, void* stream);

/* One full training step on one device (Keras train_on_batch, model.py:329-333):
 * forward, BCE, backward, deterministic embedding scatter-add and dense
 * Adam/SGD on every parameter, metrics.  Adds the batch loss/hr/dcg to
 * stats[] (double[NCF_NUM_STATS]) and increments optim->step.
 * probs_out (optional, may be NULL) receives the batch predictions. */
int ncf_train_step(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                   const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                   double* stats, float* probs_out, void* ws, size_t ws_bytes, void* stream);

/* ncf_train_step that also prepares the NEXT batch's index (next_users/next_items, n_next == n
 * samples): its contributions are counted by extra workgroups of this step's touched-row update
 * and its per-block key scan rides in this step's stats launch, so the next call — made with
 * hyper->index_ready = 2 and exactly these ids — skips both kernels.  Deferred-decay Adam only
 * (optim->row_step).  No other index-building call may come in between (the counters hold the
 * next batch's counts; ncf_workspace_init clears them). */
int ncf_train_step_ahead(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                         const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                         const int32_t* next_users, const int32_t* next_items, int64_t n_next, double* stats,
                         float* probs_out, void* ws, size_t ws_bytes, void* stream);

/* Validation batch (the evaluation pass Keras runs on validation_data inside
 * fit_generator, model.py:329-333): forward, BCE, hr/dcg over groups of
 * hyper->group; adds batch loss (BCE mean + L2 of the current weights), hr and
 * dcg to stats[] without touching the weights or optim->step. */
int ncf_evaluate(const ncf_shape_t* shape, const ncf_model_t* model, const ncf_hyper_t* hyper,
                 const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                 double* stats, float* probs_out, void* ws, size_t ws_bytes, void* stream);

/* Deferred exact decay: bring every row up to optim->step (replay its missed zero-gradient
 * Adam steps) and set row_step[r] = step (pristine rows stay NCF_ROW_PRISTINE: their state is
 * already the dense sweep's).  After it the table equals the dense-sweep state. */
int ncf_lazy_flush(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                   void* ws, size_t ws_bytes, void* stream);

/* Data-parallel split of ncf_train_step.
 * ncf_forward_backward computes this rank's gradients with the BCE mean taken
 * over hyper->inv_batch (= 1/global batch): dense embedding gradient
 * emb_grad[num_rows x row_width] (every row written, zeros where untouched),
 * mlp_grad[mlp_params], and summary[NCF_NUM_SUMMARY].  summary[NCF_SUM_REG]
 * holds the L2 loss of embedding rows [reg_row_begin, reg_row_begin +
 * reg_row_count) plus, if include_dense_reg, of the dense kernels — so that the
 * sum over ranks of disjoint row ranges is the full L2 term.  The caller sums
 * the gradients and the summary over ranks (RCCL reduce-scatter / all-reduce).
 * ncf_apply_update then applies the optimizer to embedding rows [row_begin,
 * row_begin + row_count) — emb_grad, optim->emb_m and optim->emb_v are
 * indexed from row_begin (a rank's shard; the whole table on one device) — and
 * to every dense parameter, folds the summary into stats[] and increments
 * optim->step.  Replicated data parallelism = reduce-scatter the dense
 * embedding gradient, update the own shard, all-gather the table. */
int ncf_forward_backward(const ncf_shape_t* shape, const ncf_model_t* model, const ncf_hyper_t* hyper,
                         const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                         float* emb_grad, float* mlp_grad, float* summary, float* probs_out,
                         int64_t reg_row_begin, int64_t reg_row_count, int32_t include_dense_reg,
                         void* ws, size_t ws_bytes, void* stream);
int ncf_apply_update(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                     int64_t row_begin, int64_t row_count, const float* emb_grad, const float* mlp_grad,
                     const float* summary, double* stats, void* ws, size_t ws_bytes, void* stream);

/* User-partitioned data parallelism (no reference counterpart — the
 * reference trains on one CPU).  The training ratings are partitioned by user:
 * rank r trains the users u % world == r, so rows [0, shared_row_begin) of its
 * table (its own users, local row u / world) are read and written by this rank
 * only, and rows [shared_row_begin, num_rows) (the items) are replicated.  A step:
 *   ncf_forward_backward_part  = ncf_forward_backward, but the dense embedding
 *                              gradient shared_grad is written for the replicated
 *                              rows only (indexed from shared_row_begin); the
 *                              per-sample gradient rows stay in ws
 *   all_reduce                 [shared_grad | mlp_grad | summary] (RCCL, async)
 *   ncf_update_rows            meanwhile: fused scatter-add + optimizer of the own
 *                              rows [row_begin, row_begin + row_count) from the
 *                              per-sample rows in ws (n = the batch size given to
 *                              ncf_forward_backward_part, which fixes where they
 *                              sit in ws; optim->emb_m/emb_v indexed
 *                              by table row; step *optim->step + 1, not bumped)
 *   ncf_apply_update           the replicated rows (row_begin = shared_row_begin,
 *                              moments pointers offset to that row), the dense
 *                              layers, stats, step++.
 * The result equals ncf_train_step on the concatenated global batch up to fp32
 * summation order of the cross-rank sum. */
int ncf_forward_backward_part(const ncf_shape_t* shape, const ncf_model_t* model, const ncf_hyper_t* hyper,
                              const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                              int64_t shared_row_begin, float* shared_grad, float* mlp_grad, float* summary,
                              float* probs_out, int64_t reg_row_begin, int64_t reg_row_count,
                              int32_t include_dense_reg, void* ws, size_t ws_bytes, void* stream);
int ncf_update_rows(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                    int64_t n, int64_t row_begin, int64_t row_count, void* ws, size_t ws_bytes, void* stream);
/* Build the contribution index of the NEXT batch (users/items, n samples) into ws ahead of time,
 * e.g. while the current step's all-reduce is in flight: the call replaces the index of the
 * previous batch, so it must follow that batch's ncf_update_rows on the stream.  The next
 * ncf_forward_backward_part / ncf_forward_backward with hyper->index_ready = 1 then skips its own
 * index build (the caller guarantees it passes the same ids).  hyper: that call's hyper (its group
 * and force_generic decide the user-row folding; NULL = none); a mismatch sets NCF_WSERR_FOLD. */
int ncf_build_index(const ncf_shape_t* shape, const ncf_hyper_t* hyper, const int32_t* users, const int32_t* items,
                    int64_t n, void* ws, size_t ws_bytes, void* stream);

/* The user-partitioned step with deferred exact decay of the own rows [0, hyper->lazy_rows) (the
 * rank's users; optim->row_step has lazy_rows entries; embedding L2 off), the rest as above:
 *   ncf_forward_backward_part_lazy  ncf_forward_backward_part with shared_row_begin =
 *                              hyper->lazy_rows; the batch's own rows are caught up on their
 *                              missed zero-gradient steps before the forward pass (nothing to do
 *                              with hyper->index_ready = 2: the previous ncf_update_rows_lazy counted
 *                              this batch and caught its rows up ahead; 3: the previous
 *                              ncf_user_dp_step also finished its index)
 *   all_reduce                 [shared_grad | mlp_grad | summary] (RCCL, async)
 *   ncf_update_rows_lazy       meanwhile: the touched own rows' scatter-add + Adam at step
 *                              *optim->step + 1 (row_step set; step not bumped); with next ids
 *                              (n_next == n, Adam) the same launch counts the next batch's index
 *                              and catches its own rows up ahead, then its key scan runs
 *   ncf_apply_update           the replicated rows (dense sweep), dense layers, stats, step++.
 * Bitwise the same table as the dense-sweep user-partitioned step after ncf_lazy_flush (which
 * flushes rows [0, lazy_rows) only). */
int ncf_forward_backward_part_lazy(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim,
                                   const ncf_hyper_t* hyper, const int32_t* users, const int32_t* items,
                                   const float* labels, int64_t n, float* shared_grad, float* mlp_grad, float* summary,
                                   float* probs_out, int32_t include_dense_reg, void* ws, size_t ws_bytes,
                                   void* stream);
int ncf_update_rows_lazy(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                         int64_t n, const int32_t* next_users, const int32_t* next_items, int64_t n_next, void* ws,
                         size_t ws_bytes, void* stream);

/* Native communicator (RCCL inside the library; no reference counterpart).  The ranks come from
 * the caller's process group: rank 0 takes an id with ncf_comm_unique_id (128 bytes), the caller
 * broadcasts it, every rank calls ncf_comm_init on its device (a collective: it blocks until all
 * ranks joined).  The communicator owns a side stream for its collective.
 *   ncf_comm_allreduce   in-place fp32 sum over the ranks, ordered after the work enqueued on
 *                        `stream` so far; `stream` waits for it.
 *   ncf_user_dp_step     the user-partitioned step with deferred decay in ONE call:
 *                        ncf_forward_backward_part_lazy, the all-reduce of shared =
 *                        [item-row gradient (num_rows - lazy_rows rows) | dense-layer gradient |
 *                        summary] on the side stream while the compute stream runs
 *                        ncf_update_rows_lazy (next ids optional), then ncf_apply_update of the
 *                        item rows (moments indexed by table row) and the dense layers, stats,
 *                        step++.  With next ids the next batch's index is also filled and sorted
 *                        under the collective: pass those very ids next call with
 *                        hyper->index_ready = 3 (the index is trusted: contents must not change in
 *                        between; 0 = build it now).  Bitwise the same as those calls made one by
 *                        one with any other all-reduce of the same sums. */
int ncf_comm_unique_id(void* id, size_t bytes);
int ncf_comm_init(int32_t world, int32_t rank, const void* id, size_t bytes, void** comm);
int ncf_comm_destroy(void* comm);
int ncf_comm_allreduce(void* comm, float* buf, int64_t count, void* stream);
int ncf_user_dp_step(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                     const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                     const int32_t* next_users, const int32_t* next_items, int64_t n_next, float* shared,
                     int32_t include_dense_reg, void* comm, double* stats, void* ws, size_t ws_bytes, void* stream);
/* ncf_user_dp_step with the item rows' Adam split across the ranks (item_world = the
 * communicator's ranks, item_rank = this rank; Ic = ceil(items / item_world)): shared = [item-row
 * gradient, item_world * Ic rows (rows past the items zero) | dense-layer gradient | summary];
 * model->emb holds lazy_rows + item_world * Ic rows (zero padding past num_rows).  On the side
 * stream one RCCL group reduce-scatters the item-row gradient (this rank's Ic rows into
 * slice_grad, Ic x row_width floats) and all-reduces [dense-layer gradient | summary] while the
 * compute stream runs the own-user update and the next index; then Adam on this rank's item
 * rows [lazy_rows + item_rank * Ic, + Ic) and the dense layers, stats, step++; then an in-place
 * all-gather of the item rows before the call returns control of the stream.  Same bytes on the
 * links as the all-reduce; the item Adam per rank is 1/item_world of the table.  A one-rank
 * communicator with item_world > 1 runs rank item_rank's compute of that step without the
 * exchange (slice_grad unused).  item_world == 1: bitwise ncf_user_dp_step. */
int ncf_user_dp_step_split(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                           const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                           const int32_t* next_users, const int32_t* next_items, int64_t n_next, float* shared,
                           float* slice_grad, int32_t item_world, int32_t item_rank, int32_t include_dense_reg,
                           void* comm, double* stats, void* ws, size_t ws_bytes, void* stream);
/* Exchange timing of the one-call steps (ABI 10; the bench's multi-GPU diagnostic).  every > 0:
 * from the next call on, every every-th ncf_user_dp_step[_split] records timing events — on the
 * side stream around its reduce-scatter + all-reduce group (or its all-reduce) and around its
 * all-gather, on the compute stream around its two join waits; every = 0 stops.
 * ncf_comm_timing_read waits for the recorded events and returns, summed over the sampled steps
 * since the last read, out[0] = ms of the reduce-scatter + all-reduce on the side stream, out[1]
 * = ms of the all-gather, out[2] = ms the compute stream waited for the former (exposed), out[3] =
 * ms it waited for the all-gather; *steps = the sampled steps (then cleared). */
int ncf_comm_timing(void* comm, int32_t every);
int ncf_comm_timing_read(void* comm, double* out4, int64_t* steps);

/* Row-sharded data parallelism (no reference counterpart — the
 * reference trains on one CPU).  Rank r of `world` (1..16) owns the table rows g
 * (users 0..U-1, items U..U+I-1) with g % world == r, stored at local row
 * g / world of its (shard_rows x row_width) shard, shard_rows = ceil(R/world),
 * with the Adam moments of those rows.  Dense parameters are replicated.  A step:
 *   ncf_shard_plan            unique rows of the local batch, grouped by owner
 *                             (uniq_rows[] = local row ids at the owner,
 *                             send_counts[world]); compact ids kept in ws
 *   all_to_all (host, RCCL)   row ids to their owners
 *   ncf_gather_rows           owner: rows requested by every rank
 *                             (ncf_shard_serve_rows under deferred decay)
 *   all_to_all                row values back, in uniq_rows order
 *   ncf_shard_forward_backward  fused forward/backward on the unique rows:
 *                             per-unique-row gradient uniq_grad, dense-layer
 *                             gradient, summary
 *   all_to_all                unique-row gradients to their owners;
 *                             all_reduce of the dense gradient and summary
 *   ncf_shard_apply_update    owner: sums the received gradients per row in
 *                             ascending source order, Adam/SGD over its whole
 *                             shard (dense semantics, F5) and the dense layers
 * The result equals ncf_train_step on the concatenated global batch up to fp32
 * summation order; with world == 1 it is bitwise identical.
 * The workspace comes from ncf_shard_workspace_size / _init (not
 * ncf_workspace_size) and must be used with the same world. */
int ncf_shard_rows(const ncf_shape_t* shape, int32_t world, int64_t* rows);
int ncf_shard_workspace_size(const ncf_shape_t* shape, int64_t max_batch, int32_t world, size_t* bytes);
int ncf_shard_workspace_init(const ncf_shape_t* shape, int64_t max_batch, int32_t world, void* ws, size_t ws_bytes,
                             void* stream);
/* uniq_rows: int32[2n] capacity, send_counts: int32[world] (device).  hyper: the hyper of the
 * ncf_shard_forward_backward that follows (user-row folding, as ncf_build_index); NULL for a
 * plan that only feeds ncf_shard_predict. */
int ncf_shard_plan(const ncf_shape_t* shape, const ncf_hyper_t* hyper, int32_t world, const int32_t* users,
                   const int32_t* items, int64_t n, int32_t* uniq_rows, int32_t* send_counts, void* ws,
                   size_t ws_bytes, void* stream);
/* out[j] = table[rows[j]] for j < m (rows outside [0, table_rows) give zero rows). */
int ncf_gather_rows(const ncf_shape_t* shape, const float* table, int64_t table_rows, const int32_t* rows, int64_t m,
                    float* out, void* stream);
/* model->emb = the plan's unique rows (in uniq_rows order), model->mlp the dense
 * parameters; uniq_grad: float[2n x row_width] capacity.  reg_table/reg_rows:
 * this rank's shard, whose L2 loss goes into summary[NCF_SUM_REG]. */
int ncf_shard_forward_backward(const ncf_shape_t* shape, const ncf_model_t* model, const ncf_hyper_t* hyper,
                               int32_t world, const float* labels, int64_t n, float* uniq_grad, float* mlp_grad,
                               float* summary, float* probs_out, const float* reg_table, int64_t reg_rows,
                               int32_t include_dense_reg, void* ws, size_t ws_bytes, void* stream);
/* Deferred exact decay of the shard (optim->row_step: int32[shard_rows], NCF_ROW_PRISTINE for
 * fresh rows; Adam; embedding L2 off).  The owner serves the m rows requested by every rank
 * (rows[m] = local row ids, concatenated in source-rank order; a source lists a row once): it
 * builds the owner index of those entries (its own workspace regions: the plan's index
 * survives), replays the served rows' missed zero-gradient steps (p; m, v follow in the update),
 * and gathers out[j] = shard row rows[j].  The ncf_shard_apply_update of the same step then
 * updates exactly those rows through that index (recv_grad in the order of rows[]) — bitwise
 * the dense shard sweep's result, moving only the served rows.  Replaces ncf_gather_rows on the
 * owner side of the step. */
int ncf_shard_serve_rows(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                         int32_t world, const int32_t* rows, int64_t m, float* out, void* ws, size_t ws_bytes,
                         void* stream);
/* Deferred decay: bring every shard row up to optim->step (ncf_lazy_flush of the shard). */
int ncf_shard_flush(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                    int32_t world, void* ws, size_t ws_bytes, void* stream);
/* model->emb / optim->emb_m / emb_v = this rank's shard; recv_rows[m] /
 * recv_grad[m x row_width] = the rows requested by (and gradients from) every
 * rank, concatenated in source-rank order; mlp_grad and summary summed over ranks.
 * With optim->row_step (deferred decay) only the rows of the step's ncf_shard_serve_rows are
 * updated (recv_rows is not read again); else every shard row is swept. */
int ncf_shard_apply_update(const ncf_shape_t* shape, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* hyper,
                           int32_t world, const int32_t* recv_rows, const float* recv_grad, int64_t m,
                           const float* mlp_grad, const float* summary, double* stats, void* ws, size_t ws_bytes,
                           void* stream);
/* Predictions for the batch of the last ncf_shard_plan (model->emb = its unique rows). */
int ncf_shard_predict(const ncf_shape_t* shape, const ncf_model_t* model, int32_t world, int64_t n, float* probs,
                      void* ws, size_t ws_bytes, void* stream);

/* All-item scoring + top-k (BASELINE config E).  Replaces the serving workload of
 * trt_client.py:43-57 (score items for a user with the exported model's
 * output/Sigmoid, keep the K = 10 best by np.argsort) for a whole list of users
 * against the whole catalogue.  For q < n_users: top_items[q*k .. q*k+k) = the k
 * items with the highest score for user users[q], best first, ties broken by the
 * lower item id; top_scores = their sigmoid output.  Entries past the catalogue
 * (k > num_items) and users outside [0, num_users) give item -1, score 0.
 *   NCF_SCORE_FP16: fp16 operands, fp32 accumulation on MFMA (v_mfma_f32_32x32x16_f16),
 *                   ranked by the logit; shapes where ncf_score_supported() is 1 only.
 *   NCF_SCORE_FP32: the fp32 forward of ncf_predict, ranked by probability; any shape
 *                   (slow: one generic forward per pair).
 * 1 <= k <= NCF_SCORE_MAX_K; n_users <= the max_users the workspace was sized for. */
#define NCF_SCORE_FP16 0
#define NCF_SCORE_FP32 1
#define NCF_SCORE_MAX_K 32
int ncf_score_supported(const ncf_shape_t* shape, int32_t precision);
int ncf_score_workspace_size(const ncf_shape_t* shape, int64_t max_users, size_t* bytes);
int ncf_score_topk(const ncf_shape_t* shape, const ncf_model_t* model, const int32_t* users, int64_t n_users,
                   int32_t k, int32_t precision, int32_t* top_items, float* top_scores, void* ws, size_t ws_bytes,
                   void* stream);

/* On-device negative sampling + batch assembly.  Replaces
 * MovieLensDataGenerator.__getitem__ (data_pipeline.py:115-150): for the n_pos positives
 * order[first .. first+n_pos) (indexes into pos_users/pos_items, the epoch's shuffled order,
 * data_pipeline.py:136,152-154), group g of the batch is users [u]*(negs+1), items
 * [neg_1 .. neg_negs, pos], labels [0]*negs + [1] (data_pipeline.py:141-148).  Negatives are
 * uniform over the items in [0, num_items) absent from the user's excluded list
 * (excl_items[excl_ptr[u] .. excl_ptr[u+1]), ascending and unique: the user's positives in
 * data + extra, data_pipeline.py:103-108), distinct within a group unless the user has fewer
 * candidates than negs (data_pipeline.py:111-112).  Random stream: counter-based
 * Philox4x32-10 keyed by (seed, stream), counted by the positive's slot in the order — NOT
 * numpy's stream (the host generator keeps the reference-exact mode).
 * err (device int32, OR-ed): 1 user id out of range, 2 user without candidates (item -1;
 * the reference raises), 4 attempt bound hit (a deterministic pick was used). */
typedef struct ncf_sampler_data {
    const int32_t* pos_users;   /* [num_pos] */
    const int32_t* pos_items;   /* [num_pos] */
    int64_t num_pos;
    const int32_t* excl_ptr;    /* [num_users + 1] */
    const int32_t* excl_items;  /* [excl_ptr[num_users]] */
    int32_t num_users;
    int32_t num_items;
} ncf_sampler_data_t;
int ncf_sample_batch(const ncf_sampler_data_t* data, const int32_t* order, int64_t first, int32_t n_pos,
                     int32_t negs, uint64_t seed, uint64_t stream, int32_t* x_user, int32_t* x_item, float* labels,
                     int32_t* err, void* hip_stream);

/* Profiling hook (bench.py): while enabled, every launch of a group whose bit
 * is set in `kernel_mask` (bit NCF_K_*) issued by this thread is bracketed by
 * HIP events on its own stream (up to `capacity` launches per group);
 * ncf_profile_read synchronises on the group's last event and returns the
 * summed device time (ms) and the number of launches, then resets that group.
 * kernel_mask <= 0 disables. */
#define NCF_K_INDEX 1       /* count + scan + fill + segment sorts */
#define NCF_K_FWD_BWD 2     /* gather + GMF + MLP fwd + BCE + MLP bwd (+ dense-weight partials) */
#define NCF_K_EMB_UPDATE 3  /* embedding scatter-add + optimizer sweep */
#define NCF_K_MLP_UPDATE 4  /* dense-weight gradient reduction + optimizer */
#define NCF_K_METRICS 5     /* hr/dcg + loss summary */
#define NCF_K_SCORE 6       /* all-item scoring + top-k (MFMA kernel only, not its preparation) */
#define NCF_K_SAMPLE 7      /* on-device negative sampling + batch assembly */
#define NCF_K_CATCHUP 8     /* deferred decay: replay of the batch's stale rows before the forward pass
                             * (NCF_K_EMB_UPDATE then times the touched-row update only) */
int ncf_profile_enable(int32_t kernel_mask, int32_t capacity);
int ncf_profile_read(int32_t kernel_id, double* total_ms, int64_t* launches);
/* paused != 0: launches carry no events (and take no slots) until resumed; the
 * slots already taken are kept.  bench.py times a sample of the steps of its
 * timed region this way, because the events in the dispatch packets lengthen a
 * step (measured 16 us on the config-C step). */
int ncf_profile_pause(int32_t paused);
/* Of the enabled groups, only those in kernel_mask attach events from now on (all of them after
 * ncf_profile_enable); slots already taken are kept.  bench.py times one group per sampled step,
 * so a sampled step carries one pair of events instead of one per group. */
int ncf_profile_select(int32_t kernel_mask);

#ifdef __cplusplus
}
#endif

#endif /* MOVIEREC_NCF_H */
