// RCCL inside the library: the data-parallel step's one collective enqueued by the same host call
// that enqueues its kernels (include/movierec_ncf.h "Native communicator").
//
// torch.distributed's process group forms the ranks and carries the RCCL unique id; the step's
// all-reduce then goes straight to RCCL on a side stream of this library (fork/join by events),
// beside the own-user update on the compute stream.  Per step that is one host call instead of
// the five Python-level calls (and the c10d collective's own host work) of the same step driven
// from Python — the user-partitioned step was host-issue-bound that way (a ~300 us host step
// against ~150 us of kernels at an emulated 8 ranks, rocprofv3 timeline, profiles/r03_user).
//
// librccl.so.1 is the soname the PyTorch build loads too: one RCCL serves the process.

#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "movierec_ncf.h"
#include "ncf_internal.h"

namespace {

// timing events of one sampled step: side stream c0..c1 (reduce-scatter + all-reduce), a0..a1
// (all-gather); compute stream j0..j1 (its wait for the former), g0..g1 (for the all-gather)
struct StepEvents {
    hipEvent_t e[8] = {};
    bool gather = false;
};
enum { kC0, kC1, kA0, kA1, kJ0, kJ1, kG0, kG1 };

struct Comm {
    ncclComm_t nccl = nullptr;
    hipStream_t side = nullptr;   // the collective's stream
    hipEvent_t fork = nullptr, join = nullptr;
    int world = 0, rank = 0, device = 0;
    int every = 0;                // ncf_comm_timing
    int64_t calls = 0;
    std::vector<StepEvents> sets; // recorded since the last read (events kept for reuse)
    size_t used = 0;
    StepEvents* cur = nullptr;    // the current call's, when sampled
};

int hip_ok(hipError_t e, const char* what);

// the current call's event set (nullptr: not sampled)
StepEvents* timing_begin(Comm* c) {
    c->cur = nullptr;
    if (c->every <= 0 || (c->calls++ % c->every) != 0 || c->used >= 4096) return nullptr;
    if (c->used == c->sets.size()) {
        StepEvents se;
        for (hipEvent_t& e : se.e)
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->sets.push_back(se);
    }
    c->cur = &c->sets[c->used++];
    c->cur->gather = false;
    return c->cur;
}

inline int mark(Comm* c, int which, hipStream_t st) {
    return c->cur ? hip_ok(hipEventRecord(c->cur->e[which], st), "timing event") : 0;
}

int comm_fail(int code, const char* what, const char* detail) { return ncf::set_error(code, "%s: %s", what, detail); }

int nccl_check(ncclResult_t r, const char* what) {
    return r == ncclSuccess ? 0 : comm_fail(NCF_EHIP, what, ncclGetErrorString(r));
}

int hip_ok(hipError_t e, const char* what) { return e == hipSuccess ? 0 : comm_fail(NCF_EHIP, what, hipGetErrorString(e)); }

}  // namespace

extern "C" {

int ncf_comm_unique_id(void* id, size_t bytes) {
    if (!id || bytes < sizeof(ncclUniqueId)) return comm_fail(NCF_EINVAL, "ncf_comm_unique_id", "buffer < 128 bytes");
    ncclUniqueId u;
    if (int r = nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId")) return r;
    memcpy(id, &u, sizeof(u));
    return 0;
}

int ncf_comm_init(int32_t world, int32_t rank, const void* id, size_t bytes, void** comm) {
    if (!comm || !id || bytes < sizeof(ncclUniqueId)) return comm_fail(NCF_EINVAL, "ncf_comm_init", "NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return comm_fail(NCF_EINVAL, "ncf_comm_init", "rank outside world");
    Comm* c = new Comm();
    c->world = world;
    c->rank = rank;
    if (int r = hip_ok(hipGetDevice(&c->device), "hipGetDevice")) {
        delete c;
        return r;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    int r = nccl_check(ncclCommInitRank(&c->nccl, world, u, rank), "ncclCommInitRank");
    if (!r) r = hip_ok(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking), "hipStreamCreate");
    if (!r) r = hip_ok(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming), "hipEventCreate");
    if (!r) r = hip_ok(hipEventCreateWithFlags(&c->join, hipEventDisableTiming), "hipEventCreate");
    if (r) {
        if (c->nccl) ncclCommDestroy(c->nccl);
        if (c->fork) hipEventDestroy(c->fork);
        if (c->join) hipEventDestroy(c->join);
        if (c->side) hipStreamDestroy(c->side);
        delete c;
        return r;
    }
    *comm = c;
    return 0;
}

int ncf_comm_destroy(void* comm) {
    Comm* c = static_cast<Comm*>(comm);
    if (!c) return 0;
    hipStreamSynchronize(c->side);
    int r = c->nccl ? nccl_check(ncclCommDestroy(c->nccl), "ncclCommDestroy") : 0;
    if (c->fork) hipEventDestroy(c->fork);
    if (c->join) hipEventDestroy(c->join);
    for (StepEvents& se : c->sets)
        for (hipEvent_t e : se.e)
            if (e) hipEventDestroy(e);
    if (c->side) hipStreamDestroy(c->side);
    delete c;
    return r;
}

int ncf_comm_timing(void* comm, int32_t every) {
    Comm* c = static_cast<Comm*>(comm);
    if (!c || every < 0) return comm_fail(NCF_EINVAL, "ncf_comm_timing", "NULL communicator or every < 0");
    c->every = every;
    c->calls = 0;
    return 0;
}

int ncf_comm_timing_read(void* comm, double* out4, int64_t* steps) {
    Comm* c = static_cast<Comm*>(comm);
    if (!c || !out4 || !steps) return comm_fail(NCF_EINVAL, "ncf_comm_timing_read", "NULL argument");
    double acc[4] = {0, 0, 0, 0};
    auto span = [&](const StepEvents& se, int a, int b, double* into) -> int {
        float ms = 0.f;
        if (int r = hip_ok(hipEventSynchronize(se.e[b]), "timing sync")) return r;
        if (int r = hip_ok(hipEventElapsedTime(&ms, se.e[a], se.e[b]), "timing read")) return r;
        *into += ms;
        return 0;
    };
    for (size_t i = 0; i < c->used; ++i) {
        const StepEvents& se = c->sets[i];
        if (int r = span(se, kC0, kC1, &acc[0])) return r;
        if (int r = span(se, kJ0, kJ1, &acc[2])) return r;
        if (se.gather) {
            if (int r = span(se, kA0, kA1, &acc[1])) return r;
            if (int r = span(se, kG0, kG1, &acc[3])) return r;
        }
    }
    for (int j = 0; j < 4; ++j) out4[j] = acc[j];
    *steps = (int64_t)c->used;
    c->used = 0;
    return 0;
}

// in-place sum over the ranks on the communicator's stream, ordered after everything enqueued on
// `stream` so far; `stream` waits for it before its next work
int ncf_comm_allreduce(void* comm, float* buf, int64_t count, void* stream) {
    Comm* c = static_cast<Comm*>(comm);
    if (!c || (!buf && count > 0) || count < 0) return comm_fail(NCF_EINVAL, "ncf_comm_allreduce", "invalid argument");
    hipStream_t st = (hipStream_t)stream;
    if (int r = hip_ok(hipEventRecord(c->fork, st), "fork")) return r;
    if (int r = hip_ok(hipStreamWaitEvent(c->side, c->fork, 0), "fork wait")) return r;
    if (int r = nccl_check(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, c->nccl, c->side),
                           "ncclAllReduce"))
        return r;
    if (int r = hip_ok(hipEventRecord(c->join, c->side), "join")) return r;
    return hip_ok(hipStreamWaitEvent(st, c->join, 0), "join wait");
}

// The user-partitioned step with deferred decay (ncf_forward_backward_part_lazy, all-reduce,
// ncf_update_rows_lazy, ncf_apply_update) in one call: the all-reduce of
// shared = [item-row gradient | dense-layer gradient | summary] runs on the communicator's stream
// while the compute stream applies the own-user update and prepares the next batch (counted,
// own rows caught up, index filled and sorted: the next call passes hyper->index_ready = 3).
int ncf_user_dp_step(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                     const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                     const int32_t* next_users, const int32_t* next_items, int64_t n_next, float* shared,
                     int32_t include_dense_reg, void* comm, double* stats, void* ws, size_t ws_bytes, void* stream) {
    Comm* c = static_cast<Comm*>(comm);
    if (!s || !model || !optim || !h || !shared || !c) return comm_fail(NCF_EINVAL, "ncf_user_dp_step", "NULL argument");
    if (h->lazy_rows <= 0 || h->lazy_rows > s->num_rows)
        return comm_fail(NCF_EINVAL, "ncf_user_dp_step", "hyper->lazy_rows must be the rank's user count");
    const int64_t U = h->lazy_rows, R = s->num_rows, W = s->row_width, P = s->mlp_params;
    float* item_grad = shared;
    float* mlp_grad = shared + (R - U) * W;
    float* summary = mlp_grad + P;
    hipStream_t st = (hipStream_t)stream;
    bool filled = false;
    if (int r = ncf::dp_forward_backward(s, model, optim, h, users, items, labels, n, item_grad, mlp_grad, summary,
                                         include_dense_reg, ws, ws_bytes, stream, &filled))
        return r;   // the message is set
    const int64_t count = (R - U) * W + P + NCF_NUM_SUMMARY;
    hipStream_t side = c->side;
    timing_begin(c);
    if (int r = hip_ok(hipEventRecord(c->fork, st), "fork")) return r;
    if (int r = hip_ok(hipStreamWaitEvent(side, c->fork, 0), "fork wait")) return r;
    if (int r = mark(c, kC0, side)) return r;
    if (int r = nccl_check(ncclAllReduce(shared, shared, (size_t)count, ncclFloat32, ncclSum, c->nccl, side),
                           "ncclAllReduce"))
        return r;
    if (int r = mark(c, kC1, side)) return r;
    if (int r = hip_ok(hipEventRecord(c->join, side), "join")) return r;
    // meanwhile on the compute stream: the own users' update (+ the next batch counted, its own rows
    // caught up ahead and its counts scanned) — none of it reads an item row, so all of it runs
    // under the collective; the next step fills its index inside its forward/backward
    if (int r = ncf::dp_update_rows(s, model, optim, h, n, next_users, next_items, n_next, ws, ws_bytes, stream, filled))
        return r;
    if (int r = mark(c, kJ0, st)) return r;
    if (int r = hip_ok(hipStreamWaitEvent(st, c->join, 0), "join wait")) return r;
    if (int r = mark(c, kJ1, st)) return r;
    // the replicated item rows (their moments indexed by table row) and the dense layers
    ncf_optim_t items_opt = *optim;
    if (items_opt.emb_m) items_opt.emb_m += U * W;
    if (items_opt.emb_v) items_opt.emb_v += U * W;
    items_opt.row_step = nullptr;
    if (int r = ncf_apply_update(s, model, &items_opt, h, U, R - U, item_grad, mlp_grad, summary, stats, ws, ws_bytes,
                                 stream))
        return r;
    return 0;
}

// The user-partitioned step with the item rows' optimizer split across the ranks (the item table
// stays replicated for the forward pass, but each rank applies Adam to 1/item_world of it):
//   forward/backward (as ncf_user_dp_step) -> shared = [item-row gradient, item_world x Ic rows |
//   dense-layer gradient | summary]
//   comm stream: reduce-scatter of the item-row gradient (rank r receives rows [r Ic, r Ic + Ic) in
//   slice_grad) + all-reduce of [dense-layer gradient | summary], one RCCL group ...
//   ... beside the own-user update (with the next batch counted and scanned) on the compute stream
//   join; Adam on this rank's item slice (table rows U + r Ic ..)
//   comm stream: all-gather of the updated item rows (in place: the table holds item_world x Ic
//   item rows, the rows past num_rows are zero padding) beside the dense layers' Adam and the
//   stats on the compute stream, which then waits for it
// The same bytes cross the links as the all-reduce of ncf_user_dp_step; each rank's item Adam and
// item-moment traffic shrink to 1/item_world.  item_world == 1 (or a one-rank communicator with
// item_world > 1: the per-rank compute of that layout, no exchange) is bitwise ncf_user_dp_step.
int ncf_user_dp_step_split(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                           const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                           const int32_t* next_users, const int32_t* next_items, int64_t n_next, float* shared,
                           float* slice_grad, int32_t item_world, int32_t item_rank, int32_t include_dense_reg,
                           void* comm, double* stats, void* ws, size_t ws_bytes, void* stream) {
    Comm* c = static_cast<Comm*>(comm);
    if (!s || !model || !optim || !h || !shared || !c)
        return comm_fail(NCF_EINVAL, "ncf_user_dp_step_split", "NULL argument");
    if (h->lazy_rows <= 0 || h->lazy_rows > s->num_rows)
        return comm_fail(NCF_EINVAL, "ncf_user_dp_step_split", "hyper->lazy_rows must be the rank's user count");
    if (item_world < 1 || item_rank < 0 || item_rank >= item_world || (c->world != item_world && c->world != 1) ||
        (c->world == item_world && c->rank != item_rank))
        return comm_fail(NCF_EINVAL, "ncf_user_dp_step_split", "item_world/item_rank do not match the communicator");
    const int64_t U = h->lazy_rows, R = s->num_rows, W = s->row_width, P = s->mlp_params;
    const int64_t I = R - U, Ic = (I + item_world - 1) / item_world;
    const bool exchange = c->world > 1;
    if (exchange && !slice_grad) return comm_fail(NCF_EINVAL, "ncf_user_dp_step_split", "NULL slice_grad");
    float* item_grad = shared;
    float* mlp_grad = shared + item_world * Ic * W;
    float* summary = mlp_grad + P;
    hipStream_t st = (hipStream_t)stream;
    bool filled = false;
    if (int r = ncf::dp_forward_backward(s, model, optim, h, users, items, labels, n, item_grad, mlp_grad, summary,
                                         include_dense_reg, ws, ws_bytes, stream, &filled))
        return r;
    hipStream_t side = c->side;
    timing_begin(c);
    if (int r = hip_ok(hipEventRecord(c->fork, st), "fork")) return r;
    if (int r = hip_ok(hipStreamWaitEvent(side, c->fork, 0), "fork wait")) return r;
    if (int r = mark(c, kC0, side)) return r;
    if (exchange) {
        if (int r = nccl_check(ncclGroupStart(), "ncclGroupStart")) return r;
        if (int r = nccl_check(ncclReduceScatter(item_grad, slice_grad, (size_t)(Ic * W), ncclFloat32, ncclSum,
                                                 c->nccl, side), "ncclReduceScatter"))
            return r;
        if (int r = nccl_check(ncclAllReduce(mlp_grad, mlp_grad, (size_t)(P + NCF_NUM_SUMMARY), ncclFloat32, ncclSum,
                                             c->nccl, side), "ncclAllReduce"))
            return r;
        if (int r = nccl_check(ncclGroupEnd(), "ncclGroupEnd")) return r;
    } else {
        // one rank: its slice of the (local) item gradient is the reduced one
        slice_grad = item_grad + item_rank * Ic * W;
        if (int r = nccl_check(ncclAllReduce(mlp_grad, mlp_grad, (size_t)(P + NCF_NUM_SUMMARY), ncclFloat32, ncclSum,
                                             c->nccl, side), "ncclAllReduce"))
            return r;
    }
    if (int r = mark(c, kC1, side)) return r;
    if (int r = hip_ok(hipEventRecord(c->join, side), "join")) return r;
    // the own users' update, the next batch counted (own rows caught up ahead); its counts are
    // scanned by this step's stats launch when the apply is split below (k_stats_scan), else here
    const int64_t r0 = item_rank * Ic;
    const int64_t cnt = r0 >= I ? 0 : (I - r0 < Ic ? I - r0 : Ic);
    const bool split_apply = cnt > 0 && ncf::part_tail_foldable(*s, *h, 1 << 30);
    if (int r = ncf::dp_update_rows(s, model, optim, h, n, next_users, next_items, n_next, ws, ws_bytes, stream, filled,
                                    !split_apply))
        return r;
    if (int r = mark(c, kJ0, st)) return r;
    if (int r = hip_ok(hipStreamWaitEvent(st, c->join, 0), "join wait")) return r;
    if (int r = mark(c, kJ1, st)) return r;
    // this rank's item slice (its moments indexed by table row) and the dense layers
    ncf_optim_t items_opt = *optim;
    if (items_opt.emb_m) items_opt.emb_m += (U + r0) * W;
    if (items_opt.emb_v) items_opt.emb_v += (U + r0) * W;
    items_opt.row_step = nullptr;
    // Every L2 factor zero (the fused apply): only the item slice's Adam precedes the all-gather; the
    // dense layers' Adam and the stats (step bump, the next batch's scan) run on the compute stream
    // BESIDE it — off the exchange's critical path (round 6; same kernels' arithmetic, so the states
    // stay bitwise those of ncf_apply_update).  One rank (no all-gather): both in one launch.
    if (split_apply) {
        if (int r = hip_ok(ncf::launch_apply_fused(*s, model->emb + (U + r0) * W, items_opt.emb_m, items_opt.emb_v,
                                                   slice_grad, cnt, model->mlp, optim->mlp_m, optim->mlp_v, mlp_grad,
                                                   optim->step, *h, st, exchange ? 1 : 3),
                           "item-slice update"))
            return r;
    } else if (int r = ncf_apply_update(s, model, &items_opt, h, U + (cnt ? r0 : I), cnt, slice_grad, mlp_grad, summary,
                                        stats, ws, ws_bytes, stream)) {
        return r;
    }
    auto dense_and_stats = [&]() -> int {
        if (!split_apply) return 0;
        if (exchange)
            if (int r = hip_ok(ncf::launch_apply_fused(*s, nullptr, nullptr, nullptr, nullptr, 0, model->mlp,
                                                       optim->mlp_m, optim->mlp_v, mlp_grad, optim->step, *h, st, 2),
                               "dense-layer update"))
                return r;
        // the stats (they read only the caller's summary) and the next batch's count scan in one
        // launch (k_stats_scan); the scan's regions sit where the batch's layout puts them
        const ncf::WsLayout L = ncf::make_layout(*s, n);
        return hip_ok(ncf::launch_stats(L, ws, summary, 0, 0, h->inv_batch, stats, optim->step, true, st,
                                        next_users != nullptr, s->num_rows),
                      "stats");
    };
    if (!exchange) return dense_and_stats();
    // the updated slices to every rank (in place) on the side stream, while the compute stream runs
    // the dense layers' Adam and the stats (no item row read); the compute stream waits for the
    // gather before the next forward pass can read an item row
    if (int r = hip_ok(hipEventRecord(c->fork, st), "fork")) return r;
    if (int r = hip_ok(hipStreamWaitEvent(side, c->fork, 0), "fork wait")) return r;
    if (c->cur) c->cur->gather = true;
    if (int r = mark(c, kA0, side)) return r;
    float* items0 = model->emb + U * W;
    if (int r = nccl_check(ncclAllGather(items0 + r0 * W, items0, (size_t)(Ic * W), ncclFloat32, c->nccl, side),
                           "ncclAllGather"))
        return r;
    if (int r = mark(c, kA1, side)) return r;
    if (int r = hip_ok(hipEventRecord(c->join, side), "join")) return r;
    if (int r = dense_and_stats()) return r;
    if (int r = mark(c, kG0, st)) return r;
    if (int r = hip_ok(hipStreamWaitEvent(st, c->join, 0), "join wait")) return r;
    return mark(c, kG1, st);
}

}  // extern "C"
