// Optimizer sweeps, metrics and loss summaries.
//
// Reference semantics (movierec/model.py:199-215 → Keras v1 optimizers):
//   Adam:  t += 1; lr_t = lr*sqrt(1-b2^t)/(1-b1^t)
//          m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g^2;  p -= lr_t*m/(sqrt(v)+eps)
//   SGD:   p -= lr*g
// applied DENSELY to every element of every variable (the embedding's
// IndexedSlices gradient is densified: rows absent from the batch still decay
// m, v and move p).  L2 (model.py:163,168,178) adds 2*lambda*p to the gradient
// of the whole variable and lambda*sum(p^2) to the loss.
//
// k_emb_update is the fused "scatter-add + Adam" of the embedding table: one
// HBM-bound sweep over the table (p, m, v: 24 B/param) that, per row, sums the
// row's per-sample gradient contributions in ascending sample order through
// the index built by ncf_index.hip (deterministic, no atomics).

#include <climits>
#include <cmath>

#include "ncf_adam.h"
#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

__device__ inline float block_sum_array(const float* __restrict__ a, int n, float* red) {
    float x = 0.f;
    for (int j = threadIdx.x; j < n; j += kBlock) x += a[j];
    return block_sum_256(x, red);
}

// batch summary from the per-block partials (whole block)
__device__ inline void summary_body(const float* __restrict__ part_bce, int nbce, const float* __restrict__ part_hit,
                                    const float* __restrict__ part_dcg, int nmet, float n_groups,
                                    const float* __restrict__ reg_emb, int nreg_emb,
                                    const float* __restrict__ reg_mlp, int nreg_mlp, float* __restrict__ summary,
                                    float* red) {
    const float b = block_sum_array(part_bce, nbce, red);
    const float h = block_sum_array(part_hit, nmet, red);
    const float d = block_sum_array(part_dcg, nmet, red);
    const float re = block_sum_array(reg_emb, nreg_emb, red);
    const float rm = block_sum_array(reg_mlp, nreg_mlp, red);
    if (threadIdx.x < NCF_NUM_SUMMARY) {
        const int t = threadIdx.x;
        summary[t] = t == NCF_SUM_BCE ? b : t == NCF_SUM_HIT ? h : t == NCF_SUM_DCG ? d
                   : t == NCF_SUM_GROUPS ? n_groups : t == NCF_SUM_REG ? re + rm : 0.f;
    }
}

// P-ahead rows.  The catch-up ahead (the next batch's stale rows, replayed in the touched-row
// update launch) writes p only: the next step's update reads m and v anyway and re-derives their
// missed zero-gradient decays (the moments do not depend on p), as it does after the per-step
// catch-up.  Such a row's row_step holds -(s0 + 2), s0 = the step its m and v are at; its p is at
// the step of the launch that caught it up, which every consumer knows: the next update's t - 1,
// the flush's and the stale-count gate's target (nothing else runs in between: the engine flushes
// before it discards a counted-ahead batch).  Pristine rows are never caught up, so s0 >= 0 and
// the mark is negative.
#ifndef NCF_AHEAD_P_ONLY
#define NCF_AHEAD_P_ONLY 1
#endif
__device__ __forceinline__ int pahead_mark(int s0) { return -(s0 + 2); }
__device__ __forceinline__ int pahead_s0(int rs) { return -rs - 2; }

// blocks blk of nblk stride over the table's float4 elements
template <int OPT, int SRC, bool L2>
__device__ __forceinline__ void emb_update_body(float4* __restrict__ emb, float4* __restrict__ m4,
                                                float4* __restrict__ v4, uint32_t n4, uint32_t w4,
                                                const int32_t* __restrict__ offs, const int32_t* __restrict__ list,
                                                const float4* __restrict__ gs, const float4* __restrict__ dgrad,
                                                const int32_t* __restrict__ step, float lr, float b1, float b2,
                                                float eps, float lam, float* __restrict__ part_reg, uint32_t blk,
                                                uint32_t nblk) {
    __shared__ float red[4];
    const int t = *step + 1;
    const float lr_t = (OPT == NCF_OPT_ADAM) ? adam_lr_t(lr, b1, b2, t) : lr;
    float reg = 0.0f;
    for (uint32_t e = blk * blockDim.x + threadIdx.x; e < n4; e += nblk * blockDim.x) {
        float4 p = emb[e];
        float4 g;
        if (SRC == kGradSparse) {
            const uint32_t r = e / w4;
            const uint32_t q = e - r * w4;
            const int o = offs[r];
            const int c = offs[r + 1] - o;
            g = make_float4(0.f, 0.f, 0.f, 0.f);
            int j = 0;
            for (; j + 4 <= c; j += 4) {  // four rows in flight, summed in ascending order
                const float4 g0 = gs[(size_t)list[o + j] * w4 + q], g1 = gs[(size_t)list[o + j + 1] * w4 + q];
                const float4 g2 = gs[(size_t)list[o + j + 2] * w4 + q], g3 = gs[(size_t)list[o + j + 3] * w4 + q];
                g = f4add(g, g0);
                g = f4add(g, g1);
                g = f4add(g, g2);
                g = f4add(g, g3);
            }
            for (; j < c; ++j) g = f4add(g, gs[(size_t)list[o + j] * w4 + q]);
        } else {
            g = dgrad[e];
        }
        if (L2) {
            reg += lam * (p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w);
            const float l2 = 2.0f * lam;
            g.x += l2 * p.x; g.y += l2 * p.y; g.z += l2 * p.z; g.w += l2 * p.w;
        }
        if (OPT == NCF_OPT_ADAM) {
            float4 mm = m4[e], vv = v4[e];
            adam4(p, mm, vv, g, lr_t, b1, b2, eps);
            m4[e] = mm;
            v4[e] = vv;
        } else {
            p.x -= lr * g.x; p.y -= lr * g.y; p.z -= lr * g.z; p.w -= lr * g.w;
        }
        emb[e] = p;
    }
    if (L2) {
        reg = block_sum_256(reg, red);
        if (threadIdx.x == 0) part_reg[blk] = reg;
    }
}

template <int OPT, int SRC, bool L2>
__global__ __launch_bounds__(kBlock) void k_emb_update(float4* __restrict__ emb, float4* __restrict__ m4,
                                                       float4* __restrict__ v4, uint32_t n4, uint32_t w4,
                                                       const int32_t* __restrict__ offs,
                                                       const int32_t* __restrict__ list,
                                                       const float4* __restrict__ gs,
                                                       const float4* __restrict__ dgrad,
                                                       const int32_t* __restrict__ step, float lr, float b1,
                                                       float b2, float eps, float lam, float* __restrict__ part_reg) {
    emb_update_body<OPT, SRC, L2>(emb, m4, v4, n4, w4, offs, list, gs, dgrad, step, lr, b1, b2, eps, lam, part_reg,
                                  blockIdx.x, gridDim.x);
}

#ifndef NCF_CATCHUP_P_ONLY
#define NCF_CATCHUP_P_ONLY 1
#endif
#if NCF_AHEAD_P_ONLY && !NCF_CATCHUP_P_ONLY
#error "P-ahead rows need the update's m / v re-derivation (NCF_CATCHUP_P_ONLY)"
#endif
#ifndef NCF_CATCHUP_SCALAR
#define NCF_CATCHUP_SCALAR 1
#endif
#ifndef NCF_CATCHUP_AHEAD
#define NCF_CATCHUP_AHEAD 1
#endif
#ifndef NCF_AHEAD_REP
#define NCF_AHEAD_REP 3   // replay items (rows / row slices) per wave with their loads in flight together, in the
                          // catch-up-ahead blocks and the catch-up / flush kernel (4 spills at 7 blocks/CU)
#endif
constexpr int kRep = NCF_AHEAD_REP;
#ifndef NCF_COUNT_PER_MAX
#define NCF_COUNT_PER_MAX 64   // contributions per count block and pass from 65,536 contributions
#endif
// occupancy floor of the touched-row update launch (its HBM-bound rows want many waves; the
// catch-up-ahead blocks in the same launch must not raise its register count)
#ifndef NCF_COUNT_PER_SMALL
#define NCF_COUNT_PER_SMALL 32  // contributions per count block and pass below 32,768 contributions
                                // (16 until round 5: 32 is 0.6-0.9 % faster at 8,192 and 4,095 samples, profiles/r05_cps)
#endif
#ifndef NCF_COUNT_BLOCKS_MAX
#define NCF_COUNT_BLOCKS_MAX 4096  // count (+ catch-up ahead) blocks of the touched-row update launch
#endif
#ifndef NCF_DIAG_UPD
#define NCF_DIAG_UPD 0
#endif
#ifndef NCF_TOUCHED_MIN_BLOCKS
#define NCF_TOUCHED_MIN_BLOCKS 7
#endif
#ifndef NCF_TOUCHED_MIN_BLOCKS_UNSORTED
#define NCF_TOUCHED_MIN_BLOCKS_UNSORTED NCF_TOUCHED_MIN_BLOCKS   // the unsorted-list variant (experiments)
#endif

// Deferred exact decay ("lazy" dense Adam, L2 off).  Keras' dense Adam (F5) moves EVERY row
// every step; a row no sample touches gets g = 0, so its update is a pure function of
// (p, m, v, t).  Instead of sweeping those rows, row_step[r] records how many steps row r has
// received; a row is brought up to date (its missed zero-gradient steps replayed with the
// same per-step arithmetic) only when a batch touches it (before the forward pass reads it)
// or when the whole table is read (ncf_lazy_flush).  The result is bitwise that of the dense
// sweep, and a step moves only the touched rows instead of the whole table.

// Rows are processed a wave at a time: lane l takes element l % w4 of row (l / w4) of the
// wave's group of 64 / w4 rows (w4 <= 64; wider rows loop over their elements).  Every row's
// loads are independent, so latency hides across the many waves in flight instead of inside
// a grid-stride chain of dependent index loads.
struct RowLanes {
    int rpw, sub, q, qstep;
    bool on;
    __device__ RowLanes(uint32_t w4) {
        const int lane = threadIdx.x & 63;
        rpw = w4 <= 64 ? 64 / (int)w4 : 1;
        sub = w4 <= 64 ? lane / (int)w4 : 0;
        q = w4 <= 64 ? lane % (int)w4 : lane;
        qstep = w4 <= 64 ? (int)w4 : 64;
        on = sub < rpw;
    }
};

// bias-corrected lr of the last kLrLut steps, per block in LDS (one entry per thread).  Older
// steps fall back to adam_lr_t (two powf per element-step): with fresh uniform batches a row's
// gap exceeds 64 steps often enough that the few such rows set the launch's tail
constexpr int kLrLut = kBlock;

#ifndef NCF_REPLAY_UNROLL
#define NCF_REPLAY_UNROLL 4
#endif
#ifndef NCF_FLUSH_UNROLL
#define NCF_FLUSH_UNROLL 1   // the flush (every row): the rows' joint one-step chains (79 VGPRs) beat replay2 (120) there
#endif
#ifndef NCF_FLUSH_WAVES
#define NCF_FLUSH_WAVES 1    // launch-bound minimum waves per SIMD of k_emb_flush
#endif
// The zero-gradient steps (s, t] of one element pair, U steps at a time: the U steps' moment
// chains first (two dependent operations per step), then their U step terms — independent of
// each other, so their square roots and reciprocals overlap instead of each step waiting for the
// previous one's — then p's U subtractions in step order.  Per step the operations and their
// order are adam2_zero's: bitwise the one-step loop.  A row's replay is one such chain per element
// pair, so its latency per step, not the VALU issue, set the replays' time.
template <int U>
__device__ __forceinline__ void replay2(f32x2& p, f32x2& m, f32x2& v, int s, int t, const float* lut, float lr,
                                        float b1, float b2, float eps) {
#pragma clang fp contract(off)
    int st = s + 1;
    for (; st <= t && t - st >= kLrLut; ++st) adam2_zero(p, m, v, adam_lr_t(lr, b1, b2, st), b1, b2, eps);
    for (; st + U - 1 <= t; st += U) {
        f32x2 mm[U], vv[U], r[U];
        float lrt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) lrt[u] = lut[t - st - u];
        mm[0] = m * b1 + 0.0f;
        vv[0] = v * b2;
#pragma unroll
        for (int u = 1; u < U; ++u) {
            mm[u] = mm[u - 1] * b1 + 0.0f;
            vv[u] = vv[u - 1] * b2;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = rcp_sqrt_eps2(vv[u], eps);
#pragma unroll
        for (int u = 0; u < U; ++u) p -= (mm[u] * lrt[u]) * r[u];
        m = mm[U - 1];
        v = vv[U - 1];
    }
    for (; st <= t; ++st) adam2_zero(p, m, v, lut[t - st], b1, b2, eps);
}

// replay the zero-gradient steps (s, t] of the touched rows list[0..*nlist) (ALL: every row,
// ncf_lazy_flush)
struct SortAhead {
    int ncatch;                // blocks [0, ncatch) replay rows; blocks >= ncatch sort lists
    const int32_t* offs;
    int64_t keys;
    int32_t* list;
    int nwords;
    int32_t* cnt;              // residue check of the counters (sort_rows_body)
    int32_t* err;
    const int32_t* touched;    // large key spaces: sort the touched list's rows only
    const int2* toc;
    const int32_t* nuniq;
};

// A batch whose rows the previous step caught up ahead (counted ahead, index_ready == 2) needs no
// replay — unless its ids changed after they were counted (NCF_WSERR_STALE_COUNT, raised by the
// index fill before this launch).  Then the rows of the ids actually passed that the counted set
// missed are not in the touched list, yet the forward pass reads them: the gate blocks replay
// every such row fully (p, m, v to step t, row_step = t, claimed by CAS so a row repeated in the
// batch replays once; rows already current are skipped), so the table stays exactly the dense
// sweep's state (that step's embedding gradient is still wrong, as the flag reports).  Without the
// flag the gate blocks return at once.
struct StaleGate {
    const int32_t* users;      // nullptr: no gate blocks
    const int32_t* items;
    int64_t m;                 // 2 * batch contributions
    int32_t U, I;
    int32_t* row_step;
    int64_t lazy_rows;         // rows [0, lazy_rows) are under deferred decay
    int ahead;                 // the replay target is *step + ahead (1: enqueued before the step's bump)
};

__device__ __forceinline__ void stale_replay_body(float* __restrict__ embf, float* __restrict__ mf,
                                               float* __restrict__ vf, int W, const StaleGate& sg, int t, float lr,
                                               float b1, float b2, float eps, const int32_t* __restrict__ err,
                                               int blk, int nblk) {
    if (!(__atomic_load_n(err, __ATOMIC_RELAXED) & kErrStaleCount)) return;
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blk * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)nblk * (kBlock / 64);
    // P-ahead rows of the counted batch (their p was caught up to t by the previous step's launch)
    // may now stay out of this step's batch: give every such row its m, v decays here, so that
    // row_step again tells the step of all three (the claim loop below leaves them alone)
    for (int64_t r0 = wave * 64; r0 < sg.lazy_rows; r0 += nw * 64) {
        const int64_t rr = r0 + lane;
        const int rs = rr < sg.lazy_rows ? sg.row_step[rr] : 0;
        uint64_t pm = __ballot(rs < 0);
        while (pm) {
            const int src = __ffsll((unsigned long long)pm) - 1;
            pm &= pm - 1;
            const int64_t r = r0 + src;
            const int s0 = pahead_s0(__shfl(rs, src, 64));
            for (int q = lane; 2 * q < W; q += 64) {
                const size_t e = (size_t)r * W + 2 * q;
                f32x2 m = *reinterpret_cast<const f32x2*>(mf + e);
                f32x2 v = *reinterpret_cast<const f32x2*>(vf + e);
                for (int st = s0 + 1; st <= t; ++st) decay2(m, v, b1, b2);
                *reinterpret_cast<f32x2*>(mf + e) = m;
                *reinterpret_cast<f32x2*>(vf + e) = v;
            }
            if (lane == 0) sg.row_step[r] = t;
        }
    }
    for (int64_t c0 = wave * 64; c0 < sg.m; c0 += nw * 64) {
        const int64_t c = c0 + lane;
        int key = -1;
        if (c < sg.m) {
            const int64_t i = c >> 1;
            const int id = (c & 1) ? sg.items[i] : sg.users[i];
            if ((unsigned)id < (unsigned)((c & 1) ? sg.I : sg.U)) key = (c & 1) ? sg.U + id : id;
            if (key >= sg.lazy_rows) key = -1;
        }
        claim_replay(embf, mf, vf, W, sg.row_step, key, t, lr, b1, b2, eps);
    }
}

template <bool ALL>
__device__ __forceinline__ void catchup_body(float4* __restrict__ emb, float4* __restrict__ m4,
                                                        float4* __restrict__ v4, uint32_t w4,
                                                        const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ nlist, int64_t R,
                                                        const int32_t* __restrict__ row_step,
                                                        const int32_t* __restrict__ step, float lr, float b1,
                                                        float b2, float eps, SortAhead so, StaleGate sg) {
    if (!ALL && (int)blockIdx.x >= so.ncatch) {
        // the contribution lists of this step's index, sorted while the rows replay (k_sort's work;
        // only the touched-row update after the forward pass reads them)
        if (so.touched)
            sort_rows_body<1, true>(so.offs, so.keys, so.list, so.nwords, (int)blockIdx.x - so.ncatch, so.cnt,
                                    so.err, so.touched, so.toc, so.nuniq);
        else if (sort_rpt(so.keys) == 8)
            sort_rows_body<8>(so.offs, so.keys, so.list, so.nwords, (int)blockIdx.x - so.ncatch, so.cnt, so.err);
        else
            sort_rows_body<1>(so.offs, so.keys, so.list, so.nwords, (int)blockIdx.x - so.ncatch, so.cnt, so.err);
        return;
    }
    if (!ALL && sg.users) {
        stale_replay_body(reinterpret_cast<float*>(emb), reinterpret_cast<float*>(m4), reinterpret_cast<float*>(v4),
                          4 * (int)w4, sg, *step + sg.ahead, lr, b1, b2, eps, so.err, (int)blockIdx.x, so.ncatch);
        return;
    }
    __shared__ float lut[kLrLut];
    const int t = *step;  // steps every row should have received
    if (threadIdx.x < kLrLut) lut[threadIdx.x] = t - (int)threadIdx.x >= 1 ? adam_lr_t(lr, b1, b2, t - threadIdx.x) : 0.f;
    __syncthreads();
    const int64_t n = ALL ? R : (int64_t)*nlist;
    const int64_t nblk = ALL ? gridDim.x : so.ncatch;
#if NCF_CATCHUP_SCALAR
    // One ELEMENT per lane (a row of W floats spans W lanes, 2 waves at config C): a row's replay
    // is a sequential chain per element, so the longest debt of the batch — rows untouched since
    // the start of the run — sets the launch's tail; spreading a row over 4x the lanes of the
    // float4 form cuts that tail 4x (measured: the float4 form's time grew with the longest debt
    // while the total work stayed flat, tools/catchup_probe.py).
    const int W = 4 * (int)w4;
    const int W2 = W / 2;                                                   // element pairs per row
    const int lanes_per_row = W2 < kBlock ? (W2 + 63) / 64 * 64 : kBlock;  // whole waves per row
    const int rpb = kBlock / lanes_per_row;                                // rows per block pass
    const int sub = threadIdx.x / lanes_per_row, q0 = threadIdx.x % lanes_per_row;
    float* embf = reinterpret_cast<float*>(emb);
    float* mf = reinterpret_cast<float*>(m4);
    float* vf = reinterpret_cast<float*>(v4);
    // kRep rows per pass: their steps, then their elements' loads in flight together, their step
    // chains advancing together (same per-element arithmetic: bitwise the one-row form)
    const int64_t pstride = nblk * rpb;
    for (int64_t i0 = (int64_t)blockIdx.x * rpb + sub; i0 < n; i0 += pstride * kRep) {
        int64_t r[kRep];
        int sr[kRep];
        bool pa[kRep];
#pragma unroll
        for (int j = 0; j < kRep; ++j) {
            const int64_t i = i0 + j * pstride;
            r[j] = i < n ? (ALL ? i : list[i]) : 0;
            // R: rows [0, R) are under deferred decay (touched rows past it are swept densely); a
            // pristine row (NCF_ROW_PRISTINE, past every t) is current: clamped to t, so no step loop
            // ever starts from its mark (s + 1 would overflow).  A P-ahead row's p is current (at t):
            // the flush decays its m and v from s0; the per-step catch-up leaves them to the update
            const int rs = i < n && (ALL || r[j] < R) ? row_step[r[j]] : t;
            pa[j] = ALL && rs < 0;
            sr[j] = rs < 0 ? (ALL ? pahead_s0(rs) : t) : (rs < t ? rs : t);
        }
        for (int q = q0; q < W2; q += lanes_per_row) {  // element pair q: elements 2q, 2q + 1
            const f32x2 z2 = {0.f, 0.f};
            f32x2 p[kRep], m[kRep], v[kRep];
#pragma unroll
            for (int j = 0; j < kRep; ++j) {
                const size_t e = (size_t)r[j] * W + 2 * q;
                const bool act = sr[j] < t;
                p[j] = act ? *reinterpret_cast<const f32x2*>(embf + e) : z2;
                m[j] = act ? *reinterpret_cast<const f32x2*>(mf + e) : z2;
                v[j] = act ? *reinterpret_cast<const f32x2*>(vf + e) : z2;
            }
            if constexpr ((ALL ? NCF_FLUSH_UNROLL : NCF_REPLAY_UNROLL) > 1) {
#pragma unroll
                for (int j = 0; j < kRep; ++j) {
                    if (pa[j]) {  // wave-uniform: a row spans whole waves
                        for (int st = sr[j] + 1; st <= t; ++st) decay2(m[j], v[j], b1, b2);
                    } else {
                        replay2<(ALL ? NCF_FLUSH_UNROLL : NCF_REPLAY_UNROLL)>(p[j], m[j], v[j], sr[j], t, lut, lr, b1, b2,
                                                                              eps);
                    }
                }
            } else {
                // the rows' chains advance together (same per-element arithmetic, step by step)
                int smin = t;
#pragma unroll
                for (int j = 0; j < kRep; ++j) smin = sr[j] < smin ? sr[j] : smin;
                for (int st = smin + 1; st <= t; ++st) {
                    const float lrt = t - st < kLrLut ? lut[t - st] : adam_lr_t(lr, b1, b2, st);
#pragma unroll
                    for (int j = 0; j < kRep; ++j) {
                        if (st > sr[j] && pa[j]) decay2(m[j], v[j], b1, b2);
                        else if (st > sr[j]) adam2_zero(p[j], m[j], v[j], lrt, b1, b2, eps);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kRep; ++j) {
                if (sr[j] < t) {
                    const size_t e = (size_t)r[j] * W + 2 * q;
                    if (!pa[j]) *reinterpret_cast<f32x2*>(embf + e) = p[j];
                    if (ALL || !NCF_CATCHUP_P_ONLY) {
                        *reinterpret_cast<f32x2*>(mf + e) = m[j];
                        *reinterpret_cast<f32x2*>(vf + e) = v[j];
                    }
                }
            }
        }
    }
#else
    const RowLanes rl(w4);
    if (!rl.on) return;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)nblk * kBlock) >> 6;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = wave * rl.rpw + rl.sub; i < n; i += waves * rl.rpw) {
        const int64_t r = ALL ? i : list[i];
        if (!ALL && r >= R) continue;
        int s = row_step[r];
        const bool pah = s < 0;  // P-ahead: p current; the flush decays m, v, the catch-up skips it
        if (pah && !ALL) continue;
        if (pah) s = pahead_s0(s);
        if (s >= t) continue;
        for (uint32_t q = rl.q; q < w4; q += rl.qstep) {
            const size_t e = (size_t)r * w4 + q;
            float4 p = emb[e], m = m4[e], v = v4[e];
            for (int j = s + 1; j <= t; ++j) {
                if (pah) decay4(m, v, b1, b2);
                else adam4(p, m, v, zero, t - j < kLrLut ? lut[t - j] : adam_lr_t(lr, b1, b2, j), b1, b2, eps);
            }
            if (!pah) st_stream(&emb[e], p);
            if (ALL || !NCF_CATCHUP_P_ONLY) {  // the flush leaves the dense state; with P_ONLY the
                        // per-step replay writes only p (the forward pass reads p) and
                        // k_emb_adam_touched re-derives m and v from row_step
                m4[e] = m;
                v4[e] = v;
            }
        }
    }
#endif
}

// ncf_lazy_flush: every row
__global__ __launch_bounds__(kBlock, NCF_FLUSH_WAVES) void k_emb_flush(float4* __restrict__ emb, float4* __restrict__ m4,
                                                      float4* __restrict__ v4, uint32_t w4, int64_t R,
                                                      const int32_t* __restrict__ row_step,
                                                      const int32_t* __restrict__ step, float lr, float b1, float b2,
                                                      float eps) {
    const SortAhead so{0, nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
    const StaleGate sg{nullptr, nullptr, 0, 0, 0, nullptr, 0, 0};
    catchup_body<true>(emb, m4, v4, w4, nullptr, nullptr, R, row_step, step, lr, b1, b2, eps, so, sg);
}

// the batch's touched rows (+ the index sort, + the stale-count gate): capped at 64 VGPRs, the
// 8 waves per SIMD of the latency-bound replay chains (the gate path spills a little instead)
__global__ __launch_bounds__(kBlock, 8) void k_emb_catchup(float4* __restrict__ emb, float4* __restrict__ m4,
                                                           float4* __restrict__ v4, uint32_t w4,
                                                           const int32_t* __restrict__ list,
                                                           const int32_t* __restrict__ nlist, int64_t R,
                                                           const int32_t* __restrict__ row_step,
                                                           const int32_t* __restrict__ step, float lr, float b1,
                                                           float b2, float eps, SortAhead so, StaleGate sg) {
    catchup_body<false>(emb, m4, v4, w4, list, nlist, R, row_step, step, lr, b1, b2, eps, so, sg);
}

// row_step[r] = *step for every row that is not pristine (after a flush: the replay kernel above
// only reads row_step; a pristine row is current at every step and keeps its mark)
__global__ __launch_bounds__(kBlock) void k_row_step_fill(int32_t* __restrict__ row_step, int64_t R,
                                                          const int32_t* __restrict__ step) {
    const int t = *step;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x)
        if (row_step[r] != NCF_ROW_PRISTINE) row_step[r] = t;
}

// Adam step t = *step + 1 on the touched rows, which were brought up to step t-1 before the
// forward pass; records row_step[r] = t.
struct L2Table {
    int n;
    int start[NCF_MAX_LAYERS];
    int end[NCF_MAX_LAYERS];
    float lam[NCF_MAX_LAYERS];
};

template <int OPT>
__device__ inline void mlp_update_body(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, int P,
                                       const float* __restrict__ slabs, int nslab, const float* __restrict__ grad_in,
                                       float* __restrict__ grad_out, int do_update, int want_reg,
                                       const int32_t* __restrict__ step, float lr, float b1, float b2, float eps,
                                       const L2Table& l2t, float* __restrict__ part_reg, int blk) {
    __shared__ float red[4];
    const int i = blk * kBlock + threadIdx.x;
    float reg = 0.0f;
    if (i < P) {
        float g = 0.0f;
        if (nslab > 0) {
            // fixed slab order → deterministic
            int s = 0;
            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
            for (; s + 4 <= nslab; s += 4) {
                a0 += slabs[(size_t)(s + 0) * P + i];
                a1 += slabs[(size_t)(s + 1) * P + i];
                a2 += slabs[(size_t)(s + 2) * P + i];
                a3 += slabs[(size_t)(s + 3) * P + i];
            }
            for (; s < nslab; ++s) a0 += slabs[(size_t)s * P + i];
            g = (a0 + a1) + (a2 + a3);
        } else {
            g = grad_in[i];
        }
        if (grad_out) grad_out[i] = g;
        if (do_update || want_reg) {
            float w = p[i];
            float lam = 0.0f;
            for (int l = 0; l < l2t.n; ++l)
                if (i >= l2t.start[l] && i < l2t.end[l]) lam = l2t.lam[l];
            if (lam != 0.0f) {
                reg = lam * w * w;
                g += 2.0f * lam * w;
            }
        }
        if (do_update) {
            float w = p[i];
            if (OPT == NCF_OPT_ADAM) {
                const int t = *step + 1;
                const float lr_t = adam_lr_t(lr, b1, b2, t);
                float mm = b1 * m[i] + (1.0f - b1) * g;
                float vv = b2 * v[i] + (1.0f - b2) * (g * g);
                w -= lr_t * mm / (sqrtf(vv) + eps);
                m[i] = mm;
                v[i] = vv;
            } else {
                w -= lr * g;
            }
            p[i] = w;
        }
    }
    reg = block_sum_256(reg, red);
    if (threadIdx.x == 0 && part_reg) part_reg[blk] = reg;
}

__device__ __forceinline__ void group_metrics_body(const float* __restrict__ probs, const float* __restrict__ labels,
                                                   int64_t ng, int group, int k, float* __restrict__ hit,
                                                   float* __restrict__ dcg, float* __restrict__ part_hit,
                                                   float* __restrict__ part_dcg, int blk);

struct CountAhead {
    int nupd;                  // blocks [0, nupd) update rows; [nupd, nupd + ncount) count
    int ncount;
    const int32_t* users;      // next batch (m = 2 * n_next contributions)
    const int32_t* items;
    int64_t m;
    int32_t U, I;
    int32_t* cnt;
    int replay;                // 1: also catch the next batch's stale rows up (catch-up ahead)
    int fold;                  // user-row folding of the next batch's index (fold_of)
    int per;                   // contributions per count block and pass (16, 32 or 64)
    int64_t lazy_rows;         // rows [0, lazy_rows) are under deferred decay: only they are
                               // updated here and caught up ahead (the rest are swept densely)
    const int32_t* seen;       // sparse index (sparse_index_ok): key in this step's batch <=> seen[key] ==
    const int32_t* itag;       // *itag + 1 (k_fill_touched's tag); nullptr: the offsets tell
    // replay deferred to the scan launch behind this one (claims != nullptr): pass p's claimed rows
    // (key, s0) at claims[p per ..), their number at nclaim[p], the replay target step at *claim_t
    int2* claims;
    int32_t* nclaim;
    int32_t* claim_t;
};

// The claimed rows crow[0, ncl) (their steps cstep) replayed to step t, p only under P-ahead: the
// block's 4 waves share the (row, 128-element slice) items, kRepC per wave at a time (2 in the
// update launch's count blocks keep its 72-VGPR cap unspilled).  Whole block; lut holds the bias-
// corrected lr of steps t, t - 1, ...
template <int kRepC = 2>
__device__ __forceinline__ void replay_claimed(float* __restrict__ embf, float* __restrict__ mf, float* __restrict__ vf,
                                               int W, int ncl, const int* crow, const int* cstep, int t,
                                               const float* lut, float lr, float b1, float b2, float eps,
                                               int wv, int nwv) {
    const int lane = threadIdx.x & 63;
    const int per_row = (W + 127) >> 7;
    const int items = ncl * per_row;
    // item it = row it / per_row, elements (it % per_row) * 128 + 2 lane + {0, 1} (W is a
    // multiple of 4); wave wv of the nwv sharing the rows takes it = wv + nwv j (wave-uniform: the
    // step loops do not diverge)
    const f32x2 z2 = {0.f, 0.f};
    for (int i0 = wv; i0 < items; i0 += nwv * kRepC) {
        f32x2 p[kRepC], mm[kRepC], vv[kRepC];
        size_t e[kRepC];
        int sr[kRepC];
        bool act[kRepC];
#pragma unroll
        for (int j = 0; j < kRepC; ++j) {
            const int it = i0 + nwv * j;
            const int k = it < items ? it / per_row : 0;
            const int q = (it - k * per_row) * 128 + 2 * lane;
            act[j] = it < items && q < W;
            sr[j] = it < items ? cstep[k] : t;
            e[j] = (size_t)crow[k] * W + (act[j] ? q : 0);
            p[j] = act[j] ? *reinterpret_cast<const f32x2*>(embf + e[j]) : z2;
            mm[j] = act[j] ? *reinterpret_cast<const f32x2*>(mf + e[j]) : z2;
            vv[j] = act[j] ? *reinterpret_cast<const f32x2*>(vf + e[j]) : z2;
        }
#if NCF_REPLAY_UNROLL > 1
#pragma unroll
        for (int j = 0; j < kRepC; ++j) replay2<NCF_REPLAY_UNROLL>(p[j], mm[j], vv[j], sr[j], t, lut, lr, b1, b2, eps);
#else
        // the items' chains advance together (same per-element arithmetic, step by step)
        int smin = t;
#pragma unroll
        for (int j = 0; j < kRepC; ++j) smin = sr[j] < smin ? sr[j] : smin;
        for (int st = smin + 1; st <= t; ++st) {
            const float lrt = t - st < kLrLut ? lut[t - st] : adam_lr_t(lr, b1, b2, st);
#pragma unroll
            for (int j = 0; j < kRepC; ++j)
                if (st > sr[j]) adam2_zero(p[j], mm[j], vv[j], lrt, b1, b2, eps);
        }
#endif
#pragma unroll
        for (int j = 0; j < kRepC; ++j) {
            if (act[j]) {
                *reinterpret_cast<f32x2*>(embf + e[j]) = p[j];
                if (!NCF_AHEAD_P_ONLY) {  // P-ahead: the next update re-derives m and v
                    *reinterpret_cast<f32x2*>(mf + e[j]) = mm[j];
                    *reinterpret_cast<f32x2*>(vf + e[j]) = vv[j];
                }
            }
        }
    }
}

// The replay half of the catch-up ahead in the scan launch (CountAhead::claims): one block per
// count pass, the pass's claims staged in LDS, then replay_claimed — the same items, arithmetic
// and stores as when the count blocks replay (bitwise), off the touched-row update's HBM stream.
struct ReplayAhead {
    int npass;                 // 0: none
    int per;
    const int2* claims;
    const int32_t* nclaim;
    const int32_t* claim_t;
    float *emb, *m, *v;
    int W;
    float lr, b1, b2, eps;
};
#ifndef NCF_DEFER_OWED
#define NCF_DEFER_OWED 4   // deferred replay: rows owing at most this many steps go to the scan launch
#endif
constexpr int kDeferOwed = NCF_DEFER_OWED;
#ifndef NCF_DEFER_LONG_REPC
#define NCF_DEFER_LONG_REPC 1   // items in flight per wave of the count blocks' own (long) replays
#endif
#ifndef NCF_REPLAY_PASSES
#define NCF_REPLAY_PASSES 2   // count passes per replay block of the scan launch (4 items per wave in flight)
#endif
constexpr int kReplayPasses = NCF_REPLAY_PASSES;
__device__ inline void replay_ahead_block(const ReplayAhead& ra, int blk) {
    static_assert(kReplayPasses * 64 <= kBlock, "one claim slot per thread");
    __shared__ float lut[kLrLut];
    __shared__ int crow[64 * kReplayPasses], cstep[64 * kReplayPasses];
    // this block's passes' claims, compacted into LDS (every thread reads the passes' counts)
    const int p0 = blk * kReplayPasses;
    int cnt[kReplayPasses];
#pragma unroll
    for (int j = 0; j < kReplayPasses; ++j) cnt[j] = p0 + j < ra.npass ? ra.nclaim[p0 + j] : 0;
    const int t = *ra.claim_t;
    const int jp = (int)threadIdx.x >> 6, q = (int)threadIdx.x & 63;
    int before = 0, ncl = 0;
#pragma unroll
    for (int j = 0; j < kReplayPasses; ++j) {
        before += j < jp ? cnt[j] : 0;
        ncl += cnt[j];
    }
    if (jp < kReplayPasses && q < cnt[jp]) {
        const int2 c = ra.claims[(int64_t)(p0 + jp) * ra.per + q];
        crow[before + q] = c.x;
        cstep[before + q] = c.y;
    }
    if (ncl > 0 && threadIdx.x < kLrLut)
        lut[threadIdx.x] = t - (int)threadIdx.x >= 1 ? adam_lr_t(ra.lr, ra.b1, ra.b2, t - threadIdx.x) : 0.f;
    if (ncl == 0) return;  // (block-uniform)
    __syncthreads();
    replay_claimed<2 * kReplayPasses>(ra.emb, ra.m, ra.v, ra.W, ncl, crow, cstep, t, lut, ra.lr, ra.b1, ra.b2,
                                      ra.eps, (int)threadIdx.x >> 6, kBlock / 64);
}

// the dense layers' Adam (k_mlp_update<ADAM>'s work) in blocks >= nupd + ncount of the same launch;
// two_level: in the FIRST blocks of the launch, 16 parameters per block, from the raw slabs
// the step's group metrics (groups <= 8, not computed in the forward/backward kernel) in the
// first blocks of the touched-row update launch: nblocks partials
struct MetricsTail {
    int nblocks;               // 0: none
    const float* probs;
    const float* labels;
    int64_t ng;
    int group, k;
    float *part_hit, *part_dcg;
};

struct MlpTail {
    int nblocks;               // 0: none
    float *p, *m, *v;
    int P;
    const float* slabs;
    int nslab;
    const int32_t* step;
    float lr, b1, b2, eps;
    L2Table l2t;
    float* part_reg;
    int two_level;
};

// Both levels of the slab reduction for 16 parameters (16 P0 .. 16 P0 + 15, P0 = blk): thread
// (c, j) sums chunk c of the slabs for parameter j (k_slab_partial's chunks and order), then the
// threads c == 0 add the chunk sums (k_mlp_update's order) and return the gradient — bitwise the
// k_slab_partial + k_mlp_update pair.  Whole block; the value is meaningful where c == 0, i < P.
__device__ __forceinline__ float slab_grad16(const float* __restrict__ slabs, int P, int nslab, int blk) {
    __shared__ float part[16][17];
    const int c = threadIdx.x >> 4, j = threadIdx.x & 15, i = blk * 16 + j;
    const int per = (nslab + kSlabSplit - 1) / kSlabSplit, nch = (nslab + per - 1) / per;
    if (c < nch && i < P) {
        const int s0 = c * per, s1 = min(nslab, s0 + per);
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int s = s0;
        for (; s + 4 <= s1; s += 4) {
            a0 += slabs[(size_t)(s + 0) * P + i];
            a1 += slabs[(size_t)(s + 1) * P + i];
            a2 += slabs[(size_t)(s + 2) * P + i];
            a3 += slabs[(size_t)(s + 3) * P + i];
        }
        for (; s < s1; ++s) a0 += slabs[(size_t)s * P + i];
        part[c][j] = (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
    float g = 0.f;
    if (c == 0 && i < P) {
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int s = 0;
        for (; s + 4 <= nch; s += 4) {
            a0 += part[s + 0][j];
            a1 += part[s + 1][j];
            a2 += part[s + 2][j];
            a3 += part[s + 3][j];
        }
        for (; s < nch; ++s) a0 += part[s][j];
        g = (a0 + a1) + (a2 + a3);
    }
    return g;
}

// Dense-layer Adam straight from the fused kernel's slabs (every L2 factor zero), 16 parameters
// per block: slab_grad16, then mlp_update_body's Adam (the same expressions)
__device__ __forceinline__ void mlp_slabs_adam(const MlpTail& mt, int blk) {
    const float g = slab_grad16(mt.slabs, mt.P, mt.nslab, blk);
    const int i = blk * 16 + (threadIdx.x & 15);
    if ((threadIdx.x >> 4) == 0 && i < mt.P) {
        const int t = *mt.step + 1;
        const float lr_t = adam_lr_t(mt.lr, mt.b1, mt.b2, t);
        float w = mt.p[i];
        const float mm = mt.b1 * mt.m[i] + (1.0f - mt.b1) * g;
        const float vv = mt.b2 * mt.v[i] + (1.0f - mt.b2) * (g * g);
        w -= lr_t * mm / (sqrtf(vv) + mt.eps);
        mt.m[i] = mm;
        mt.v[i] = vv;
        mt.p[i] = w;
    }
}

// Lists left unsorted by the in-kernel fill (FillArgs, ncf_internal.h): the touched-row update
// orders each row's contributions itself.  A row of c <= hc entries: lane q of its row group holds
// entry q, its rank (how many of the row's entries are smaller; the entries are distinct
// contribution ids) comes from c shuffles and one ds_permute puts it at lane rank, so the sum
// reads the ids in ascending order from the lanes — the order of a sorted list, so the same sum
// bitwise.  Longer rows (heavy: listed by the fill) go to the launch's first blocks, which sort
// block-wide by rank through LDS into slist and update the row.  A counter left at a touched row
// (a batch counted ahead whose ids changed since) is flagged and cleared here, as k_sort does.
struct SortRows {
    int on;                    // 0: the lists are sorted (a fill + sort launch built the index)
    int hc;                    // rows of more entries are heavy
    int nheavy;                // heavy blocks (the first blocks of the launch)
    const int32_t* heavy;      // touched-list positions of the heavy rows
    const int32_t* heavy_n;
    int32_t* cursor;           // ws cnt
    int32_t* err;
    int32_t* slist;            // heavy rows' lists, sorted (indexed like the list)
    int mcap;                  // contribution ids are below this (2 * max batch): a stale list slot is clamped
    const int32_t* drop;       // ws stale_step: nonzero — the step is dropped (fill_wave): only the next
                               // batch's count and catch-up ahead run, the latter to *step
    const int32_t* local;      // this step's per-block key offsets and block totals (a key's count:
    const int32_t* tot;        // the next key's offset minus its own; the fill writes no offs array)
};
constexpr int kHeavyChunk = 1024;  // heavy-row list entries staged in LDS per round

// Row r's Adam step t from its c contributions, ids id(j) ascending; lanes q, q + qstep, ... of
// its w4 float4 elements.  k: the m / v decays it still owes (P-ahead / caught-up rows), fresh:
// pristine (m = v = 0, only p read).  The element expressions of every touched-row path.
template <class ID>
__device__ __forceinline__ void row_adam(float4* __restrict__ emb, float4* __restrict__ m4, float4* __restrict__ v4,
                                         const float4* __restrict__ gs, uint32_t w4, int64_t r, int c, uint32_t q0,
                                         uint32_t qstep, int k, bool fresh, float lr_t, float b1, float b2, float eps,
                                         ID id) {
    for (uint32_t q = q0; q < w4; q += qstep) {
        const size_t e = (size_t)r * w4 + q;
        float4 p = emb[e], m = make_float4(0.f, 0.f, 0.f, 0.f), v = m;
        if (!fresh) {
            m = m4[e];
            v = v4[e];
        }
        for (int j = 0; j < k; ++j) decay4(m, v, b1, b2);
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        int j = 0;
        for (; j + 4 <= c; j += 4) {
            const int c0 = id(j), c1 = id(j + 1), c2 = id(j + 2), c3 = id(j + 3);
            const float4 g0 = gs[(size_t)c0 * w4 + q], g1 = gs[(size_t)c1 * w4 + q];
            const float4 g2 = gs[(size_t)c2 * w4 + q], g3 = gs[(size_t)c3 * w4 + q];
            g = f4add(g, g0);
            g = f4add(g, g1);
            g = f4add(g, g2);
            g = f4add(g, g3);
        }
        for (; j < c; ++j) g = f4add(g, gs[(size_t)id(j) * w4 + q]);
        adam4(p, m, v, g, lr_t, b1, b2, eps);
        st_stream(&emb[e], p);
        st_stream(&m4[e], m);
        st_stream(&v4[e], v);
    }
}

// A heavy row's list [o, o + c) (in-kernel fill: unsorted; its lowest `res` slots unfilled) sorted
// ascending into slist[o, o + c - res), block-wide: each entry's rank among the row's from the
// list staged through LDS a chunk at a time.  Whole block; ends with a barrier (the sorted list is
// the workgroup's own stores).
__device__ inline void sort_heavy_list(const int32_t* __restrict__ clist, int o, int c, int res, int mcap,
                                       int32_t* __restrict__ slist, int* chunk) {
    int e[4], rk[4];
    for (int j0 = 0; j0 < c; j0 += 4 * kBlock) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int j = j0 + a * kBlock + (int)threadIdx.x;
            e[a] = j >= res && j < c ? (int)min((unsigned)clist[o + j], (unsigned)(mcap - 1)) : INT_MAX;
            rk[a] = 0;
        }
        for (int i0 = 0; i0 < c; i0 += kHeavyChunk) {
            const int ni = min(kHeavyChunk, c - i0);
            __syncthreads();
            for (int i = threadIdx.x; i < ni; i += kBlock)
                chunk[i] = i0 + i >= res ? (int)min((unsigned)clist[o + i0 + i], (unsigned)(mcap - 1)) : INT_MAX;
            __syncthreads();
            for (int i = 0; i < ni; ++i) {
                const int x = chunk[i];
#pragma unroll
                for (int a = 0; a < 4; ++a) rk[a] += x < e[a];
            }
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int j = j0 + a * kBlock + (int)threadIdx.x;
            if (j >= res && j < c) slist[o + rk[a]] = e[a];
        }
    }
    __syncthreads();
}

template <bool UNSORTED>
__global__ __launch_bounds__(kBlock, UNSORTED ? NCF_TOUCHED_MIN_BLOCKS_UNSORTED : NCF_TOUCHED_MIN_BLOCKS) void k_emb_adam_touched(float4* __restrict__ emb, float4* __restrict__ m4,
                                                             float4* __restrict__ v4, uint32_t w4,
                                                             const int32_t* __restrict__ list,
                                                             const int2* __restrict__ toc,
                                                             const int32_t* __restrict__ nlist,
                                                             const int32_t* __restrict__ offs,
                                                             const int32_t* __restrict__ clist,
                                                             const float4* __restrict__ gs,
                                                             int32_t* __restrict__ row_step, const int32_t* step,
                                                             float lr, float b1, float b2, float eps,
                                                             CountAhead ca, MlpTail mt, MetricsTail mm,
                                                             SortRows so) {
    // block order: [count (+ catch-up ahead)] [touched-row update] [dense-layer Adam]: the
    // latency-bound replay blocks are dispatched first, so they run under the HBM-bound update
    // (interleaving them one in every (nupd + ncount) / ncount blocks was measured slower: 60.2
    // vs 53.3 us at config C — their chains are the launch's long pole)
    // (two_level: the dense-layer blocks come first — each waits one round of slab loads, under
    // everything else)
    int b = (int)blockIdx.x;
    // a dropped step (stale counted set, unsorted lists only): nothing of it is applied
    const bool dropped = UNSORTED && so.drop && *so.drop != 0;
    if (UNSORTED && b < so.nheavy) {
        if (dropped) return;
        // heavy rows (lists longer than so.hc, unsorted): one per block and pass
        __shared__ int chunk[kHeavyChunk];
        const int t = *step + 1;
        const float lr_t = adam_lr_t(lr, b1, b2, t);
        const int nh = *so.heavy_n;
        for (int hi = b; hi < nh; hi += so.nheavy) {
            const int u = so.heavy[hi];
            const int64_t r = list[u];
            const int2 oc = toc[u];
            const int o = oc.x, c = oc.y;
#if NCF_DEBUG_BOUNDS == 1
            if (u < 0 || u >= so.mcap || r < 0 || r >= ca.lazy_rows || o < 0 || c < 0 || o + c > so.mcap) {
                if (threadIdx.x == 0) printf("heavy %d: u %d nlist %d r %lld o %d c %d (skipped)\n", hi, u, *nlist, (long long)r, o, c);
                continue;
            }
#endif
            // the key's residue: slots [0, res) were never filled (fill_wave; the light rows' rule)
            const int res = min(max(so.cursor[r], 0), c);
            sort_heavy_list(clist, o, c, res, so.mcap, so.slist, chunk);
            const bool mine = r < ca.lazy_rows;
            int rs = mine ? row_step[r] : 0;
            const bool fresh = rs == NCF_ROW_PRISTINE;
            if (rs < 0) rs = pahead_s0(rs);
            const int k = NCF_CATCHUP_P_ONLY && mine && !fresh ? t - 1 - rs : 0;
            if (mine)
                row_adam(emb, m4, v4, gs, w4, r, c - res, threadIdx.x, kBlock, k, fresh, lr_t, b1, b2, eps,
                         [&](int j) { return so.slist[o + j]; });
            if (threadIdx.x == 0) {
                if (mine) row_step[r] = t;
                if (so.cursor[r] != 0) {
                    atomicOr(so.err, kErrStaleCount);
                    so.cursor[r] = 0;
                }
            }
        }
        return;
    }
    b -= so.nheavy;
    // the step's hr/dcg partials (k_group_metrics' work, groups <= 8) in the first blocks: the
    // probabilities are final once the forward/backward launch before this one is done
    if (b < mm.nblocks) {
        if (dropped) return;
        group_metrics_body(mm.probs, mm.labels, mm.ng, mm.group, mm.k, nullptr, nullptr, mm.part_hit, mm.part_dcg, b);
        return;
    }
    b -= mm.nblocks;
    if (mt.two_level) {
        if (b < mt.nblocks) {
            if (!dropped) mlp_slabs_adam(mt, b);
            return;
        }
        b -= mt.nblocks;
    } else if (b >= ca.nupd + ca.ncount) {
        if (dropped) return;
        mlp_update_body<NCF_OPT_ADAM>(mt.p, mt.m, mt.v, mt.P, mt.slabs, mt.nslab, nullptr, nullptr, 1, 0, mt.step,
                                      mt.lr, mt.b1, mt.b2, mt.eps, mt.l2t, mt.part_reg,
                                      b - ca.nupd - ca.ncount);
        return;
    }
    if (b < ca.ncount) {
        const int cblk = b;  // this block's index among the count blocks
        // count the NEXT batch's contributions (k_count's work) while this step's rows stream; the
        // counters are free here (the fill of this step's index emptied them).
        // Catch-up ahead (ca.replay): a row of the next batch that this step does not touch owes
        // the zero-gradient steps (row_step, t] — this step's included — and nothing else in this
        // launch reads or writes it, so it is replayed here (k_emb_catchup's work, same per-step
        // arithmetic: bitwise) under the touched-row update, instead of in a launch of its own
        // before the next forward pass.  One lane claims a row (CAS on row_step: a user's
        // repeated contributions replay it once) and leaves p, m, v and row_step at step t.
        // (A dropped step applies nothing: the next batch's rows are caught up to *step instead.)
        __shared__ float lut[kLrLut];
        const int t = *step + (dropped ? 0 : 1);
        const int tagc = ca.seen ? *ca.itag + 1 : 0;
        const bool defer = ca.claims != nullptr;
        if (ca.replay && threadIdx.x < kLrLut)
            lut[threadIdx.x] = t - (int)threadIdx.x >= 1 ? adam_lr_t(lr, b1, b2, t - threadIdx.x) : 0.f;
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const int W = 4 * (int)w4;
        // one pass of one wave: count contributions [cb, cb + per) and claim their stale rows;
        // returns the claims' ballot (the claiming lanes in ascending order)
        const int per = ca.per;
        auto count_pass = [&](int64_t cb, int& key, int& s0) -> uint64_t {
            const int64_t c = cb + lane;
            bool ok = false;
            key = 0;
            if (lane < per && c < ca.m) {
                const int64_t i = c >> 1;
                const int id = (c & 1) ? ca.items[i] : ca.users[i];
                const int bound = (c & 1) ? ca.I : ca.U;
                ok = (unsigned)id < (unsigned)bound && ((c & 1) || !folded_user(ca.users, i, ca.fold));
                key = (c & 1) ? ca.U + id : id;
            }
            // the row's step and offsets go out before the count's atomic returns (one memory
            // round trip); the lane whose run is the key's first occurrence in the next batch
            // (its count was 0) owns the row's replay — no claim atomic of its own
            int o0 = 0, o1 = 0, sv = t;
            if (ca.replay && ok && key < ca.lazy_rows) {
                if (UNSORTED) {   // (the in-kernel fill writes no offs array: the key's count instead)
                    o0 = so.local[key];
                    o1 = (key + 1) % kScanBlock != 0 ? so.local[key + 1] : so.tot[key / kScanBlock];
                } else if (ca.seen) {   // sparse index: no offsets at keys outside the batch
                    o1 = ca.seen[key] == tagc;
                } else {
                    o0 = offs[key];
                    o1 = offs[key + 1];
                }
                sv = row_step[key];
            }
            const bool first = wave_run_count<true>(ca.cnt, key, ok);
            // not in this step's batch (this launch's update blocks do not touch it) and behind
            // (a P-ahead mark, negative, never occurs here: the previous step's update consumed it)
            const bool claim = ca.replay && first && key < ca.lazy_rows && o1 == o0 && (unsigned)sv < (unsigned)t;
            s0 = sv;
            if (claim) row_step[key] = NCF_AHEAD_P_ONLY ? pahead_mark(s0) : t;
            return __ballot(claim);
        };
        float* embf = reinterpret_cast<float*>(emb);
        float* mf = reinterpret_cast<float*>(m4);
        float* vf = reinterpret_cast<float*>(v4);
        if (defer) {
            // replay in the scan launch behind this one (ReplayAhead): every wave counts passes of
            // its own and writes the claims (key, s0) of rows owing at most kDeferOwed steps at the
            // pass's slots, their number per pass; it replays the rest itself (the long chains stay
            // under this launch's HBM stream — in the short scan launch they would be its critical path)
            __shared__ int wrow[kBlock / 64][64], wstep[kBlock / 64][64];
            __syncthreads();  // lut
            const int64_t nw = (int64_t)ca.ncount * (kBlock / 64);
            const uint64_t below = (1ull << lane) - 1;
            for (int64_t ps = (int64_t)cblk * (kBlock / 64) + wv; ps * per < ca.m; ps += nw) {
                int key, s0;
                const uint64_t cm = count_pass(ps * per, key, s0);
                const bool mine = (cm >> lane) & 1ull;
                const bool near = mine && t - s0 <= kDeferOwed;
                const uint64_t sm = __ballot(near), lm = cm & ~sm;
                if (near) ca.claims[ps * per + __popcll(sm & below)] = make_int2(key, s0);
                if (lane == 0) ca.nclaim[ps] = __popcll(sm);
                if (lm) {  // (wave-uniform)
                    if (mine && !near) {
                        const int slot = __popcll(lm & below);
                        wrow[wv][slot] = key;
                        wstep[wv][slot] = s0;
                    }
                    __builtin_amdgcn_wave_barrier();
                    replay_claimed<NCF_DEFER_LONG_REPC>(embf, mf, vf, W, __popcll(lm), wrow[wv], wstep[wv], t, lut, lr,
                                                        b1, b2, eps, 0, 1);
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (cblk == 0 && threadIdx.x == 0) *ca.claim_t = t;
            return;
        }
        // a block takes ca.per contributions per pass: wave 0 counts them and claims the stale
        // rows, then the block's 4 waves share the claimed rows' replay, kRep (row, 64-element
        // slice) items per wave at a time with all their loads in flight and their step chains
        // interleaved — many short replay chains in flight (small batches get 16 contributions
        // per block: their rows owe many steps each), one memory round trip per batch of items
        __shared__ int crow[64], cstep[64], ncl;
        for (int64_t cb = (int64_t)cblk * per; cb < ca.m; cb += (int64_t)ca.ncount * per) {
            __syncthreads();  // lut ready, the previous pass's replay done
            if (wv == 0) {
                int key, s0;
                const uint64_t cm = count_pass(cb, key, s0);
                if ((cm >> lane) & 1ull) {
                    const int slot = __popcll(cm & ((1ull << lane) - 1));
                    crow[slot] = key;
                    cstep[slot] = s0;
                }
                if (lane == 0) ncl = __popcll(cm);
            }
            __syncthreads();
            replay_claimed(embf, mf, vf, W, ncl, crow, cstep, t, lut, lr, b1, b2, eps, wv, kBlock / 64);
        }
        return;
    }
    if (dropped) {
        // Nothing of the step is applied; the fill's leftover cursors (entries counted but absent:
        // every counted key is a touched row) go back to zero for the next index.  The counted rows
        // the previous launch caught up ahead are P-ahead (p at *step, m and v owed from s0): with
        // the step gone, a row that the next batch does not touch would keep that mark past the
        // next bump, its p a step behind what the mark promises.  Settle them here — m and v
        // decayed to *step (the per-step decay's arithmetic, as the stale gate does), row_step =
        // *step — so that row_step again tells the step of all three.  (This launch's count blocks
        // never claim a negative or current mark, so nothing else writes these rows.)
        const int64_t nt = *nlist;
        const int tdrop = *step;
        const int lane = threadIdx.x & 63;
        const int W = 4 * (int)w4;
        float* mf = reinterpret_cast<float*>(m4);
        float* vf = reinterpret_cast<float*>(v4);
        const int64_t wave = ((int64_t)(b - ca.ncount) * kBlock + threadIdx.x) >> 6;
        const int64_t nw = ((int64_t)ca.nupd * kBlock) >> 6;
        for (int64_t i0 = wave * 64; i0 < nt; i0 += nw * 64) {  // wave-uniform
            const int64_t i = i0 + lane;
            const int r = i < nt ? list[i] : -1;
            int rs = 0;
            if (r >= 0) {
                if (so.cursor[r] != 0) {
                    atomicOr(so.err, kErrStaleCount);
                    so.cursor[r] = 0;
                }
                if (r < ca.lazy_rows) rs = row_step[r];
            }
            uint64_t pm = __ballot(rs < 0);
            while (pm) {
                const int src = __ffsll((unsigned long long)pm) - 1;
                pm &= pm - 1;
                const int64_t rr = __shfl(r, src, 64);
                const int s0 = pahead_s0(__shfl(rs, src, 64));
                for (int q = lane; 2 * q < W; q += 64) {
                    const size_t e = (size_t)rr * W + 2 * q;
                    f32x2 m = *reinterpret_cast<const f32x2*>(mf + e);
                    f32x2 v = *reinterpret_cast<const f32x2*>(vf + e);
                    for (int st = s0 + 1; st <= tdrop; ++st) decay2(m, v, b1, b2);
                    *reinterpret_cast<f32x2*>(mf + e) = m;
                    *reinterpret_cast<f32x2*>(vf + e) = v;
                }
                if (lane == 0) row_step[rr] = tdrop;
            }
        }
        return;
    }
#if NCF_DIAG_UPD == 2  // diagnostic timing builds only (wrong numerics): no touched-row update
    return;
#endif
    const int ublk = b - ca.ncount;   // this block's index among the update blocks
    const RowLanes rl(w4);
    const int t = *step + 1;
    if constexpr (UNSORTED) {
        // unsorted lists (in-kernel fill): every lane runs the row loop (its shuffles), a lane outside
        // a row group (w4 not dividing 64) or past the list with c = 0
        const float lr_t = adam_lr_t(lr, b1, b2, t);
        const int64_t n = *nlist;
        const int lane = threadIdx.x & 63;
        const int gsz = w4 <= 64 ? (int)w4 : 64;            // lanes of a row group
        const int base = w4 <= 64 ? rl.sub * (int)w4 : 0;   // its first lane
        const int ql = lane - base;                          // this lane's entry slot
        const int64_t wave = ((int64_t)ublk * kBlock + threadIdx.x) >> 6;
        const int64_t wstride = ((int64_t)ca.nupd * kBlock) >> 6;
        const int64_t istep = wstride * rl.rpw;
        // software pipeline: the next row's (row, list offset, count) load while this row runs
        int r = 0;
        int2 oc = make_int2(0, 0);
        if (rl.on && wave * rl.rpw + rl.sub < n) {
            r = list[wave * rl.rpw + rl.sub];
            oc = toc[wave * rl.rpw + rl.sub];
        }
        for (int64_t i0 = wave * rl.rpw; i0 < n; i0 += istep) {  // wave-uniform
            const int64_t i = i0 + rl.sub;
            bool has = rl.on && i < n;
            int rn = 0;
            int2 ocn = make_int2(0, 0);
            if (rl.on && i + istep < n) {
                rn = list[i + istep];
                ocn = toc[i + istep];
            }
#if NCF_DEBUG_BOUNDS == 1
            if (has && (i >= so.mcap || r < 0 || r >= ca.lazy_rows || oc.x < 0 || oc.y < 0 || oc.x + oc.y > so.mcap)) {
                if (ql == 0) printf("row %lld of %lld: r %d o %d c %d (skipped)\n", (long long)i, (long long)n, r, oc.x, oc.y);
                has = false;
                r = 0;
                oc = make_int2(0, 0);
            }
#endif
            const bool heavy = oc.y > so.hc;
            const int c = heavy ? 0 : oc.y;
            const bool mine = has && !heavy && r < ca.lazy_rows;
            int rs = mine ? row_step[r] : 0;
            // the key's residue (normally 0): its lowest `res` slots were never filled — ids changed
            // after they were counted, with fewer contributions here and no overflow anywhere (else
            // the step is dropped) — so the row sums the slots [res, c) only (fill_wave)
            const int res = has && !heavy ? min(max(so.cursor[r], 0), c) : 0;
            const bool valid = ql >= res && ql < c;
            int e = valid ? (int)min((unsigned)clist[oc.x + ql], (unsigned)(so.mcap - 1)) : INT_MAX;
            // the wave's longest light list (its row groups' counts, read lane by lane)
            int cmax = 0;
            for (int g = 0; g < rl.rpw; ++g) cmax = max(cmax, __builtin_amdgcn_readlane(c, g * (int)w4));
            int rank = 0;
            for (int j = 0; j < cmax; ++j) {
                const int x = __shfl(e, base + j, 64);
                rank += j < c && x < e;
            }
            // entry ql goes to lane base + rank (a permutation of the group's first c lanes: the
            // unfilled slots' lanes to [c - res, c); the other lanes keep their own value)
            const int cv = c - res;
            const int to = valid ? base + rank : ql < res ? base + cv + ql : lane;
            const int srt = __builtin_amdgcn_ds_permute(to * 4, e);
            if (res != 0 && ql == 0) {
                atomicOr(so.err, kErrStaleCount);
                so.cursor[r] = 0;
            }
            const bool fresh = rs == NCF_ROW_PRISTINE;
            if (rs < 0) rs = pahead_s0(rs);
            const int k = NCF_CATCHUP_P_ONLY && mine && !fresh ? t - 1 - rs : 0;
            // the sum's ids from the lanes: a wave-uniform loop over the longest list, masked per row
            for (uint32_t q = w4 <= 64 ? (uint32_t)ql : (uint32_t)lane; ; q += 64) {
                const bool act = mine && q < w4 && ql < gsz;
                const size_t ee = (size_t)r * w4 + (act ? q : 0);
                // (explicit branches, no `c ? a[i] : local` lvalue selects: those compile to a flat load
                // through a selected pointer, the local's being a scratch address)
                float4 p = make_float4(0.f, 0.f, 0.f, 0.f), m = p, v = p;
                if (act) {
                    p = emb[ee];
                    if (!fresh) {
                        m = m4[ee];
                        v = v4[ee];
                    }
                }
                for (int j = 0; j < k; ++j) decay4(m, v, b1, b2);
                float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
                for (int j = 0; j < cmax; j += 4) {
                    const int c0 = __shfl(srt, base + j, 64), c1 = __shfl(srt, base + min(j + 1, gsz - 1), 64);
                    const int c2 = __shfl(srt, base + min(j + 2, gsz - 1), 64);
                    const int c3 = __shfl(srt, base + min(j + 3, gsz - 1), 64);
                    const bool v0 = act && j < cv, v1 = act && j + 1 < cv, v2 = act && j + 2 < cv, v3 = act && j + 3 < cv;
#if NCF_DEBUG_BOUNDS == 1
                    if ((v0 && (unsigned)c0 >= (unsigned)so.mcap) || (v1 && (unsigned)c1 >= (unsigned)so.mcap) ||
                        (v2 && (unsigned)c2 >= (unsigned)so.mcap) || (v3 && (unsigned)c3 >= (unsigned)so.mcap))
                        printf("sum r %d j %d c %d ids %d %d %d %d\n", r, j, c, c0, c1, c2, c3);
#endif
                    float4 g0, g1, g2, g3;
                    if (v0) g0 = gs[(size_t)c0 * w4 + q];
                    if (v1) g1 = gs[(size_t)c1 * w4 + q];
                    if (v2) g2 = gs[(size_t)c2 * w4 + q];
                    if (v3) g3 = gs[(size_t)c3 * w4 + q];
                    if (v0) g = f4add(g, g0);
                    if (v1) g = f4add(g, g1);
                    if (v2) g = f4add(g, g2);
                    if (v3) g = f4add(g, g3);
                }
                if (act) {
                    adam4(p, m, v, g, lr_t, b1, b2, eps);
                    st_stream(&emb[ee], p);
                    st_stream(&m4[ee], m);
                    st_stream(&v4[ee], v);
                }
                if (w4 <= 64 || q + 64 >= w4) break;
            }
            if (ql == 0 && mine) row_step[r] = t;
            r = rn;
            oc = ocn;
        }
        return;
    }
    if (rl.on) {
        const float lr_t = adam_lr_t(lr, b1, b2, t);
        const int64_t n = *nlist;
        const int64_t wave = ((int64_t)ublk * kBlock + threadIdx.x) >> 6;
        const int64_t stride = (((int64_t)ca.nupd * kBlock) >> 6) * rl.rpw;
        int64_t i = wave * rl.rpw + rl.sub;
        // software pipeline over this lane group's rows: the next row's id and (list offset,
        // count) are loaded while the current row is processed, so the list -> contribution
        // chain of row i+1 overlaps row i's state and gradient traffic
        int r = i < n ? list[i] : 0;
        int2 oc = i < n ? toc[i] : make_int2(0, 0);
        for (; i < n; i += stride) {
            const int rn = i + stride < n ? list[i + stride] : 0;
            const int2 ocn = i + stride < n ? toc[i + stride] : make_int2(0, 0);
            const int o = oc.x;
            const int c = oc.y;
            // rows past lazy_rows (the list is ascending: its tail) are the caller's dense sweep's
            const bool mine = r < ca.lazy_rows;
            int rs = mine ? row_step[r] : 0;
            // a pristine row's moments are +0 (NCF_ROW_PRISTINE): only p is read
            const bool fresh = rs == NCF_ROW_PRISTINE;
            // a P-ahead row (caught up ahead by the previous step's launch): p at t - 1, m / v at s0
            if (rs < 0) rs = pahead_s0(rs);
            const int k = NCF_CATCHUP_P_ONLY && mine && !fresh ? t - 1 - rs : 0;  // m/v decay steps still owed
            for (uint32_t q = rl.q; mine && q < w4; q += rl.qstep) {
                const size_t e = (size_t)r * w4 + q;
                // the row's state does not depend on the gradient chain: its loads go out first
                const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                float4 p = emb[e], m = fresh ? z : m4[e], v = fresh ? z : v4[e];
                // k_emb_catchup brought p up to step t-1 and left m, v at row_step: the same
                // per-step decay adam4 applies with g = 0 (b1*m + 0, b2*v + 0), bitwise
                for (int j = 0; j < k; ++j) decay4(m, v, b1, b2);
                // contributions summed in ascending order; four gradient rows in flight at a time
                float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
                int j = 0;
                for (; j + 4 <= c; j += 4) {
                    const int c0 = clist[o + j], c1 = clist[o + j + 1], c2 = clist[o + j + 2], c3 = clist[o + j + 3];
                    const float4 g0 = gs[(size_t)c0 * w4 + q], g1 = gs[(size_t)c1 * w4 + q];
                    const float4 g2 = gs[(size_t)c2 * w4 + q], g3 = gs[(size_t)c3 * w4 + q];
                    g = f4add(g, g0);
                    g = f4add(g, g1);
                    g = f4add(g, g2);
                    g = f4add(g, g3);
                }
                for (; j < c; ++j) g = f4add(g, gs[(size_t)clist[o + j] * w4 + q]);
                adam4(p, m, v, g, lr_t, b1, b2, eps);
                st_stream(&emb[e], p);
                st_stream(&m4[e], m);
                st_stream(&v4[e], v);
            }
            if (rl.q == 0 && mine) row_step[r] = t;
            r = rn;
            oc = ocn;
        }
    }
}

// SGD on the hot rows only (cold rows: p - lr*0 = p, bitwise)
__global__ __launch_bounds__(kBlock) void k_emb_sgd_hot(float4* __restrict__ emb, uint32_t n4, uint32_t w4,
                                                        const int32_t* __restrict__ offs,
                                                        const int32_t* __restrict__ list,
                                                        const float4* __restrict__ gs, float lr) {
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += gridDim.x * blockDim.x) {
        const uint32_t r = e / w4;
        const int o = offs[r];
        const int c = offs[r + 1] - o;
        if (c == 0) continue;
        const uint32_t q = e - r * w4;
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < c; ++j) g = f4add(g, gs[(size_t)list[o + j] * w4 + q]);
        float4 p = emb[e];
        p.x -= lr * g.x; p.y -= lr * g.y; p.z -= lr * g.z; p.w -= lr * g.w;
        emb[e] = p;
    }
}

// lambda * sum(p^2) over the table (evaluation loss; no update)
__global__ __launch_bounds__(kBlock) void k_emb_reg(const float4* __restrict__ emb, uint32_t n4, float lam,
                                                    float* __restrict__ part_reg) {
    __shared__ float red[4];
    float reg = 0.0f;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += gridDim.x * blockDim.x) {
        const float4 p = emb[e];
        reg += lam * (p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w);
    }
    reg = block_sum_256(reg, red);
    if (threadIdx.x == 0) part_reg[blockIdx.x] = reg;
}

// Dense embedding gradient (data-parallel path): every row written.  Blocks stride over the
// elements with `nblk` blocks (the folded launch below adds blocks of other work after them).
__device__ __forceinline__ void emb_grad_dense_body(float4* __restrict__ out, uint32_t n4, uint32_t w4,
                                                    const int32_t* __restrict__ offs,
                                                    const int32_t* __restrict__ list,
                                                    const float4* __restrict__ gs, uint32_t blk, uint32_t nblk) {
    for (uint32_t e = blk * blockDim.x + threadIdx.x; e < n4; e += nblk * blockDim.x) {
        const uint32_t r = e / w4;
        const uint32_t q = e - r * w4;
        const int o = offs[r];
        const int c = offs[r + 1] - o;
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        int j = 0;
        for (; j + 4 <= c; j += 4) {  // four rows in flight, summed in ascending order
            const float4 g0 = gs[(size_t)list[o + j] * w4 + q], g1 = gs[(size_t)list[o + j + 1] * w4 + q];
            const float4 g2 = gs[(size_t)list[o + j + 2] * w4 + q], g3 = gs[(size_t)list[o + j + 3] * w4 + q];
            g = f4add(g, g0);
            g = f4add(g, g1);
            g = f4add(g, g2);
            g = f4add(g, g3);
        }
        for (; j < c; ++j) g = f4add(g, gs[(size_t)list[o + j] * w4 + q]);
        out[e] = g;
    }
}

__global__ __launch_bounds__(kBlock) void k_emb_grad_dense(float4* __restrict__ out, uint32_t n4, uint32_t w4,
                                                           const int32_t* __restrict__ offs,
                                                           const int32_t* __restrict__ list,
                                                           const float4* __restrict__ gs) {
    emb_grad_dense_body(out, n4, w4, offs, list, gs, blockIdx.x, gridDim.x);
}

// Replicated-row Adam/SGD with the all-reduced gradient in one launch: blocks [0, nupd) sweep the
// table rows with their dense gradient (k_emb_update<OPT, kGradDense, false>'s work), blocks
// >= nupd step the dense layers with theirs (k_mlp_update's work, no L2).  Used only with every
// L2 factor zero; bitwise the two separate launches.
template <int OPT>
__global__ __launch_bounds__(kBlock) void k_emb_update_mlp(float4* __restrict__ emb, float4* __restrict__ m4,
                                                           float4* __restrict__ v4, uint32_t n4, uint32_t w4,
                                                           const float4* __restrict__ dgrad, uint32_t nupd,
                                                           float* __restrict__ mp, float* __restrict__ mm,
                                                           float* __restrict__ mv, int P,
                                                           const float* __restrict__ mlp_grad,
                                                           const int32_t* __restrict__ step, float lr, float b1,
                                                           float b2, float eps) {
    if (blockIdx.x >= nupd) {
        const L2Table none{};
        mlp_update_body<OPT>(mp, mm, mv, P, nullptr, 0, mlp_grad, nullptr, 1, 0, step, lr, b1, b2, eps, none, nullptr,
                             (int)(blockIdx.x - nupd));
        return;
    }
    emb_update_body<OPT, kGradDense, false>(emb, m4, v4, n4, w4, nullptr, nullptr, nullptr, dgrad, step, lr, b1, b2,
                                            eps, 0.f, nullptr, blockIdx.x, nupd);
}

// Compact gradient of a row-sharded plan: out[u] = sum of unique row u's contributions
// (ascending c through the plan's sorted list); nuniq is read on the device.
__global__ __launch_bounds__(kBlock) void k_uniq_grad(float4* __restrict__ out, const int32_t* __restrict__ nuniq,
                                                      uint32_t w4, const int32_t* __restrict__ uoffs,
                                                      const int32_t* __restrict__ list,
                                                      const float4* __restrict__ gs) {
    const uint32_t n4 = (uint32_t)*nuniq * w4;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += gridDim.x * blockDim.x) {
        const uint32_t u = e / w4;
        const uint32_t q = e - u * w4;
        const int o = uoffs[u];
        const int c = uoffs[u + 1] - o;
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = 0; j < c; ++j) g = f4add(g, gs[(size_t)list[o + j] * w4 + q]);
        out[e] = g;
    }
}

// out[j] = table[rows[j]] (rows outside [0, nrows) give zero rows)
__global__ __launch_bounds__(kBlock) void k_gather_rows(float4* __restrict__ out, const float4* __restrict__ table,
                                                        int64_t nrows, const int32_t* __restrict__ rows, uint32_t n4,
                                                        uint32_t w4) {
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += gridDim.x * blockDim.x) {
        const uint32_t j = e / w4;
        const uint32_t q = e - j * w4;
        const int r = rows[j];
        out[e] = (r >= 0 && r < nrows) ? table[(size_t)r * w4 + q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// First level of the slab reduction: group c sums slabs [c*per, (c+1)*per) in order.
struct SummaryArgs {
    float* summary;            // nullptr: no summary block
    const float* part_bce;
    const float* part_hit;
    const float* part_dcg;
    int nbce, nmet;
    float n_groups;
    int32_t* drop;             // (stats launches) nonzero: the step was dropped — no summary, stats or
                               // bump; cleared here
};

__global__ __launch_bounds__(kBlock) void k_slab_partial(const float* __restrict__ slabs, int P, int nslab, int per,
                                                         float* __restrict__ part, SummaryArgs sa) {
    if (sa.summary && blockIdx.x == gridDim.x - 1) {  // the extra column: the batch summary
        if (blockIdx.y == 0) {
            __shared__ float red[4];
            summary_body(sa.part_bce, sa.nbce, sa.part_hit, sa.part_dcg, sa.nmet, sa.n_groups, nullptr, 0, nullptr, 0,
                         sa.summary, red);
        }
        return;
    }
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int s0 = blockIdx.y * per;
    const int s1 = min(nslab, s0 + per);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
        a0 += slabs[(size_t)(s + 0) * P + p];
        a1 += slabs[(size_t)(s + 1) * P + p];
        a2 += slabs[(size_t)(s + 2) * P + p];
        a3 += slabs[(size_t)(s + 3) * P + p];
    }
    for (; s < s1; ++s) a0 += slabs[(size_t)s * P + p];
    part[(size_t)blockIdx.y * P + p] = (a0 + a1) + (a2 + a3);
}


// The data-parallel gradient tail in one launch, both slab levels included: blocks [0, nmlp)
// reduce the slabs of 16 dense-layer parameters each into their gradient (slab_grad16: the
// k_slab_partial + k_mlp_update pair's order, bitwise), block nmlp writes the batch summary (when
// asked), the rest write the dense embedding gradient (ngrad blocks).  Dispatch order puts the
// short slab blocks first.
__global__ __launch_bounds__(kBlock) void k_part_tail(float4* __restrict__ out, uint32_t n4, uint32_t w4,
                                                      const int32_t* __restrict__ offs, const int32_t* __restrict__ list,
                                                      const float4* __restrict__ gs, uint32_t ngrad, int P,
                                                      const float* __restrict__ slabs, int nslab, int nmlp,
                                                      float* __restrict__ mlp_grad, SummaryArgs sa) {
    int b = (int)blockIdx.x;
    if (b < nmlp) {
        const float g = slab_grad16(slabs, P, nslab, b);
        const int i = b * 16 + (threadIdx.x & 15);
        if ((threadIdx.x >> 4) == 0 && i < P) mlp_grad[i] = g;
        return;
    }
    b -= nmlp;
    if (sa.summary) {
        if (b == 0) {
            __shared__ float red[4];
            summary_body(sa.part_bce, sa.nbce, sa.part_hit, sa.part_dcg, sa.nmet, sa.n_groups, nullptr, 0, nullptr, 0,
                         sa.summary, red);
            return;
        }
        --b;
    }
    emb_grad_dense_body(out, n4, w4, offs, list, gs, (uint32_t)b, ngrad);
}


// The dense gradient of the replicated rows [U, R) (the user-partitioned step's item rows) from the
// in-kernel fill's UNSORTED lists (FillArgs): each row's contributions ordered by the touched-row
// update's rules — a light row's entries ranked across the lanes of its row group, a heavy row's
// (more than hc entries) sorted block-wide into slist by the first blocks — so every row sums in
// ascending contribution order, bitwise the sorted index's emb_grad_dense_body; a counted key's
// unfilled slots (its residue, left for the update launch to clear) are skipped; a row without
// contributions gets zeros.  Offsets come from the scan ahead's per-block offsets (offs_local) and
// the block totals' prefixes (no offs array exists).
struct ItemGradArgs {
    const int32_t* local;      // ws offs_local
    const int32_t* tot;        // ws tot
    int nscan;                 // scan blocks (<= kMaxFillScan)
    const int32_t* clist;      // ws list
    const int32_t* cursor;     // ws cnt (residues; read only)
    const int32_t* touched;    // the fill's touched rows and their (offset, count)
    const int2* toc;
    const int32_t* heavy;      // touched-list positions of the heavy rows
    const int32_t* heavy_n;
    int nheavy;                // heavy blocks (the first blocks of the launch)
    int32_t* slist;            // sorted heavy lists (this launch writes the item rows' ranges)
    int hc, mcap;
};

__global__ __launch_bounds__(kBlock) void k_part_tail_unsorted(float4* __restrict__ out, int64_t U, int64_t R,
                                                               uint32_t w4, const float4* __restrict__ gs,
                                                               uint32_t ngrad, int P, const float* __restrict__ slabs,
                                                               int nslab, int nmlp, float* __restrict__ mlp_grad,
                                                               SummaryArgs sa, ItemGradArgs ig) {
    int b = (int)blockIdx.x;
    if (b < ig.nheavy) {
        __shared__ int chunk[kHeavyChunk];
        const int nh = *ig.heavy_n;
        for (int hi = b; hi < nh; hi += ig.nheavy) {
            const int u = ig.heavy[hi];
            const int64_t r = ig.touched[u];
            if (r < U || r >= R) continue;  // a user row: the touched-row update's (block-uniform)
            const int2 oc = ig.toc[u];
            const int res = min(max(ig.cursor[r], 0), oc.y);
            sort_heavy_list(ig.clist, oc.x, oc.y, res, ig.mcap, ig.slist, chunk);
            const int cv = oc.y - res;
            for (uint32_t q = threadIdx.x; q < w4; q += kBlock) {
                float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
                int j = 0;
                for (; j + 4 <= cv; j += 4) {
                    const int c0 = ig.slist[oc.x + j], c1 = ig.slist[oc.x + j + 1];
                    const int c2 = ig.slist[oc.x + j + 2], c3 = ig.slist[oc.x + j + 3];
                    const float4 g0 = gs[(size_t)c0 * w4 + q], g1 = gs[(size_t)c1 * w4 + q];
                    const float4 g2 = gs[(size_t)c2 * w4 + q], g3 = gs[(size_t)c3 * w4 + q];
                    g = f4add(g, g0);
                    g = f4add(g, g1);
                    g = f4add(g, g2);
                    g = f4add(g, g3);
                }
                for (; j < cv; ++j) g = f4add(g, gs[(size_t)ig.slist[oc.x + j] * w4 + q]);
                out[(size_t)(r - U) * w4 + q] = g;
            }
            __syncthreads();  // slist / chunk reused by the block's next heavy row
        }
        return;
    }
    b -= ig.nheavy;
    if (b < nmlp) {
        const float g = slab_grad16(slabs, P, nslab, b);
        const int i = b * 16 + (threadIdx.x & 15);
        if ((threadIdx.x >> 4) == 0 && i < P) mlp_grad[i] = g;
        return;
    }
    b -= nmlp;
    if (sa.summary) {
        if (b == 0) {
            __shared__ float red[4];
            summary_body(sa.part_bce, sa.nbce, sa.part_hit, sa.part_dcg, sa.nmet, sa.n_groups, nullptr, 0, nullptr, 0,
                         sa.summary, red);
            return;
        }
        --b;
    }
    // the dense pass: block prefixes of the scan-block totals in LDS, then row groups over [U, R)
    __shared__ int pre[kMaxFillScan];
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const int t0 = lane < ig.nscan ? ig.tot[lane] : 0, t1 = lane + 64 < ig.nscan ? ig.tot[lane + 64] : 0;
        int a0 = t0, a1 = t1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int x0 = __shfl_up(a0, d, 64), x1 = __shfl_up(a1, d, 64);
            if (lane >= d) a0 += x0, a1 += x1;
        }
        pre[lane] = a0 - t0;
        pre[lane + 64] = __shfl(a0, 63, 64) + a1 - t1;
    }
    __syncthreads();
    const RowLanes rl(w4);
    const int lane = threadIdx.x & 63;
    const int gsz = w4 <= 64 ? (int)w4 : 64;
    const int base = w4 <= 64 ? rl.sub * (int)w4 : 0;
    const int ql = lane - base;
    const int64_t wave = ((int64_t)b * kBlock + threadIdx.x) >> 6;
    const int64_t istep = (((int64_t)ngrad * kBlock) >> 6) * rl.rpw;
    for (int64_t i0 = U + wave * rl.rpw; i0 < R; i0 += istep) {  // wave-uniform
        const int64_t r = i0 + rl.sub;
        const bool has = rl.on && r < R;
        int c = 0, o = 0;
        if (has) {
            const int lo = ig.local[r];
            const int hi = (r + 1) % kScanBlock != 0 ? ig.local[r + 1] : ig.tot[r / kScanBlock];
            c = hi - lo;
            o = lo + pre[r / kScanBlock];
        }
        const bool heavy = c > ig.hc;
        const int cl = heavy ? 0 : c;
        const int res = has && cl > 0 ? min(max(ig.cursor[r], 0), cl) : 0;
        const bool valid = ql >= res && ql < cl;
        const int e = valid ? (int)min((unsigned)ig.clist[o + ql], (unsigned)(ig.mcap - 1)) : INT_MAX;
        int cmax = 0;
        for (int g = 0; g < rl.rpw; ++g) cmax = max(cmax, __builtin_amdgcn_readlane(cl, g * (int)w4));
        int rank = 0;
        for (int j = 0; j < cmax; ++j) {
            const int x = __shfl(e, base + j, 64);
            rank += j < cl && x < e;
        }
        const int cv = cl - res;
        const int to = valid ? base + rank : ql < res ? base + cv + ql : lane;
        const int srt = __builtin_amdgcn_ds_permute(to * 4, e);
        for (uint32_t q = w4 <= 64 ? (uint32_t)ql : (uint32_t)lane; ; q += 64) {
            const bool act = has && !heavy && q < w4 && ql < gsz;
            float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int j = 0; j < cmax; j += 4) {
                const int c0 = __shfl(srt, base + j, 64), c1 = __shfl(srt, base + min(j + 1, gsz - 1), 64);
                const int c2 = __shfl(srt, base + min(j + 2, gsz - 1), 64);
                const int c3 = __shfl(srt, base + min(j + 3, gsz - 1), 64);
                const bool v0 = act && j < cv, v1 = act && j + 1 < cv, v2 = act && j + 2 < cv, v3 = act && j + 3 < cv;
                float4 g0, g1, g2, g3;
                if (v0) g0 = gs[(size_t)c0 * w4 + q];
                if (v1) g1 = gs[(size_t)c1 * w4 + q];
                if (v2) g2 = gs[(size_t)c2 * w4 + q];
                if (v3) g3 = gs[(size_t)c3 * w4 + q];
                if (v0) g = f4add(g, g0);
                if (v1) g = f4add(g, g1);
                if (v2) g = f4add(g, g2);
                if (v3) g = f4add(g, g3);
            }
            if (act) out[(size_t)(r - U) * w4 + q] = g;
            if (w4 <= 64 || q + 64 >= w4) break;
        }
    }
}

template <int OPT>
__global__ __launch_bounds__(kBlock) void k_mlp_update(float* __restrict__ p, float* __restrict__ m,
                                                       float* __restrict__ v, int P, const float* __restrict__ slabs,
                                                       int nslab, const float* __restrict__ grad_in,
                                                       float* __restrict__ grad_out, int do_update, int want_reg,
                                                       const int32_t* __restrict__ step, float lr, float b1, float b2,
                                                       float eps, L2Table l2t, float* __restrict__ part_reg) {
    mlp_update_body<OPT>(p, m, v, P, slabs, nslab, grad_in, grad_out, do_update, want_reg, step, lr, b1, b2, eps, l2t,
                         part_reg, (int)blockIdx.x);
}

// Per-group hit@k / dcg@k: the label's position in the stable descending
// order equals #(p_j > p_lab) + #(j < lab with p_j == p_lab)  (top_k ties →
// lower index first; test/test_model.py:121-149).
__device__ __forceinline__ void group_metrics_body(const float* __restrict__ probs, const float* __restrict__ labels,
                                                   int64_t ng, int group, int k, float* __restrict__ hit,
                                                   float* __restrict__ dcg, float* __restrict__ part_hit,
                                                   float* __restrict__ part_dcg, int blk) {
    __shared__ float red[4];
    const int64_t g = (int64_t)blk * kBlock + threadIdx.x;
    float h = 0.f, d = 0.f;
    if (g < ng) {
        const float* pr = probs + g * group;
        const float* lb = labels + g * group;
        int lab = 0;
        float best = lb[0];
        for (int j = 1; j < group; ++j)
            if (lb[j] > best) { best = lb[j]; lab = j; }
        const float pl = pr[lab];
        int pos = 0;
        for (int j = 0; j < group; ++j) {
            const float pj = pr[j];
            pos += (pj > pl) || (pj == pl && j < lab);
        }
        h = pos < k ? 1.0f : 0.0f;
        d = h * (logf(2.0f) / logf((float)pos + 2.0f));
        if (hit) hit[g] = h;
        if (dcg) dcg[g] = d;
    }
    h = block_sum_256(h, red);
    d = block_sum_256(d, red);
    if (threadIdx.x == 0) {
        if (part_hit) part_hit[blk] = h;
        if (part_dcg) part_dcg[blk] = d;
    }
}
__global__ __launch_bounds__(kBlock) void k_group_metrics(const float* __restrict__ probs,
                                                          const float* __restrict__ labels, int64_t ng, int group,
                                                          int k, float* __restrict__ hit, float* __restrict__ dcg,
                                                          float* __restrict__ part_hit, float* __restrict__ part_dcg) {
    group_metrics_body(probs, labels, ng, group, k, hit, dcg, part_hit, part_dcg, (int)blockIdx.x);
}

__global__ __launch_bounds__(kBlock) void k_rank(const float* __restrict__ probs, int64_t ng, int group,
                                                 int32_t* __restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    const float* pr = probs + g * group;
    int32_t* o = out + g * group;
    for (int e = 0; e < group; ++e) {
        const float pe = pr[e];
        int pos = 0;
        for (int j = 0; j < group; ++j) {
            const float pj = pr[j];
            pos += (pj > pe) || (pj == pe && j < e);
        }
        o[pos] = e;
    }
}


__global__ __launch_bounds__(kBlock) void k_summary(const float* __restrict__ part_bce, int nbce,
                                                    const float* __restrict__ part_hit,
                                                    const float* __restrict__ part_dcg, int nmet, float n_groups,
                                                    const float* __restrict__ reg_emb, int nreg_emb,
                                                    const float* __restrict__ reg_mlp, int nreg_mlp,
                                                    float* __restrict__ summary) {
    __shared__ float red[4];
    summary_body(part_bce, nbce, part_hit, part_dcg, nmet, n_groups, reg_emb, nreg_emb, reg_mlp, nreg_mlp, summary,
                 red);
}

// Block 0 of a stats launch in one round trip: k_stats' work (the drop word, the batch summary when
// sa.summary, the stats fold and the step bump) with every load issued before the first barrier and
// the five block sums reduced together — the same per-thread orders and the same tree as
// block_sum_256 per value, so the results are bitwise the earlier per-value block sums.  (Those chained a
// load round trip and two barriers per value; this block was the stats launch's critical path.)
__device__ inline void summary_stats_block(const SummaryArgs& sa, float* __restrict__ summary,
                                           const float* __restrict__ reg_emb, int nreg_emb,
                                           const float* __restrict__ reg_mlp, int nreg_mlp, float inv_batch,
                                           double* __restrict__ stats, int32_t* step, int bump) {
    __shared__ float red[5][4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int dropped = sa.drop ? *sa.drop : 0;
    float x[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // bce, hit, dcg, reg_emb, reg_mlp
    if (sa.summary) {
        for (int j = tid; j < sa.nbce; j += kBlock) x[0] += sa.part_bce[j];
        for (int j = tid; j < sa.nmet; j += kBlock) x[1] += sa.part_hit[j];
        for (int j = tid; j < sa.nmet; j += kBlock) x[2] += sa.part_dcg[j];
    }
    for (int j = tid; j < nreg_emb; j += kBlock) x[3] += reg_emb[j];
    for (int j = tid; j < nreg_mlp; j += kBlock) x[4] += reg_mlp[j];
    // thread 0's operands of the fold, in flight with the sums
    double s[NCF_NUM_STATS];
    float sb = 0.f, sh = 0.f, sd = 0.f, sg = sa.n_groups, sreg = 0.f;
    if (tid == 0) {
        if (stats)
#pragma unroll
            for (int k = 0; k < NCF_NUM_STATS; ++k) s[k] = stats[k];
        if (!sa.summary) {
            sb = summary[NCF_SUM_BCE], sh = summary[NCF_SUM_HIT], sd = summary[NCF_SUM_DCG];
            sg = summary[NCF_SUM_GROUPS], sreg = summary[NCF_SUM_REG];
        }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) x[k] = wave_sum(x[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 5; ++k) red[k][w] = x[k];
    __syncthreads();
    if (tid != 0) return;
    float r[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) r[k] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    if (dropped) {  // the step was dropped (fill_wave): no summary, stats or bump; clear the word
        *sa.drop = 0;
        return;
    }
    if (sa.summary) {
        sb = r[0], sh = r[1], sd = r[2];
        sreg = 0.f + 0.f;  // summary_body's reg terms: empty sums
        summary[NCF_SUM_BCE] = sb;
        summary[NCF_SUM_HIT] = sh;
        summary[NCF_SUM_DCG] = sd;
        summary[NCF_SUM_GROUPS] = sg;
        summary[NCF_SUM_REG] = sreg;
#pragma unroll
        for (int k = NCF_SUM_REG + 1; k < NCF_NUM_SUMMARY; ++k) summary[k] = 0.f;
    }
    const float loss = sb * inv_batch + sreg + (r[3] + r[4]);
    const float hr = sg > 0.f ? sh / sg : 0.f;
    const float dc = sg > 0.f ? sd / sg : 0.f;
    if (stats) {
        stats[NCF_STAT_LOSS_SUM] = s[NCF_STAT_LOSS_SUM] + (double)loss;
        stats[NCF_STAT_HR_SUM] = s[NCF_STAT_HR_SUM] + (double)hr;
        stats[NCF_STAT_DCG_SUM] = s[NCF_STAT_DCG_SUM] + (double)dc;
        stats[NCF_STAT_STEPS] = s[NCF_STAT_STEPS] + 1.0;
        stats[NCF_STAT_LAST_LOSS] = loss;
        stats[NCF_STAT_LAST_HR] = hr;
        stats[NCF_STAT_LAST_DCG] = dc;
        stats[NCF_STAT_BCE_SUM] = s[NCF_STAT_BCE_SUM] + (double)(sb * inv_batch);
    }
    if (bump) *step += 1;
}

__global__ __launch_bounds__(kBlock) void k_stats(float* __restrict__ summary,
                                                  const float* __restrict__ reg_emb, int nreg_emb,
                                                  const float* __restrict__ reg_mlp, int nreg_mlp, float inv_batch,
                                                  double* __restrict__ stats, int32_t* step, int bump, SummaryArgs sa) {
    summary_stats_block(sa, summary, reg_emb, nreg_emb, reg_mlp, nreg_mlp, inv_batch, stats, step, bump);
}

// The in-kernel fill's body (FillArgs) as a launch of its own, before the forward/backward (a stale
// counted set drops the step: fill_wave).  The rows part and the contributions part run in waves of their own (the first nr waves, the
// rest), so the launch waits on the longer of the two dependency chains instead of their sum.
__global__ __launch_bounds__(kBlock) void k_fill_ahead(FillArgs f, const int32_t* __restrict__ users,
                                                       const int32_t* __restrict__ items, int64_t n, int fold, int nr) {
    const int gw = (int)blockIdx.x * (kBlock / 64) + (int)(threadIdx.x >> 6);
    if (gw < nr)
        fill_wave<1>(f, users, items, n, fold, gw, nr);
    else
        fill_wave<2>(f, users, items, n, fold, gw - nr, (int)gridDim.x * (kBlock / 64) - nr);
}

hipError_t launch_fill_ahead(const FillArgs& f,const int32_t* users, const int32_t* items, int64_t n, int fold,
                             hipStream_t st) {
    if (f.nscan < 1 || f.nscan > kMaxFillScan || n < 1) return hipErrorInvalidValue;
    // one pass per wave where the grid allows (4 waves per block)
    auto waves = [](int64_t work, int per) { return (work + 64 * per - 1) / (64 * per); };
    int64_t nr = (int64_t)f.nscan * (kScanBlock / 64), nc = waves(2 * n, kFillContribPerLane);
    const int64_t cap = 2048 * (kBlock / 64) / 2;  // at most 2048 blocks, half for each part
    nr = nr > cap ? cap : nr;
    nc = nc > cap ? cap : nc;
    const int64_t blocks = (nr + nc + kBlock / 64 - 1) / (kBlock / 64);
    // (the contributions part gets the waves past nr: at least nc of them)
    launch(k_fill_ahead, (unsigned)blocks, kBlock, 0, st, f, users, items, n, fold, (int)nr);
    return hipGetLastError();
}

// Block 0: k_stats; blocks 1..: the next batch's per-block key scan (k_scan_local<true>) over the
// counts the touched update took ahead — one launch instead of two.
struct ScanAhead {
    const int32_t* cnt;        // the counts taken ahead (ws cnt_ahead): moved to cursor, then zeroed
    int64_t r1;
    int32_t *offs, *tot, *uloc, *utot;
    int32_t* cursor;           // ws cnt
    int32_t* heavy_n;          // the in-kernel fill's heavy-row count (FillArgs), zeroed here
    TouchedOut to;             // the next index's per-block touched rows (single-table workspaces)
    int sparse;                // scan_local_body<true, true> (sparse_index_ok): occupied keys only
    int32_t* itag;             // sparse: the seen tag, bumped by block 0 (after this step's update read it)
};
__global__ __launch_bounds__(kBlock) void k_stats_scan(float* __restrict__ summary,
                                                       const float* __restrict__ reg_emb, int nreg_emb,
                                                       const float* __restrict__ reg_mlp, int nreg_mlp,
                                                       float inv_batch, double* __restrict__ stats, int32_t* step,
                                                       int bump, ScanAhead sc, SummaryArgs sa, ReplayAhead ra) {
    // block order: [stats] [replay ahead: the latency-bound chains first] [scan]
    const int b = (int)blockIdx.x - 1 - (ra.npass + kReplayPasses - 1) / kReplayPasses;
    if (blockIdx.x == 0) {
        summary_stats_block(sa, summary, reg_emb, nreg_emb, reg_mlp, nreg_mlp, inv_batch, stats, step, bump);
        if (sc.itag && threadIdx.x == 0) *sc.itag += 1;
    } else if (b < 0) {
        replay_ahead_block(ra, (int)blockIdx.x - 1);
    } else if (sc.sparse) {
        scan_local_body<true, true>(sc.cnt, sc.r1, sc.offs, sc.tot, sc.uloc, sc.utot, b, sc.cursor, sc.heavy_n, sc.to);
    } else {
        scan_local_body<true>(sc.cnt, sc.r1, sc.offs, sc.tot, sc.uloc, sc.utot, b, sc.cursor, sc.heavy_n, sc.to);
    }
}

// The next batch's per-block key scan alone (k_stats_scan's blocks >= 1), for a counting-ahead
// update that has no stats launch of its own behind it (user-partitioned data parallelism).
__global__ __launch_bounds__(kBlock) void k_scan_ahead(ScanAhead sc) {
    scan_local_body<true>(sc.cnt, sc.r1, sc.offs, sc.tot, sc.uloc, sc.utot, (int)blockIdx.x, sc.cursor, sc.heavy_n,
                          sc.to);
}

static TouchedOut touched_out(const WsLayout& L, void* ws) {
    return L.world == 0 ? TouchedOut{at<int32_t>(ws, L.tl), at<int2>(ws, L.tocl)} : TouchedOut{};
}

hipError_t launch_scan_ahead(const WsLayout& L, void* ws, int64_t keys, hipStream_t st) {
    const int64_t r1 = keys + 1;
    const int nscan = (int)((r1 + kScanBlock - 1) / kScanBlock);
    ScanAhead sc{at<const int32_t>(ws, L.cnt_ahead), r1, at<int32_t>(ws, L.offs_local), at<int32_t>(ws, L.tot),
                 at<int32_t>(ws, L.uloc), at<int32_t>(ws, L.utot), at<int32_t>(ws, L.cnt), at<int32_t>(ws, L.heavy_n),
                 touched_out(L, ws), 0, nullptr};
    launch(k_scan_ahead, nscan, kBlock, 0, st, sc);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------

static L2Table make_l2_table(const ncf_shape_t& s, const ncf_hyper_t& h) {
    L2Table t{};
    t.n = 0;
    for (int l = 1; l < s.num_layers; ++l) {
        if (h.l2[l] == 0.0f) continue;
        t.start[t.n] = s.layer_off[l];
        t.end[t.n] = s.layer_off[l] + s.layers[l - 1] * s.layers[l];
        t.lam[t.n] = h.l2[l];
        ++t.n;
    }
    return t;
}

hipError_t launch_emb_update(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m, float* v,
                             const int32_t* step, const ncf_hyper_t& h, const float* dense_grad, int64_t rows,
                             hipStream_t st, const float* gs_rows, int64_t offs_row) {
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const uint32_t n4 = (uint32_t)(rows * w4);
    if (n4 == 0) return hipSuccess;
    const int32_t* offs = at<int32_t>(ws, L.offs) + offs_row;
    const int32_t* list = at<int32_t>(ws, L.list);
    const float4* gs = gs_rows ? (const float4*)gs_rows : at<const float4>(ws, L.gs);
    float* part = at<float>(ws, L.part_reg);
    const bool l2 = h.l2[0] != 0.0f;
    const int src = dense_grad ? kGradDense : kGradSparse;
    dim3 grid(kUpdateGrid), blk(kBlock);
#define NCF_EMB_LAUNCH(OPT, SRC, L2)                                                                          \
    launch(k_emb_update<OPT, SRC, L2>, grid, blk, 0, st, (float4*)emb, (float4*)m, (float4*)v, n4, w4, offs, list, gs, \
                                                     (const float4*)dense_grad, step, h.lr, h.beta_1, h.beta_2,    \
                                                     h.epsilon, h.l2[0], part)
    if (h.optimizer == NCF_OPT_ADAM) {
        if (src == kGradSparse) { if (l2) NCF_EMB_LAUNCH(NCF_OPT_ADAM, kGradSparse, true); else NCF_EMB_LAUNCH(NCF_OPT_ADAM, kGradSparse, false); }
        else { if (l2) NCF_EMB_LAUNCH(NCF_OPT_ADAM, kGradDense, true); else NCF_EMB_LAUNCH(NCF_OPT_ADAM, kGradDense, false); }
    } else {
        if (src == kGradSparse) { if (l2) NCF_EMB_LAUNCH(NCF_OPT_SGD, kGradSparse, true); else NCF_EMB_LAUNCH(NCF_OPT_SGD, kGradSparse, false); }
        else { if (l2) NCF_EMB_LAUNCH(NCF_OPT_SGD, kGradDense, true); else NCF_EMB_LAUNCH(NCF_OPT_SGD, kGradDense, false); }
    }
#undef NCF_EMB_LAUNCH
    return hipGetLastError();
}

// Block caps of the row kernels (measured on MI355X, config C): the replay kernel runs best
// with few, long-lived waves (2048 blocks: 17.7 us vs 21 us at 8192), the touched update with
// one pass over the rows (8192).
#ifndef NCF_CATCHUP_GRID_MAX
#define NCF_CATCHUP_GRID_MAX 2048
#endif
#ifndef NCF_TOUCHED_GRID_MAX
#define NCF_TOUCHED_GRID_MAX 8192
#endif
// count (+ catch-up ahead) blocks: 64 contributions per pass, 32 below 65,536 contributions
// (NCF_COUNT_PER_SMALL below 32,768)
static int count_per(int64_t mc) { return mc >= 65536 ? NCF_COUNT_PER_MAX : mc >= 32768 ? 32 : NCF_COUNT_PER_SMALL; }
int64_t count_ahead_passes(int64_t mc) {
    const int per = count_per(mc);
    return (mc + per - 1) / per;
}

static unsigned row_grid(int64_t rows, uint32_t w4, int64_t cap) {
    const int64_t rpw = w4 <= 64 ? 64 / w4 : 1;
    int64_t g = (rows + rpw * 4 - 1) / (rpw * 4);  // 4 waves per block
    return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_emb_catchup(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m, float* v,
                              int32_t* row_step, const int32_t* step, const ncf_hyper_t& h, bool all_rows,
                              hipStream_t st, bool sort_lists, int64_t n, bool rows_current, const int32_t* users,
                              const int32_t* items, int gate_ahead) {
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const int64_t R = s.num_rows;
    const int64_t nmax = R < 2 * L.max_batch ? R : 2 * L.max_batch;
    SortAhead so{0, nullptr, 0, nullptr, 0, nullptr, at<int32_t>(ws, L.err), nullptr, nullptr, nullptr};
    const StaleGate nogate{nullptr, nullptr, 0, 0, 0, nullptr, 0, 0};
    const int64_t bound = lazy_bound(s, h);  // rows under deferred decay
    unsigned nsort = 0;
    size_t lds = 0;
    if (sort_lists && !all_rows) {
        so = SortAhead{0, at<const int32_t>(ws, L.offs), R, at<int32_t>(ws, L.list), (int)((2 * n + 31) / 32),
                       at<int32_t>(ws, L.cnt), at<int32_t>(ws, L.err), nullptr, nullptr, nullptr};
        if (sort_rpt(R) == 8 || (L.nscan > kFillBigScan && L.nscan <= kBlock * kPrefixPer)) {
            // large key spaces (k_fill_big / k_fill_touched, which give back what a run takes below
            // zero, so residues sit at counted keys only): the touched list's rows (at most 2n) — the
            // sparse index (k_fill_touched) writes no per-key offsets
            so.touched = at<const int32_t>(ws, L.touched);
            so.toc = at<const int2>(ws, L.touched_oc);
            so.nuniq = at<const int32_t>(ws, L.nuniq);
            const int64_t nt = R < 2 * n ? R : 2 * n;
            nsort = (unsigned)((nt + kBlock - 1) / kBlock);
        } else {
            nsort = (unsigned)((R + kBlock - 1) / kBlock);
        }
        lds = (size_t)so.nwords * 4;
        static bool lds_cfg = false;
        if (!lds_cfg && lds > 65536) {
            hipError_t e = hipFuncSetAttribute((const void*)k_emb_catchup,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)((kMaxBatch * 2 / 32) * 4));
            if (e != hipSuccess) return e;
            lds_cfg = true;
        }
    }
    // rows_current: the previous step's update launch caught this batch's rows up ahead
    if (h.optimizer != NCF_OPT_ADAM || (rows_current && NCF_CATCHUP_AHEAD)) {
        // SGD (an untouched row does not move) or rows already current: only the sort remains,
        // plus (Adam, rows current) the stale-count gate blocks
        StaleGate sg = nogate;
        unsigned ngate = 0;
        if (h.optimizer == NCF_OPT_ADAM && users && items && n > 0) {
            sg = StaleGate{users, items, 2 * n, s.num_users, s.num_items, row_step, bound, gate_ahead};
            ngate = 64;
        }
        if (nsort + ngate) {
            so.ncatch = (int)ngate;
            launch(k_emb_catchup, ngate + nsort, kBlock, lds, st, (float4*)emb, (float4*)m, (float4*)v, w4,
                   at<const int32_t>(ws, L.touched), at<const int32_t>(ws, L.nuniq), bound, (const int32_t*)row_step,
                   step, h.lr, h.beta_1, h.beta_2, h.epsilon, so, sg);
        }
        return hipGetLastError();
    }
#if NCF_CATCHUP_SCALAR
    auto cgrid = [&](int64_t rows, int64_t cap) {
        const int W2 = 2 * (int)w4;  // element pairs per row (one per lane)
        const int64_t lanes = W2 < kBlock ? (W2 + 63) / 64 * 64 : kBlock;
        const int64_t rpb = kBlock / lanes;
        int64_t g = (rows + rpb - 1) / rpb;
        return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
    };
#else
    auto cgrid = [&](int64_t rows, int64_t cap) { return row_grid(rows, w4, cap); };
#endif
    if (all_rows) {
        launch(k_emb_flush, cgrid(bound, 8192), kBlock, 0, st, (float4*)emb, (float4*)m, (float4*)v, w4, bound,
               (const int32_t*)row_step, step, h.lr, h.beta_1, h.beta_2, h.epsilon);
    } else {
        const unsigned ncatch = cgrid(nmax, NCF_CATCHUP_GRID_MAX);
        so.ncatch = (int)ncatch;
        launch(k_emb_catchup, ncatch + nsort, kBlock, lds, st, (float4*)emb, (float4*)m, (float4*)v, w4,
               at<const int32_t>(ws, L.touched), at<const int32_t>(ws, L.nuniq), bound, (const int32_t*)row_step,
               step, h.lr, h.beta_1, h.beta_2, h.epsilon, so, nogate);
    }
    return hipGetLastError();
}

hipError_t launch_row_step_fill(int32_t* row_step, int64_t R, const int32_t* step, hipStream_t st) {
    launch(k_row_step_fill, kUpdateGrid, kBlock, 0, st, row_step, R, step);
    return hipGetLastError();
}

hipError_t launch_emb_update_touched(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m,
                                     float* v, int32_t* row_step, int32_t* step, const ncf_hyper_t& h,
                                     hipStream_t st, const int32_t* next_users, const int32_t* next_items,
                                     int64_t n_next, const MlpDeferred* mlp, int next_fold, const MetricsDeferred* met,
                                     const float* grad_rows, bool unsorted_lists, bool may_drop, bool sparse_index,
                                     bool* defer_replay) {
#if NCF_DIAG_UPD == 1  // diagnostic timing builds only (wrong numerics): no catch-up ahead
    const bool replay_ahead = false;
#else
    const bool replay_ahead = next_users != nullptr && NCF_CATCHUP_AHEAD;
#endif
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const uint32_t n4 = (uint32_t)(lazy_bound(s, h) * w4);  // SGD: the rows under deferred decay
    const int32_t* offs = at<int32_t>(ws, L.offs);
    const int32_t* list = at<int32_t>(ws, L.list);
    const float4* gs = grad_rows ? reinterpret_cast<const float4*>(grad_rows) : at<const float4>(ws, L.gs);
    const int64_t R = s.num_rows;
    if (h.optimizer == NCF_OPT_ADAM) {
        const unsigned nupd = row_grid(R < 2 * L.max_batch ? R : 2 * L.max_batch, w4, NCF_TOUCHED_GRID_MAX);
        const int64_t mc = next_users ? 2 * n_next : 0;
        const int per = count_per(mc);
        const int64_t npass = count_ahead_passes(mc);
        // deferred replay: the count blocks' 4 waves take a pass each (no replay to share)
        const bool defer = defer_replay && *defer_replay && replay_ahead && mc > 0;
        if (defer_replay) *defer_replay = defer;
        if (defer && (L.world != 0 || mc > 2 * L.max_batch)) return hipErrorInvalidValue;
        const int64_t nblk = defer ? (npass + kBlock / 64 - 1) / (kBlock / 64) : npass;
        const unsigned ncount = mc > 0 ? (unsigned)(nblk < NCF_COUNT_BLOCKS_MAX ? nblk : NCF_COUNT_BLOCKS_MAX) : 0u;
        if (sparse_index && (unsorted_lists || !sparse_index_ok(L))) return hipErrorInvalidValue;
        CountAhead ca{(int)nupd, (int)ncount, next_users, next_items, mc, s.num_users, s.num_items,
                      at<int32_t>(ws, L.cnt_ahead), replay_ahead ? 1 : 0, next_fold, per, lazy_bound(s, h),
                      sparse_index ? at<const int32_t>(ws, L.seen) : nullptr,
                      sparse_index ? at<const int32_t>(ws, L.itag) : nullptr,
                      defer ? at<int2>(ws, L.claims) : nullptr, defer ? at<int32_t>(ws, L.nclaim) : nullptr,
                      defer ? at<int32_t>(ws, L.claim_t) : nullptr};
        MlpTail mt{};
        if (mlp) {
            mt = MlpTail{mlp->two_level ? (s.mlp_params + 15) / 16 : (s.mlp_params + kBlock - 1) / kBlock, mlp->p,
                         mlp->m, mlp->v, s.mlp_params, mlp->slabs, mlp->nslab, step, h.lr, h.beta_1, h.beta_2,
                         h.epsilon, make_l2_table(s, h), at<float>(ws, L.part_reg) + kUpdateGrid, mlp->two_level};
        }
        MetricsTail mm{};
        if (met) mm = MetricsTail{met->nblocks, met->probs, met->labels, met->ng, met->group, met->k,
                                  at<float>(ws, L.part_hit), at<float>(ws, L.part_dcg)};
        SortRows so{};
        if (unsorted_lists) {
            if (L.world != 0 || unsorted_heavy_c(s) < kHeavyMin) return hipErrorInvalidValue;
            // heavy rows are rare (lists longer than a row group's lanes): a few blocks stride over them
            so = SortRows{1, unsorted_heavy_c(s), 32, at<const int32_t>(ws, L.heavy), at<const int32_t>(ws, L.heavy_n),
                          at<int32_t>(ws, L.cnt), at<int32_t>(ws, L.err), at<int32_t>(ws, L.slist),
                          (int)(2 * L.max_batch), may_drop ? at<const int32_t>(ws, L.stale_step) : nullptr,
                          at<const int32_t>(ws, L.offs_local), at<const int32_t>(ws, L.tot)};
        }
        launch(unsorted_lists ? k_emb_adam_touched<true> : k_emb_adam_touched<false>, (unsigned)so.nheavy + nupd + ncount + (unsigned)mt.nblocks + (unsigned)mm.nblocks,
               kBlock, 0, st, (float4*)emb, (float4*)m, (float4*)v, w4, at<const int32_t>(ws, L.touched),
               at<const int2>(ws, L.touched_oc), at<const int32_t>(ws, L.nuniq), offs, list, gs, row_step,
               (const int32_t*)step, h.lr, h.beta_1, h.beta_2, h.epsilon, ca, mt, mm, so);
    } else
        launch(k_emb_sgd_hot, kUpdateGrid, kBlock, 0, st, (float4*)emb, n4, w4, offs, list, gs, h.lr);
    return hipGetLastError();
}

hipError_t launch_emb_grad_dense(const ncf_shape_t& s, const WsLayout& L, void* ws, float* out, hipStream_t st,
                                  int64_t row_begin) {
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const uint32_t n4 = (uint32_t)((s.num_rows - row_begin) * w4);
    if (n4 == 0) return hipSuccess;
    launch(k_emb_grad_dense, kUpdateGrid, kBlock, 0, st, (float4*)out, n4, w4, at<int32_t>(ws, L.offs) + row_begin,
                                                     at<int32_t>(ws, L.list), at<const float4>(ws, L.gs));
    return hipGetLastError();
}

bool part_tail_foldable(const ncf_shape_t& s, const ncf_hyper_t& h, int nslab) {
    return h.l2[0] == 0.0f && make_l2_table(s, h).n == 0 && nslab > 2 * kSlabSplit;
}

hipError_t launch_part_tail(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb_grad, int64_t row_begin,
                            float* mlp_grad, int nslab, int nbce, int nmet, float n_groups, float* summary,
                            hipStream_t st) {
    const int P = s.mlp_params;
    const int nmlp = (P + 15) / 16;
    SummaryArgs sa{summary, at<float>(ws, L.part_bce), at<float>(ws, L.part_hit), at<float>(ws, L.part_dcg), nbce,
                   nmet, n_groups};
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const uint32_t n4 = (uint32_t)((s.num_rows - row_begin) * w4);
    const uint32_t ngrad = n4 ? (uint32_t)kUpdateGrid : 0u;
    launch(k_part_tail, ngrad + (uint32_t)nmlp + (summary ? 1u : 0u), kBlock, 0, st, (float4*)emb_grad, n4, w4,
           at<int32_t>(ws, L.offs) + row_begin, at<int32_t>(ws, L.list), at<const float4>(ws, L.gs), ngrad, P,
           at<const float>(ws, L.slabs), nslab, nmlp, mlp_grad, sa);
    return hipGetLastError();
}

hipError_t launch_part_tail_unsorted(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb_grad,
                                     int64_t row_begin, float* mlp_grad, int nslab, int nbce, int nmet, float n_groups,
                                     float* summary, hipStream_t st) {
    if (L.world != 0 || L.nscan > kMaxFillScan || unsorted_heavy_c(s) < kHeavyMin || row_begin > s.num_rows)
        return hipErrorInvalidValue;
    const int P = s.mlp_params;
    const int nmlp = (P + 15) / 16;
    SummaryArgs sa{summary, at<float>(ws, L.part_bce), at<float>(ws, L.part_hit), at<float>(ws, L.part_dcg), nbce,
                   nmet, n_groups};
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const int64_t rows = s.num_rows - row_begin;
    const unsigned ngrad = rows > 0 ? row_grid(rows, w4, kUpdateGrid) : 0u;
    const ItemGradArgs ig{at<const int32_t>(ws, L.offs_local), at<const int32_t>(ws, L.tot), L.nscan,
                          at<const int32_t>(ws, L.list), at<const int32_t>(ws, L.cnt), at<const int32_t>(ws, L.touched),
                          at<const int2>(ws, L.touched_oc), at<const int32_t>(ws, L.heavy),
                          at<const int32_t>(ws, L.heavy_n), 32, at<int32_t>(ws, L.slist), unsorted_heavy_c(s),
                          (int)(2 * L.max_batch)};
    launch(k_part_tail_unsorted, (unsigned)ig.nheavy + (unsigned)nmlp + (summary ? 1u : 0u) + ngrad, kBlock, 0, st,
           (float4*)emb_grad, (int64_t)row_begin, (int64_t)s.num_rows, w4, at<const float4>(ws, L.gs), ngrad, P,
           at<const float>(ws, L.slabs), nslab, nmlp, mlp_grad, sa, ig);
    return hipGetLastError();
}

hipError_t launch_apply_fused(const ncf_shape_t& s, float* emb, float* m, float* v, const float* emb_grad,
                              int64_t rows, float* mlp, float* mlp_m, float* mlp_v, const float* mlp_grad,
                              const int32_t* step, const ncf_hyper_t& h, hipStream_t st, int parts) {
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    const uint32_t n4 = (parts & 1) ? (uint32_t)(rows * w4) : 0u;
    const int P = s.mlp_params;
    const unsigned gridp = (parts & 2) ? (unsigned)((P + kBlock - 1) / kBlock) : 0u;
    const uint32_t nupd = n4 ? (uint32_t)kUpdateGrid : 0u;
    if (nupd + gridp == 0) return hipSuccess;
    if (h.optimizer == NCF_OPT_ADAM)
        launch(k_emb_update_mlp<NCF_OPT_ADAM>, nupd + gridp, kBlock, 0, st, (float4*)emb, (float4*)m, (float4*)v, n4,
               w4, (const float4*)emb_grad, nupd, mlp, mlp_m, mlp_v, P, mlp_grad, step, h.lr, h.beta_1, h.beta_2,
               h.epsilon);
    else
        launch(k_emb_update_mlp<NCF_OPT_SGD>, nupd + gridp, kBlock, 0, st, (float4*)emb, (float4*)m, (float4*)v, n4,
               w4, (const float4*)emb_grad, nupd, mlp, mlp_m, mlp_v, P, mlp_grad, step, h.lr, h.beta_1, h.beta_2,
               h.epsilon);
    return hipGetLastError();
}

hipError_t launch_uniq_grad(const ncf_shape_t& s, const WsLayout& L, void* ws, int64_t n, float* out,
                            hipStream_t st) {
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    int64_t g = (2 * n * w4 + kBlock - 1) / kBlock;
    if (g > kUpdateGrid) g = kUpdateGrid;
    launch(k_uniq_grad, (unsigned)g, kBlock, 0, st, (float4*)out, at<int32_t>(ws, L.nuniq), w4, at<int32_t>(ws, L.uoffs),
                                                at<int32_t>(ws, L.list), at<const float4>(ws, L.gs));
    return hipGetLastError();
}

hipError_t launch_gather_rows(const ncf_shape_t& s, const float* table, int64_t table_rows, const int32_t* rows,
                              int64_t m, float* out, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    const uint32_t w4 = (uint32_t)(s.row_width / 4);
    int64_t g = (m * w4 + kBlock - 1) / kBlock;
    if (g > kUpdateGrid) g = kUpdateGrid;
    launch(k_gather_rows, (unsigned)g, kBlock, 0, st, (float4*)out, (const float4*)table, table_rows, rows,
                                                  (uint32_t)(m * w4), w4);
    return hipGetLastError();
}

hipError_t launch_emb_reg(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, int64_t rows,
                          float lam, hipStream_t st) {
    const uint32_t n4 = (uint32_t)(rows * (s.row_width / 4));
    launch(k_emb_reg, kUpdateGrid, kBlock, 0, st, (const float4*)emb, n4, lam, at<float>(ws, L.part_reg));
    return hipGetLastError();
}

hipError_t launch_mlp_update(const ncf_shape_t& s, const WsLayout& L, void* ws, float* mlp, float* m, float* v,
                             const int32_t* step, const ncf_hyper_t& h, int nslab, const float* grad_in,
                             float* grad_out, bool do_update, int* nreg, hipStream_t st, bool want_reg,
                             int summary_nbce, int summary_nmet, float n_groups, float* summary,
                             MlpDeferred* defer) {
    const int P = s.mlp_params;
    const int grid = (P + kBlock - 1) / kBlock;
    float* part = at<float>(ws, L.part_reg) + kUpdateGrid;
    const L2Table t = make_l2_table(s, h);
    const float* slabs = at<float>(ws, L.slabs);
    bool summary_done = summary == nullptr || summary_nbce < 0;
    if (defer && defer->two_level && h.optimizer == NCF_OPT_ADAM && do_update && !grad_out && !want_reg &&
        nslab > 2 * kSlabSplit && t.n == 0 && summary_done) {
        // the touched-row update launch does both slab-reduction levels and the Adam step
        *defer = MlpDeferred{mlp, m, v, slabs, nslab, 1};
        *nreg = 0;
        return hipSuccess;
    }
    if (defer) defer->two_level = 0;
    if (nslab > 2 * kSlabSplit) {
        const int per = (nslab + kSlabSplit - 1) / kSlabSplit;
        const int nch = (nslab + per - 1) / per;
        float* sp = at<float>(ws, L.slab_part);
        SummaryArgs sa{nullptr, nullptr, nullptr, nullptr, 0, 0, 0.f};
        if (!summary_done)
            sa = SummaryArgs{summary, at<float>(ws, L.part_bce), at<float>(ws, L.part_hit), at<float>(ws, L.part_dcg),
                             summary_nbce, summary_nmet, n_groups};
        launch(k_slab_partial, dim3(grid + (summary_done ? 0 : 1), nch), kBlock, 0, st, slabs, P, nslab, per, sp, sa);
        summary_done = true;
        slabs = sp;
        nslab = nch;
    }
    if (!summary_done) {
        hipError_t e = launch_summary(L, ws, summary_nbce, summary_nmet, n_groups, 0, 0, summary, st);
        if (e != hipSuccess) return e;
    }
    if (defer && h.optimizer == NCF_OPT_ADAM && do_update && !grad_out && !want_reg && nslab > 0) {
        // the caller runs the Adam step of the dense layers inside the touched-row update launch
        *defer = MlpDeferred{mlp, m, v, slabs, nslab, 0};
        *nreg = t.n > 0 ? grid : 0;
        return hipGetLastError();
    }
    if (defer) defer->p = nullptr;
    if (h.optimizer == NCF_OPT_ADAM)
        launch(k_mlp_update<NCF_OPT_ADAM>, grid, kBlock, 0, st, mlp, m, v, P, slabs, nslab, grad_in,
                                                            grad_out, do_update ? 1 : 0, want_reg ? 1 : 0, step,
                                                            h.lr, h.beta_1, h.beta_2, h.epsilon, t, part);
    else
        launch(k_mlp_update<NCF_OPT_SGD>, grid, kBlock, 0, st, mlp, m, v, P, slabs, nslab, grad_in,
                                                           grad_out, do_update ? 1 : 0, want_reg ? 1 : 0, step,
                                                           h.lr, h.beta_1, h.beta_2, h.epsilon, t, part);
    *nreg = ((do_update || want_reg) && t.n > 0) ? grid : 0;
    return hipGetLastError();
}

// Groups wider than 8 (evaluation: 1 positive + 99 negatives): one wave per group, its elements
// on the lanes (coalesced reads, chunks of 64), label = first max of y and position = #(p > p_lab)
// + #(earlier ties) from wave reductions — the per-group hit and dcg of k_group_metrics, with
// every lane of the machine busy instead of one thread per group.  A block's 4 waves loop over
// groups with the block's stride and add their sums into one partial per block.
__global__ __launch_bounds__(kBlock) void k_group_metrics_wave(const float* __restrict__ probs,
                                                               const float* __restrict__ labels, int64_t ng,
                                                               int group, int k, float* __restrict__ hit,
                                                               float* __restrict__ dcg, float* __restrict__ part_hit,
                                                               float* __restrict__ part_dcg) {
    __shared__ float red[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float h_acc = 0.f, d_acc = 0.f;
    for (int64_t g = (int64_t)blockIdx.x * 4 + wv; g < ng; g += (int64_t)gridDim.x * 4) {
        const float* pr = probs + g * group;
        const float* lb = labels + g * group;
        float best = -INFINITY;
        for (int j = lane; j < group; j += 64) best = fmaxf(best, lb[j]);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) best = fmaxf(best, __shfl_xor(best, m, 64));
        int first = INT_MAX;
        for (int j = lane; j < group; j += 64) first = lb[j] == best && j < first ? j : first;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) first = min(first, __shfl_xor(first, m, 64));
        const int lab = first;
        const float pl = pr[lab];
        int cnt = 0;
        for (int j = lane; j < group; j += 64) {
            const float pj = pr[j];
            cnt += (pj > pl) || (pj == pl && j < lab);
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) cnt += __shfl_xor(cnt, m, 64);
        const float h = cnt < k ? 1.0f : 0.0f;
        const float d = h * (logf(2.0f) / logf((float)cnt + 2.0f));
        if (lane == 0) {
            if (hit) hit[g] = h;
            if (dcg) dcg[g] = d;
        }
        h_acc += h;
        d_acc += d;
    }
    if (lane == 0) red[wv] = h_acc;
    __syncthreads();
    const float hs = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    if (lane == 0) red[wv] = d_acc;
    __syncthreads();
    const float ds = (red[0] + red[1]) + (red[2] + red[3]);
    if (threadIdx.x == 0) {
        if (part_hit) part_hit[blockIdx.x] = hs;
        if (part_dcg) part_dcg[blockIdx.x] = ds;
    }
}

hipError_t launch_group_metrics(const float* probs, const float* labels, int64_t n_groups, int group, int k,
                                float* hit, float* dcg, float* part_hit, float* part_dcg, int* nparts,
                                hipStream_t st) {
    if (group > 8) {
        // a wave per group; at most ceil(samples / kBlock) partials (the workspace's nmetric)
        const int64_t by_groups = (n_groups + 3) / 4, cap = (n_groups * group + kBlock - 1) / kBlock;
        const int grid = (int)(by_groups < cap ? by_groups : cap);
        *nparts = grid;
        if (grid == 0) return hipSuccess;
        launch(k_group_metrics_wave, grid, kBlock, 0, st, probs, labels, n_groups, group, k, hit, dcg, part_hit,
               part_dcg);
        return hipGetLastError();
    }
    const int grid = (int)((n_groups + kBlock - 1) / kBlock);
    *nparts = grid;
    if (grid == 0) return hipSuccess;
    launch(k_group_metrics, grid, kBlock, 0, st, probs, labels, n_groups, group, k, hit, dcg, part_hit, part_dcg);
    return hipGetLastError();
}

hipError_t launch_rank(const float* probs, int64_t n_groups, int group, int32_t* rank_idx, hipStream_t st) {
    const int grid = (int)((n_groups + kBlock - 1) / kBlock);
    if (grid == 0) return hipSuccess;
    launch(k_rank, grid, kBlock, 0, st, probs, n_groups, group, rank_idx);
    return hipGetLastError();
}

hipError_t launch_summary(const WsLayout& L, void* ws, int nbce, int nmet, float n_groups, int nreg_emb,
                          int nreg_mlp, float* summary, hipStream_t st) {
    const float* reg = at<float>(ws, L.part_reg);
    launch(k_summary, 1, kBlock, 0, st, at<float>(ws, L.part_bce), nbce, at<float>(ws, L.part_hit),
                                    at<float>(ws, L.part_dcg), nmet, n_groups, reg, nreg_emb, reg + kUpdateGrid,
                                    nreg_mlp, summary);
    return hipGetLastError();
}

hipError_t launch_stats(const WsLayout& L, void* ws, const float* summary_in, int nreg_emb, int nreg_mlp,
                        float inv_batch, double* stats, int32_t* step, bool bump_step, hipStream_t st,
                        bool scan_ahead, int64_t scan_keys, SummaryFirst sf, int32_t* drop, bool sparse_scan,
                        const ReplayDeferred* replay) {
    const float* reg = at<float>(ws, L.part_reg);
    // written only by the summary_first block (the workspace's summary); read-only otherwise
    float* summary = const_cast<float*>(summary_in);
    SummaryArgs sa{nullptr, nullptr, nullptr, nullptr, 0, 0, 0.f, drop};
    if (sf.nbce >= 0)
        sa = SummaryArgs{summary, at<float>(ws, L.part_bce), at<float>(ws, L.part_hit), at<float>(ws, L.part_dcg),
                         sf.nbce, sf.nmet, sf.n_groups, drop};
    if (scan_ahead) {
        const int64_t r1 = scan_keys + 1;
        const int nscan = (int)((r1 + kScanBlock - 1) / kScanBlock);
        ScanAhead sc{at<const int32_t>(ws, L.cnt_ahead), r1, at<int32_t>(ws, L.offs_local), at<int32_t>(ws, L.tot),
                     at<int32_t>(ws, L.uloc), at<int32_t>(ws, L.utot), at<int32_t>(ws, L.cnt), at<int32_t>(ws, L.heavy_n),
                     touched_out(L, ws), sparse_scan ? 1 : 0, sparse_scan ? at<int32_t>(ws, L.itag) : nullptr};
        if (sparse_scan && (!sparse_index_ok(L) || r1 != L.keys + 1)) return hipErrorInvalidValue;
        ReplayAhead ra{};
        if (replay && replay->contributions > 0) {
            if (L.world != 0 || replay->contributions > 2 * L.max_batch) return hipErrorInvalidValue;
            const int64_t mc = replay->contributions;
            ra = ReplayAhead{(int)count_ahead_passes(mc), count_per(mc), at<const int2>(ws, L.claims),
                             at<const int32_t>(ws, L.nclaim), at<const int32_t>(ws, L.claim_t), replay->emb, replay->m,
                             replay->v, replay->row_width, replay->lr, replay->beta_1, replay->beta_2, replay->epsilon};
        }
        launch(k_stats_scan, 1 + (ra.npass + kReplayPasses - 1) / kReplayPasses + nscan, kBlock, 0, st, summary, reg, nreg_emb, reg + kUpdateGrid, nreg_mlp,
               inv_batch, stats, step, bump_step ? 1 : 0, sc, sa, ra);
        return hipGetLastError();
    }
    if (replay && replay->contributions > 0) return hipErrorInvalidValue;  // (the replay rides on the scan)
    launch(k_stats, 1, kBlock, 0, st, summary, reg, nreg_emb, reg + kUpdateGrid, nreg_mlp, inv_batch, stats, step,
                                  bump_step ? 1 : 0, sa);
    return hipGetLastError();
}

}  // namespace ncf
