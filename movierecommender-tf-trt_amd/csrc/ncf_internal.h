// Internal declarations shared by the HIP translation units of libmovierec_ncf.
// Not part of the ABI (see include/movierec_ncf.h).
#pragma once

#include <climits>
#include <cstdlib>

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "movierec_ncf.h"
#include "ncf_common.h"

namespace ncf {

constexpr int kBlock = 256;            // threads per workgroup for the streaming kernels
constexpr int kScanBlock = 2048;       // keys per block of the offset scan (8 per thread)
constexpr int kSmallSeg = 16;          // segments up to this length are sorted in registers
constexpr int kMaxSlabs = 1024;        // partial dense-gradient slabs (one per producing block)
constexpr int kSlabSplit = 16;         // first-level slab reduction fan-in groups
constexpr int kUpdateGrid = 2048;      // grid of the embedding-table sweep (fixed: deterministic partials)
constexpr int64_t kMaxBatch = 262144;  // heavy-segment bitmap must fit the LDS (2*B bits = 64 KB)
constexpr int kFillBigScan = 256;      // scan blocks above which the index fill uses k_prefix + k_fill_big
constexpr int kMaxFillScan = 128;      // scan blocks (262,144 keys) the in-kernel index fill holds (FillArgs)
constexpr int kPrefixPer = 32;         // k_prefix's chunk length cap: at most 8,192 scan blocks (16.7 M keys)
constexpr int kHeavyMin = 8;           // smallest list length the touched-row update leaves to its heavy blocks

#ifndef NCF_DEBUG_BOUNDS
#define NCF_DEBUG_BOUNDS 0   // 1: printf + skip on out-of-range index-path accesses (diagnostic builds)
#endif

// Kernel-selection switches for A/B experiments (NCF_FB_KERNEL, NCF_WAVE_SPLIT, NCF_FOLD_USERS,
// NCF_UNIT_SCHED, NCF_SIDE_STREAM): read from the environment only by a library built with
// -DNCF_EXPERIMENT_ENV=1 (tools/ variants); the product library ignores them
#ifndef NCF_EXPERIMENT_ENV
#define NCF_EXPERIMENT_ENV 0
#endif
inline const char* experiment_env(const char* name) { return NCF_EXPERIMENT_ENV ? getenv(name) : nullptr; }

// Scalars every kernel of a step reads (device copy of hyper + derived).
struct StepScalars {
    int32_t t;       // optimizer iteration being applied (1-based)
    float lr_t;      // Adam bias-corrected lr (Keras v1 formula)
};

// Byte offsets of the workspace regions (host-computed, passed by value).
struct WsLayout {
    size_t cnt;       // int32[R+1]  persistent, all-zero between calls: the index fill's per-key cursors
    size_t cnt_ahead; // int32[R+1]  persistent, all-zero between calls: the NEXT batch's counts, taken by
                      // the touched-row update; the scan ahead copies them into cnt and zeroes them, so
                      // the fill of one batch and the count of the next never share a counter
    size_t heavy_n;   // int32       persistent
    size_t err;       // int32       persistent (sticky id-out-of-range flag)
    size_t persistent_end;
    size_t probs;     // float[B]
    size_t gs;        // float[2B * W] per-contribution gradient rows
    size_t list;      // int32[list_cap] contributions grouped by key (sorted inside a key)
    size_t offs_local;// int32[R+1]  per-2048-row local exclusive scan
    size_t offs;      // int32[R+1]  row -> first list slot
    size_t tot;       // int32[nscan]
    size_t pre;       // int32[2 * nscan]  exclusive prefixes of tot / utot (large key spaces: k_prefix)
    size_t part_bce;  // float[kMaxSlabs]
    size_t part_hit;  // float[nmetric]
    size_t part_dcg;  // float[nmetric]
    size_t part_reg;  // float[kUpdateGrid + mlp blocks]
    size_t summary;   // float[NCF_NUM_SUMMARY]
    size_t slabs;     // float[kMaxSlabs * P]
    size_t mlp_grad;  // float[P] (reduced dense-layer gradient, single-device path)
    size_t slab_part; // float[kSlabSplit * P] first-level slab sums
    // row-sharded plan (world > 0 only; else empty): unique table rows of the batch
    size_t uloc;      // int32[K+1]  per-2048-key local exclusive scan of (cnt > 0)
    size_t utot;      // int32[nscan]
    size_t ifold;     // int32       user-row folding of the last index build (persistent)
    size_t stale_step;// int32      persistent: nonzero while the current step is dropped (fill_wave)
    size_t seen;      // int32[K+1] persistent (single table): the sparse index's tag of the batch that last
                      // touched each key (sparse_index_ok: k_fill_touched writes it, the count blocks read it)
    size_t itag;      // int32      persistent: the last sparse index's tag (bumped by the stats launch)
    size_t claims;    // int2[2B]    single table: the catch-up-ahead claims (key, s0) per count pass
    size_t nclaim;    // int32[2B / 16 + 1] their number per pass
    size_t claim_t;   // int32       their replay target step
    size_t cid_u;     // int32[B]    compact (unique-row) id of each sample's user row
    size_t cid_i;     // int32[B]    compact id of each sample's item row
    size_t uoffs;     // int32[2B+1] compact row -> first list slot
    size_t nuniq;     // int32       number of unique rows (single table: of touched rows)
    size_t touched;   // int32[min(R, 2B)] single table, deferred decay: the touched rows, ascending
    size_t touched_oc;  // int2[min(R, 2B)] their (list offset, contribution count): the update needs no offs
    size_t heavy;     // int32[2B / kHeavyMin + 1] single table: touched-list positions of the rows whose
                      // lists the touched-row update sorts block-wide (FillArgs); count in heavy_n
    size_t tl;        // int32[nscan * kScanBlock] single table: the scan ahead's touched rows per scan block
    size_t tocl;      // int2[nscan * kScanBlock]  their (offset inside the block's list part, count)
    size_t slist;     // int32[2B] single table: the heavy rows' sorted lists (indexed like list)
    size_t act;       // float[B * A] generic kernel activations
    size_t dz;        // float[B * D] generic kernel pre-activation grad
    size_t ones;      // float[B] layered path: all-ones vector (column sums as GEMV)ients
    // row-sharded owner index (world > 0 only): the rows this rank serves, keyed by local shard row;
    // every region sized by the shard alone (placed before the per-batch regions, so serving rows
    // and updating them use the same offsets whatever the requesters' batch size)
    size_t ocnt;      // int32[S+1]  persistent, all-zero between calls
    size_t oheavy;    // int32       persistent
    size_t oifold;    // int32       persistent (written by the index build, never read)
    size_t ooffs_local, ooffs, ouloc;  // int32[S+1]
    size_t otot, outot;                // int32[onscan]
    size_t opre;                       // int32[2 * onscan]
    size_t olist;     // int32[world * S] received entries grouped by local row (ascending entry)
    size_t otouched;  // int32[S] the served rows, ascending
    size_t otoc;      // int2[S] their (list offset, entry count)
    size_t onuniq;    // int32
    int onscan;
    size_t total;
    int64_t max_batch;
    int nscan;        // blocks of the offset scan
    int nmetric;      // max blocks of the metrics kernel
    int act_w;        // A
    int dz_w;         // D
    int world;        // 0: single table; > 0: row-sharded plan layout for this many ranks
    int64_t shard_rows;  // S = ceil(R / world) (R when world == 0)
    int64_t keys;     // key space of the index: world * S (R when world == 0)
    int64_t list_cap; // contribution capacity of list (2B, or world * min(2B, S) for the owner index)
};

// Per-kScanBlock-key exclusive scan of cnt into offs (+ block total), and for UNIQ of the flags
// cnt > 0 into uloc / utot: the body of k_scan_local for scan block `blk` (whole workgroup).
// cnt[key] += 1 for every lane with ok, called by all 64 lanes of a wave together.  Equal keys
// two lanes apart (a user group's contributions c = 2i, 2i+2, ...) form runs: the run's head
// adds the run length with one atomic, so a group does not queue on one counter.
// FIRST: the head lane returns whether its run is the key's first occurrence in the counted set
// (the count it added to was 0: the counters start at zero for a batch), every other lane false.
template <bool FIRST = false>
__device__ __forceinline__ bool wave_run_count(int32_t* __restrict__ cnt, int key, bool ok) {
    const int lane = threadIdx.x & 63;
    const uint64_t par = (lane & 1) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int kk = ok ? key : -2 - lane;
    const int prev = __shfl_up(kk, 2, 64);
    const uint64_t heads = ~__ballot(lane >= 2 && prev == kk) & par;
    const uint64_t later = heads & ~upto;
    const int next = later ? __ffsll((unsigned long long)later) - 1 : 64 + (lane & 1);
    if (ok && ((heads >> lane) & 1ull)) {
        if constexpr (FIRST) return atomicAdd(&cnt[key], (next - lane) >> 1) == 0;
        atomicAdd(&cnt[key], (next - lane) >> 1);
    }
    return false;
}

// The scan ahead's share of the next index's row side: scan block b's touched rows, in key order,
// at [b * kScanBlock, + utot[b]) of tl, with their (offset inside the block's part of the list,
// count) in tocl — the fill compacts them into the touched list (fill_wave), touching occupied
// keys only instead of every key of the table
struct TouchedOut {
    int32_t* tl;
    int2* tocl;
};

// move_to (optional): the counts were taken ahead (ws cnt_ahead); they also move to the fill's
// cursors move_to (ws cnt) and cnt is zeroed for the next batch's count
// SPARSE (large key spaces, sparse_index_ok): the move, the zeroing and the local offsets are written
// for the occupied keys only (every other key's cursor and count are zero already — the fill and
// the update leave them so — and its offset is never read: the fill reads the offsets of listed
// keys, the count blocks test membership with the seen tags), the occupied-key numbering (uloc) not
// at all: the scan's dense writes were 4 x 4 bytes per key of the table (11 M keys at config D)
// scan block blk's counts, 8 keys per thread: two int4 loads when all 8 are inside (the workspace
// regions are 256-byte aligned and the thread's first key a multiple of 8), else key by key
__device__ __forceinline__ void scan_local_load(const int32_t* cnt, int64_t r1, int blk, int (&v)[8]) {
    const int64_t base = (int64_t)blk * kScanBlock + threadIdx.x * 8;
    if (base + 8 <= r1) {
        const int4 a = *reinterpret_cast<const int4*>(cnt + base), b = *reinterpret_cast<const int4*>(cnt + base + 4);
        v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (base + j < r1) ? cnt[base + j] : 0;
    }
}

// the scan of block blk from its loaded counts v (scan_local_load)
template <bool UNIQ, bool SPARSE = false>
// (cnt is written through when moving: not a const __restrict__ pointer, whose memory the compiler
// may assume nothing writes)
__device__ inline void scan_local_apply(const int (&v)[8], const int32_t* cnt, int64_t r1, int32_t* __restrict__ offs,
                                        int32_t* __restrict__ tot, int32_t* __restrict__ uloc,
                                        int32_t* __restrict__ utot, int blk, int32_t* __restrict__ move_to = nullptr,
                                        int32_t* __restrict__ zero_at_end = nullptr, TouchedOut to = TouchedOut{}) {
    __shared__ int sw[4];
    const int64_t base = (int64_t)blk * kScanBlock + threadIdx.x * 8;
    const bool full = base + 8 <= r1;
    int sum = 0, nz = 0;
    if (SPARSE && move_to) {
        int32_t* zc = const_cast<int32_t*>(cnt);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (v[j] != 0) move_to[base + j] = v[j], zc[base + j] = 0;
    } else if (move_to) {
        int32_t* zc = const_cast<int32_t*>(cnt);
        if (full) {
            *reinterpret_cast<int4*>(move_to + base) = make_int4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<int4*>(move_to + base + 4) = make_int4(v[4], v[5], v[6], v[7]);
            *reinterpret_cast<int4*>(zc + base) = make_int4(0, 0, 0, 0);
            *reinterpret_cast<int4*>(zc + base + 4) = make_int4(0, 0, 0, 0);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (base + j < r1) move_to[base + j] = v[j], zc[base + j] = 0;
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        sum += v[j];
        nz += v[j] > 0;
    }
    int total;
    int run = block_exscan_256(sum, sw, &total);
    int o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        o[j] = run;
        run += v[j];
    }
    if (SPARSE) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (v[j] != 0) offs[base + j] = o[j];
    } else if (full) {
        *reinterpret_cast<int4*>(offs + base) = make_int4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<int4*>(offs + base + 4) = make_int4(o[4], o[5], o[6], o[7]);
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (base + j < r1) offs[base + j] = o[j];
    }
    if (threadIdx.x == 0) tot[blk] = total;
    if constexpr (UNIQ) {
        int utotal;
        int urun = block_exscan_256(nz, sw, &utotal);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            o[j] = urun;
            urun += v[j] > 0;
        }
        if (SPARSE) {
        } else if (full) {
            *reinterpret_cast<int4*>(uloc + base) = make_int4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<int4*>(uloc + base + 4) = make_int4(o[4], o[5], o[6], o[7]);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (base + j < r1) uloc[base + j] = o[j];
        }
        if (threadIdx.x == 0) utot[blk] = utotal;
        if (to.tl) {
            int ro = run - sum;  // this thread's first list offset inside the block (o[] is the numbering now)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (v[j] > 0) {
                    const int64_t e = (int64_t)blk * kScanBlock + o[j];
                    to.tl[e] = (int)(base + j);
                    to.tocl[e] = make_int2(ro, v[j]);
                }
                ro += v[j];
            }
        }
    }
    // last, after every use of threadIdx.x: a `blockIdx.x == 1 && threadIdx.x == 0` store ahead of
    // the body made hipcc (ROCm 7.2) feed the later blocks an undefined thread id
    if (zero_at_end && blk == 0 && threadIdx.x == 0) *zero_at_end = 0;
}

template <bool UNIQ, bool SPARSE = false>
__device__ inline void scan_local_body(const int32_t* cnt, int64_t r1, int32_t* __restrict__ offs,
                                       int32_t* __restrict__ tot, int32_t* __restrict__ uloc,
                                       int32_t* __restrict__ utot, int blk, int32_t* __restrict__ move_to = nullptr,
                                       int32_t* __restrict__ zero_at_end = nullptr, TouchedOut to = TouchedOut{}) {
    int v[8];
    scan_local_load(cnt, r1, blk, v);
    scan_local_apply<UNIQ, SPARSE>(v, cnt, r1, offs, tot, uloc, utot, blk, move_to, zero_at_end, to);
}

// User-row folding (the north star's duplicate-index reduction, done where the gradients are
// made): the reference's batches are groups of group = negs + 1 samples sharing one user
// (data_pipeline.py:141).  With fold = group (a power of two <= 32, fused kernel only), the
// user-gradient rows of a group's samples whose user equals the group head's are summed inside
// the kernel (lanes of one wave, fixed butterfly order) and written once, as the head's
// contribution c = 2 * head; the others' user contributions do not exist.  Samples whose user
// differs from the head's keep their own contribution, so any batch stays exact.  Fold widths
// 2, 4 (the reference's default: 3 negatives) and 8 have fused-kernel variants.
// fused: the step runs a kernel that folds (the fused MFMA kernels and the layered path's k_lay_l1b)
inline int fold_of(int group, bool fused) { return fused && (group == 2 || group == 4 || group == 8) ? group : 0; }
__device__ __forceinline__ bool folded_user(const int32_t* __restrict__ users, int64_t i, int fold) {
    if (fold <= 1) return false;
    const int64_t hd = i - i % fold;
    return i != hd && users[i] == users[hd];
}

// Workspace error flags (L.err, sticky until ncf_workspace_flags reads them).
constexpr int kErrIdRange = 1;     // an index build met an id outside the table
constexpr int kErrStaleCount = 4;  // a counted-ahead index met ids that differ from the counted ones
constexpr int kErrFold = 8;        // an index built ahead folds user rows differently than the step
                                   // using it (ncf_build_index / ncf_shard_plan hyper mismatch)

// cnt/err (optional): every row's counter must be back at zero after k_fill; a residue means the
// ids changed after they were counted ahead (ncf_train_step_ahead) — flagged, and the counter
// cleared so that the next build starts from zero.
// RPT rows per thread (8 for very large key spaces, config D's 11 M rows: int4 loads of the
// offsets and counters, an eighth of the workgroups)
constexpr int64_t kSortRpt8Rows = 1 << 20;
__host__ __device__ inline int sort_rpt(int64_t R) { return R > kSortRpt8Rows ? 8 : 1; }
// LISTED: the rows of the touched list (counted keys; (offset, count) from the list) instead of
// every row: large key spaces, where k_fill_big adds back what it takes below zero, so a residue
// can only sit at a counted key
template <int RPT = 1, bool LISTED = false>
__device__ inline void sort_rows_body(const int32_t* __restrict__ offs, int64_t R, int32_t* __restrict__ list,
                                      int nwords, int blk, int32_t* __restrict__ cnt = nullptr,
                                      int32_t* __restrict__ err = nullptr, const int32_t* __restrict__ touched = nullptr,
                                      const int2* __restrict__ toc = nullptr, const int32_t* __restrict__ nuniq = nullptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned bm[];
    __shared__ int2 hrows[kBlock * RPT];  // (offset, count) of the longer lists
    __shared__ int2 mrows[kBlock * RPT];
    __shared__ int nh, nm;
    __shared__ int sw[4];
    if (threadIdx.x == 0) nh = nm = 0;
    __syncthreads();
    const int64_t r0 = ((int64_t)blk * kBlock + threadIdx.x) * RPT;
    int ov[RPT + 1], cv[RPT];
    int64_t rl = -1;  // LISTED: this thread's row
    if constexpr (LISTED) {
        static_assert(RPT == 1, "listed rows: one per thread");
        const int64_t i = (int64_t)blk * kBlock + threadIdx.x;
        if (i < *nuniq) {
            rl = touched[i];
            const int2 oc = toc[i];
            ov[0] = oc.x;
            ov[1] = oc.x + oc.y;
            cv[0] = cnt ? cnt[rl] : 0;
        } else {
            ov[0] = ov[1] = cv[0] = 0;
        }
    } else if (RPT > 1 && r0 + RPT < R) {
        const int4 a = *reinterpret_cast<const int4*>(offs + r0), b = *reinterpret_cast<const int4*>(offs + r0 + 4);
        ov[0] = a.x, ov[1] = a.y, ov[2] = a.z, ov[3] = a.w, ov[4] = b.x, ov[5] = b.y, ov[6] = b.z, ov[7] = b.w;
        ov[RPT] = offs[r0 + RPT];
        if (cnt) {
            const int4 x = *reinterpret_cast<const int4*>(cnt + r0), y = *reinterpret_cast<const int4*>(cnt + r0 + 4);
            cv[0] = x.x, cv[1] = x.y, cv[2] = x.z, cv[3] = x.w, cv[4] = y.x, cv[5] = y.y, cv[6] = y.z, cv[7] = y.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j <= RPT; ++j) ov[j] = r0 + j <= R ? offs[r0 + j] : 0;
#pragma unroll
        for (int j = 0; j < RPT; ++j) cv[j] = cnt && r0 + j < R ? cnt[r0 + j] : 0;
    }
#pragma unroll
    for (int jr = 0; jr < RPT; ++jr) {
    const int64_t r = LISTED ? rl : r0 + jr;
    if (cnt && r >= 0 && r < R && cv[jr] != 0) {
        atomicOr(err, kErrStaleCount);
        cnt[r] = 0;
    }
    if (r >= 0 && r < R) {
        const int o = ov[jr];
        const int c = ov[jr + 1] - o;
        if (c > 64) {
            hrows[atomicAdd(&nh, 1)] = make_int2(o, c);
        } else if (c > kSmallSeg) {
            mrows[atomicAdd(&nm, 1)] = make_int2(o, c);
        } else if (c >= 2) {
            int v[kSmallSeg];
#pragma unroll
            for (int j = 0; j < kSmallSeg; ++j) v[j] = (j < c) ? list[o + j] : INT_MAX;
#pragma unroll
            for (int round = 0; round < kSmallSeg; ++round) {
#pragma unroll
                for (int j = round & 1; j + 1 < kSmallSeg; j += 2) {
                    const int a = min(v[j], v[j + 1]);
                    const int b = max(v[j], v[j + 1]);
                    v[j] = a;
                    v[j + 1] = b;
                }
            }
#pragma unroll
            for (int j = 0; j < kSmallSeg; ++j)
                if (j < c) list[o + j] = v[j];
        }
    }
    }
    __syncthreads();
    // rows of 17..64 entries (frequent when a rank's users are few — user-partitioned DP): one
    // wave each, a bitonic network across the 64 lanes (one entry per lane, INT_MAX padding)
    {
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        for (int hh = wv; hh < nm; hh += kBlock / 64) {
            const int o = mrows[hh].x;
            const int c = mrows[hh].y;
            int x = lane < c ? list[o + lane] : INT_MAX;
#pragma unroll
            for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const int y = __shfl_xor(x, j, 64);
                    const bool asc = (lane & k) == 0;
                    const bool lower = (lane & j) == 0;
                    x = (lower == asc) ? min(x, y) : max(x, y);
                }
            }
            if (lane < c) list[o + lane] = x;
        }
    }
    const int count = nh;
    const int per = (nwords + kBlock - 1) / kBlock;
    for (int hh = 0; hh < count; ++hh) {
        const int o = hrows[hh].x;
        const int c = hrows[hh].y;
        for (int w = threadIdx.x; w < nwords; w += kBlock) bm[w] = 0u;
        __syncthreads();
        for (int j = threadIdx.x; j < c; j += kBlock) {
            const unsigned v = (unsigned)list[o + j];
            atomicOr(&bm[v >> 5], 1u << (v & 31));
        }
        __syncthreads();
        const int w0 = threadIdx.x * per;
        const int w1 = min(w0 + per, nwords);
        int mine = 0;
        for (int w = w0; w < w1; ++w) mine += __popc(bm[w]);
        int total;
        int pos = o + block_exscan_256(mine, sw, &total);
        for (int w = w0; w < w1; ++w) {
            unsigned b = bm[w];
            while (b) {
                const int bit = __ffs(b) - 1;
                list[pos++] = w * 32 + bit;
                b &= b - 1;
            }
        }
        __syncthreads();
    }
}

// In-kernel index fill (a batch counted and scanned ahead; single-table keys, touched list):
// k_fill's outputs, computed by the waves of another launch that would otherwise wait (the wave
// kernel's weight-gradient waves before their first unit), so the step has no fill launch.  The
// lists are left UNSORTED: the touched-row update orders each row's list itself (rows of up to hc
// entries across the lanes of their row group, longer ones — listed in `heavy` — block-wide).  A
// run that takes a counter below zero gives the excess back (k_fill_big's rule): a residue can
// only sit at a counted key, i.e. in the touched list, where the update checks it.
struct FillArgs {
    int32_t* cnt;             // per-key cursors: the counts the scan ahead copied (ws cnt)
    const int32_t* local;     // per-scan-block exclusive offsets (ws offs_local)
    const int32_t* tot;       // scan-block totals
    const int32_t* utot;      // occupied keys per scan block
    const int32_t* tl;        // the scan ahead's touched rows per block (TouchedOut)
    const int2* tocl;
    int nscan;                // <= kMaxFillScan
    int64_t r1;               // keys + 1
    int32_t* list;
    int32_t* touched;         // touched rows, ascending
    int2* toc;                // their (list offset, count)
    int32_t* nuniq;
    int32_t* heavy;           // touched-list positions of the rows with more than hc entries
    int32_t* heavy_n;         // zeroed by the scan ahead
    int hc;
    int32_t* err;
    int32_t* ifold;
    int32_t U, I;             // user u -> key u, item v -> key U + v
    int64_t list_cap, touched_cap, heavy_cap;  // region sizes (debug bound checks)
    int32_t* stale_step;      // set when a contribution finds no slot: the step is dropped (below);
                              // nullptr: never dropped (data parallelism: flagged only)
};
#if NCF_DEBUG_BOUNDS == 1
#define NCF_BOUND(cond, ...)          \
    if (!(cond)) {                    \
        printf(__VA_ARGS__);          \
    } else
#elif NCF_DEBUG_BOUNDS == 2
// no printf (the kernel's code stays close to the release build): flag bit 0x100 and skip
#define NCF_BOUND(cond, ...)          \
    if (!(cond)) {                    \
        atomicOr(f.err, 0x100);       \
    } else
#else
#define NCF_BOUND(cond, ...)
#endif

constexpr int kFillContribPerLane = 2;  // its CU: contributions per lane and pass

// Wave gw of nw: its share of the fill of batch (users, items, n) folded by `fold`.  The
// exclusive prefixes of the scan-block totals stay in registers (lane l: blocks l and l + 64) and
// are read with lane shuffles, so every loop below is wave-uniform.  PART: 1 the rows, 2 the
// contributions, 3 both.
// A contribution that finds no slot means the ids changed after they were counted (a write that
// bypassed torch's version counter): the forward pass of this very launch or the next may have
// read rows the counted set missed, at their deferred step.  Such a step is DROPPED — f.stale_step
// tells the touched-row update and the stats launch to apply nothing of it (the table, moments,
// dense layers, stats and step counter stay as they were: a consistent deferred-decay state) —
// and reported (NCF_WSERR_STALE_COUNT, RuntimeError from check_errors).
// Changed ids that overflow no counted row — fewer valid, unfolded contributions at some keys than
// were counted (ids moved out of the table, users that now fold into their group head), none more
// anywhere — read no row outside the counted set.  Such a step is exact as it stands: a key's
// run takes slots from the top of its range down, so its unfilled slots are the lowest `residue`
// ones (the cursor a key keeps after the fill); the touched-row update sums only the slots above
// them (a counted row left with no contribution takes the zero-gradient step, as in the dense
// sweep) and clears the residue, and the error is still reported.  (the update used to
// read those stale slots as contributions.)
template <int PART = 3>
__device__ inline void fill_wave(const FillArgs& f, const int32_t* __restrict__ users,
                                 const int32_t* __restrict__ items, int64_t n, int fold, int gw, int nw);
template <int PART>
__device__ inline void fill_wave(const FillArgs& f, const int32_t* __restrict__ users,
                                 const int32_t* __restrict__ items, int64_t n, int fold, int gw, int nw) {
    const int lane = threadIdx.x & 63;
    int p0, p1, q0, q1;  // pre[lane], pre[lane + 64], upre[lane], upre[lane + 64]
    int u0, u1, ntouched;  // utot[lane], utot[lane + 64], their sum
    {
        const int t0 = lane < f.nscan ? f.tot[lane] : 0, t1 = lane + 64 < f.nscan ? f.tot[lane + 64] : 0;
        u0 = lane < f.nscan ? f.utot[lane] : 0;
        u1 = lane + 64 < f.nscan ? f.utot[lane + 64] : 0;
        int a0 = t0, a1 = t1, b0 = u0, b1 = u1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int x0 = __shfl_up(a0, d, 64), x1 = __shfl_up(a1, d, 64);
            const int y0 = __shfl_up(b0, d, 64), y1 = __shfl_up(b1, d, 64);
            if (lane >= d) a0 += x0, a1 += x1, b0 += y0, b1 += y1;
        }
        const int ca = __shfl(a0, 63, 64), cb = __shfl(b0, 63, 64);
        p0 = a0 - t0;
        p1 = ca + a1 - t1;
        q0 = b0 - u0;
        q1 = cb + b1 - u1;
        ntouched = cb + __shfl(b1, 63, 64);
#if NCF_DEBUG_BOUNDS == 1
        if (gw == 0 && lane < 4 && lane < f.nscan)
            printf("fill lane %d: tot %d utot %d pre %d upre %d nscan %d\n", lane, t0, u0, p0, q0, f.nscan);
#endif
    }
    // prefix of scan block b (b < kMaxFillScan), every lane its own b
    auto pre = [&](int64_t key) {
        const int b = (int)(key / kScanBlock);
        const int x = __shfl(p0, b & 63, 64), y = __shfl(p1, b & 63, 64);
        return b < 64 ? x : y;
    };
    const int64_t rstep = (int64_t)nw * 64;
    // rows: the scan ahead's per-block touched rows compacted into the touched list with (list
    // offset, count), and the heavy rows — one 64-slot chunk of a block's row slots per wave and
    // pass; a chunk past the block's occupied keys costs a compare (its count from a register)
    const int64_t nchunk = (int64_t)f.nscan * (kScanBlock / 64);
    for (int64_t ch = gw; (PART & 1) && ch < nchunk; ch += nw) {
        const int b = (int)(ch / (kScanBlock / 64));
        const int j = (int)(ch % (kScanBlock / 64)) * 64 + lane;
        // the block's count and prefixes, read while every lane is active: v_readlane takes the
        // named lane's register whatever the exec mask, and inside the branch below that lane may
        // be inactive — its copy of the register then holds whatever the allocator put there (a
        // first version read them there and wrote a row at another block's position)
        const int ub = __builtin_amdgcn_readlane(b < 64 ? u0 : u1, b & 63);     // utot[b]
        const int ubase = __builtin_amdgcn_readlane(b < 64 ? q0 : q1, b & 63);  // upre(b)
        const int obase = __builtin_amdgcn_readlane(b < 64 ? p0 : p1, b & 63);  // pre(b)
        if ((int)(ch % (kScanBlock / 64)) * 64 >= ub) continue;                 // wave-uniform
        if (j < ub) {
            const int64_t e = (int64_t)b * kScanBlock + j;
            const int key = f.tl[e];
            const int2 lc = f.tocl[e];
            const int u = ubase + j;
            const int o = obase + lc.x;
            NCF_BOUND(u >= 0 && u < f.touched_cap && o >= 0 && o + lc.y <= f.list_cap,
                      "fill row %d: u %d (cap %lld) o %d c %d (list cap %lld)\n", key, u,
                      (long long)f.touched_cap, o, lc.y, (long long)f.list_cap) {
            f.touched[u] = key;
            f.toc[u] = make_int2(o, lc.y);
            if (lc.y > f.hc) {
                const int hx = atomicAdd(f.heavy_n, 1);
                NCF_BOUND(hx < f.heavy_cap, "fill heavy %d cap %lld\n", hx, (long long)f.heavy_cap)
                f.heavy[hx] = u;
            }
            }
        }
    }
    if constexpr ((PART & 1) != 0) {
        if (gw == 0 && lane == 0) {
            *f.nuniq = ntouched;
            *f.ifold = fold;
        }
    }
    // contributions c = 2i + side, a wave at a time (k_fill's runs: equal keys two lanes apart share
    // one atomic; slot order inside a key is free, the update sorts)
    const int64_t m = 2 * n;
    const uint64_t par = (lane & 1) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    constexpr int CU = kFillContribPerLane;
    for (int64_t cb = (int64_t)gw * 64; (PART & 2) && cb < m; cb += CU * rstep) {
        int id[CU], hid[CU];
#pragma unroll
        for (int j = 0; j < CU; ++j) {
            const int64_t c = cb + j * rstep + lane;
            const int64_t i = c >> 1;
            id[j] = c < m ? ((c & 1) ? items[i] : users[i]) : 0;
            hid[j] = c < m && !(c & 1) && fold > 1 ? users[i - i % fold] : 0;
        }
#pragma unroll
        for (int j = 0; j < CU; ++j) {
            const int64_t c0 = cb + j * rstep;
            if (c0 >= m) break;
            const int64_t c = c0 + lane;
            const int64_t i = c >> 1;
            bool ok = false;
            int key = 0;
            if (c < m) {
                if (c & 1) {
                    ok = (unsigned)id[j] < (unsigned)f.I;
                    key = f.U + id[j];
                } else {
                    ok = (unsigned)id[j] < (unsigned)f.U;
                    key = id[j];
                }
                if (!ok) atomicOr(f.err, kErrIdRange);
                // a user contribution folded into its group head's has no slot
                if (!(c & 1) && fold > 1 && i % fold != 0 && hid[j] == id[j]) ok = false;
            }
            const int kp = pre(ok ? key : 0);
            const int kk = ok ? key : -2 - lane;  // inactive lanes: unique keys
            const int prev = __shfl_up(kk, 2, 64);
            const uint64_t heads = ~__ballot(lane >= 2 && prev == kk) & par;
            const int head = 63 - __clzll(heads & upto);
            const uint64_t later = heads & ~upto;
            const int next = later ? __ffsll((unsigned long long)later) - 1 : 64 + (lane & 1);
            int top = 0, loc = 0;
            if (ok) loc = f.local[key];
            if (ok && lane == head) {
                top = atomicSub(&f.cnt[key], (next - head) >> 1);
                const int over = ((next - head) >> 1) - max(top, 0);
                if (over > 0) atomicAdd(&f.cnt[key], over);
            }
            top = __shfl(top, head, 64);
            const int slot = top - 1 - ((lane - head) >> 1);
            if (ok && slot >= 0) {
                const int64_t li = (int64_t)loc + kp + slot;
                NCF_BOUND(li >= 0 && li < f.list_cap && key < f.r1 - 1, "fill c %lld key %d list %lld cap %lld\n",
                          (long long)c, key, (long long)li, (long long)f.list_cap)
                f.list[li] = (int)c;
            }
            if (ok && slot < 0) {
                atomicOr(f.err, kErrStaleCount);
                if (f.stale_step) atomicOr(f.stale_step, 1);
            }
        }
    }
}

// ncf_user_dp_step's halves (ncf_capi.hip): forward/backward + gradient tail (*filled: the in-kernel
// fill built this step's index), then the own-user update + the next batch counted and scanned
int dp_forward_backward(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                        const int32_t* users, const int32_t* items, const float* labels, int64_t n, float* shared_grad,
                        float* mlp_grad, float* summary, int32_t include_dense_reg, void* ws, size_t ws_bytes,
                        void* stream, bool* filled);
int dp_update_rows(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h, int64_t n,
                   const int32_t* next_users, const int32_t* next_items, int64_t n_next, void* ws, size_t ws_bytes,
                   void* stream, bool filled, bool scan_ahead = true);

// the thread's ncf_last_error() text (printf format); returns code
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// world == 0: single-table layout; world >= 1: row-sharded layout (ncf_shard_*)
WsLayout make_layout(const ncf_shape_t& s, int64_t max_batch, int world = 0);

// Timing events attached to kernel dispatches by the profiler (ncf_profile_enable): while set,
// every dispatch through launch() carries them in its AQL packet (hipExtLaunchKernel), so a
// launch group is timed from its first kernel's start to its last kernel's end without the
// marker packets a hipEventRecord would add to the stream.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
    int launches = 0;
};
LaunchEvents& launch_events();  // thread-local

template <typename... KArgs, typename... Args>
inline void launch(void (*k)(KArgs...), dim3 grid, dim3 block, size_t shmem, hipStream_t st, Args... args) {
    static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel argument count");
    LaunchEvents& ev = launch_events();
    if (ev.stop) {
        hipEvent_t s0 = ev.start;
        ev.start = nullptr;  // the group's first dispatch carries the start stamp
        ++ev.launches;
        hipExtLaunchKernelGGL(k, grid, block, (std::uint32_t)shmem, st, s0, ev.stop, 0u, static_cast<KArgs>(args)...);
    } else {
        hipLaunchKernelGGL(k, grid, block, shmem, st, static_cast<KArgs>(args)...);
    }
}

// Table row numbering of the row-sharded layout: global row g (users 0..U-1,
// items U..U+I-1) is owned by rank g % world at local row g / world.  The plan's index keys
// rows by owner first: key = (g % world) * S + g / world.
inline int64_t shard_rows_of(int64_t R, int world) { return world > 0 ? (R + world - 1) / world : R; }

// Rows under deferred exact decay (hyper->lazy_rows; 0 = every row of the table).
inline int64_t lazy_bound(const ncf_shape_t& s, const ncf_hyper_t& h) {
    return h.lazy_rows > 0 && h.lazy_rows < s.num_rows ? (int64_t)h.lazy_rows : s.num_rows;
}

// Which ids a forward/backward kernel reads: table rows (user u -> row u, item v -> row
// ibase + v, bounds ubound/ibound), or the compact unique-row ids of a row-sharded plan.
struct IdSpace {
    int ubound, ibound, ibase;
};
inline IdSpace table_ids(const ncf_shape_t& s) { return IdSpace{s.num_users, s.num_items, s.num_users}; }
inline IdSpace compact_ids(int64_t n) { return IdSpace{(int)(2 * n), (int)(2 * n), 0}; }

template <typename T>
__host__ __device__ inline T* at(void* base, size_t off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}

// Launchers (return hipError_t of the launch). ------------------------------

// index build: contribution c = 2*i + side (0 user row, 1 item row) grouped by table row
// touched_list: also the ascending list of the touched rows (ws touched, count in nuniq)
// fold: user-row folding group (fold_of), 0 = every sample's user row is a contribution
// sparse (touched_list && counted && sparse_index_ok): the previous step's stats launch scanned the
// counts sparsely (launch_stats sparse_scan); the rows come from its per-block touched lists and
// the keys' seen tags are set (k_fill_touched) — no pass over every key of the table
hipError_t launch_index_build(const ncf_shape_t& s, const WsLayout& L, void* ws, const int32_t* users,
                              const int32_t* items, int64_t n, hipStream_t st, bool touched_list = false,
                              bool counted = false, bool skip_sort = false, int fold = 0, bool sparse = false);
// the counted-ahead index of a single-table step without any pass over every key: large key spaces
// (more scan blocks than k_fill holds, at most what k_prefix scans); the touched-row update's count
// blocks then test "in this step's batch" with the seen tags instead of the offsets
// (-DNCF_SPARSE_INDEX=0: the dense k_fill_big path, for A/B)
#ifndef NCF_SPARSE_INDEX
#define NCF_SPARSE_INDEX 1
#endif
inline bool sparse_index_ok(const WsLayout& L) {
    return NCF_SPARSE_INDEX && L.world == 0 && L.nscan > kFillBigScan && L.nscan <= kBlock * kPrefixPer;
}
// row-sharded plan: index over owner-major keys + unique-row compaction (uniq_rows = local row
// ids grouped by owner, send_counts[world], cid_u/cid_i/uoffs/nuniq in the workspace)
// flags kErrFold unless the last index build folded with `fold` (an index built in another call)
hipError_t launch_fold_check(const WsLayout& L, void* ws, int fold, hipStream_t st);
hipError_t launch_shard_plan(const ncf_shape_t& s, const WsLayout& L, void* ws, const int32_t* users,
                             const int32_t* items, int64_t n, int32_t* uniq_rows, int32_t* send_counts,
                             hipStream_t st, int fold = 0);
// owner index: m received local row ids keys[j] grouped by row (ascending j), S = L.shard_rows keys
hipError_t launch_owner_index(const WsLayout& L, void* ws, const int32_t* keys, int64_t m, hipStream_t st);
// The owner index of the deferred-decay shard (world > 0): its own regions (WsLayout o*), so the
// plan's index of the same workspace survives it; also the ascending list of the served rows.
// owner_view: the layout with the index regions pointed at the owner's, keys = S, max_batch
// sized for m entries (grid sizing of the catch-up and update launches over them)
WsLayout owner_view(const WsLayout& L, int64_t m);
hipError_t launch_owner_touched_index(const WsLayout& L, void* ws, const int32_t* keys, int64_t m, hipStream_t st);
// compact gradient: out[u] = sum over the plan's contributions of unique row u (ascending c)
hipError_t launch_uniq_grad(const ncf_shape_t& s, const WsLayout& L, void* ws, int64_t n, float* out,
                            hipStream_t st);
hipError_t launch_gather_rows(const ncf_shape_t& s, const float* table, int64_t table_rows, const int32_t* rows,
                              int64_t m, float* out, hipStream_t st);

// forward+backward, generic per-sample kernel: writes probs, gs rows, bce partials, dense slabs.
// returns number of slabs written in *nslab, bce partial count in *nbce
hipError_t launch_fb_generic(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                             const float* mlp, const int32_t* users, const int32_t* items,
                             const float* labels, int64_t n, float inv_batch, IdSpace ids, int* nslab, int* nbce,
                             hipStream_t st);
// forward only; with labels also writes per-block BCE partials (*nbce of them)
hipError_t launch_predict_generic(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                                  const float* mlp, const int32_t* users, const int32_t* items,
                                  const float* labels, int64_t n, float* probs, IdSpace ids, int* nbce,
                                  hipStream_t st);

// fused MFMA forward+backward (shapes with s.fast_path); same outputs as the generic kernel
// also computes the hr/dcg group metrics in-kernel when group divides 32 (*nmet = partial count, else 0)
// fold (fold_of(group, true) or 0): user-row folding, as the index was built with
hipError_t launch_fb_fused(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                           const float* mlp, const int32_t* users, const int32_t* items, const float* labels,
                           int64_t n, float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce,
                           int* nmet, hipStream_t st, int fold = 0);
bool fused_supported(const ncf_shape_t& s);
// sample-unit kernel (ncf_unit.hip): the fused shapes, 32-sample units split across a
// workgroup's waves by output feature; same outputs and folding as launch_fb_fused
bool unit_supported(const ncf_shape_t& s);
// wave-chain kernel (ncf_wave.hip): outputs as launch_fb_unit (fp32 operands only); one_wave: the
// form without separate weight-gradient waves (else chosen by shape and NCF_WAVE_SPLIT)
bool wave_supported(const ncf_shape_t& s);
hipError_t launch_fb_wave(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                          const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                          float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                          hipStream_t st, int fold, bool check_fold, bool one_wave = false,
                          const FillArgs* fill = nullptr);
// the split form runs for this shape (its weight-gradient waves can build the index: FillArgs)
bool wave_fill_supported(const ncf_shape_t& s);
// the in-kernel fill as a launch of its own (ncf_update.hip)
hipError_t launch_fill_ahead(const FillArgs& f, const int32_t* users, const int32_t* items, int64_t n, int fold,
                             hipStream_t st);
// fill (optional): the batch's index filled by extra workgroups of the unit launch, on the CUs its
// unit grid leaves idle (unit_fill_fits)
hipError_t launch_fb_unit(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                          const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                          float inv_batch, IdSpace ids, int group, int topk, int* nslab, int* nbce, int* nmet,
                          hipStream_t st, int fold, bool bf16, bool check_fold = false, const FillArgs* fill = nullptr);
bool unit_fill_fits(const ncf_shape_t& s, int64_t n, bool bf16, int64_t r1);
// fused MFMA forward only (shapes with s.fast_path): probs; with labels also one BCE partial per
// workgroup in ws part_bce (*nbce of them)
hipError_t launch_fwd_fused(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                            const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                            float* probs, IdSpace ids, int* nbce, hipStream_t st);
// layer-by-layer path (ncf_layered.hip): hand-written fp32 MFMA kernels (k_lay_l1f, k_lay_mid,
// k_lay_dw1, k_lay_l1b) for the shapes they hold (config D's widths); same outputs as
// launch_fb_generic (probs, gs, part_bce, slabs).  Other shapes run the generic kernel.
bool layered_supported(const ncf_shape_t& s);
bool layered_all_mfma(const ncf_shape_t& s);  // == layered_supported (no vendor-GEMM variant remains)
hipError_t launch_fb_layered(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, const float* mlp,
                             const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                             float inv_batch, IdSpace ids, int* nslab, int* nbce, hipStream_t st, int fold = 0);
// layer 1 of the layered path on hand-written MFMA (ncf_layer1.hip, config D's widths):
// forward = gather + X0 + (gmf != nullptr) GMF product + relu(W1^T x + b1); backward = dX = W1 G1 into the
// gradient rows gs with their GMF part (the replaced gather / GEMM / bias / scatter kernels' outputs)
bool layer1_supported(const ncf_shape_t& s);
// fold (2, 4, 8) with gpart ([n / fold][L1] floats of scratch): the user half once per group
// (k_lay_l1f_gu); else per sample
hipError_t launch_layer1_fwd(const ncf_shape_t& s, const float* emb, const float* mlp, const int32_t* users,
                             const int32_t* items, int64_t n, IdSpace ids, float* x0, float* gmf, float* h1,
                             hipStream_t st, int fold = 0, float* gpart = nullptr);
// dW1 = X0^T G1 per batch chunk of `chunk` samples into slab c (hidden_1 kernel at offset 0), c < nchunks
// fold (2, 4, 8) with the ids: the user half per group (k_lay_dw1<FOLD>, with k_lay_l1f_gu's X0)
hipError_t launch_layer1_dw(const ncf_shape_t& s, const float* x0, const float* g1, int64_t n, int64_t chunk,
                            int nchunks, float* slabs, hipStream_t st, int fold = 0, const int32_t* users = nullptr,
                            const int32_t* items = nullptr, IdSpace ids = IdSpace{});
hipError_t launch_layer1_bwd(const ncf_shape_t& s, const float* emb, const float* mlp, const int32_t* users,
                             const int32_t* items, int64_t n, IdSpace ids, const float* dzo, const float* g1,
                             float* gs, hipStream_t st, int fold = 0);  // fold: user-row folding (fold_of)
// layers 2.. of the layered path in one hand-written MFMA kernel (ncf_laymid.hip, config D's widths):
// from H1 and the rows' GMF vectors to probs, dz, G1 (row-major), the BCE partials and, per workgroup
// (grid of them), one slab of every dense parameter after layer 1
bool laymid_supported(const ncf_shape_t& s);
hipError_t launch_laymid(const ncf_shape_t& s, const float* mlp, const float* h1, const float* emb,
                         const float* labels, const int32_t* users, const int32_t* items, int64_t n, IdSpace ids,
                         float inv_batch, float* probs, float* dzo, float* g1, float* slabs, float* part_bce,
                         int grid, hipStream_t st);
// (dzo nullptr: the forward half alone — probs, and with labels the BCE partials; predict / evaluate)
hipError_t launch_predict_layered(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb,
                                  const float* mlp, const int32_t* users, const int32_t* items, const float* labels,
                                  int64_t n, float* probs, IdSpace ids, int* nbce, hipStream_t st);

// metrics / summaries
hipError_t launch_group_metrics(const float* probs, const float* labels, int64_t n_groups, int group, int k,
                                float* hit, float* dcg, float* part_hit, float* part_dcg, int* nparts,
                                hipStream_t st);
hipError_t launch_rank(const float* probs, int64_t n_groups, int group, int32_t* rank_idx, hipStream_t st);
hipError_t launch_summary(const WsLayout& L, void* ws, int nbce, int nmet, float n_groups, int nreg_emb,
                          int nreg_mlp, float* summary, hipStream_t st);

// updates
enum GradSource { kGradSparse = 0, kGradDense = 1 };
// sparse mode (dense_grad == nullptr): per-row sums of gs rows (nullptr: the workspace's
// per-contribution rows) through the workspace index
hipError_t launch_emb_update(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m, float* v,
                             const int32_t* step, const ncf_hyper_t& h, const float* dense_grad, int64_t rows,
                             hipStream_t st, const float* gs = nullptr, int64_t offs_row = 0);
// deferred exact decay (ncf_update.hip, L2 off): replay the missed zero-gradient Adam steps of
// the touched rows (all_rows: every row, ncf_lazy_flush) up to *step; then the step's update of
// the touched rows, which records row_step[r] = *step + 1.  Bitwise the dense sweep.
// sort_lists (touched rows only): extra blocks of the same launch run k_sort over the index the
// build left unsorted (launch_index_build(..., skip_sort = true)), for batch size n
// rows_current: the batch's rows were caught up ahead by the previous step's update launch
// (launch_emb_update_touched with next ids): only the sort blocks run, plus gate blocks that —
// only if the index fill flagged kErrStaleCount — fully replay the rows of users/items (the ids
// actually passed, n samples) the counted set missed
hipError_t launch_emb_catchup(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m, float* v,
                              int32_t* row_step, const int32_t* step, const ncf_hyper_t& h, bool all_rows,
                              hipStream_t st, bool sort_lists = false, int64_t n = 0, bool rows_current = false,
                              const int32_t* users = nullptr, const int32_t* items = nullptr, int gate_ahead = 0);
// (gate_ahead 1: enqueued before the step counter's bump — ncf_user_dp_step's next index — so the
// gate replays to *step + 1, the step the next forward pass reads)
hipError_t launch_row_step_fill(int32_t* row_step, int64_t R, const int32_t* step, hipStream_t st);
// next_users/next_items (optional, n_next samples): extra blocks of the same launch count the NEXT
// batch's contributions into the index counters (the next build skips its k_count) and replay the
// missed zero-gradient steps of its rows that this step does not touch (catch-up ahead)
// The dense layers' Adam step handed from launch_mlp_update to launch_emb_update_touched
// (same stream): it then runs in extra workgroups of the touched-row update launch.
struct MlpDeferred {
    float *p, *m, *v;          // p == nullptr: not deferred (launch_mlp_update launched it)
    const float* slabs;        // reduced slab partials (two_level: the raw slabs)
    int nslab;
    int two_level;             // 1: the launch also does the first-level slab reduction
                               // (k_slab_partial's work, same order: bitwise) — no launch of its own
};
// The step's group metrics handed from the forward/backward to the touched-row update launch
// (groups <= 8 that the kernel did not compute): nblocks partials into ws part_hit / part_dcg
struct MetricsDeferred {
    int nblocks;
    const float* probs;
    const float* labels;
    int64_t ng;
    int group, k;
};
hipError_t launch_emb_update_touched(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb, float* m,
                                     float* v, int32_t* row_step, int32_t* step, const ncf_hyper_t& h,
                                     hipStream_t st, const int32_t* next_users = nullptr,
                                     const int32_t* next_items = nullptr, int64_t n_next = 0,
                                     const MlpDeferred* mlp = nullptr, int next_fold = 0,
                                     const MetricsDeferred* met = nullptr, const float* grad_rows = nullptr,
                                     bool unsorted_lists = false, bool may_drop = true, bool sparse_index = false,
                                     bool* defer_replay = nullptr);
// *defer_replay (in: asked, out: done): the count blocks only claim the next batch's stale rows (ws
// claims / nclaim / claim_t); the stats launch behind this one must replay them (launch_stats'
// ReplayDeferred with 2 n_next contributions)
int64_t count_ahead_passes(int64_t contributions);
// (may_drop false: a fill overflow does not drop the step — data parallelism, where a rank that
// skipped its step would leave the replicas apart; the error is still reported)
// (grad_rows: the contribution rows the list indexes; default the workspace's per-sample rows gs)
// (unsorted_lists: the index came from the in-kernel fill (FillArgs): the launch orders each row's
// list itself and checks the touched rows' counters for a stale count)
// heavy-row threshold of the touched-row update over unsorted lists (FillArgs::hc)
inline int unsorted_heavy_c(const ncf_shape_t& s) { return s.row_width / 4 < 64 ? s.row_width / 4 : 64; }
// dense gradient of rows [row_begin, num_rows) into out (indexed from row_begin)
hipError_t launch_emb_grad_dense(const ncf_shape_t& s, const WsLayout& L, void* ws, float* out, hipStream_t st,
                                  int64_t row_begin = 0);
// Launch folding of the data-parallel gradient/update tails (every L2 factor zero and the slab
// count large enough for the two-level reduction): launch_part_tail = slab partials + batch
// summary, then dense embedding gradient of rows [row_begin, num_rows) + dense-layer gradient in
// one launch; launch_apply_fused = table-row update with a dense gradient + dense-layer update in
// one launch.  Bitwise the unfolded sequences.
bool part_tail_foldable(const ncf_shape_t& s, const ncf_hyper_t& h, int nslab);
// launch_part_tail over the in-kernel fill's unsorted lists (FillArgs): the dense gradient of rows
// [row_begin, num_rows) with each row's contributions in ascending order (bitwise launch_part_tail
// over the sorted index), heavy rows in the first blocks
hipError_t launch_part_tail_unsorted(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb_grad,
                                     int64_t row_begin, float* mlp_grad, int nslab, int nbce, int nmet, float n_groups,
                                     float* summary, hipStream_t st);
hipError_t launch_part_tail(const ncf_shape_t& s, const WsLayout& L, void* ws, float* emb_grad, int64_t row_begin,
                            float* mlp_grad, int nslab, int nbce, int nmet, float n_groups, float* summary,
                            hipStream_t st);
// parts: 1 the table rows only, 2 the dense layers only, 3 both (the split user-partitioned step runs
// the item rows before its all-gather and the dense layers beside it)
hipError_t launch_apply_fused(const ncf_shape_t& s, float* emb, float* m, float* v, const float* emb_grad,
                              int64_t rows, float* mlp, float* mlp_m, float* mlp_v, const float* mlp_grad,
                              const int32_t* step, const ncf_hyper_t& h, hipStream_t st, int parts = 3);
// mlp: reduce slabs (if nslab > 0) or read grad_in; optionally write grad_out; optionally update
// summary_nbce >= 0: the first-level slab reduction also writes the batch summary (what
// launch_summary(L, ws, summary_nbce, summary_nmet, n_groups, 0, 0, summary) does)
hipError_t launch_mlp_update(const ncf_shape_t& s, const WsLayout& L, void* ws, float* mlp, float* m, float* v,
                             const int32_t* step, const ncf_hyper_t& h, int nslab, const float* grad_in,
                             float* grad_out, bool do_update, int* nreg, hipStream_t st, bool want_reg = false,
                             int summary_nbce = -1, int summary_nmet = 0, float n_groups = 0.f,
                             float* summary = nullptr, MlpDeferred* defer = nullptr);
hipError_t launch_emb_reg(const ncf_shape_t& s, const WsLayout& L, void* ws, const float* emb, int64_t rows,
                          float lam, hipStream_t st);
// the next batch's per-block key scan (k_scan_local<true>) over counts taken ahead, alone
hipError_t launch_scan_ahead(const WsLayout& L, void* ws, int64_t keys, hipStream_t st);
// scan_ahead: the same launch also runs the next batch's per-block key scan (k_scan_local<true>
// over the counts the touched update took ahead)
// summary_first (nbce >= 0): block 0 first writes the batch summary (launch_summary's work with
// no L2 partials) and then folds it into stats
// the catch-up-ahead replay a defer_replay update left to the stats launch: the tables, the
// hyperparameters and the counted contributions (2 n_next)
struct ReplayDeferred {
    float *emb, *m, *v;
    int row_width;
    float lr, beta_1, beta_2, epsilon;
    int64_t contributions;
};
struct SummaryFirst {
    int nbce, nmet;
    float n_groups;
};
// drop (in-kernel fill steps: ws stale_step): nonzero — the step is dropped: no stats, no bump; the
// launch clears it
hipError_t launch_stats(const WsLayout& L, void* ws, const float* summary, int nreg_emb, int nreg_mlp,
                        float inv_batch, double* stats, int32_t* step, bool bump_step, hipStream_t st,
                        bool scan_ahead = false, int64_t scan_keys = 0, SummaryFirst sf = SummaryFirst{-1, 0, 0.f},
                        int32_t* drop = nullptr, bool sparse_scan = false, const ReplayDeferred* replay = nullptr);

// on-device negative sampling (ncf_sample.hip)
hipError_t launch_sample_batch(const int32_t* pos_users, const int32_t* pos_items, const int32_t* excl_ptr,
                               const int32_t* excl_items, int num_users, int num_items, const int32_t* order,
                               int64_t first, int n_pos, int negs, uint64_t seed, uint64_t stream,
                               int32_t* x_user, int32_t* x_item, float* labels, int32_t* err, hipStream_t st);

// all-item scoring + top-k (ncf_score.hip) ---------------------------------------------------
struct ScoreDims {
    int U, I, W, gmf_stride, du, di, G, L0, L1, L2, L3;
    int off_w2, off_w3, off_out;  // flat offsets of hidden_2 / hidden_3 / output kernels
    int ks2, ks3, nr3, ksg;       // MFMA k-steps of layer 2 / layer 3 / GMF, layer-3 output registers
    bool fast;                    // dimensions within the MFMA scorer's limits
};
struct ScoreLayout {
    // MFMA path (empty when the shape is not supported)
    size_t ic, ig, nega, init2, ug, a2, a3, init3, wh, bo, uok, part, gthr;
    // exact path: pair lists + probabilities of `chunk` users x all items, generic-forward ws
    size_t pu, pi, probs, pred_ws, pred_ws_bytes;
    int64_t chunk;
    int64_t max_users;
    size_t total;
};
ScoreDims score_dims(const ncf_shape_t& s);
ScoreLayout make_score_layout(const ncf_shape_t& s, int64_t max_users);
bool score_fast_supported(const ncf_shape_t& s);
hipError_t launch_score_prep(const ncf_shape_t& s, const ScoreLayout& L, void* ws, const float* emb,
                             const float* mlp, const int32_t* users, int64_t n, hipStream_t st);
hipError_t launch_score_main(const ncf_shape_t& s, const ScoreLayout& L, void* ws, int64_t n, int k,
                             int32_t* top_items, float* top_scores, hipStream_t st);
hipError_t launch_score_pairs(const int32_t* users, int64_t nq, int I, int32_t* pu, int32_t* pi, hipStream_t st);
hipError_t launch_topk_rows(const float* probs, int64_t rows, int I, int k, int32_t* top_items, float* top_scores,
                            hipStream_t st);

}  // namespace ncf
