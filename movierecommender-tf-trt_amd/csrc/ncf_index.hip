// Index build for the deterministic embedding scatter-add.
//
// The reference's embedding backward is the autodiff of ResourceGather
// (movierec/model.py:161-170): an IndexedSlices gradient that Keras' dense
// Adam densifies, duplicates summed.  Here every batch sample i
// contributes two gradient rows (c = 2i: user row, c = 2i+1: item row) to the
// combined table.  This TU groups the contributions by table row so that the
// optimizer sweep can sum each row's contributions in ascending c order —
// deterministic, no float atomics:
//
//   k_count       cnt[row]++                     (int atomics; order-free)
//   k_scan_local  per-2048-row exclusive scan + block totals
//   k_fill        offs[row] = local + prefix(block totals);
//                 list[offs[row] + --cnt[row]] = c        (cnt back to 0)
//   k_sort        sort each row's list: <=16 entries in registers (one
//                 thread), 17..64 by one wave (bitonic network across lanes),
//                 longer rows by the whole workgroup through an LDS bitmap
//                 over c (popcount scan, ascending write-back).
//
// All HBM traffic here is O(B + R) int32 (R = table rows); see DESIGN.md.

#include <climits>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

// Where contribution c's key comes from.
enum KeyMode {
    kKeyPair = 0,      // c = 2i + side: user row users[i] / item row U + items[i]
    kKeyPairPerm = 1,  // same rows, keyed owner-major for a row-sharded plan
    kKeyList = 2,      // c indexes keys[] directly (owner index over received row ids)
};

struct KeySrc {
    const int32_t* users;
    const int32_t* items;
    const int32_t* keys;
    int32_t U, I;
    int32_t world;
    int32_t S;     // shard rows (kKeyPairPerm) / key count (kKeyList)
    int32_t fold;  // > 1: user rows folded per group of this size (fold_of, ncf_internal.h)
};

// Key of contribution c; *ok = the id is inside its table.  *own = false: a user contribution
// folded into its group head's (it has a key — the plan's compact ids need it — but no slot).
template <int MODE>
__device__ inline int contrib_key(int64_t c, const KeySrc& k, bool* ok, bool* own) {
    *own = true;
    if constexpr (MODE == kKeyList) {
        const int v = k.keys[c];
        *ok = (unsigned)v < (unsigned)k.S;
        return v;
    } else {
        const int64_t i = c >> 1;
        int g;
        if (c & 1) {
            const int v = k.items[i];
            *ok = (unsigned)v < (unsigned)k.I;
            g = k.U + v;
        } else {
            const int u = k.users[i];
            *ok = (unsigned)u < (unsigned)k.U;
            *own = !folded_user(k.users, i, k.fold);
            g = u;
        }
        if constexpr (MODE == kKeyPairPerm) {
            const int q = g / k.world;
            g = (g - q * k.world) * k.S + q;
        }
        return g;
    }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_count(KeySrc ks, int64_t m, int32_t* __restrict__ cnt, int32_t* heavy_n,
                                                  int32_t* err) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *heavy_n = 0;
    const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t cb = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); cb < m; cb += gstride) {
        const int64_t c = cb + (threadIdx.x & 63);
        bool ok = false, own = true;
        int key = 0;
        if (c < m) {
            key = contrib_key<MODE>(c, ks, &ok, &own);
            if (!ok) atomicOr(err, kErrIdRange);
        }
        wave_run_count(cnt, key, ok && own);
    }
}

// Per-2048-key exclusive scan of cnt (and, for a plan, of the occupied-key flags cnt > 0): the
// body (scan_local_body, ncf_internal.h) is shared with the stats launch that scans ahead.
template <bool UNIQ>
__global__ __launch_bounds__(kBlock) void k_scan_local(const int32_t* __restrict__ cnt, int64_t r1,
                                                       int32_t* __restrict__ offs, int32_t* __restrict__ tot,
                                                       int32_t* __restrict__ uloc, int32_t* __restrict__ utot) {
    scan_local_body<UNIQ>(cnt, r1, offs, tot, uloc, utot, (int)blockIdx.x);
}

// Plan outputs of k_fill (UNIQ only).
struct PlanOut {
    const int32_t* uloc;
    const int32_t* utot;
    int32_t* uniq_rows;    // [nuniq] local row id at the owner, grouped by owner
    int32_t* send_counts;  // [world]
    int32_t* cid_u;        // [n]
    int32_t* cid_i;        // [n]
    int32_t* uoffs;        // [nuniq + 1]
    int32_t* nuniq;
    int2* uniq_oc;         // LIST: [nuniq] (list offset, contribution count) of each touched row
};

// Finalise the key offsets (offs_g = local scan + prefix of block totals) and scatter every
// contribution into its key's list slot; the per-key counter runs back down to zero.  A plan
// (UNIQ) also numbers the occupied keys (compact ids) and writes the per-owner counts.
// LIST (single table): also the compact list of the occupied keys (touched rows, ascending) and
// its length, for the deferred-decay kernels.
//
// Latency: a thread's first row and first contribution are handled before the block prefixes
// exist wherever they do not need them (single-table keys): the ids, the row's local offsets,
// the block totals and — once the ids are in — the contribution's counter atomic and its key's
// local offset all go out together, so the launch waits on two memory round trips instead of
// five.  Later grid-stride passes (more keys or contributions than threads) take the plain path.
template <int MODE, bool UNIQ, bool LIST>
__global__ __launch_bounds__(kBlock) void k_fill(KeySrc ks, int64_t m, int32_t* __restrict__ cnt,
                                                 const int32_t* __restrict__ local, const int32_t* __restrict__ tot,
                                                 int nscan, int64_t r1, int32_t* __restrict__ offs_g,
                                                 int32_t* __restrict__ list, PlanOut po, int32_t* __restrict__ err,
                                                 int32_t* __restrict__ ifold) {
    extern __shared__ __attribute__((aligned(16))) int pre[];  // [nscan] (+ [nscan] unique prefix)
    __shared__ int sw[4];
    constexpr bool U2 = UNIQ || LIST;
    constexpr bool EARLY = MODE == kKeyPair && !UNIQ;
    int* upre = pre + nscan;
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
    const int64_t K = r1 - 1;
    const int lane = threadIdx.x & 63;
    const uint64_t par = (lane & 1) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);

    // ---- early loads (EARLY): first contribution's key, first row's local offsets, the totals
    int e_key = 0, e_top = 0, e_head = 0, e_loc = 0;
    bool e_ok = false;
    int r_loc = 0, r_loc1 = 0, r_uloc = 0;
    int t_first = 0, u_first = 0;
    if constexpr (EARLY) {
        const int64_t c = gt;  // cb = gt - lane, c = cb + lane
        bool own = true;
        if (c < m) {
            e_key = contrib_key<MODE>(c, ks, &e_ok, &own);
            if (!e_ok) atomicOr(err, kErrIdRange);
        }
        if (gt < r1) {
            r_loc = local[gt];
            if constexpr (U2) {
                if (gt < K) r_loc1 = local[gt + 1];
                r_uloc = po.uloc[gt];
            }
        }
        if ((int)threadIdx.x < nscan) {
            t_first = tot[threadIdx.x];
            if constexpr (U2) u_first = po.utot[threadIdx.x];
        }
        e_ok = e_ok && own;
        const int kk = e_ok ? e_key : -2 - lane;  // inactive lanes: unique keys
        const int prev = __shfl_up(kk, 2, 64);
        const uint64_t heads = ~__ballot(lane >= 2 && prev == kk) & par;
        e_head = 63 - __clzll(heads & upto);
        const uint64_t later = heads & ~upto;
        const int next = later ? __ffsll((unsigned long long)later) - 1 : 64 + (lane & 1);
        if (e_ok && lane == e_head) e_top = atomicSub(&cnt[e_key], (next - e_head) >> 1);
        if (e_ok) e_loc = local[e_key];
    }

    // ---- exclusive prefixes of the scan-block totals into LDS (pre, upre)
    {
        int carry = 0, ucarry = 0;
        for (int base = 0; base < nscan; base += kBlock) {
            const bool in = base + (int)threadIdx.x < nscan;
            int x, y = 0;
            if (EARLY && base == 0) {
                x = t_first;
                y = u_first;
            } else {
                x = in ? tot[base + threadIdx.x] : 0;
                if constexpr (U2) y = in ? po.utot[base + threadIdx.x] : 0;
            }
            int total;
            const int ex = block_exscan_256(x, sw, &total);
            if (in) pre[base + threadIdx.x] = carry + ex;
            carry += total;
            if constexpr (U2) {
                int utotal;
                const int uex = block_exscan_256(y, sw, &utotal);
                if (in) upre[base + threadIdx.x] = ucarry + uex;
                ucarry += utotal;
            }
        }
        __syncthreads();
    }
    if (gt == 0) *ifold = ks.fold;
    for (int64_t r = gt; r < r1; r += gstride) {
        const bool first = EARLY && r == gt;
        const int o = (first ? r_loc : local[r]) + pre[r / kScanBlock];
        offs_g[r] = o;
        if constexpr (U2) {
            if (r < K) {
                const int o1 = (first ? r_loc1 : local[r + 1]) + pre[(r + 1) / kScanBlock];
                if (o1 > o) {
                    const int u = (first ? r_uloc : po.uloc[r]) + upre[r / kScanBlock];
                    if constexpr (UNIQ) {
                        po.uniq_rows[u] = (int)(r % ks.S);
                        po.uoffs[u] = o;
                    } else {
                        po.uniq_rows[u] = (int)r;
                        po.uniq_oc[u] = make_int2(o, o1 - o);
                    }
                }
            }
        }
    }
    if constexpr (LIST) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *po.nuniq = po.uloc[K] + upre[K / kScanBlock];
    }
    if constexpr (UNIQ) {
        if (blockIdx.x == 0) {
            auto uprefix = [&](int64_t x) { return po.uloc[x] + upre[x / kScanBlock]; };
            for (int d = threadIdx.x; d < ks.world; d += kBlock)
                po.send_counts[d] = uprefix((int64_t)(d + 1) * ks.S) - uprefix((int64_t)d * ks.S);
            if (threadIdx.x == 0) {
                const int nu = uprefix(K);
                *po.nuniq = nu;
                po.uoffs[nu] = local[K] + pre[K / kScanBlock];  // listed contributions (folded ones are not)
            }
        }
    }
    // Contributions a wave at a time (lane l takes c = base + l).  Equal keys two lanes apart
    // (a user group's samples: c = 2i, 2i+2, ...) form runs; the run's head takes all of its
    // slots with one atomic and hands them out, so a group's user contributions do not queue on
    // one counter.  Slot order within a key does not matter: the lists are sorted afterwards.
    // A slot below the key's range means the key was counted fewer times than it occurs
    // (counted-ahead ids changed since): flagged, never written outside the key's slots.
    if constexpr (EARLY) {
        if (gt - lane < m) {
            const int top = __shfl(e_top, e_head, 64);
            const int slot = top - 1 - ((lane - e_head) >> 1);
            if (e_ok && slot >= 0) list[e_loc + pre[e_key / kScanBlock] + slot] = (int)gt;
            else if (e_ok) atomicOr(err, kErrStaleCount);
        }
    }
    for (int64_t cb = gt - lane + (EARLY ? gstride : 0); cb < m; cb += gstride) {
        const int64_t c = cb + lane;
        bool ok = false, own = true;
        int key = 0;
        if (c < m) {
            key = contrib_key<MODE>(c, ks, &ok, &own);
            if (!ok) atomicOr(err, kErrIdRange);
            if constexpr (UNIQ) {
                const int u = ok ? po.uloc[key] + upre[key / kScanBlock] : -1;
                ((c & 1) ? po.cid_i : po.cid_u)[c >> 1] = u;
            }
            ok = ok && own;
        }
        const int kk = ok ? key : -2 - lane;                 // inactive lanes: unique keys
        const int prev = __shfl_up(kk, 2, 64);
        const uint64_t heads = ~__ballot(lane >= 2 && prev == kk) & par;
        const int head = 63 - __clzll(heads & upto);
        const uint64_t later = heads & ~upto;
        const int next = later ? __ffsll((unsigned long long)later) - 1 : 64 + (lane & 1);
        int top = 0;
        if (ok && lane == head) top = atomicSub(&cnt[key], (next - head) >> 1);
        top = __shfl(top, head, 64);
        const int slot = top - 1 - ((lane - head) >> 1);
        if (ok && slot >= 0) list[local[key] + pre[key / kScanBlock] + slot] = (int)c;
        else if (ok) atomicOr(err, kErrStaleCount);
    }
}

// Large key spaces (config D: 11 M rows, 5,371 scan blocks).  k_fill derives the exclusive prefix
// of the scan-block totals in every workgroup (O(nscan) each), which caps its grid at 1,024
// workgroups and leaves each thread a grid-stride chain of ~40 dependent row passes.  Here one
// workgroup writes the prefixes to the workspace once (k_prefix) and the fill runs one workgroup
// per scan block (8 rows per thread) — same outputs as k_fill.
// One workgroup per array (tot, and utot when given): the totals go through LDS — loaded (all in flight at once) and stored back
// coalesced (a thread's contiguous chunk read straight from memory put 64 different cache lines
// behind every wave instruction) — thread t scans its chunk of ceil(nscan / 256)
// scan blocks (at most kPrefixPer), one block scan of the chunk sums, then the chunk's prefixes.
__global__ __launch_bounds__(kBlock) void k_prefix(const int32_t* __restrict__ tot, const int32_t* __restrict__ utot,
                                                   int nscan, int32_t* __restrict__ pre, int32_t* __restrict__ upre) {
    __shared__ int sw[4];
    __shared__ int buf[kBlock * kPrefixPer];   // 32 KB: one of the two arrays at a time
    const int per = (nscan + kBlock - 1) / kBlock;
    const int i0 = (int)threadIdx.x * per;
    {   // workgroup 0: tot -> pre; workgroup 1 (launched when utot is given): utot -> upre
        const int pass = (int)blockIdx.x;
        const int32_t* src = pass ? utot : tot;
        int32_t* dst = pass ? upre : pre;
        {   // every load in flight before the first LDS store (a load-store loop waits a round trip each)
            int x[kPrefixPer];
#pragma unroll
            for (int j = 0; j < kPrefixPer; ++j) {
                const int i = (int)threadIdx.x + kBlock * j;
                x[j] = i < nscan ? src[i] : 0;
            }
#pragma unroll
            for (int j = 0; j < kPrefixPer; ++j) {
                const int i = (int)threadIdx.x + kBlock * j;
                if (i < nscan) buf[i] = x[j];
            }
        }
        __syncthreads();
        int ts = 0;
        for (int j = 0; j < per; ++j) ts += i0 + j < nscan ? buf[i0 + j] : 0;
        int total;
        int run = block_exscan_256(ts, sw, &total);
        __syncthreads();   // every chunk read before the prefixes overwrite the buffer
        for (int j = 0; j < per; ++j) {
            if (i0 + j < nscan) {
                const int t = buf[i0 + j];
                buf[i0 + j] = run;
                run += t;
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nscan; i += kBlock) dst[i] = buf[i];
    }
}

template <int MODE, bool UNIQ, bool LIST>
__global__ __launch_bounds__(kBlock) void k_fill_big(KeySrc ks, int64_t m, int32_t* __restrict__ cnt,
                                                     const int32_t* __restrict__ local, const int32_t* __restrict__ pre,
                                                     const int32_t* __restrict__ upre, int nscan, int64_t r1,
                                                     int32_t* __restrict__ offs_g, int32_t* __restrict__ list, PlanOut po,
                                                     int32_t* __restrict__ err, int32_t* __restrict__ ifold) {
    constexpr bool U2 = UNIQ || LIST;
    const int64_t K = r1 - 1;
    const int lane = threadIdx.x & 63;
    const uint64_t par = (lane & 1) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int b = (int)blockIdx.x;
    if (b == 0 && threadIdx.x == 0) *ifold = ks.fold;
    if (b < nscan) {
        // this scan block's keys, 8 per thread: their offsets (and, for a plan or the touched
        // list, the compact numbering of the occupied keys)
        const int pb = pre[b];
        const int ub = U2 ? upre[b] : 0;
        const int pn = b + 1 < nscan ? pre[b + 1] : 0;  // the next scan block's prefix (key r + 1)
        const int64_t r0 = (int64_t)b * kScanBlock + threadIdx.x * 8;
        int loc[9], ul[8];
        const bool full = r0 + 9 <= r1;  // int4 pairs (256-byte aligned regions, r0 a multiple of 8)
        if (full) {
            const int4 a = *reinterpret_cast<const int4*>(local + r0), c = *reinterpret_cast<const int4*>(local + r0 + 4);
            loc[0] = a.x, loc[1] = a.y, loc[2] = a.z, loc[3] = a.w, loc[4] = c.x, loc[5] = c.y, loc[6] = c.z, loc[7] = c.w;
            loc[8] = U2 ? local[r0 + 8] : 0;
            if constexpr (U2) {
                const int4 x = *reinterpret_cast<const int4*>(po.uloc + r0), y = *reinterpret_cast<const int4*>(po.uloc + r0 + 4);
                ul[0] = x.x, ul[1] = x.y, ul[2] = x.z, ul[3] = x.w, ul[4] = y.x, ul[5] = y.y, ul[6] = y.z, ul[7] = y.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 9; ++j) loc[j] = r0 + j < r1 && (j < 8 || U2) ? local[r0 + j] : 0;
            if constexpr (U2) {
#pragma unroll
                for (int j = 0; j < 8; ++j) ul[j] = r0 + j < r1 ? po.uloc[r0 + j] : 0;
            }
        }
        if (full) {
            *reinterpret_cast<int4*>(offs_g + r0) = make_int4(loc[0] + pb, loc[1] + pb, loc[2] + pb, loc[3] + pb);
            *reinterpret_cast<int4*>(offs_g + r0 + 4) = make_int4(loc[4] + pb, loc[5] + pb, loc[6] + pb, loc[7] + pb);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t r = r0 + j;
            if (r >= r1) break;
            const int o = loc[j] + pb;
            if (!full) offs_g[r] = o;
            if constexpr (U2) {
                if (r < K) {
                    // key r + 1 opens the next scan block for the last thread's last key
                    const int o1 = loc[j + 1] + ((r + 1) % kScanBlock == 0 ? pn : pb);
                    if (o1 > o) {
                        const int u = ul[j] + ub;
                        if constexpr (UNIQ) {
                            po.uniq_rows[u] = (int)(r % ks.S);
                            po.uoffs[u] = o;
                        } else {
                            po.uniq_rows[u] = (int)r;
                            po.uniq_oc[u] = make_int2(o, o1 - o);
                        }
                    }
                }
            }
        }
        if constexpr (LIST) {
            if (K / kScanBlock == b && threadIdx.x == 0) *po.nuniq = po.uloc[K] + ub;
        }
    }
    if constexpr (UNIQ) {
        if (b == 0) {
            auto uprefix = [&](int64_t x) { return po.uloc[x] + upre[x / kScanBlock]; };
            for (int d = threadIdx.x; d < ks.world; d += kBlock)
                po.send_counts[d] = uprefix((int64_t)(d + 1) * ks.S) - uprefix((int64_t)d * ks.S);
            if (threadIdx.x == 0) {
                const int nu = uprefix(K);
                *po.nuniq = nu;
                po.uoffs[nu] = local[K] + pre[K / kScanBlock];
            }
        }
    }
    // contributions a wave at a time (k_fill's scheme: a run's head takes its slots with one atomic)
    const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t cb = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); cb < m; cb += gstride) {
        const int64_t c = cb + lane;
        bool ok = false, own = true;
        int key = 0;
        if (c < m) {
            key = contrib_key<MODE>(c, ks, &ok, &own);
            if (!ok) atomicOr(err, kErrIdRange);
            if constexpr (UNIQ) {
                const int u = ok ? po.uloc[key] + upre[key / kScanBlock] : -1;
                ((c & 1) ? po.cid_i : po.cid_u)[c >> 1] = u;
            }
            ok = ok && own;
        }
        const int kk = ok ? key : -2 - lane;
        const int prev = __shfl_up(kk, 2, 64);
        const uint64_t heads = ~__ballot(lane >= 2 && prev == kk) & par;
        const int head = 63 - __clzll(heads & upto);
        const uint64_t later = heads & ~upto;
        const int next = later ? __ffsll((unsigned long long)later) - 1 : 64 + (lane & 1);
        int top = 0;
        if (ok && lane == head) {
            top = atomicSub(&cnt[key], (next - head) >> 1);
            // what the run takes below zero (a key counted fewer times than it occurs) goes back:
            // a counter ends at max(0, counted - placed), so a residue can only sit at a counted
            // key (the list sort checks those only, sort_rows_body<..., LISTED>)
            const int over = ((next - head) >> 1) - max(top, 0);
            if (over > 0) atomicAdd(&cnt[key], over);
        }
        top = __shfl(top, head, 64);
        const int slot = top - 1 - ((lane - head) >> 1);
        if (ok && slot >= 0) list[local[key] + pre[key / kScanBlock] + slot] = (int)c;
        else if (ok) atomicOr(err, kErrStaleCount);
    }
}

// The sparse counted index (sparse_index_ok: large key spaces, a batch counted and scanned ahead by
// the previous step with scan_local_body<true, true>): the touched rows come from the scan's
// per-block lists (TouchedOut: block b's occupied keys in key order at tl[b 2048 ..], their
// (offset inside the block, count) in tocl) — block b writes its rows at upre[b] .. of the touched
// list with offsets pre[b] + the block's, and tags each with this index's seen tag (*itag + 1: the
// touched-row update's count blocks test "in this step's batch" with it); then the contributions,
// k_fill_big's scheme.  Same list, touched rows (key order) and cursors as k_fill_big<.., LIST>;
// no pass over the keys of the table (k_fill_big writes every key's offset: 44 MB at config D).
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_fill_touched(KeySrc ks, int64_t m, int32_t* __restrict__ cnt,
                                                         const int32_t* __restrict__ local,
                                                         const int32_t* __restrict__ pre, const int32_t* __restrict__ upre,
                                                         const int32_t* __restrict__ utot, int nscan,
                                                         const int32_t* __restrict__ tl, const int2* __restrict__ tocl,
                                                         int32_t* __restrict__ touched, int2* __restrict__ toc,
                                                         int32_t* __restrict__ nuniq, int32_t* __restrict__ seen,
                                                         const int32_t* __restrict__ itag, int32_t* __restrict__ list,
                                                         int32_t* __restrict__ err, int32_t* __restrict__ ifold) {
    const int lane = threadIdx.x & 63;
    const int b = (int)blockIdx.x;
    if (b == 0 && threadIdx.x == 0) *ifold = ks.fold;
    if (b < nscan) {
        const int nb = utot[b];
        const int pb = pre[b], ub = upre[b];
        const int tag = *itag + 1;
        for (int i = threadIdx.x; i < nb; i += kBlock) {
            const int64_t e = (int64_t)b * kScanBlock + i;
            const int key = tl[e];
            const int2 oc = tocl[e];
            touched[ub + i] = key;
            toc[ub + i] = make_int2(pb + oc.x, oc.y);
            seen[key] = tag;
        }
        if (b == nscan - 1 && threadIdx.x == 0) *nuniq = ub + nb;
    }
    const uint64_t par = (lane & 1) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t cb = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); cb < m; cb += gstride) {
        const int64_t c = cb + lane;
        bool ok = false, own = true;
        int key = 0;
        if (c < m) {
            key = contrib_key<MODE>(c, ks, &ok, &own);
            if (!ok) atomicOr(err, kErrIdRange);
            ok = ok && own;
        }
        const int kk = ok ? key : -2 - lane;
        const int prev = __shfl_up(kk, 2, 64);
        const uint64_t heads = ~__ballot(lane >= 2 && prev == kk) & par;
        const int head = 63 - __clzll(heads & upto);
        const uint64_t later = heads & ~upto;
        const int next = later ? __ffsll((unsigned long long)later) - 1 : 64 + (lane & 1);
        int top = 0;
        if (ok && lane == head) {
            top = atomicSub(&cnt[key], (next - head) >> 1);
            const int over = ((next - head) >> 1) - max(top, 0);   // k_fill_big's give-back
            if (over > 0) atomicAdd(&cnt[key], over);
        }
        top = __shfl(top, head, 64);
        const int slot = top - 1 - ((lane - head) >> 1);
        if (ok && slot >= 0) list[local[key] + pre[key / kScanBlock] + slot] = (int)c;
        else if (ok) atomicOr(err, kErrStaleCount);
    }
}

// Sort each key's contribution list ascending.  Keys of <= kSmallSeg entries: one thread,
// odd-even network in registers.  Longer keys: queued in LDS and sorted by the whole
// workgroup with a bitmap over the contribution ids (set bits, popcount scan, write back).
template <int RPT>
__global__ __launch_bounds__(kBlock) void k_sort(const int32_t* __restrict__ offs, int64_t R,
                                                 int32_t* __restrict__ list, int nwords, int32_t* __restrict__ cnt,
                                                 int32_t* __restrict__ err) {
    sort_rows_body<RPT>(offs, R, list, nwords, (int)blockIdx.x, cnt, err);
}

static int grid_for(int64_t work, int cap) {
    int64_t g = (work + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

static hipError_t set_sort_lds(int nwords) {
    static bool lds_cfg = false;
    if (!lds_cfg && (size_t)nwords * 4 > 65536) {
        for (const void* f : {(const void*)k_sort<1>, (const void*)k_sort<8>}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)((kMaxBatch * 2 / 32) * 4));
            if (e != hipSuccess) return e;
        }
        lds_cfg = true;
    }
    return hipSuccess;
}

// count -> scan -> fill -> sort over K keys for m contributions.
template <int MODE, bool UNIQ, bool LIST = false>
static hipError_t build(const WsLayout& L, void* ws, const KeySrc& ks, int64_t m, int64_t K, PlanOut po,
                        int nwords, hipStream_t st, bool counted = false, bool skip_sort = false,
                        bool sparse = false) {
    // skip_sort: the caller's next launch (the touched-row catch-up) sorts the lists in extra blocks
    // counted: the previous step counted AND scanned these ids (touched update + stats launch)
    const int64_t r1 = K + 1;
    int32_t* cnt = at<int32_t>(ws, L.cnt);
    int32_t* local = at<int32_t>(ws, L.offs_local);
    int32_t* offs = at<int32_t>(ws, L.offs);
    int32_t* tot = at<int32_t>(ws, L.tot);
    int32_t* list = at<int32_t>(ws, L.list);
    const int nscan = (int)((r1 + kScanBlock - 1) / kScanBlock);
    if (m > 0 && !counted)  // counted: the previous step's touched update already counted these ids
        launch(k_count<MODE>, grid_for(m, 1024), kBlock, 0, st, ks, m, cnt, at<int32_t>(ws, L.heavy_n),
                                                            at<int32_t>(ws, L.err));
    constexpr bool U2 = UNIQ || LIST;
    if (!counted)
        launch(k_scan_local<U2>, nscan, kBlock, 0, st, cnt, r1, local, tot, U2 ? at<int32_t>(ws, L.uloc) : nullptr,
                                                   U2 ? at<int32_t>(ws, L.utot) : nullptr);
    if (sparse) {
        if (UNIQ || !LIST || !counted || !sparse_index_ok(L) || r1 != L.keys + 1) return hipErrorInvalidValue;
        int32_t* pre = at<int32_t>(ws, L.pre);
        launch(k_prefix, 2, kBlock, 0, st, (const int32_t*)tot, (const int32_t*)at<int32_t>(ws, L.utot), nscan, pre,
               pre + nscan);
        const int64_t gc = (m + kBlock - 1) / kBlock;
        launch(k_fill_touched<MODE>, (unsigned)(gc > nscan ? gc : nscan), kBlock, 0, st, ks, m, cnt,
               (const int32_t*)local, (const int32_t*)pre, (const int32_t*)(pre + nscan),
               (const int32_t*)at<int32_t>(ws, L.utot), nscan, (const int32_t*)at<int32_t>(ws, L.tl),
               (const int2*)at<int2>(ws, L.tocl), po.uniq_rows, po.uniq_oc, po.nuniq, at<int32_t>(ws, L.seen),
               (const int32_t*)at<int32_t>(ws, L.itag), list, at<int32_t>(ws, L.err), at<int32_t>(ws, L.ifold));
    } else if (nscan > kFillBigScan && nscan <= kBlock * kPrefixPer) {
        int32_t* pre = at<int32_t>(ws, L.pre);
        launch(k_prefix, U2 ? 2 : 1, kBlock, 0, st, (const int32_t*)tot, U2 ? (const int32_t*)at<int32_t>(ws, L.utot) : nullptr,
               nscan, pre, pre + nscan);
        const int64_t gc = (m + kBlock - 1) / kBlock;
        launch(k_fill_big<MODE, UNIQ, LIST>, (unsigned)(gc > nscan ? gc : nscan), kBlock, 0, st, ks, m, cnt,
               (const int32_t*)local, (const int32_t*)pre, (const int32_t*)(pre + nscan), nscan, r1, offs, list, po,
               at<int32_t>(ws, L.err), at<int32_t>(ws, L.ifold));
    } else {
        const size_t pre_bytes = (size_t)nscan * 4 * (U2 ? 2 : 1);
        launch(k_fill<MODE, UNIQ, LIST>, grid_for(m > r1 ? m : r1, 1024), kBlock, pre_bytes, st, ks, m, cnt, local,
               tot, nscan, r1, offs, list, po, at<int32_t>(ws, L.err), at<int32_t>(ws, L.ifold));
    }
    if (skip_sort) return hipGetLastError();
    if (hipError_t e = set_sort_lds(nwords)) return e;
    const int rpt = sort_rpt(K);
    const unsigned gs = (unsigned)((K + (int64_t)kBlock * rpt - 1) / ((int64_t)kBlock * rpt));
    if (rpt == 8)
        launch(k_sort<8>, gs, kBlock, (size_t)nwords * 4, st, offs, K, list, nwords, cnt, at<int32_t>(ws, L.err));
    else
        launch(k_sort<1>, gs, kBlock, (size_t)nwords * 4, st, offs, K, list, nwords, cnt, at<int32_t>(ws, L.err));
    return hipGetLastError();
}

hipError_t launch_index_build(const ncf_shape_t& s, const WsLayout& L, void* ws, const int32_t* users,
                              const int32_t* items, int64_t n, hipStream_t st, bool touched_list, bool counted,
                              bool skip_sort, int fold, bool sparse) {
    KeySrc ks{users, items, nullptr, s.num_users, s.num_items, 1, 0, fold};
    if (touched_list) {
        PlanOut po{};
        po.uloc = at<int32_t>(ws, L.uloc);
        po.utot = at<int32_t>(ws, L.utot);
        po.uniq_rows = at<int32_t>(ws, L.touched);
        po.nuniq = at<int32_t>(ws, L.nuniq);
        po.uniq_oc = at<int2>(ws, L.touched_oc);
        return build<kKeyPair, false, true>(L, ws, ks, 2 * n, s.num_rows, po, (int)((2 * n + 31) / 32), st,
                                            counted, skip_sort, sparse);
    }
    if (sparse) return hipErrorInvalidValue;
    return build<kKeyPair, false>(L, ws, ks, 2 * n, s.num_rows, PlanOut{}, (int)((2 * n + 31) / 32), st, counted);
}

hipError_t launch_shard_plan(const ncf_shape_t& s, const WsLayout& L, void* ws, const int32_t* users,
                             const int32_t* items, int64_t n, int32_t* uniq_rows, int32_t* send_counts,
                             hipStream_t st, int fold) {
    KeySrc ks{users, items, nullptr, s.num_users, s.num_items, L.world, (int32_t)L.shard_rows, fold};
    PlanOut po{at<int32_t>(ws, L.uloc), at<int32_t>(ws, L.utot), uniq_rows, send_counts, at<int32_t>(ws, L.cid_u),
               at<int32_t>(ws, L.cid_i), at<int32_t>(ws, L.uoffs), at<int32_t>(ws, L.nuniq)};
    return build<kKeyPairPerm, true>(L, ws, ks, 2 * n, L.keys, po, (int)((2 * n + 31) / 32), st);
}

__global__ void k_fold_check(const int32_t* __restrict__ ifold, int fold, int32_t* __restrict__ err) {
    if (threadIdx.x == 0 && *ifold != fold) atomicOr(err, kErrFold);
}

hipError_t launch_fold_check(const WsLayout& L, void* ws, int fold, hipStream_t st) {
    launch(k_fold_check, 1, 64, 0, st, at<const int32_t>(ws, L.ifold), fold, at<int32_t>(ws, L.err));
    return hipGetLastError();
}

hipError_t launch_owner_index(const WsLayout& L, void* ws, const int32_t* keys, int64_t m, hipStream_t st) {
    KeySrc ks{nullptr, nullptr, keys, 0, 0, L.world, (int32_t)L.shard_rows, 0};
    // every source sends a row at most once: a key has <= world entries, so keys longer than
    // kSmallSeg (bitmap sort over m ids) exist only for world > kSmallSeg
    const int nwords = L.world > kSmallSeg ? (int)((m + 31) / 32) : 0;
    return build<kKeyList, false>(L, ws, ks, m, L.shard_rows, PlanOut{}, nwords, st);
}

hipError_t launch_owner_touched_index(const WsLayout& L, void* ws, const int32_t* keys, int64_t m, hipStream_t st) {
    const WsLayout O = owner_view(L, m);
    KeySrc ks{nullptr, nullptr, keys, 0, 0, L.world, (int32_t)L.shard_rows, 0};
    PlanOut po{};
    po.uloc = at<int32_t>(ws, O.uloc);
    po.utot = at<int32_t>(ws, O.utot);
    po.uniq_rows = at<int32_t>(ws, O.touched);
    po.nuniq = at<int32_t>(ws, O.nuniq);
    po.uniq_oc = at<int2>(ws, O.touched_oc);
    // a row gets at most one entry per source rank: <= world <= kSmallSeg entries, no bitmap sort
    return build<kKeyList, false, true>(O, ws, ks, m, L.shard_rows, po, 0, st);
}

}  // namespace ncf
