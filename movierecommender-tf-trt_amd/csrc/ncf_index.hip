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
//                 thread), longer rows by the whole workgroup through an
//                 LDS bitmap over c (popcount scan, ascending write-back).
//
// All HBM traffic here is O(B + R) int32 (R = table rows); see DESIGN.md.

#include <climits>

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

__device__ inline int contrib_key(int64_t c, const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                                  int32_t U, int32_t I, bool* ok) {
    const int64_t i = c >> 1;
    if (c & 1) {
        const int v = items[i];
        *ok = (unsigned)v < (unsigned)I;
        return U + v;
    }
    const int u = users[i];
    *ok = (unsigned)u < (unsigned)U;
    return u;
}

__global__ __launch_bounds__(kBlock) void k_count(const int32_t* __restrict__ users,
                                                  const int32_t* __restrict__ items, int64_t n, int32_t U,
                                                  int32_t I, int32_t* __restrict__ cnt, int32_t* heavy_n,
                                                  int32_t* err) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *heavy_n = 0;
    const int64_t m = 2 * n;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += (int64_t)gridDim.x * blockDim.x) {
        bool ok;
        const int key = contrib_key(c, users, items, U, I, &ok);
        if (ok)
            atomicAdd(&cnt[key], 1);
        else
            atomicOr(err, 1);
    }
}

__global__ __launch_bounds__(kBlock) void k_scan_local(const int32_t* __restrict__ cnt, int64_t r1,
                                                       int32_t* __restrict__ offs, int32_t* __restrict__ tot) {
    __shared__ int sw[4];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * 8;
    int v[8];
    int sum = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        v[j] = (base + j < r1) ? cnt[base + j] : 0;
        sum += v[j];
    }
    int total;
    int run = block_exscan_256(sum, sw, &total);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (base + j < r1) offs[base + j] = run;
        run += v[j];
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = total;
}

// Exclusive prefix of the scan-block totals into LDS pre[0..nscan) (every thread participates).
__device__ inline void block_prefix_of_totals(const int32_t* __restrict__ tot, int nscan, int* pre, int* sw) {
    int carry = 0;
    for (int base = 0; base < nscan; base += kBlock) {
        const int x = base + (int)threadIdx.x < nscan ? tot[base + threadIdx.x] : 0;
        int total;
        const int ex = block_exscan_256(x, sw, &total);
        if (base + (int)threadIdx.x < nscan) pre[base + threadIdx.x] = carry + ex;
        carry += total;
    }
    __syncthreads();
}

// Finalise the row offsets (offs_g = local scan + prefix of block totals) and scatter every
// contribution into its row's list slot; the per-row counter runs back down to zero.
__global__ __launch_bounds__(kBlock) void k_fill(const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                                                 int64_t n, int32_t U, int32_t I, int32_t* __restrict__ cnt,
                                                 const int32_t* __restrict__ local, const int32_t* __restrict__ tot,
                                                 int nscan, int64_t r1, int32_t* __restrict__ offs_g,
                                                 int32_t* __restrict__ list) {
    extern __shared__ __attribute__((aligned(16))) int pre[];
    __shared__ int sw[4];
    block_prefix_of_totals(tot, nscan, pre, sw);
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = gt; r < r1; r += gstride) offs_g[r] = local[r] + pre[r / kScanBlock];
    const int64_t m = 2 * n;
    for (int64_t c = gt; c < m; c += gstride) {
        bool ok;
        const int key = contrib_key(c, users, items, U, I, &ok);
        if (!ok) continue;
        const int slot = atomicSub(&cnt[key], 1) - 1;
        list[local[key] + pre[key / kScanBlock] + slot] = (int)c;
    }
}

// Sort each row's contribution list ascending.  Rows of <= kSmallSeg entries: one thread,
// odd-even network in registers.  Longer rows: queued in LDS and sorted by the whole
// workgroup with a bitmap over the contribution ids (set bits, popcount scan, write back).
__global__ __launch_bounds__(kBlock) void k_sort(const int32_t* __restrict__ offs, int64_t R,
                                                 int32_t* __restrict__ list, int nwords) {
    extern __shared__ __attribute__((aligned(16))) unsigned bm[];
    __shared__ int hrows[kBlock];
    __shared__ int nh;
    __shared__ int sw[4];
    if (threadIdx.x == 0) nh = 0;
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (r < R) {
        const int o = offs[r];
        const int c = offs[r + 1] - o;
        if (c > kSmallSeg) {
            hrows[atomicAdd(&nh, 1)] = (int)r;
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
    __syncthreads();
    const int count = nh;
    const int per = (nwords + kBlock - 1) / kBlock;
    for (int hh = 0; hh < count; ++hh) {
        const int row = hrows[hh];
        const int o = offs[row];
        const int c = offs[row + 1] - o;
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

static int grid_for(int64_t work, int cap) {
    int64_t g = (work + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

hipError_t launch_index_build(const ncf_shape_t& s, const WsLayout& L, void* ws, const int32_t* users,
                              const int32_t* items, int64_t n, hipStream_t st) {
    const int64_t R = s.num_rows;
    const int64_t r1 = R + 1;
    int32_t* cnt = at<int32_t>(ws, L.cnt);
    int32_t* heavy_n = at<int32_t>(ws, L.heavy_n);
    int32_t* err = at<int32_t>(ws, L.err);
    int32_t* local = at<int32_t>(ws, L.offs_local);
    int32_t* offs = at<int32_t>(ws, L.offs);
    int32_t* tot = at<int32_t>(ws, L.tot);
    int32_t* list = at<int32_t>(ws, L.list);
    const int gc = grid_for(2 * n, 1024);
    k_count<<<gc, kBlock, 0, st>>>(users, items, n, s.num_users, s.num_items, cnt, heavy_n, err);
    const int nscan = (int)((r1 + kScanBlock - 1) / kScanBlock);
    k_scan_local<<<nscan, kBlock, 0, st>>>(cnt, r1, local, tot);
    const int gf = grid_for(2 * n > r1 ? 2 * n : r1, 1024);
    k_fill<<<gf, kBlock, (size_t)nscan * 4, st>>>(users, items, n, s.num_users, s.num_items, cnt, local, tot, nscan,
                                                  r1, offs, list);
    const int nwords = (int)((2 * n + 31) / 32);
    static bool lds_cfg = false;
    if (!lds_cfg && (size_t)nwords * 4 > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)k_sort, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)((kMaxBatch * 2 / 32) * 4));
        if (e != hipSuccess) return e;
        lds_cfg = true;
    }
    k_sort<<<(unsigned)((R + kBlock - 1) / kBlock), kBlock, (size_t)nwords * 4, st>>>(offs, R, list, nwords);
    return hipGetLastError();
}

}  // namespace ncf
