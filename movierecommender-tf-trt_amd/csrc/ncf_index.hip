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
//   k_scan_final  add the prefix of the block totals      -> offs[row]
//   k_fill        list[offs[row] + --cnt[row]] = c        (cnt back to 0)
//   k_sort_small  sort each row's list (<=16) in registers; longer rows
//                 are queued for
//   k_sort_heavy  one workgroup per long row: LDS bitmap over c, popcount
//                 scan, write back in ascending order.
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

__global__ __launch_bounds__(kBlock) void k_scan_final(int32_t* __restrict__ offs, int64_t r1,
                                                       const int32_t* __restrict__ tot) {
    __shared__ int sw[4];
    if (blockIdx.x == 0) return;
    int part = 0;
    for (int j = threadIdx.x; j < (int)blockIdx.x; j += blockDim.x) part += tot[j];
    int pre;
    block_exscan_256(part, sw, &pre);
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (base + j < r1) offs[base + j] += pre;
}

__global__ __launch_bounds__(kBlock) void k_fill(const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                                                 int64_t n, int32_t U, int32_t I, int32_t* __restrict__ cnt,
                                                 const int32_t* __restrict__ offs, int32_t* __restrict__ list) {
    const int64_t m = 2 * n;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += (int64_t)gridDim.x * blockDim.x) {
        bool ok;
        const int key = contrib_key(c, users, items, U, I, &ok);
        if (!ok) continue;
        const int slot = atomicSub(&cnt[key], 1) - 1;
        list[offs[key] + slot] = (int)c;
    }
}

__global__ __launch_bounds__(kBlock) void k_sort_small(const int32_t* __restrict__ offs, int64_t R,
                                                       int32_t* __restrict__ list, int32_t* __restrict__ heavy,
                                                       int32_t* heavy_n) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
        const int o = offs[r];
        const int c = offs[r + 1] - o;
        if (c < 2) continue;
        if (c > kSmallSeg) {
            heavy[atomicAdd(heavy_n, 1)] = (int)r;
            continue;
        }
        int v[kSmallSeg];
#pragma unroll
        for (int j = 0; j < kSmallSeg; ++j) v[j] = (j < c) ? list[o + j] : INT_MAX;
        // odd-even transposition network (static indexing keeps v[] in VGPRs)
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

__global__ __launch_bounds__(kBlock) void k_sort_heavy(const int32_t* __restrict__ offs, int32_t* __restrict__ list,
                                                       const int32_t* __restrict__ heavy,
                                                       const int32_t* __restrict__ heavy_n, int nwords) {
    extern __shared__ __attribute__((aligned(16))) unsigned bm[];
    __shared__ int sw[4];
    const int nh = *heavy_n;
    const int per = (nwords + kBlock - 1) / kBlock;
    for (int h = blockIdx.x; h < nh; h += gridDim.x) {
        const int r = heavy[h];
        const int o = offs[r];
        const int c = offs[r + 1] - o;
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
    int32_t* offs = at<int32_t>(ws, L.offs);
    int32_t* tot = at<int32_t>(ws, L.tot);
    int32_t* list = at<int32_t>(ws, L.list);
    int32_t* heavy = at<int32_t>(ws, L.heavy);
    const int gc = grid_for(2 * n, 2048);
    k_count<<<gc, kBlock, 0, st>>>(users, items, n, s.num_users, s.num_items, cnt, heavy_n, err);
    const int nscan = (int)((r1 + kScanBlock - 1) / kScanBlock);
    k_scan_local<<<nscan, kBlock, 0, st>>>(cnt, r1, offs, tot);
    k_scan_final<<<nscan, kBlock, 0, st>>>(offs, r1, tot);
    k_fill<<<gc, kBlock, 0, st>>>(users, items, n, s.num_users, s.num_items, cnt, offs, list);
    k_sort_small<<<grid_for(R, 4096), kBlock, 0, st>>>(offs, R, list, heavy, heavy_n);
    const int nwords = (int)((2 * n + 31) / 32);
    static bool lds_cfg = false;
    if (!lds_cfg && (size_t)nwords * 4 > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)k_sort_heavy, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)((kMaxBatch * 2 / 32) * 4));
        if (e != hipSuccess) return e;
        lds_cfg = true;
    }
    k_sort_heavy<<<256, kBlock, (size_t)nwords * 4, st>>>(offs, list, heavy, heavy_n, nwords);
    return hipGetLastError();
}

}  // namespace ncf
