// On-device negative sampling and batch assembly.
//
// Reference: MovieLensDataGenerator.__getitem__ (movierec/data_pipeline.py:115-150) builds
// a batch of groups [neg_1 .. neg_n, pos] (users repeated n+1 times, labels [0]*n + [1],
// :141-148); the negatives of a positive are drawn from the items the user has in neither
// `data` nor `extra` (np.setdiff1d, :103-108), without replacement unless there are fewer
// candidates than n (np.random.choice(..., replace=len < n), :111-112).
//
// Here one thread assembles one group.  Candidate c (0 <= c < C = num_items - |excluded|)
// is the c-th item missing from the user's sorted excluded list; it is found by a binary
// search over that list (p[m] - m counts the candidates below p[m]), so no candidate array is
// materialised.  c is drawn uniformly (Lemire's multiply with rejection of the biased
// remainder) from a counter-based Philox4x32-10 stream keyed by (seed, stream) and counted
// by (global positive slot, draw, attempt): batches are reproducible and independent of the
// launch configuration.  Duplicates inside a group are redrawn (without replacement) unless
// C < n.  The same algorithm is restated in numpy by oracle/ncf_oracle.py (sample_batch).

#include "ncf_common.h"
#include "ncf_internal.h"

namespace ncf {

constexpr uint32_t kMaxAttempts = 1u << 16;

__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                             uint32_t k1) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    c0 = h1 ^ c1 ^ k0;
    c1 = l1;
    c2 = h0 ^ c3 ^ k1;
    c3 = l0;
}

// first word of Philox4x32-10(counter = (a, b, c, d), key = (k0, k1))
__device__ __forceinline__ uint32_t philox_u32(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k0,
                                               uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        philox_round(a, b, c, d, k0, k1);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return a;
}

// the c-th (0-based) item in [0, I) that is not in the ascending list p[0..d)
__device__ __forceinline__ int kth_candidate(const int32_t* __restrict__ p, int d, uint32_t c) {
    int lo = 0, hi = d;  // count of m with p[m] - m <= c
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)p[mid] - mid <= (int64_t)c) lo = mid + 1;
        else hi = mid;
    }
    return (int)c + lo;
}

__global__ __launch_bounds__(kBlock) void k_sample_batch(const int32_t* __restrict__ pos_users,
                                                         const int32_t* __restrict__ pos_items,
                                                         const int32_t* __restrict__ excl_ptr,
                                                         const int32_t* __restrict__ excl_items, int num_users,
                                                         int num_items, const int32_t* __restrict__ order,
                                                         int64_t first, int n_pos, int negs, uint32_t k0, uint32_t k1,
                                                         uint32_t s0, uint32_t s1, int32_t* __restrict__ x_user,
                                                         int32_t* __restrict__ x_item, float* __restrict__ labels,
                                                         int32_t* __restrict__ err) {
    const int g = blockIdx.x * kBlock + threadIdx.x;
    if (g >= n_pos) return;
    const int64_t slot = first + g;  // position in the epoch order
    const int32_t pidx = order[slot];
    const int u = pos_users[pidx];
    const int ip = pos_items[pidx];
    const int64_t base = (int64_t)g * (negs + 1);
    int32_t* xi = x_item + base;
    for (int k = 0; k <= negs; ++k) {
        x_user[base + k] = u;
        labels[base + k] = k == negs ? 1.0f : 0.0f;
    }
    xi[negs] = ip;
    if ((unsigned)u >= (unsigned)num_users) {
        atomicOr(err, 1);
        for (int k = 0; k < negs; ++k) xi[k] = -1;
        return;
    }
    const int32_t* p = excl_items + excl_ptr[u];
    const int d = excl_ptr[u + 1] - excl_ptr[u];
    const uint32_t C = (uint32_t)(num_items - d);
    if (C == 0) {  // np.random.choice on an empty candidate array raises (data_pipeline.py:111-112)
        atomicOr(err, 2);
        for (int k = 0; k < negs; ++k) xi[k] = -1;
        return;
    }
    const bool replace = C < (uint32_t)negs;
    const uint32_t thresh = (0u - C) % C;  // Lemire: reject low words below 2^32 mod C
    const uint32_t sl = (uint32_t)slot, sh = (uint32_t)((uint64_t)slot >> 32) ^ s1;
    for (int k = 0; k < negs; ++k) {
        int item = -1;
        for (uint32_t a = 0; a < kMaxAttempts; ++a) {
            const uint32_t r = philox_u32((uint32_t)k, a, sl, sh, k0 ^ s0, k1);
            const uint64_t m = (uint64_t)r * C;
            if ((uint32_t)m < thresh) continue;
            const int cand = kth_candidate(p, d, (uint32_t)(m >> 32));
            bool dup = false;
            if (!replace)
                for (int q = 0; q < k; ++q) dup |= xi[q] == cand;
            if (dup) continue;
            item = cand;
            break;
        }
        if (item < 0) {  // bounded: never reached in practice (acceptance >= 1/C per attempt)
            atomicOr(err, 4);
            for (uint32_t c = 0; c < C && item < 0; ++c) {
                const int cand = kth_candidate(p, d, c);
                bool dup = false;
                for (int q = 0; q < k; ++q) dup |= xi[q] == cand;
                if (!dup) item = cand;
            }
        }
        xi[k] = item;
    }
}

hipError_t launch_sample_batch(const int32_t* pos_users, const int32_t* pos_items, const int32_t* excl_ptr,
                               const int32_t* excl_items, int num_users, int num_items, const int32_t* order,
                               int64_t first, int n_pos, int negs, uint64_t seed, uint64_t stream,
                               int32_t* x_user, int32_t* x_item, float* labels, int32_t* err, hipStream_t st) {
    if (n_pos <= 0) return hipSuccess;
    launch(k_sample_batch, (n_pos + kBlock - 1) / kBlock, kBlock, 0, st, pos_users, pos_items, excl_ptr, excl_items,
           num_users, num_items, order, first, n_pos, negs, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)stream,
           (uint32_t)(stream >> 32), x_user, x_item, labels, err);
    return hipGetLastError();
}

}  // namespace ncf
