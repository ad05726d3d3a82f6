// Device helpers shared by the kernels (wave64 reductions and scans).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ncf {

// Deterministic sum over a 256-thread block (fixed tree order).  All threads
// get the result.  `red` is a __shared__ float[kBlock/64] scratch.
__device__ inline float wave_sum(float x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__device__ inline float block_sum_256(float x, float* red) {
    x = wave_sum(x);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = x;
    __syncthreads();
    float r = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return r;
}

// Exclusive scan of one int per thread over a 256-thread block.
// Returns the exclusive prefix; *total receives the block sum.
__device__ inline int block_exscan_256(int x, int* sw, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    __syncthreads();
    if (lane == 63) sw[w] = incl;
    __syncthreads();
    int pre = 0;
    for (int j = 0; j < w; ++j) pre += sw[j];
    *total = sw[0] + sw[1] + sw[2] + sw[3];
    __syncthreads();
    return pre + incl - x;
}

__device__ inline float4 f4add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

}  // namespace ncf

#ifndef NCF_NT_STORES
#define NCF_NT_STORES 0
#endif
namespace ncf {
// Store of a streamed result nothing re-reads soon.  NCF_NT_STORES=1 makes it non-temporal:
// measured on MI355X it slows the fused kernel's gradient-row stores 80 -> 130 us per launch
// (config C) and the touched update 34 -> 37 us, so it is off.
__device__ __forceinline__ void st_stream(float4* p, const float4& v) {
#if NCF_NT_STORES
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(p));
#else
    *p = v;
#endif
}
}  // namespace ncf
