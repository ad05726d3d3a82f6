// All-item scoring + top-k (BASELINE.json config E).
//
// Reference workload: movierec/trt_client.py:43-57 sends one user with
// NUM_ITEMS_PREDICT random items to the served model (output/Sigmoid of
// model.py:184-194) and keeps the K = 10 best by np.argsort.  Here every user
// of a list is scored against the WHOLE catalogue and the k best items are
// kept, best first, ties broken by the lower item id.
//
// Fast path (NCF_SCORE_FP16, 4-layer models with layers[1] <= 64,
// layers[2] <= 32, layers[3] <= 32, gmf_dim <= 64): fp16 operands, fp32
// accumulation on v_mfma_f32_32x32x16_f16.  The first layer splits over the
// concatenated input (model.py:171-181):
//     h1 = relu(a_u + c_i),  a_u = b1 + W1[:du]^T e_u,  c_i = W1[du:]^T e_i
// and relu(a + c) = a + max(c, -a), so
//     W2^T h1 = W2^T a_u + W2^T max(c_i, -a_u).
// W2^T a_u + b2 is a per-user vector (prepared once, fp32) that initialises
// the layer-2 accumulator; the per-pair operand is a single v_pk_max_f16 of
// the item term and the negated user term.  Layer 2 and 3 are feature-major
// MFMA chains (item on the lane, features in registers; a D tile feeds the
// next MFMA's B operand register-for-register), the GMF term
// (w_g ⊙ e_u^g) · e_i^g is one 32-user x 32-item MFMA tile per item tile.
// One wave owns 32 users and sweeps all items in 32-item tiles (the item
// tiles stream from L2 for every wave of an XCD); a running per-user
// threshold (the k-th best so far) filters candidates with one compare and
// a ballot, and the rare insertions into the per-user list (LDS) run after
// the tile.  Ranking is by the logit z (sigmoid is monotonic); the reported
// score is sigmoid(z).
//
// Exact path (NCF_SCORE_FP32, any shape): the generic fp32 forward
// (ncf_predict) over (user, item) pairs for a chunk of users, then a per-user
// top-k by probability — the reference's own ranking quantity.

#include <cmath>

#include "ncf_common.h"
#include "ncf_internal.h"

#ifndef NCF_SCORE_OUT_DEFER
#define NCF_SCORE_OUT_DEFER 1
#endif
#ifndef NCF_DIAG_SCORE
#define NCF_DIAG_SCORE 0
#endif

namespace ncf {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float sf32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t su32x4 __attribute__((ext_vector_type(4)));

constexpr int kScoreTopMax = 32;  // largest k of the MFMA path

__device__ __forceinline__ int drow_s(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ sf32x16 mfma16(f16x8 a, f16x8 b, sf32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// elementwise max of packed halves: v_pk_maximum3_f16 (a, b, b), no canonicalisation of the
// inputs, and visible to the compiler's MFMA hazard checks (no inline asm)
__device__ __forceinline__ f16x8 pkmax(f16x8 a, f16x8 b) { return __builtin_elementwise_maximum(a, b); }

__device__ __forceinline__ f16x8 relu_f16(f16x8 a) { return __builtin_elementwise_maximum(a, f16x8{}); }

// ----------------------------------------------------------------------------- preparation

// Weight fragments.  a2[s][lane][e] = W2[k][i] (lane (i, h), k = 16s + 8h + e);
// a3[s][lane][e] = W3[x][i] with x = 16s + 8(e>>2) + 4h + (e&3), the row of the layer-2 D
// tile that register 8s+e of lane half h holds; init3/wh[h][r] = b3 / w_out at row drow(r, h).
__global__ __launch_bounds__(kBlock) void k_score_weights(const float* __restrict__ mlp, ScoreDims d,
                                                          _Float16* __restrict__ a2, _Float16* __restrict__ a3,
                                                          float* __restrict__ init3, float* __restrict__ wh,
                                                          float* __restrict__ bo) {
    const float* W2 = mlp + d.off_w2;
    const float* W3 = mlp + d.off_w3;
    const float* b3 = W3 + d.L2 * d.L3;
    const float* wout = mlp + d.off_out;
    for (int x = threadIdx.x; x < d.ks2 * 512; x += kBlock) {
        const int s = x >> 9, lane = (x >> 3) & 63, e = x & 7;
        const int i = lane & 31, k = 16 * s + 8 * (lane >> 5) + e;
        a2[x] = (_Float16)((k < d.L1 && i < d.L2) ? W2[k * d.L2 + i] : 0.0f);
    }
    for (int x = threadIdx.x; x < d.ks3 * 512; x += kBlock) {
        const int s = x >> 9, lane = (x >> 3) & 63, e = x & 7;
        const int i = lane & 31, row = 16 * s + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
        a3[x] = (_Float16)((row < d.L2 && i < d.L3) ? W3[row * d.L3 + i] : 0.0f);
    }
    if (threadIdx.x < 32) {
        const int h = threadIdx.x >> 4, r = threadIdx.x & 15, row = drow_s(r, h);
        init3[threadIdx.x] = row < d.L3 ? b3[row] : 0.0f;
        wh[threadIdx.x] = row < d.L3 ? wout[d.G + row] : 0.0f;
    }
    if (threadIdx.x == 0) bo[0] = wout[d.G + d.L3];
}

// Item tiles, fragment-major: ic[((t*ks2 + s)*64 + lane)*8 + e] = c_i[16s + 8h + e] for item
// i = 32t + (lane & 31), h = lane >> 5 (zero past num_items / L1); ig likewise for e_i^g.
__global__ __launch_bounds__(kBlock) void k_score_items(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                        ScoreDims d, _Float16* __restrict__ ic,
                                                        _Float16* __restrict__ ig) {
    __shared__ float xe[32][65];  // the tile's item MLP vectors (di <= 64)
    const int t = blockIdx.x;
    const float* W1 = mlp;  // hidden_1 kernel [L0][L1] at offset 0
    for (int x = threadIdx.x; x < 32 * 64; x += kBlock) {
        const int j = x >> 6, k = x & 63, item = 32 * t + j;
        xe[j][k] = (item < d.I && k < d.di) ? emb[(int64_t)(d.U + item) * d.W + d.gmf_stride + k] : 0.0f;
    }
    __syncthreads();
    const int L1P = 16 * d.ks2;
    for (int x = threadIdx.x; x < 32 * L1P; x += kBlock) {
        const int j = x / L1P, f = x - j * L1P;
        float c = 0.0f;
        if (f < d.L1)
            for (int k = 0; k < d.di; ++k) c = fmaf(W1[(d.du + k) * d.L1 + f], xe[j][k], c);
        const int s = f >> 4, h = (f >> 3) & 1, e = f & 7;
        ic[(((int64_t)t * d.ks2 + s) * 64 + h * 32 + j) * 8 + e] = (_Float16)c;
    }
    const int GP = 16 * d.ksg;
    for (int x = threadIdx.x; x < 32 * GP; x += kBlock) {
        const int j = x / GP, f = x - j * GP, item = 32 * t + j;
        const float g = (item < d.I && f < d.G) ? emb[(int64_t)(d.U + item) * d.W + f] : 0.0f;
        const int s = f >> 4, h = (f >> 3) & 1, e = f & 7;
        ig[(((int64_t)t * d.ksg + s) * 64 + h * 32 + j) * 8 + e] = (_Float16)g;
    }
}

// Per-user terms (one 64-thread block per user slot q; slots past n are zero):
// nega[q][f] = -(b1 + W1[:du]^T e_u)[f]; init2[q][h][r] = (b2 + W2^T a_u)[drow(r, h)];
// ug = GMF A fragments (w_g ⊙ e_u^g) of the 32-user block.
__global__ __launch_bounds__(64) void k_score_users(const float* __restrict__ emb, const float* __restrict__ mlp,
                                                    ScoreDims d, const int32_t* __restrict__ users, int64_t n,
                                                    _Float16* __restrict__ nega, float* __restrict__ init2,
                                                    _Float16* __restrict__ ug, int32_t* __restrict__ uok,
                                                    int32_t* __restrict__ gthr) {
    __shared__ float a[64];
    __shared__ float xu[64];
    const int64_t q = blockIdx.x;
    const int uid = q < n ? users[q] : -1;
    const bool valid = uid >= 0 && uid < d.U;  // out-of-range ids: no recommendations (items -1)
    const int u = valid ? uid : 0;
    if (threadIdx.x == 0) {
        uok[q] = valid ? 1 : 0;
        gthr[q] = (int32_t)0x807fffff;  // key of -inf
    }
    const float* W1 = mlp;
    const float* b1 = mlp + d.L0 * d.L1;
    const float* W2 = mlp + d.off_w2;
    const float* b2 = W2 + d.L1 * d.L2;
    const float* wout = mlp + d.off_out;
    const int f = threadIdx.x;
    xu[f] = (valid && f < d.du) ? emb[(int64_t)u * d.W + d.gmf_stride + f] : 0.0f;
    __syncthreads();
    float av = 0.0f;
    if (valid && f < d.L1) {
        av = b1[f];
        for (int k = 0; k < d.du; ++k) av = fmaf(W1[k * d.L1 + f], xu[k], av);
    }
    a[f] = av;
    if (f < 16 * d.ks2) nega[q * 16 * d.ks2 + f] = (_Float16)(-av);
    __syncthreads();
    if (f < 32) {
        const int h = f >> 4, r = f & 15, row = drow_s(r, h);
        float v = 0.0f;
        if (valid && row < d.L2) {
            v = b2[row];
            for (int k = 0; k < d.L1; ++k) v = fmaf(W2[k * d.L2 + row], a[k], v);
        }
        init2[q * 32 + f] = v;
    }
    if (f < 16 * d.ksg) {
        const float g = (valid && f < d.G) ? wout[f] * emb[(int64_t)u * d.W + f] : 0.0f;
        const int64_t ub = q >> 5;
        const int i = (int)(q & 31), s = f >> 4, h = (f >> 3) & 1, e = f & 7;
        ug[((ub * d.ksg + s) * 64 + h * 32 + i) * 8 + e] = (_Float16)g;
    }
}

// ----------------------------------------------------------------------------- MFMA scorer

struct ScoreArgs {
    const f16x8* ic;
    const f16x8* ig;
    const _Float16* nega;
    const float4* init2;
    const f16x8* ug;
    const f16x8* a2;
    const f16x8* a3;
    const float* init3;
    const float* wh;
    const float* bo;
    const int32_t* uok;
    int64_t n;
    int nub, ntiles, num_items, k;
    int splits, tiles_per;  // the catalogue is cut into `splits` ranges of tiles_per 32-item tiles
    int32_t* top_items;
    float* top_scores;
    float2* part;           // splits > 1: per-range lists [split][nub*32][k] of (logit, item)
    int32_t* gthr;          // per user: best k-th logit published by any of its ranges (ordered key)
};

// float <-> int key with the same order (atomicMax on floats of either sign)
__device__ __forceinline__ int fkey(float f) {
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float unkey(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }
// admission bound from another range's k-th best g: admit z >= g (ties resolve in the merge)
__device__ __forceinline__ float below(float g) { return g - fmaxf(fabsf(g) * 1e-6f, 1e-30f); }

template <int KS2, int KS3, int NR3, int KSG>
__global__ __launch_bounds__(kBlock, 2) void k_score_topk(ScoreArgs a) {
    constexpr int L1P = 16 * KS2;
    __shared__ __attribute__((aligned(16))) _Float16 s_nega[4][32][L1P];
    __shared__ float4 s_init2[4][32][8];
    __shared__ float2 s_top[4][32][kScoreTopMax];
    __shared__ float s_z[4][32][32];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
    // wave g: users block g % nub, item range g / nub (waves in flight together share a range:
    // its tiles stay in L2)
    const int g = blockIdx.x * 4 + w;
    const bool active = g < a.nub * a.splits;
    const int ub = active ? g % a.nub : 0;
    const int sp = active ? g / a.nub : 0;
    const int t0 = sp * a.tiles_per;
    const int t1 = min(a.ntiles, t0 + a.tiles_per);
    const int64_t q0 = (int64_t)ub * 32;
    const int K = a.k;
    // stage this wave's users
    {
        const float4* src = reinterpret_cast<const float4*>(a.nega + q0 * L1P);
        float4* dst = reinterpret_cast<float4*>(&s_nega[w][0][0]);
        for (int x = lane; x < 32 * L1P / 8; x += 64) dst[x] = src[x];
        for (int x = lane; x < 32 * 8; x += 64) s_init2[w][x >> 3][x & 7] = a.init2[q0 * 8 + x];
        for (int x = lane; x < 32 * kScoreTopMax; x += 64)
            s_top[w][x / kScoreTopMax][x % kScoreTopMax] = make_float2(-INFINITY, __int_as_float(-1));
    }
    __syncthreads();
    if (!active) return;

    f16x8 A2[KS2], A3[KS3];
#pragma unroll
    for (int s = 0; s < KS2; ++s) A2[s] = a.a2[s * 64 + lane];
#pragma unroll
    for (int s = 0; s < KS3; ++s) A3[s] = a.a3[s * 64 + lane];
    // GMF A fragments of the wave's 32 users, in registers for the whole sweep
    f16x8 AG[KSG > 0 ? KSG : 1];
#pragma unroll
    for (int s = 0; s < KSG; ++s) AG[s] = a.ug[((int64_t)ub * KSG + s) * 64 + lane];
    sf32x16 init3;
#pragma unroll
    for (int r = 0; r < 16; ++r) init3[r] = a.init3[h * 16 + r];
    // output layer as one MFMA (K = 16, the layer-3 D rows of lane half h as B): rows 0 and 4
    // of its A operand hold w_out, so register 0 of EVERY lane ends up with its item's dot
    f16x8 AO;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        AO[e] = ((j == 0 || j == 4) && e < NR3) ? (_Float16)a.wh[h * 16 + e] : (_Float16)0.0f;
    const float bo = a.bo[0];
    // lane q (< 32): user q0+q's own k-th best so far (thr) and admission bound (adm >= thr is
    // raised further by the k-th best any other range of the user has published: an item
    // below it cannot make the user's final top k)
    float thr = (lane < 32 && a.uok[q0 + (lane & 31)]) ? -INFINITY : INFINITY;
    int32_t* gth = a.gthr + q0 + (lane & 31);
    float adm = thr;
    int pub = fkey(-INFINITY);  // last key this wave published for its lane's user

    f16x8 BC[KS2], BG[KSG > 0 ? KSG : 1];
#pragma unroll
    for (int s = 0; s < KS2; ++s) BC[s] = a.ic[((int64_t)t0 * KS2 + s) * 64 + lane];
#pragma unroll
    for (int s = 0; s < KSG; ++s) BG[s] = a.ig[((int64_t)t0 * KSG + s) * 64 + lane];

    // the other ranges' published k-th best, read one tile ahead of its use (a bound: a late
    // value only admits more candidates, which the exact insertion test then rejects)
    int gk = fkey(-INFINITY);
    if (a.splits > 1 && lane < 32) gk = __hip_atomic_load(gth, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = t0; t < t1; ++t) {
        if (a.splits > 1 && lane < 32) {
            if (gk > pub) adm = fmaxf(adm, below(unkey(gk)));
            gk = __hip_atomic_load(gth, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // GMF + output bias of the 32 users x 32 items, parked in LDS ([user][item]) for the
        // user loop; a user's slot is then reused for its flagged logits
        {
            sf32x16 accg;
#pragma unroll
            for (int r = 0; r < 16; ++r) accg[r] = bo;
#pragma unroll
            for (int s = 0; s < KSG; ++s) accg = mfma16(AG[s], BG[s], accg);
#pragma unroll
            for (int r = 0; r < 16; ++r) s_z[w][drow_s(r, h)][j] = accg[r];
        }
        // the next tile's GMF operands: a whole tile in flight
        if (t + 1 < t1) {
#pragma unroll
            for (int s = 0; s < KSG; ++s) BG[s] = a.ig[((int64_t)(t + 1) * KSG + s) * 64 + lane];
        }

        const bool item_ok = h == 0 && 32 * t + j < a.num_items;
        const uint64_t okm = __builtin_amdgcn_ballot_w64(item_ok);
        uint32_t flagged = 0;
        // per-user operands from LDS, fetched one user ahead of their use
        // software pipeline over the 32 users: iteration q runs layer 3 + output of user q beside
        // layer 2 of user q+1, whose operands were read from LDS one iteration earlier (the reads
        // for user q+2 are in flight meanwhile); a scheduling barrier closes each iteration, so
        // the register footprint stays that of one
        float4 ui[4], vi[4];
        f16x8 un[KS2], vn[KS2];
        float ug = s_z[w][0][j], ugn = s_z[w][1][j];
#define NCF_SCORE_USER_OPS(UI, UN, Q)                                                           \
    {                                                                                           \
        if (NCF_DIAG_SCORE != 5)                                                                \
            _Pragma("unroll") for (int c = 0; c < 4; ++c) UI[c] = s_init2[w][Q][h * 4 + c];     \
        _Pragma("unroll") for (int s = 0; s < KS2; ++s)                                         \
            UN[s] = *reinterpret_cast<const f16x8*>(&s_nega[w][Q][16 * s + 8 * h]);             \
    }
#define NCF_SCORE_LAYER2(ACC)                                                                   \
    {                                                                                           \
        _Pragma("unroll") for (int c = 0; c < 4; ++c) {                                         \
            ACC[4 * c + 0] = ui[c].x; ACC[4 * c + 1] = ui[c].y;                                 \
            ACC[4 * c + 2] = ui[c].z; ACC[4 * c + 3] = ui[c].w;                                 \
        }                                                                                       \
        _Pragma("unroll") for (int s = 0; s < KS2; ++s)                                         \
            ACC = mfma16(A2[s], NCF_DIAG_SCORE == 6 ? BC[s] : pkmax(BC[s], un[s]), ACC);        \
    }
        NCF_SCORE_USER_OPS(ui, un, 0)
        sf32x16 acc2;
        NCF_SCORE_LAYER2(acc2)
        NCF_SCORE_USER_OPS(ui, un, 1)
#if NCF_SCORE_OUT_DEFER
        // the output MFMA of user q is consumed in iteration q + 1 (its latency hidden behind that
        // iteration's work instead of an s_nop before the logit's add)
        sf32x16 acc4p;
        float ugp = 0.0f;
#endif
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            float ugnn = 0.0f;
            if (q + 2 < 32) {
                ugnn = s_z[w][q + 2][j];
#if NCF_DIAG_SCORE != 1  // diagnostic builds only (wrong results)
                NCF_SCORE_USER_OPS(vi, vn, q + 2)
#endif
            }
            // keep those reads at the top of the iteration (the scheduler would sink them to the
            // end, next to their use, and expose the LDS latency)
            __builtin_amdgcn_sched_barrier(0);
            sf32x16 acc3 = init3;
#pragma unroll
            for (int s = 0; s < KS3; ++s) {
                f16x8 x;
#pragma unroll
                for (int e = 0; e < 8; ++e) x[e] = (_Float16)acc2[8 * s + e];
                acc3 = mfma16(A3[s], relu_f16(x), acc3);
            }
            if (q + 1 < 32) NCF_SCORE_LAYER2(acc2)
            // output layer: one MFMA over relu(h3) (zero accumulator), then the GMF term + bias
            f16x8 x3;
#pragma unroll
            for (int e = 0; e < 8; ++e) x3[e] = e < NR3 ? (_Float16)acc3[e] : (_Float16)0.0f;
#if NCF_SCORE_OUT_DEFER
            if (q > 0) {
                const float z = acc4p[0] + ugp;
                s_z[w][q - 1][j] = z;
                const float tq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(adm), q - 1));
                flagged |= (__builtin_amdgcn_ballot_w64(z > tq) & okm) ? (1u << (q - 1)) : 0u;
            }
            acc4p = mfma16(AO, relu_f16(x3), sf32x16{});
            ugp = ug;
#else
#if NCF_DIAG_SCORE == 7
            const float z = acc3[0] + ug;
#else
            const sf32x16 acc4 = mfma16(AO, relu_f16(x3), sf32x16{});
            const float z = acc4[0] + ug;
#endif
            // branch-free: both lane halves hold the same z (rows 0 and 4) and store it to the
            // user's slot (its GMF value was read two users ahead); the flag is a scalar select
            s_z[w][q][j] = z;
            const float tq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(adm), q));
            flagged |= (__builtin_amdgcn_ballot_w64(z > tq) & okm) ? (1u << q) : 0u;
#endif
            ug = ugn;
            ugn = ugnn;
            if (q + 2 < 32) {
#pragma unroll
                for (int c = 0; c < 4; ++c) ui[c] = vi[c];
#pragma unroll
                for (int s = 0; s < KS2; ++s) un[s] = vn[s];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#if NCF_SCORE_OUT_DEFER
        {   // the last user's logit
            const float z = acc4p[0] + ugp;
            s_z[w][31][j] = z;
            const float tq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(adm), 31));
            flagged |= (__builtin_amdgcn_ballot_w64(z > tq) & okm) ? (1u << 31) : 0u;
        }
#endif
#undef NCF_SCORE_LAYER2
#undef NCF_SCORE_USER_OPS
        // the next tile's item operands: loads in flight over the insertions below
#if NCF_DIAG_SCORE == 2
        flagged = 0;
#endif
#if NCF_DIAG_SCORE == 4
        if (false) {
#else
        if (t + 1 < t1) {
#endif
#pragma unroll
            for (int s = 0; s < KS2; ++s) BC[s] = a.ic[((int64_t)(t + 1) * KS2 + s) * 64 + lane];
        }
        // insertions (rare once the lists fill): ascending item order, ties keep the earlier item
        while (flagged) {
            const int q = __builtin_ctz(flagged);
            flagged &= flagged - 1;
            float tq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(adm), q));
            float tk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(thr), q));
            const float zl = s_z[w][q][j];
            uint64_t m = __ballot(item_ok && zl > tq);
            float2 ent = lane < K ? s_top[w][q][lane] : make_float2(-INFINITY, __int_as_float(-1));
            while (m) {
                const int c = __builtin_ctzll(m);
                m &= m - 1;
                const float zc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zl), c));
                if (!(zc > tq)) continue;
                const int p = __popcll(__ballot(lane < K && ent.x >= zc));
                // lane i <- lane i-1 (DPP wave_shr:1; lane 0 keeps its own, and never takes it)
                const float px = __int_as_float(__builtin_amdgcn_update_dpp(
                    __float_as_int(ent.x), __float_as_int(ent.x), 0x138, 0xf, 0xf, false));
                const float py = __int_as_float(__builtin_amdgcn_update_dpp(
                    __float_as_int(ent.y), __float_as_int(ent.y), 0x138, 0xf, 0xf, false));
                if (lane == p) ent = make_float2(zc, __int_as_float(32 * t + c));
                else if (lane > p) ent = make_float2(px, py);
                tk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ent.x), K - 1));
                tq = fmaxf(tq, tk);
            }
            if (lane < K) s_top[w][q][lane] = ent;
            if (lane == q) {
                thr = tk;
                adm = tq;
                // publish a full list's k-th best for the user's other ranges
                if (a.splits > 1 && tk > -INFINITY && fkey(tk) > pub) {
                    pub = fkey(tk);
                    atomicMax(gth, pub);
                }
            }
        }
    }
    for (int q = 0; q < 32; ++q) {
        if (q0 + q >= a.n) break;
        if (lane < K) {
            const float2 e = s_top[w][q][lane];
            if (a.splits > 1) {
                a.part[((int64_t)sp * a.nub * 32 + q0 + q) * K + lane] = e;
            } else {
                const int item = __float_as_int(e.y);
                a.top_items[(q0 + q) * K + lane] = item;
                a.top_scores[(q0 + q) * K + lane] = item >= 0 ? 1.0f / (1.0f + expf(-e.x)) : 0.0f;
            }
        }
    }
}

// Merge the per-range lists of each user (one thread per user): k rounds of a max over the
// splits*k entries that come after the previous pick in (logit desc, item asc) order.
__global__ __launch_bounds__(kBlock) void k_score_merge(const float2* __restrict__ part, int64_t n, int64_t stride,
                                                        int splits, int K, int32_t* __restrict__ top_items,
                                                        float* __restrict__ top_scores) {
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= n) return;
    float pv = INFINITY;
    int pi = -1;
    for (int r = 0; r < K; ++r) {
        float bv = -INFINITY;
        int bi = INT32_MAX;
        for (int sp = 0; sp < splits; ++sp) {
            const float2* l = part + ((int64_t)sp * stride + q) * K;
            for (int e = 0; e < K; ++e) {
                const float2 x = l[e];
                const int it = __float_as_int(x.y);
                if (it < 0) break;  // lists are sorted; -1 entries only at the tail
                const bool after = x.x < pv || (x.x == pv && it > pi);
                if (after && (x.x > bv || (x.x == bv && it < bi))) { bv = x.x; bi = it; }
            }
        }
        const bool ok = bi != INT32_MAX;
        top_items[q * K + r] = ok ? bi : -1;
        top_scores[q * K + r] = ok ? 1.0f / (1.0f + expf(-bv)) : 0.0f;
        pv = bv;
        pi = bi;
    }
}

// ----------------------------------------------------------------------------- exact path

// pair lists of users [q0, q0 + nq) x all items
__global__ __launch_bounds__(kBlock) void k_score_pairs(const int32_t* __restrict__ users, int64_t nq, int I,
                                                        int32_t* __restrict__ pu, int32_t* __restrict__ pi) {
    const int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (x >= nq * I) return;
    const int64_t q = x / I;
    pu[x] = users[q];
    pi[x] = (int32_t)(x - q * I);
}

// per row of I probabilities: the k best (descending, ties: lower item), k rounds of a
// block-wide arg-max over the items that come after the previous pick in that order
__global__ __launch_bounds__(kBlock) void k_topk_rows(const float* __restrict__ probs, int I, int K,
                                                      int32_t* __restrict__ top_items,
                                                      float* __restrict__ top_scores) {
    __shared__ float sv[kBlock / 64];
    __shared__ int si[kBlock / 64];
    const float* p = probs + (int64_t)blockIdx.x * I;
    float pv = INFINITY;
    int pidx = -1;
    for (int r = 0; r < K; ++r) {
        float bv = -INFINITY;
        int bi = INT32_MAX;
        for (int i = threadIdx.x; i < I; i += kBlock) {
            const float v = p[i];
            const bool after = v < pv || (v == pv && i > pidx);
            if (after && (v > bv || (v == bv && i < bi))) { bv = v; bi = i; }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const float ov = __shfl_xor(bv, d, 64);
            const int oi = __shfl_xor(bi, d, 64);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        __syncthreads();
        if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = bv; si[threadIdx.x >> 6] = bi; }
        __syncthreads();
        bv = sv[0];
        bi = si[0];
        for (int x = 1; x < kBlock / 64; ++x)
            if (sv[x] > bv || (sv[x] == bv && si[x] < bi)) { bv = sv[x]; bi = si[x]; }
        if (threadIdx.x == 0) {
            const bool ok = bi != INT32_MAX;
            top_items[(int64_t)blockIdx.x * K + r] = ok ? bi : -1;
            top_scores[(int64_t)blockIdx.x * K + r] = ok ? bv : 0.0f;
        }
        pv = bv;
        pidx = bi;
    }
}

// ----------------------------------------------------------------------------- host side

static inline int cdiv_i(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Item ranges per user block: enough waves (users/32 x splits) to fill the 2048 wave slots of the
// chip many times over, so the last round of waves is short; ranges of >= 64 tiles.
static inline int score_splits(int ntiles) {
    int s = cdiv_i(ntiles, 64);
    return s < 1 ? 1 : (s > 8 ? 8 : s);
}

ScoreDims score_dims(const ncf_shape_t& s) {
    ScoreDims d{};
    d.U = s.num_users;
    d.I = s.num_items;
    d.W = s.row_width;
    d.gmf_stride = s.gmf_stride;
    d.du = s.du;
    d.di = s.di;
    d.G = s.gmf_dim;
    d.L0 = s.layers[0];
    d.L1 = s.num_layers > 1 ? s.layers[1] : 0;
    d.L2 = s.num_layers > 2 ? s.layers[2] : 0;
    d.L3 = s.num_layers > 3 ? s.layers[3] : 0;
    d.off_w2 = s.num_layers > 2 ? s.layer_off[2] : 0;
    d.off_w3 = s.num_layers > 3 ? s.layer_off[3] : 0;
    d.off_out = s.layer_off[0];
    d.ks2 = cdiv_i(d.L1, 16);
    d.ks3 = cdiv_i(d.L2, 16);
    d.nr3 = 4 * cdiv_i(d.L3, 8);
    d.ksg = cdiv_i(d.G, 16);
    d.fast = s.num_layers == 4 && d.L1 <= 64 && d.L2 <= 32 && d.L3 <= 32 && d.G <= 64 && d.du <= 64 &&
             d.di <= 64;
    return d;
}

ScoreLayout make_score_layout(const ncf_shape_t& s, int64_t max_users) {
    ScoreLayout L{};
    const ScoreDims d = score_dims(s);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = (off + bytes + 255) / 256 * 256;
        return o;
    };
    L.max_users = max_users;
    const int64_t nub = (max_users + 31) / 32;
    const int64_t nt = (s.num_items + 31) / 32;
    if (d.fast) {
        L.ic = take((size_t)nt * d.ks2 * 64 * 16);
        L.ig = take((size_t)nt * (d.ksg > 0 ? d.ksg : 1) * 64 * 16);
        L.nega = take((size_t)nub * 32 * d.ks2 * 16 * 2);
        L.init2 = take((size_t)nub * 32 * 32 * 4);
        L.ug = take((size_t)nub * (d.ksg > 0 ? d.ksg : 1) * 64 * 16);
        L.a2 = take((size_t)d.ks2 * 64 * 16);
        L.a3 = take((size_t)d.ks3 * 64 * 16);
        L.init3 = take(32 * 4);
        L.wh = take(32 * 4);
        L.bo = take(4);
        L.uok = take((size_t)nub * 32 * 4);
        L.part = take((size_t)score_splits((int)nt) * nub * 32 * kScoreTopMax * 8);
        L.gthr = take((size_t)nub * 32 * 4);
    }
    // exact path: chunks of users x all items through the generic forward
    int64_t chunk = kMaxBatch / s.num_items;
    if (chunk < 1) chunk = 1;
    if (chunk > max_users) chunk = max_users;
    L.chunk = chunk;
    const int64_t np = chunk * s.num_items;
    L.pu = take((size_t)np * 4);
    L.pi = take((size_t)np * 4);
    L.probs = take((size_t)np * 4);
    L.pred_ws = off;
    L.pred_ws_bytes = make_layout(s, np > kMaxBatch ? kMaxBatch : np).total;
    L.total = off + L.pred_ws_bytes;
    return L;
}

hipError_t launch_score_prep(const ncf_shape_t& s, const ScoreLayout& L, void* ws, const float* emb,
                             const float* mlp, const int32_t* users, int64_t n, hipStream_t st) {
    const ScoreDims d = score_dims(s);
    const int nt = cdiv_i(s.num_items, 32);
    const int nub = cdiv_i(n, 32);
    launch(k_score_weights, 1, kBlock, 0, st, mlp, d, at<_Float16>(ws, L.a2), at<_Float16>(ws, L.a3),
           at<float>(ws, L.init3), at<float>(ws, L.wh), at<float>(ws, L.bo));
    launch(k_score_items, nt, kBlock, 0, st, emb, mlp, d, at<_Float16>(ws, L.ic), at<_Float16>(ws, L.ig));
    launch(k_score_users, nub * 32, 64, 0, st, emb, mlp, d, users, n, at<_Float16>(ws, L.nega),
           at<float>(ws, L.init2), at<_Float16>(ws, L.ug), at<int32_t>(ws, L.uok), at<int32_t>(ws, L.gthr));
    return hipGetLastError();
}

hipError_t launch_score_main(const ncf_shape_t& s, const ScoreLayout& L, void* ws, int64_t n, int k,
                             int32_t* top_items, float* top_scores, hipStream_t st) {
    const ScoreDims d = score_dims(s);
    const int nub = cdiv_i(n, 32);
    ScoreArgs a;
    a.ic = at<const f16x8>(ws, L.ic);
    a.ig = at<const f16x8>(ws, L.ig);
    a.nega = at<const _Float16>(ws, L.nega);
    a.init2 = at<const float4>(ws, L.init2);
    a.ug = at<const f16x8>(ws, L.ug);
    a.a2 = at<const f16x8>(ws, L.a2);
    a.a3 = at<const f16x8>(ws, L.a3);
    a.init3 = at<const float>(ws, L.init3);
    a.wh = at<const float>(ws, L.wh);
    a.bo = at<const float>(ws, L.bo);
    a.uok = at<const int32_t>(ws, L.uok);
    a.n = n;
    a.nub = nub;
    a.ntiles = cdiv_i(s.num_items, 32);
    a.num_items = s.num_items;
    a.k = k;
    a.top_items = top_items;
    a.top_scores = top_scores;
    a.splits = score_splits(a.ntiles);
    a.tiles_per = cdiv_i(a.ntiles, a.splits);
    a.part = at<float2>(ws, L.part);
    a.gthr = at<int32_t>(ws, L.gthr);
    const int grid = cdiv_i((int64_t)nub * a.splits, 4);
#define NCF_SCORE_LAUNCH(A, B, C, D) launch(k_score_topk<A, B, C, D>, grid, kBlock, 0, st, a)
    if (d.ks2 == 4 && d.ks3 == 2 && d.nr3 == 8 && d.ksg == 4) NCF_SCORE_LAUNCH(4, 2, 8, 4);       // ml-20m NeuMF (configs C/E)
    else if (d.ks2 == 4 && d.ks3 == 2 && d.nr3 == 8 && d.ksg == 0) NCF_SCORE_LAUNCH(4, 2, 8, 0);  // its MLP-only form
    else if (d.ks2 == 2 && d.ks3 == 1 && d.nr3 == 4 && d.ksg == 1) NCF_SCORE_LAUNCH(2, 1, 4, 1);  // ml-1m NeuMF (config B)
    else if (d.ks2 == 2 && d.ks3 == 1 && d.nr3 == 4 && d.ksg == 0) NCF_SCORE_LAUNCH(2, 1, 4, 0);  // trainer default [64,32,16,8]
    else return hipErrorInvalidValue;
#undef NCF_SCORE_LAUNCH
    if (a.splits > 1)
        launch(k_score_merge, cdiv_i(n, kBlock), kBlock, 0, st, (const float2*)a.part, n, (int64_t)nub * 32,
               a.splits, k, top_items, top_scores);
    return hipGetLastError();
}

bool score_fast_supported(const ncf_shape_t& s) {
    const ScoreDims d = score_dims(s);
    if (!d.fast) return false;
    return (d.ks2 == 4 && d.ks3 == 2 && d.nr3 == 8 && (d.ksg == 4 || d.ksg == 0)) ||
           (d.ks2 == 2 && d.ks3 == 1 && d.nr3 == 4 && (d.ksg == 1 || d.ksg == 0));
}

hipError_t launch_score_pairs(const int32_t* users, int64_t nq, int I, int32_t* pu, int32_t* pi, hipStream_t st) {
    const int64_t np = nq * I;
    launch(k_score_pairs, cdiv_i(np, kBlock), kBlock, 0, st, users, nq, I, pu, pi);
    return hipGetLastError();
}

hipError_t launch_topk_rows(const float* probs, int64_t rows, int I, int k, int32_t* top_items, float* top_scores,
                            hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    launch(k_topk_rows, (unsigned)rows, kBlock, 0, st, probs, I, k, top_items, top_scores);
    return hipGetLastError();
}

}  // namespace ncf
