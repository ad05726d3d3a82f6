// C ABI entry points (include/movierec_ncf.h).  Host orchestration only:
// argument validation, workspace carving and the launch sequence of each call.

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "movierec_ncf.h"
#include "ncf_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return fail(NCF_EHIP, "%s: %s", what, hipGetErrorString(e));
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int check_shape(const ncf_shape_t* s) {
    if (!s) return fail(NCF_EINVAL, "shape is NULL");
    if (s->row_width <= 0 || s->mlp_params <= 0) return fail(NCF_EINVAL, "shape not initialised (ncf_shape_init)");
    return 0;
}

int check_ws(const ncf_shape_t& s, int64_t n, void* ws, size_t ws_bytes, ncf::WsLayout* L, int world = 0) {
    if (!ws) return fail(NCF_EINVAL, "workspace is NULL");
    if (n <= 0) return fail(NCF_EINVAL, "batch size must be > 0, got %lld", (long long)n);
    if (n > ncf::kMaxBatch) return fail(NCF_EINVAL, "batch size %lld exceeds %lld", (long long)n,
                                        (long long)ncf::kMaxBatch);
    // the layout depends on max_batch only through per-batch regions; recover it from ws_bytes
    // by requiring the caller to size ws for at least n samples
    ncf::WsLayout need = ncf::make_layout(s, n, world);
    if (ws_bytes < need.total)
        return fail(NCF_EINVAL, "workspace too small: %zu bytes for batch %lld (need %zu)", ws_bytes,
                    (long long)n, need.total);
    *L = need;
    return 0;
}

int check_world(int world) {
    if (world < 1 || world > ncf::kSmallSeg)
        return fail(NCF_EINVAL, "world must be in [1, %d] for the row-sharded path, got %d", ncf::kSmallSeg, world);
    return 0;
}

int check_hyper(const ncf_hyper_t* h) {
    if (!h) return fail(NCF_EINVAL, "hyper is NULL");
    if (h->optimizer != NCF_OPT_ADAM && h->optimizer != NCF_OPT_SGD)
        return fail(NCF_EINVAL, "Optimizer %d is not implemented.", h->optimizer);
    if (h->group <= 0) return fail(NCF_EINVAL, "group must be > 0");
    return 0;
}

struct ProfSlot {
    std::vector<hipEvent_t> start, stop;
    size_t used = 0;
};
struct Profiler {
    uint32_t mask = 0;  // bit k set: time launch group k
    uint32_t select = ~0u;  // of those, the ones currently attaching events (ncf_profile_select)
    bool paused = false;
    ProfSlot slot[16];
};
thread_local Profiler g_prof;

// A profiled launch group's events ride on its kernels' dispatch packets (ncf::launch).
void prof_begin(int k, hipStream_t) {
    ProfSlot& p = g_prof.slot[k & 15];
    if (g_prof.paused || !((g_prof.mask & g_prof.select) >> k & 1u) || p.used >= p.start.size()) return;
    ncf::LaunchEvents& ev = ncf::launch_events();
    ev.start = p.start[p.used];
    ev.stop = p.stop[p.used];
    ev.launches = 0;
}
void prof_end(int k, hipStream_t) {
    ProfSlot& p = g_prof.slot[k & 15];
    if (g_prof.paused || !((g_prof.mask & g_prof.select) >> k & 1u) || p.used >= p.start.size()) return;
    ncf::LaunchEvents& ev = ncf::launch_events();
    if (ev.launches > 0) ++p.used;
    ev = ncf::LaunchEvents{};
}

// Side stream (one per device, created on first use, opt-in with NCF_SIDE_STREAM=1): the
// index build and the dense-layer tail run on it beside the forward/backward and the
// embedding sweep.  Measured on MI355X the cross-stream fork/join packets cost more than the
// overlap gains (225 vs 232 us per config-C step), so one stream is the default.
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};

#ifndef NCF_UNIT_MAX_BATCH
// batches up to this run the sample-unit kernel: it is faster than the tile kernel at every size
// measured (config C: 8192 22.4 vs 42.3 us, 65536 72 vs 80 us; profiles/r02_unit), so by default all
#define NCF_UNIT_MAX_BATCH (1LL << 40)
#endif
#ifndef NCF_WAVE_MIN_BATCH
// fp32 batches from this size run the wave-chain kernel instead (config C: 16384 28.2 vs 29.3 us,
// 65536 63.7 vs 73.4, 131072 108.7 vs 130.2; 8192 26.5 vs 23.1 — too few 16-sample units to give
// every SIMD work; profiles/r02_wave)
#define NCF_WAVE_MIN_BATCH 16384
#endif

int side_stream_mode() {
    static const int mode = [] {
        const char* e = ncf::experiment_env("NCF_SIDE_STREAM");
        return e ? atoi(e) : 0;
    }();
    return mode;
}

SideStream* side_stream() {
    if (side_stream_mode() == 0) return nullptr;
    static std::mutex mu;
    static std::map<int, SideStream> streams;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    SideStream& ss = streams[dev];
    if (!ss.s) {
        if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ss.join, hipEventDisableTiming) != hipSuccess) {
            ss.s = nullptr;
            return nullptr;
        }
    }
    return &ss;
}

// fork: the side stream waits for everything enqueued on `st` so far; returns the stream to use
hipStream_t fork_side(hipStream_t st, SideStream** out) {
    SideStream* ss = side_stream();
    *out = ss;
    if (!ss) return st;
    if (hipEventRecord(ss->fork, st) != hipSuccess || hipStreamWaitEvent(ss->s, ss->fork, 0) != hipSuccess) {
        *out = nullptr;
        return st;
    }
    return ss->s;
}

hipError_t join_side(hipStream_t st, SideStream* ss) {
    if (!ss) return hipSuccess;
    hipError_t e = hipEventRecord(ss->join, ss->s);
    if (e != hipSuccess) return e;
    return hipStreamWaitEvent(st, ss->join, 0);
}

bool use_fused(const ncf_shape_t& s, const ncf_hyper_t* h) {
    return s.fast_path && !(h && (h->force_generic == 1 || h->force_generic == 2)) && ncf::fused_supported(s);
}

// the layered kernels hold config D's widths only (ncf_layered.hip); any other shape whose weights
// outgrow the fused kernels — or asked for the layered path (force_generic == 2) — runs the
// generic per-sample kernel: no vendor-GEMM path exists
bool use_layered(const ncf_shape_t& s, const ncf_hyper_t* h) {
    if (!ncf::layered_supported(s)) return false;
    if (h && h->force_generic == 2) return true;
    if (h && h->force_generic == 1) return false;
    return !use_fused(s, h) && s.mlp_params > 12288;
}

// forward only: the fused MFMA forward when the shape has it, else the generic per-sample kernel
hipError_t launch_predict(const ncf_shape_t& s, const ncf_hyper_t* h, const ncf::WsLayout& L, void* ws,
                          const float* emb, const float* mlp, const int32_t* users, const int32_t* items,
                          const float* labels, int64_t n, float* probs, ncf::IdSpace ids, int* nbce, hipStream_t st) {
    if (use_fused(s, h)) return ncf::launch_fwd_fused(s, L, ws, emb, mlp, users, items, labels, n, probs, ids, nbce, st);
    // shapes whose weights outgrow the fused kernels (config D): the layered GEMM forward
    if (use_layered(s, h)) return ncf::launch_predict_layered(s, L, ws, emb, mlp, users, items, labels, n, probs, ids, nbce, st);
    return ncf::launch_predict_generic(s, L, ws, emb, mlp, users, items, labels, n, probs, ids, nbce, st);
}

// Shapes the fused kernel does not hold: the layer-by-layer GEMM path when the dense weights
// outgrow the generic kernel's LDS staging (config D), or when asked for (force_generic == 2);
// the per-sample generic kernel for small models (the reference's test shapes) or force_generic == 1.
// MFMA forward/backward kernel for a fused shape: the sample-unit kernel (ncf_unit.hip), the
// wave-chain kernel (ncf_wave.hip) or the 128-sample tile kernel (ncf_fused.hip).
// NCF_FB_KERNEL=unit|wave|tile forces one; hyper->force_generic 3 / 4 / 5 pick tile / unit / wave
// per call (6: the wave kernel's one-wave form).  bf16 operands run on the unit kernel only.
int fb_variant(const ncf_shape_t& s, const ncf_hyper_t* h, int64_t n) {
    static const int mode = [] {
        const char* e = ncf::experiment_env("NCF_FB_KERNEL");
        if (!e) return 0;
        return strcmp(e, "tile") == 0 ? NCF_FB_TILE : strcmp(e, "unit") == 0 ? NCF_FB_UNIT
                                                    : strcmp(e, "wave") == 0 ? NCF_FB_WAVE : 0;
    }();
    const bool bf16 = h && h->mlp_bf16;
    const int fg = h ? h->force_generic : 0;
    if (!ncf::unit_supported(s)) return NCF_FB_TILE;
    if (fg == 3) return NCF_FB_TILE;
    if (fg == 4) return NCF_FB_UNIT;
    if (fg == 5 || fg == 6) return ncf::wave_supported(s) && !bf16 ? NCF_FB_WAVE : NCF_FB_UNIT;
    int v = mode                      ? mode
            : n > NCF_UNIT_MAX_BATCH      ? NCF_FB_TILE
            : n >= NCF_WAVE_MIN_BATCH     ? NCF_FB_WAVE
                                          : NCF_FB_UNIT;
    if (v == NCF_FB_WAVE && (bf16 || !ncf::wave_supported(s))) v = NCF_FB_UNIT;
    return v;
}

// user-row folding of a step's index and fused kernel (ncf_internal.h fold_of); h NULL: none.
// NCF_FOLD_USERS=0 turns it off (A/B measurements).  The layered path (config D) folds in
// k_lay_l1b since round 6; -DNCF_LAYERED_FOLD=0 builds the unfolded layered step (A/B)
#ifndef NCF_LAYERED_FOLD
#define NCF_LAYERED_FOLD 1
#endif
#ifndef NCF_REPLAY_IN_SCAN
#define NCF_REPLAY_IN_SCAN 1   // short catch-up-ahead replays in the stats launch (0: all in the update's count blocks)
#endif
int index_fold(const ncf_shape_t& s, const ncf_hyper_t* h) {
    static const bool on = [] {
        const char* e = ncf::experiment_env("NCF_FOLD_USERS");
        return !e || atoi(e) != 0;
    }();
    return h && on ? ncf::fold_of(h->group, use_fused(s, h) || (NCF_LAYERED_FOLD && use_layered(s, h))) : 0;
}


}  // namespace

namespace ncf {

WsLayout make_layout(const ncf_shape_t& s, int64_t B, int world) {
    WsLayout L{};
    const int64_t R = s.num_rows;
    const size_t a = 256;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes, a);
        return o;
    };
    L.max_batch = B;
    L.world = world;
    L.shard_rows = shard_rows_of(R, world);
    L.keys = world > 0 ? (int64_t)world * L.shard_rows : R;
    const int64_t K = L.keys;
    L.list_cap = 2 * B;
    if (world > 0) {
        const int64_t per = 2 * B < L.shard_rows ? 2 * B : L.shard_rows;
        if ((int64_t)world * per > L.list_cap) L.list_cap = (int64_t)world * per;
    }
    L.cnt = take((size_t)(K + 1) * 4);
    L.cnt_ahead = take((size_t)(K + 1) * 4);  // right behind cnt: one memset clears both
    L.heavy_n = take(4);
    L.err = take(4);
    L.ifold = take(4);
    L.stale_step = take(4);
    if (world == 0) {
        L.seen = take((size_t)(K + 1) * 4);
        L.itag = take(4);
    }
    const int64_t S = L.shard_rows;
    if (world > 0) {
        L.ocnt = take((size_t)(S + 1) * 4);
        L.oheavy = take(4);
        L.oifold = take(4);
    }
    L.persistent_end = off;
    if (world == 0) {
        L.claims = take((size_t)2 * B * 8);
        L.nclaim = take((size_t)(2 * B / 16 + 1) * 4);
        L.claim_t = take(4);
    }
    if (world > 0) {
        // the owner index: sized by the shard only, ahead of every per-batch region
        L.onscan = (int)((S + 1 + kScanBlock - 1) / kScanBlock);
        L.ooffs_local = take((size_t)(S + 1) * 4);
        L.ooffs = take((size_t)(S + 1) * 4);
        L.ouloc = take((size_t)(S + 1) * 4);
        L.otot = take((size_t)L.onscan * 4);
        L.outot = take((size_t)L.onscan * 4);
        L.opre = take((size_t)2 * L.onscan * 4);
        L.olist = take((size_t)world * S * 4);
        L.otouched = take((size_t)S * 4);
        L.otoc = take((size_t)S * 8);
        L.onuniq = take(4);
    }
    L.nscan = (int)((K + 1 + kScanBlock - 1) / kScanBlock);
    L.nmetric = (int)((B + kBlock - 1) / kBlock);
    int A = 0;
    for (int l = 0; l < s.num_layers; ++l) A += s.layers[l];
    A += s.gmf_dim;
    int D = 1;
    for (int l = 1; l < s.num_layers; ++l) D += s.layers[l];
    L.act_w = A;
    L.dz_w = D;
    L.probs = take((size_t)B * 4);
    L.gs = take((size_t)2 * B * s.row_width * 4);
    L.list = take((size_t)L.list_cap * 4);
    L.offs_local = take((size_t)(K + 1) * 4);
    L.offs = take((size_t)(K + 1) * 4);
    L.tot = take((size_t)L.nscan * 4);
    L.pre = take((size_t)2 * L.nscan * 4);
    L.part_bce = take((size_t)kMaxSlabs * 4 + (size_t)L.nmetric * 4);
    // one partial per metrics block or per fused workgroup (up to kMaxSlabs)
    L.part_hit = take((size_t)(L.nmetric > kMaxSlabs ? L.nmetric : kMaxSlabs) * 4);
    L.part_dcg = take((size_t)(L.nmetric > kMaxSlabs ? L.nmetric : kMaxSlabs) * 4);
    L.part_reg = take((size_t)(kUpdateGrid + (s.mlp_params + kBlock - 1) / kBlock) * 4);
    L.summary = take(NCF_NUM_SUMMARY * 4);
    L.slabs = take((size_t)kMaxSlabs * s.mlp_params * 4);
    L.mlp_grad = take((size_t)s.mlp_params * 4);
    L.slab_part = take((size_t)kSlabSplit * s.mlp_params * 4);
    L.uloc = take((size_t)(K + 1) * 4);
    L.utot = take((size_t)L.nscan * 4);
    L.nuniq = take(4);
    if (world > 0) {
        L.cid_u = take((size_t)B * 4);
        L.cid_i = take((size_t)B * 4);
        L.uoffs = take((size_t)(2 * B + 1) * 4);
    } else {
        L.touched = take((size_t)(R < 2 * B ? R : 2 * B) * 4);
        L.touched_oc = take((size_t)(R < 2 * B ? R : 2 * B) * 8);
        L.heavy = take((size_t)(2 * B / kHeavyMin + 1) * 4);
        L.tl = take((size_t)L.nscan * kScanBlock * 4);
        L.tocl = take((size_t)L.nscan * kScanBlock * 8);
        L.slist = take((size_t)2 * B * 4);
    }
    L.act = take((size_t)B * A * 4);
    L.dz = take((size_t)B * D * 4);
    L.ones = take((size_t)B * 4);
    L.total = off;
    return L;
}

WsLayout owner_view(const WsLayout& L, int64_t m) {
    WsLayout o = L;
    o.cnt = L.ocnt;
    o.cnt_ahead = L.ocnt;  // (the owner index never counts ahead)
    o.heavy_n = L.oheavy;
    o.ifold = L.oifold;
    o.offs_local = L.ooffs_local;
    o.offs = L.ooffs;
    o.uloc = L.ouloc;
    o.tot = L.otot;
    o.utot = L.outot;
    o.pre = L.opre;
    o.list = L.olist;
    o.touched = L.otouched;
    o.touched_oc = L.otoc;
    o.nuniq = L.onuniq;
    o.nscan = L.onscan;
    o.keys = L.shard_rows;
    o.list_cap = (int64_t)L.world * L.shard_rows;
    o.max_batch = m > 1 ? (m + 1) / 2 : 1;
    o.world = 0;
    return o;
}

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

LaunchEvents& launch_events() {
    thread_local LaunchEvents ev;
    return ev;
}

}  // namespace ncf

extern "C" {

int ncf_abi_version(void) { return NCF_ABI_VERSION; }

// Provenance (csrc/build.py passes the tree's source hash and the build's -D defines; a build by
// other means reports "unknown").  The marker string lets build.py read the hash from the file.
#ifndef NCF_BUILD_HASH
#define NCF_BUILD_HASH "unknown"
#endif
#ifndef NCF_BUILD_DEFINES
#define NCF_BUILD_DEFINES ""
#endif
#define NCF_STR2(x) #x
#define NCF_STR(x) NCF_STR2(x)
__attribute__((used)) static const char kNcfHashMark[] = "NCF_SRC_SHA256=" NCF_BUILD_HASH;
static const char kNcfBuildInfo[] = "{\"src_sha256\": \"" NCF_BUILD_HASH "\", \"defines\": \"" NCF_BUILD_DEFINES
                                    "\", \"arch\": \"gfx950\", \"abi\": " NCF_STR(NCF_ABI_VERSION) "}";

const char* ncf_build_info(void) { return kNcfBuildInfo + 0 * sizeof(kNcfHashMark); }

int ncf_fb_kernel(const ncf_shape_t* s, const ncf_hyper_t* h, int64_t n) {
    if (int r = check_shape(s)) return r;
    if (use_fused(*s, h)) return fb_variant(*s, h, n);
    return use_layered(*s, h) ? NCF_FB_LAYERED_MFMA : NCF_FB_GENERIC;
}

const char* ncf_last_error(void) { return g_err.c_str(); }

int ncf_shape_init(ncf_shape_t* s, int32_t num_users, int32_t num_items, const int32_t* layers, int32_t num_layers,
                   int32_t gmf_dim) {
    if (!s || (num_layers > 0 && !layers)) return fail(NCF_EINVAL, "NULL argument");
    if (num_layers < 0 || num_layers > NCF_MAX_LAYERS)
        return fail(NCF_EINVAL, "num_layers must be in [0, %d], got %d", NCF_MAX_LAYERS, num_layers);
    if (num_layers == 0 && gmf_dim <= 0)
        return fail(NCF_EINVAL, "a model needs an MLP (layers_sizes) or a GMF branch (gmf_dim > 0)");
    if (num_users <= 0 || num_items <= 0) return fail(NCF_EINVAL, "num_users and num_items must be > 0");
    if (gmf_dim < 0) return fail(NCF_EINVAL, "gmf_dim must be >= 0");
    for (int l = 0; l < num_layers; ++l)
        if (layers[l] <= 0) return fail(NCF_EINVAL, "layers_sizes[%d] must be > 0", l);
    if (num_layers > 0 && layers[0] < 2) return fail(NCF_EINVAL, "layers_sizes[0] must be >= 2 (user and item halves)");
    memset(s, 0, sizeof(*s));
    s->num_users = num_users;
    s->num_items = num_items;
    s->num_layers = num_layers;
    s->gmf_dim = gmf_dim;
    for (int l = 0; l < num_layers; ++l) s->layers[l] = layers[l];
    // GMF-only model (num_layers == 0, BASELINE config A): no MLP embedding halves, the output
    // layer reads the GMF product alone
    s->du = num_layers > 0 ? layers[0] / 2 : 0;
    s->di = num_layers > 0 ? layers[0] - s->du : 0;
    s->gmf_stride = (gmf_dim + 3) / 4 * 4;
    const int mlpw = ((s->du > s->di ? s->du : s->di) + 3) / 4 * 4;
    s->row_width = s->gmf_stride + mlpw;
    s->num_rows = (int64_t)num_users + num_items;
    s->out_features = gmf_dim + (num_layers > 0 ? layers[num_layers - 1] : 0);
    int off = 0;
    for (int l = 1; l < num_layers; ++l) {
        s->layer_off[l] = off;
        off += layers[l - 1] * layers[l] + layers[l];
    }
    s->layer_off[0] = off;
    off += s->out_features + 1;
    s->mlp_params = off;
    if (s->num_rows * (int64_t)(s->row_width / 4) >= (int64_t)1 << 31)
        return fail(NCF_EINVAL, "embedding table too large for one device (%lld rows)", (long long)s->num_rows);
    s->fast_path = ncf::fused_supported(*s) ? 1 : 0;
    return 0;
}

int ncf_workspace_size(const ncf_shape_t* s, int64_t max_batch, size_t* bytes) {
    if (int r = check_shape(s)) return r;
    if (!bytes) return fail(NCF_EINVAL, "bytes is NULL");
    if (max_batch <= 0 || max_batch > ncf::kMaxBatch)
        return fail(NCF_EINVAL, "max_batch must be in [1, %lld]", (long long)ncf::kMaxBatch);
    *bytes = ncf::make_layout(*s, max_batch).total;
    return 0;
}

int ncf_workspace_init(const ncf_shape_t* s, int64_t max_batch, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    ncf::WsLayout L = ncf::make_layout(*s, max_batch);
    if (!ws || ws_bytes < L.total) return fail(NCF_EINVAL, "workspace too small");
    static bool configured = false;
    if (!configured) {
        // the heavy-segment sort needs up to 2*kMaxBatch/8 bytes of dynamic LDS
        configured = true;
    }
    return hip_check(hipMemsetAsync(ws, 0, L.persistent_end, (hipStream_t)stream), "hipMemsetAsync");
}

int ncf_workspace_flags(const ncf_shape_t* s, int64_t max_batch, void* ws, size_t ws_bytes, int32_t* flags,
                        void* stream) {
    if (int r = check_shape(s)) return r;
    if (!flags) return fail(NCF_EINVAL, "flags is NULL");
    ncf::WsLayout L = ncf::make_layout(*s, max_batch);
    if (!ws || ws_bytes < L.total) return fail(NCF_EINVAL, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    if (hipError_t e = hipMemcpyAsync(flags, ncf::at<int32_t>(ws, L.err), 4, hipMemcpyDeviceToDevice, st))
        return hip_check(e, "flags copy");
    return hip_check(hipMemsetAsync(ncf::at<int32_t>(ws, L.err), 0, 4, st), "flags clear");
}

int ncf_shard_workspace_flags(const ncf_shape_t* s, int64_t max_batch, int32_t world, void* ws, size_t ws_bytes,
                              int32_t* flags, void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_world(world)) return r;
    if (!flags) return fail(NCF_EINVAL, "flags is NULL");
    ncf::WsLayout L = ncf::make_layout(*s, max_batch, world);
    if (!ws || ws_bytes < L.total) return fail(NCF_EINVAL, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    if (hipError_t e = hipMemcpyAsync(flags, ncf::at<int32_t>(ws, L.err), 4, hipMemcpyDeviceToDevice, st))
        return hip_check(e, "flags copy");
    return hip_check(hipMemsetAsync(ncf::at<int32_t>(ws, L.err), 0, 4, st), "flags clear");
}

// Diagnostics (tools/, not in the ABI header): byte offsets of the single-table index regions
// cnt, cnt_ahead, heavy_n, err, offs_local, offs, tot, uloc, utot, nuniq, touched, touched_oc,
// heavy, list, slist, then nscan and list_cap
extern "C" int ncf_debug_index_regions(const ncf_shape_t* s, int64_t max_batch, int64_t* out17) {
    if (int r = check_shape(s)) return r;
    if (!out17) return fail(NCF_EINVAL, "out is NULL");
    const ncf::WsLayout L = ncf::make_layout(*s, max_batch);
    const size_t v[] = {L.cnt, L.cnt_ahead, L.heavy_n, L.err, L.offs_local, L.offs, L.tot, L.uloc, L.utot,
                        L.nuniq, L.touched, L.touched_oc, L.heavy, L.list, L.slist};
    for (int j = 0; j < 15; ++j) out17[j] = (int64_t)v[j];
    out17[15] = L.nscan;
    out17[16] = L.list_cap;
    return 0;
}

int ncf_workspace_discard_counts(const ncf_shape_t* s, int64_t max_batch, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    ncf::WsLayout L = ncf::make_layout(*s, max_batch);
    if (!ws || ws_bytes < L.total) return fail(NCF_EINVAL, "workspace too small");
    // the index counters only (cursors and counts taken ahead, adjacent): the sticky error flags and
    // the last build's fold stay
    return hip_check(hipMemsetAsync(ncf::at<int32_t>(ws, L.cnt), 0, L.cnt_ahead - L.cnt + (size_t)(L.keys + 1) * 4,
                                    (hipStream_t)stream),
                     "counter clear");
}

int ncf_predict(const ncf_shape_t* s, const ncf_model_t* model, const int32_t* users, const int32_t* items,
                int64_t n, float* probs, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    if (!model || !model->emb || !model->mlp || !users || !items || !probs)
        return fail(NCF_EINVAL, "NULL device pointer");
    int nbce = 0;
    return hip_check(launch_predict(*s, nullptr, L, ws, model->emb, model->mlp, users, items, nullptr, n, probs,
                                    ncf::table_ids(*s), &nbce, (hipStream_t)stream),
                     "ncf_predict");
}

int ncf_rank(const float* probs, int64_t n_groups, int32_t group, int32_t* rank_idx, void* stream) {
    if (!probs || !rank_idx) return fail(NCF_EINVAL, "NULL device pointer");
    if (group <= 0 || n_groups < 0) return fail(NCF_EINVAL, "invalid group/n_groups");
    return hip_check(ncf::launch_rank(probs, n_groups, group, rank_idx, (hipStream_t)stream), "ncf_rank");
}

int ncf_group_metrics(const float* probs, const float* labels, int64_t n_groups, int32_t group, int32_t k,
                      float* hit, float* dcg, void* stream) {
    if (!probs || !labels) return fail(NCF_EINVAL, "NULL device pointer");
    if (group <= 0 || n_groups < 0) return fail(NCF_EINVAL, "invalid group/n_groups");
    int np = 0;
    return hip_check(ncf::launch_group_metrics(probs, labels, n_groups, group, k, hit, dcg, nullptr, nullptr, &np,
                                               (hipStream_t)stream),
                     "ncf_group_metrics");
}

struct FbOut {
    int nslab = 0, nbce = 0, nmet = 0;
    float n_groups = 0.f;
    bool defer_metrics = false;         // in: groups <= 8 may leave their metrics to the update launch
    ncf::MetricsDeferred met{0, nullptr, nullptr, 0, 0, 0};  // out: deferred (nblocks > 0)
    SideStream* index_side = nullptr;  // index built on this side stream: join before using it
};

// deferred exact decay: bring the batch's rows up to date before the forward pass reads them
struct CatchupCtx {
    const ncf_shape_t* s;
    const ncf::WsLayout* L;
    ncf_model_t* model;
    ncf_optim_t* optim;
    const ncf_hyper_t* h;
    void* ws;
    hipStream_t st;
    int64_t n;  // batch size (the catch-up launch also sorts the index lists)
    const int32_t* users;
    const int32_t* items;
};
static int catchup_touched(void* p) {
    const CatchupCtx& c = *static_cast<CatchupCtx*>(p);
    prof_begin(NCF_K_CATCHUP, c.st);
    // counted ahead (index_ready == 2): the previous step's update launch also caught these rows up
    // (if the ids changed since, the launch's gate blocks replay the rows the counted set missed)
    hipError_t e = ncf::launch_emb_catchup(*c.s, *c.L, c.ws, c.model->emb, c.optim->emb_m, c.optim->emb_v,
                                           c.optim->row_step, c.optim->step, *c.h, false, c.st, true, c.n,
                                           c.h->index_ready == 2, c.users, c.items);
    prof_end(NCF_K_CATCHUP, c.st);
    return hip_check(e, "touched-row catch-up");
}

// make `st` wait for an index built on the side stream
static int index_join(hipStream_t st, FbOut& fb) {
    if (!fb.index_side) return 0;
    hipError_t e = join_side(st, fb.index_side);
    fb.index_side = nullptr;
    return hip_check(e, "index join");
}

// index build + forward/backward (+ group metrics): shared by train_step and forward_backward
// sharded: ids are the compact ids of the last ncf_shard_plan (model->emb = its unique rows)
// after_index(ctx) (optional) runs once the index is enqueued, before the forward/backward
// fill (optional): the wave kernel's weight-gradient waves build the index (a batch counted and
// scanned ahead; fill_in_kernel): no index launch, no catch-up / sort launch
static int run_fb(const ncf_shape_t& s, const ncf::WsLayout& L, const ncf_model_t* model, const ncf_hyper_t* h,
                  const int32_t* users, const int32_t* items, const float* labels, int64_t n, void* ws,
                  float* probs_out, FbOut* out, hipStream_t st, bool sharded = false,
                  int (*after_index)(void*) = nullptr, void* ctx = nullptr, const ncf::FillArgs* fill = nullptr,
                  bool index_filled = false, bool sparse_index = false) {
    hipError_t e = hipSuccess;
    ncf::IdSpace ids = ncf::table_ids(s);
    const int fold = index_fold(s, h);
    const int variant = use_fused(s, h) ? fb_variant(s, h, n) : -1;
    const bool unit = variant == NCF_FB_UNIT || variant == NCF_FB_WAVE;
    bool check_fold = false;  // the unit / wave kernels check an earlier call's index fold themselves
    if (fill) {
        if ((variant != NCF_FB_WAVE && variant != NCF_FB_UNIT) || sharded)
            return fail(NCF_EINVAL, "in-kernel index fill: wave or unit kernel only");
    } else if (index_filled) {
        // k_fill_ahead has just filled this step's index (its fold is the kernel's)
    } else if (sharded || (h->index_ready == 1 && !after_index) || h->index_ready == 3) {
        // the index was built by an earlier call — ncf_shard_plan (compact ids), ncf_build_index
        // (the deferred-decay step needs the touched-row list too and builds its own), or the
        // previous ncf_user_dp_step (index_ready 3: list, touched rows and catch-up all done): it
        // must fold the user rows as this step's kernel does
        if (sharded) {
            users = ncf::at<int32_t>(ws, L.cid_u);
            items = ncf::at<int32_t>(ws, L.cid_i);
            ids = ncf::compact_ids(n);
        }
        if (unit) {
            check_fold = true;
        } else {
            e = ncf::launch_fold_check(L, ws, fold, st);
            if (e != hipSuccess) return hip_check(e, "fold check");
        }
    } else {
        // the index depends only on the ids: it is built on the side stream while the
        // forward/backward runs (the fused kernel leaves registers and a little LDS free on every
        // CU); the caller's next launch on `st` that needs it comes after index_join
        SideStream* ss = nullptr;
        // NCF_SIDE_STREAM=2: only the dense-layer tail leaves the main stream
        hipStream_t sti = side_stream_mode() == 2 ? st : fork_side(st, &ss);
        prof_begin(NCF_K_INDEX, sti);
        // deferred decay: the catch-up launch (after_index) sorts the lists in extra workgroups
        e = ncf::launch_index_build(s, L, ws, users, items, n, sti, after_index != nullptr, h->index_ready == 2,
                                    after_index != nullptr, fold, sparse_index);
        prof_end(NCF_K_INDEX, sti);
        if (e != hipSuccess) return hip_check(e, "index build");
        out->index_side = ss;
        if (after_index) {
            if (int r = index_join(st, *out)) return r;
            if (int r = after_index(ctx)) return r;
        }
    }
    prof_begin(NCF_K_FWD_BWD, st);
    if (h->mlp_bf16 && variant != NCF_FB_UNIT)
        return fail(NCF_EINVAL, "bf16 MLP operands need a fused-kernel shape and the unit kernel");
    if (variant == NCF_FB_WAVE)
        e = ncf::launch_fb_wave(s, L, ws, model->emb, model->mlp, users, items, labels, n, h->inv_batch, ids,
                                h->group, h->k, &out->nslab, &out->nbce, &out->nmet, st, fold, check_fold,
                                h->force_generic == 6, fill);
    else if (unit)
        e = ncf::launch_fb_unit(s, L, ws, model->emb, model->mlp, users, items, labels, n, h->inv_batch, ids,
                                h->group, h->k, &out->nslab, &out->nbce, &out->nmet, st, fold, h->mlp_bf16 != 0,
                                check_fold, fill);
    else if (use_fused(s, h))
        e = ncf::launch_fb_fused(s, L, ws, model->emb, model->mlp, users, items, labels, n, h->inv_batch, ids,
                                 h->group, h->k, &out->nslab, &out->nbce, &out->nmet, st, fold);
    else if (use_layered(s, h))
        e = ncf::launch_fb_layered(s, L, ws, model->emb, model->mlp, users, items, labels, n, h->inv_batch, ids,
                                   &out->nslab, &out->nbce, st, fold);
    else
        e = ncf::launch_fb_generic(s, L, ws, model->emb, model->mlp, users, items, labels, n, h->inv_batch, ids,
                                   &out->nslab, &out->nbce, st);
    prof_end(NCF_K_FWD_BWD, st);
    if (e != hipSuccess) return hip_check(e, "forward/backward");
    float* probs = ncf::at<float>(ws, L.probs);
    const int64_t ng = n / h->group;
    out->n_groups = (float)ng;
    if (out->nmet == 0 && out->defer_metrics && h->group <= 8 && ng > 0) {
        // the touched-row update launch computes them (MetricsDeferred, when the batch summary
        // is written after it; else the caller launches them): one launch fewer
        const int grid = (int)((ng + ncf::kBlock - 1) / ncf::kBlock);
        out->met = ncf::MetricsDeferred{grid, probs, labels, ng, h->group, h->k};
        out->nmet = grid;
    } else if (out->nmet == 0) {
        prof_begin(NCF_K_METRICS, st);
        e = ncf::launch_group_metrics(probs, labels, ng, h->group, h->k, nullptr, nullptr,
                                      ncf::at<float>(ws, L.part_hit), ncf::at<float>(ws, L.part_dcg), &out->nmet, st);
        prof_end(NCF_K_METRICS, st);
        if (e != hipSuccess) return hip_check(e, "metrics");
    }
    if (probs_out) {
        e = hipMemcpyAsync(probs_out, probs, (size_t)n * 4, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return hip_check(e, "probs copy");
    }
    return 0;
}

static int check_train_args(const ncf_shape_t* s, const ncf_model_t* model, const ncf_hyper_t* h,
                            const int32_t* users, const int32_t* items, const float* labels, int64_t n) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (!model || !model->emb || !model->mlp || !users || !items || !labels)
        return fail(NCF_EINVAL, "NULL device pointer");
    if (n % h->group)
        return fail(NCF_EINVAL, "Batch size must be divisible by (num_negs_per_pos + 1). Found: batch_size=%lld, "
                    "group=%d", (long long)n, h->group);
    return 0;
}

#ifndef NCF_FILL_IN_KERNEL
// 1: the wave kernel's weight-gradient waves fill the index; 2: a fill launch of its own
// (k_fill_ahead) before the forward/backward; either way the touched-row update orders the lists.
// 0: round 4's fill and list-sort launches (timing comparisons)
#define NCF_FILL_IN_KERNEL 1
#endif
// The step's index built inside a launch that runs anyway (FillArgs): a batch counted and scanned
// ahead by the previous step (index_ready 2, deferred-decay Adam), a key space the fill's prefix
// table holds, one stream — by the split wave kernel's weight-gradient waves where that kernel
// runs (1), else by a fill launch ahead of the forward/backward (2).  The lists stay unsorted (the
// touched-row update orders them), and the counted rows were caught up by the previous step's
// update launch.  A batch whose ids changed after they were counted (a write that bypassed torch's
// version counter: NCF_WSERR_STALE_COUNT) is DROPPED: the forward pass may have read rows the
// counted set missed at their deferred step, so the update and stats launches apply nothing of
// the step (ws stale_step, fill_wave) — table, moments, dense layers, stats and step counter stay
// as they were, a consistent deferred-decay state — and check_errors raises.
// Returns 0: the index launches; 1: the forward/backward launch fills (the wave kernel's weight-gradient
// waves, or spare workgroups of a unit launch that leaves CUs idle); 2: k_fill_ahead fills
static int fill_in_kernel(const ncf_shape_t& s, const ncf::WsLayout& L, const ncf_hyper_t* h, int64_t n) {
    if (!NCF_FILL_IN_KERNEL || h->index_ready != 2 || h->optimizer != NCF_OPT_ADAM || side_stream_mode() != 0 ||
        L.world != 0 || L.nscan > ncf::kMaxFillScan || ncf::unsorted_heavy_c(s) < ncf::kHeavyMin)
        return 0;
    if (NCF_FILL_IN_KERNEL == 1 && use_fused(s, h) && fb_variant(s, h, n) == NCF_FB_WAVE && h->force_generic != 6 &&
        ncf::wave_fill_supported(s))
        return 1;
    // the unit kernel's grid leaves CUs idle (small batches, e.g. config B): fill workgroups there
    if (NCF_FILL_IN_KERNEL == 1 && use_fused(s, h) && fb_variant(s, h, n) == NCF_FB_UNIT &&
        ncf::unit_fill_fits(s, n, h->mlp_bf16 != 0, L.keys + 1))
        return 1;
    return 2;
}

static ncf::FillArgs fill_args(const ncf_shape_t& s, const ncf::WsLayout& L, void* ws) {
    using ncf::at;
    return ncf::FillArgs{at<int32_t>(ws, L.cnt), at<const int32_t>(ws, L.offs_local), at<const int32_t>(ws, L.tot),
                         at<const int32_t>(ws, L.utot), at<const int32_t>(ws, L.tl), at<const int2>(ws, L.tocl),
                         L.nscan, L.keys + 1, at<int32_t>(ws, L.list), at<int32_t>(ws, L.touched),
                         at<int2>(ws, L.touched_oc), at<int32_t>(ws, L.nuniq), at<int32_t>(ws, L.heavy),
                         at<int32_t>(ws, L.heavy_n), ncf::unsorted_heavy_c(s), at<int32_t>(ws, L.err),
                         at<int32_t>(ws, L.ifold), s.num_users, s.num_items, L.list_cap,
                         L.keys < 2 * L.max_batch ? L.keys : 2 * L.max_batch, 2 * L.max_batch / ncf::kHeavyMin + 1,
                         at<int32_t>(ws, L.stale_step)};
}

static int train_step_impl(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                           const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                           const int32_t* next_users, const int32_t* next_items, int64_t n_next, double* stats,
                           float* probs_out, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_train_args(s, model, h, users, items, labels, n)) return r;
    if (!optim || !optim->step || (h->optimizer == NCF_OPT_ADAM &&
                                   (!optim->emb_m || !optim->emb_v || !optim->mlp_m || !optim->mlp_v)))
        return fail(NCF_EINVAL, "NULL optimizer state");
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    float* summary = ncf::at<float>(ws, L.summary);
    FbOut fb;
    // Deferred exact decay (optim->row_step set, L2 off): untouched rows are not swept; the
    // batch's rows catch up on their missed zero-gradient steps right after the index build
    const bool lazy = optim->row_step != nullptr;
    if (lazy && h->lazy_rows > 0 && h->lazy_rows < s->num_rows)
        return fail(NCF_EINVAL, "hyper->lazy_rows < num_rows is the user-partitioned step's (ncf_*_lazy)");
    if (lazy && h->l2[0] != 0.0f)
        return fail(NCF_EINVAL, "deferred decay (row_step) needs the embedding L2 off: the loss sums the whole table");
    CatchupCtx cc{s, &L, model, optim, h, ws, st, n, users, items};
    // deferred decay on one stream: the group metrics (groups <= 8 the kernel does not compute)
    // ride in the touched-row update launch
    fb.defer_metrics = lazy && side_stream_mode() == 0;
    const int fmode = lazy ? fill_in_kernel(*s, L, h, n) : 0;
    const bool kfill = fmode != 0;
    // large key spaces (config D): the counted-ahead index without a pass over every key — the
    // previous step's stats launch scanned sparsely (sparse_scan below), k_fill_touched builds from
    // its per-block lists, and this step's update tests "in the batch" with the seen tags
    const bool sparse_ok = lazy && !kfill && h->optimizer == NCF_OPT_ADAM && ncf::sparse_index_ok(L);
    const bool sparse_build = sparse_ok && h->index_ready == 2;
    const ncf::FillArgs fa = kfill ? fill_args(*s, L, ws) : ncf::FillArgs{};
    if (fmode == 2) {
        prof_begin(NCF_K_INDEX, st);
        hipError_t e = ncf::launch_fill_ahead(fa, users, items, n, index_fold(*s, h), st);
        prof_end(NCF_K_INDEX, st);
        if (e != hipSuccess) return hip_check(e, "index fill");
    }
    if (int r = run_fb(*s, L, model, h, users, items, labels, n, ws, probs_out, &fb, st, false,
                       lazy && !kfill ? catchup_touched : nullptr, &cc, fmode == 1 ? &fa : nullptr,
                       fmode == 2, sparse_build))
        return r;
    // the index (side stream) must be complete before the side stream takes the dense tail
    if (int r = index_join(st, fb)) return r;
    // dense-layer tail on the side stream, embedding sweep on the main stream
    SideStream* ss = nullptr;
    hipStream_t st2 = fork_side(st, &ss);
    // one stream (the default): the batch summary rides in the slab reduction's launch.  (Folding
    // the stats into the touched update's last block was measured 8x slower: a device-scope fence
    // per block on a multi-XCD part writes back L2.)
    const bool fold = ss == nullptr;
    hipError_t e = hipSuccess;
    if (!fold) {
        e = ncf::launch_summary(L, ws, fb.nbce, fb.nmet, fb.n_groups, 0, 0, summary, st2);
        if (e != hipSuccess) return hip_check(e, "summary");
    }
    int nreg_mlp = 0;
    // one stream + deferred decay: the dense layers' Adam step runs in extra workgroups of the
    // touched-row update launch (one launch fewer)
    ncf::MlpDeferred mlp_def{nullptr, nullptr, nullptr, nullptr, 0, 0};
    const bool defer_mlp = fold && lazy;
    // every L2 factor zero and enough slabs: both slab-reduction levels run in the touched-row
    // update launch too, and the batch summary in the stats launch (two launches fewer)
    const bool two_level = defer_mlp && h->optimizer == NCF_OPT_ADAM && ncf::part_tail_foldable(*s, *h, fb.nslab);
    mlp_def.two_level = two_level ? 1 : 0;
    if (fb.met.nblocks > 0 && !two_level) {
        // the summary is written before the touched-row update launch: the metrics go first
        int nm = 0;
        prof_begin(NCF_K_METRICS, st);
        e = ncf::launch_group_metrics(fb.met.probs, fb.met.labels, fb.met.ng, fb.met.group, fb.met.k, nullptr, nullptr,
                                      ncf::at<float>(ws, L.part_hit), ncf::at<float>(ws, L.part_dcg), &nm, st);
        prof_end(NCF_K_METRICS, st);
        if (e != hipSuccess) return hip_check(e, "metrics");
        fb.met.nblocks = 0;
    }
    prof_begin(NCF_K_MLP_UPDATE, st2);
    e = ncf::launch_mlp_update(*s, L, ws, model->mlp, optim->mlp_m, optim->mlp_v, optim->step, *h, fb.nslab, nullptr,
                               nullptr, true, &nreg_mlp, st2, false, fold && !two_level ? fb.nbce : -1, fb.nmet,
                               fb.n_groups, fold && !two_level ? summary : nullptr, defer_mlp ? &mlp_def : nullptr);
    prof_end(NCF_K_MLP_UPDATE, st2);
    if (e != hipSuccess) return hip_check(e, "dense update");
    // counting ahead: the next batch's stale rows are claimed in the touched-row update launch; those
    // owing a few steps are replayed in the stats launch behind it (off the update's HBM stream),
    // the long chains stay under the update (profiles/r06_ab/replay_in_scan)
    bool defer_replay = NCF_REPLAY_IN_SCAN && lazy && next_users != nullptr && L.world == 0 &&
                        h->optimizer == NCF_OPT_ADAM;
    prof_begin(NCF_K_EMB_UPDATE, st);
    if (lazy)
        e = ncf::launch_emb_update_touched(*s, L, ws, model->emb, optim->emb_m, optim->emb_v, optim->row_step,
                                           optim->step, *h, st, next_users, next_items, n_next,
                                           mlp_def.p ? &mlp_def : nullptr, index_fold(*s, h),
                                           fb.met.nblocks > 0 ? &fb.met : nullptr, nullptr, kfill, true, sparse_build,
                                           &defer_replay);
    else
        e = ncf::launch_emb_update(*s, L, ws, model->emb, optim->emb_m, optim->emb_v, optim->step, *h, nullptr,
                                   s->num_rows, st);
    prof_end(NCF_K_EMB_UPDATE, st);
    if (e != hipSuccess) return hip_check(e, "embedding update");
    e = join_side(st, ss);
    if (e != hipSuccess) return hip_check(e, "side-stream join");
    const int nreg_emb = h->l2[0] != 0.0f ? ncf::kUpdateGrid : 0;
    const ncf::ReplayDeferred rdef{model->emb, optim->emb_m, optim->emb_v, s->row_width, h->lr, h->beta_1, h->beta_2,
                                   h->epsilon, lazy && defer_replay ? 2 * n_next : 0};
    // counting ahead: the stats launch also scans the next batch's counts
    // (an in-kernel fill's step may have been dropped: the stats launch then adds nothing, bumps
    // nothing and clears the word)
    e = ncf::launch_stats(L, ws, summary, nreg_emb, nreg_mlp, h->inv_batch, stats, optim->step, true, st,
                          lazy && next_users != nullptr, s->num_rows,
                          two_level ? ncf::SummaryFirst{fb.nbce, fb.nmet, fb.n_groups} : ncf::SummaryFirst{-1, 0, 0.f},
                          kfill ? ncf::at<int32_t>(ws, L.stale_step) : nullptr, sparse_ok && next_users != nullptr,
                          &rdef);
    return hip_check(e, "stats");
}

int ncf_train_step(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                   const int32_t* users, const int32_t* items, const float* labels, int64_t n, double* stats,
                   float* probs_out, void* ws, size_t ws_bytes, void* stream) {
    return train_step_impl(s, model, optim, h, users, items, labels, n, nullptr, nullptr, 0, stats, probs_out, ws,
                           ws_bytes, stream);
}

int ncf_train_step_ahead(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                         const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                         const int32_t* next_users, const int32_t* next_items, int64_t n_next, double* stats,
                         float* probs_out, void* ws, size_t ws_bytes, void* stream) {
    if (!s || !optim || !h) return fail(NCF_EINVAL, "NULL argument");
    // the scan ahead lands in workspace regions placed by the batch size: the next batch must
    // have this batch's size
    if (!next_users || !next_items || n_next != n)
        return fail(NCF_EINVAL, "next batch: NULL ids or n_next != n");
    if (!optim->row_step || h->optimizer != NCF_OPT_ADAM)
        return fail(NCF_EINVAL, "counting ahead needs deferred-decay Adam (optim->row_step)");
    return train_step_impl(s, model, optim, h, users, items, labels, n, next_users, next_items, n_next, stats,
                           probs_out, ws, ws_bytes, stream);
}

// lazy (optional): deferred exact decay of rows [0, h->lazy_rows) — the index carries the touched
// list and the batch's stale rows are caught up before the forward pass (user-partitioned DP)
static int forward_backward_rows(const ncf_shape_t* s, const ncf_model_t* model, const ncf_hyper_t* h,
                                 const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                                 int64_t grad_row_begin, float* emb_grad, float* mlp_grad, float* summary,
                                 float* probs_out, int64_t reg_row_begin, int64_t reg_row_count,
                                 int32_t include_dense_reg, void* ws, size_t ws_bytes, void* stream,
                                 ncf_optim_t* lazy = nullptr) {
    if (int r = check_train_args(s, model, h, users, items, labels, n)) return r;
    if (!emb_grad || !mlp_grad || !summary) return fail(NCF_EINVAL, "NULL gradient output");
    if (reg_row_begin < 0 || reg_row_count < 0 || reg_row_begin > s->num_rows)
        return fail(NCF_EINVAL, "invalid regulariser row range");
    if (reg_row_begin + reg_row_count > s->num_rows) reg_row_count = s->num_rows - reg_row_begin;
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    FbOut fb;
    CatchupCtx cc{s, &L, const_cast<ncf_model_t*>(model), lazy, h, ws, st, n, users, items};
    if (int r = run_fb(*s, L, model, h, users, items, labels, n, ws, probs_out, &fb, st, false,
                       lazy ? catchup_touched : nullptr, &cc))
        return r;
    // the index (side stream) must be complete before the side stream takes the dense tail
    if (int r = index_join(st, fb)) return r;
    if (side_stream_mode() == 0 && ncf::part_tail_foldable(*s, *h, fb.nslab)) {
        // L2 off, one stream: slab partials + summary, then the dense embedding gradient with the
        // dense-layer gradient in extra workgroups: 2 launches instead of 4
        hipError_t e = ncf::launch_part_tail(*s, L, ws, emb_grad, grad_row_begin, mlp_grad, fb.nslab, fb.nbce, fb.nmet,
                                             fb.n_groups, summary, st);
        return hip_check(e, "gradient tail");
    }
    SideStream* ss = nullptr;
    hipStream_t st2 = fork_side(st, &ss);
    int nreg_mlp = 0, nreg_emb = 0;
    hipError_t e = ncf::launch_mlp_update(*s, L, ws, model->mlp, nullptr, nullptr, nullptr, *h, fb.nslab, nullptr,
                                          mlp_grad, false, &nreg_mlp, st2, include_dense_reg != 0);
    if (e != hipSuccess) return hip_check(e, "dense-layer gradient");
    if (h->l2[0] != 0.0f && reg_row_count > 0) {
        e = ncf::launch_emb_reg(*s, L, ws, model->emb + reg_row_begin * s->row_width, reg_row_count, h->l2[0], st2);
        if (e != hipSuccess) return hip_check(e, "embedding l2");
        nreg_emb = ncf::kUpdateGrid;
    }
    e = ncf::launch_summary(L, ws, fb.nbce, fb.nmet, fb.n_groups, nreg_emb, nreg_mlp, summary, st2);
    if (e != hipSuccess) return hip_check(e, "summary");
    e = ncf::launch_emb_grad_dense(*s, L, ws, emb_grad, st, grad_row_begin);
    if (e != hipSuccess) return hip_check(e, "dense embedding gradient");
    return hip_check(join_side(st, ss), "side-stream join");
}

int ncf_forward_backward(const ncf_shape_t* s, const ncf_model_t* model, const ncf_hyper_t* h, const int32_t* users,
                         const int32_t* items, const float* labels, int64_t n, float* emb_grad, float* mlp_grad,
                         float* summary, float* probs_out, int64_t reg_row_begin, int64_t reg_row_count,
                         int32_t include_dense_reg, void* ws, size_t ws_bytes, void* stream) {
    return forward_backward_rows(s, model, h, users, items, labels, n, 0, emb_grad, mlp_grad, summary, probs_out,
                                 reg_row_begin, reg_row_count, include_dense_reg, ws, ws_bytes, stream);
}

int ncf_forward_backward_part(const ncf_shape_t* s, const ncf_model_t* model, const ncf_hyper_t* h,
                              const int32_t* users, const int32_t* items, const float* labels, int64_t n,
                              int64_t shared_row_begin, float* shared_grad, float* mlp_grad, float* summary,
                              float* probs_out, int64_t reg_row_begin, int64_t reg_row_count,
                              int32_t include_dense_reg, void* ws, size_t ws_bytes, void* stream) {
    if (!s) return fail(NCF_EINVAL, "NULL shape");
    if (shared_row_begin < 0 || shared_row_begin > s->num_rows) return fail(NCF_EINVAL, "invalid shared row range");
    return forward_backward_rows(s, model, h, users, items, labels, n, shared_row_begin, shared_grad, mlp_grad, summary,
                                 probs_out, reg_row_begin, reg_row_count, include_dense_reg, ws, ws_bytes, stream);
}

static int check_lazy_dp(const ncf_shape_t* s, const ncf_model_t* model, const ncf_optim_t* optim,
                         const ncf_hyper_t* h) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (!model || !model->emb) return fail(NCF_EINVAL, "NULL device pointer");
    if (!optim || !optim->step || !optim->row_step ||
        (h->optimizer == NCF_OPT_ADAM && (!optim->emb_m || !optim->emb_v)))
        return fail(NCF_EINVAL, "deferred decay needs the optimizer state and row_step");
    if (h->lazy_rows <= 0 || h->lazy_rows > s->num_rows)
        return fail(NCF_EINVAL, "hyper->lazy_rows must be in [1, num_rows], got %d", h->lazy_rows);
    if (h->l2[0] != 0.0f)
        return fail(NCF_EINVAL, "deferred decay (row_step) needs the embedding L2 off: the loss sums the whole table");
    return 0;
}

int ncf_forward_backward_part_lazy(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim,
                                   const ncf_hyper_t* h, const int32_t* users, const int32_t* items,
                                   const float* labels, int64_t n, float* shared_grad, float* mlp_grad, float* summary,
                                   float* probs_out, int32_t include_dense_reg, void* ws, size_t ws_bytes,
                                   void* stream) {
    if (int r = check_lazy_dp(s, model, optim, h)) return r;
    if (h->index_ready == 1) return fail(NCF_EINVAL, "index_ready = 1 (ncf_build_index) is not used here: count ahead");
    return forward_backward_rows(s, model, h, users, items, labels, n, h->lazy_rows, shared_grad, mlp_grad, summary,
                                 probs_out, 0, 0, include_dense_reg, ws, ws_bytes, stream, optim);
}

int ncf_update_rows_lazy(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                         int64_t n, const int32_t* next_users, const int32_t* next_items, int64_t n_next, void* ws,
                         size_t ws_bytes, void* stream) {
    if (int r = check_lazy_dp(s, model, optim, h)) return r;
    if ((next_users || next_items) && (!next_users || !next_items || n_next != n || h->optimizer != NCF_OPT_ADAM))
        return fail(NCF_EINVAL, "next batch: NULL ids, n_next != n, or not Adam");
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    prof_begin(NCF_K_EMB_UPDATE, st);
    hipError_t e = ncf::launch_emb_update_touched(*s, L, ws, model->emb, optim->emb_m, optim->emb_v, optim->row_step,
                                                  optim->step, *h, st, next_users, next_items,
                                                  next_users ? n_next : 0, nullptr, index_fold(*s, h));
    prof_end(NCF_K_EMB_UPDATE, st);
    if (e != hipSuccess) return hip_check(e, "touched-row update");
    if (next_users) {
        e = ncf::launch_scan_ahead(L, ws, s->num_rows, st);
        if (e != hipSuccess) return hip_check(e, "scan ahead");
    }
    return 0;
}

}  // extern "C"

namespace ncf {

// The one-call user-partitioned step's halves (ncf_comm.hip).  hyper->index_ready 3: the previous
// one-call step counted this batch, scanned the counts and caught its own stale rows up, so —
// where the in-kernel fill runs (fill_in_kernel; batches of 2,048 samples and up, every L2 factor
// zero, one stream) — the forward/backward launch fills the index (its unsorted lists), the
// gradient tail orders each item row's list itself (launch_part_tail_unsorted) and the own-user
// update orders the user rows' (k_emb_adam_touched<true>): no index-build, list-sort or catch-up
// launch in the step (round 6; the round-5 step built the next index with two more launches).
// Otherwise (or index_ready 2, the call-by-call path's state) the index is built here from the
// counts as ncf_forward_backward_part_lazy does.  A fill overflow (ids changed after they were
// counted) is flagged, never dropped: a rank that skipped its step would leave the replicas apart.
int dp_forward_backward(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                        const int32_t* users, const int32_t* items, const float* labels, int64_t n, float* shared_grad,
                        float* mlp_grad, float* summary, int32_t include_dense_reg, void* ws, size_t ws_bytes,
                        void* stream, bool* filled) {
    *filled = false;
    if (int r = check_lazy_dp(s, model, optim, h)) return r;
    if (int r = check_train_args(s, model, h, users, items, labels, n)) return r;
    if (!shared_grad || !mlp_grad || !summary) return fail(NCF_EINVAL, "NULL gradient output");
    ncf_hyper_t h2 = *h;
    if (h->index_ready == 3) h2.index_ready = 2;  // counted and scanned ahead
    WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    const int fmode = h->index_ready == 3 && n >= 2048 && side_stream_mode() == 0 &&
                              part_tail_foldable(*s, *h, 1 << 30)
                          ? fill_in_kernel(*s, L, &h2, n)
                          : 0;
    if (!fmode)
        return forward_backward_rows(s, model, &h2, users, items, labels, n, h->lazy_rows, shared_grad, mlp_grad,
                                     summary, nullptr, 0, 0, include_dense_reg, ws, ws_bytes, stream, optim);
    hipStream_t st = (hipStream_t)stream;
    FillArgs fa = fill_args(*s, L, ws);
    fa.stale_step = nullptr;  // flagged, not dropped
    if (fmode == 2) {
        prof_begin(NCF_K_INDEX, st);
        hipError_t e = launch_fill_ahead(fa, users, items, n, index_fold(*s, &h2), st);
        prof_end(NCF_K_INDEX, st);
        if (e != hipSuccess) return hip_check(e, "index fill");
    }
    FbOut fb;
    if (int r = run_fb(*s, L, model, &h2, users, items, labels, n, ws, nullptr, &fb, st, false, nullptr, nullptr,
                       fmode == 1 ? &fa : nullptr, fmode == 2))
        return r;
    if (!part_tail_foldable(*s, *h, fb.nslab))
        return fail(NCF_EHIP, "in-kernel fill: %d slabs do not take the two-level reduction", fb.nslab);
    *filled = true;
    return hip_check(launch_part_tail_unsorted(*s, L, ws, shared_grad, h->lazy_rows, mlp_grad, fb.nslab, fb.nbce,
                                               fb.nmet, fb.n_groups, summary, st),
                     "gradient tail");
}

// The own users' touched-row update (+ the next batch counted, its own stale rows caught up ahead,
// and its counts scanned for the next fill): `filled` — this step's lists came from the in-kernel
// fill (dp_forward_backward)
int dp_update_rows(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h, int64_t n,
                   const int32_t* next_users, const int32_t* next_items, int64_t n_next, void* ws, size_t ws_bytes,
                   void* stream, bool filled, bool scan_ahead) {
    if (int r = check_lazy_dp(s, model, optim, h)) return r;
    if ((next_users || next_items) && (!next_users || !next_items || n_next != n || h->optimizer != NCF_OPT_ADAM))
        return fail(NCF_EINVAL, "next batch: NULL ids, n_next != n, or not Adam");
    WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    prof_begin(NCF_K_EMB_UPDATE, st);
    hipError_t e = launch_emb_update_touched(*s, L, ws, model->emb, optim->emb_m, optim->emb_v, optim->row_step,
                                             optim->step, *h, st, next_users, next_items, next_users ? n_next : 0,
                                             nullptr, index_fold(*s, h), nullptr, nullptr, filled, false);
    prof_end(NCF_K_EMB_UPDATE, st);
    if (e != hipSuccess) return hip_check(e, "touched-row update");
    if (next_users && scan_ahead) {  // (else the caller's stats launch scans: launch_stats(..., scan_ahead))
        e = launch_scan_ahead(L, ws, s->num_rows, st);
        if (e != hipSuccess) return hip_check(e, "scan ahead");
    }
    return 0;
}

}  // namespace ncf

extern "C" {

int ncf_build_index(const ncf_shape_t* s, const ncf_hyper_t* h, const int32_t* users, const int32_t* items,
                    int64_t n, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    if (h)
        if (int r = check_hyper(h)) return r;
    if (!users || !items) return fail(NCF_EINVAL, "NULL device pointer");
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    prof_begin(NCF_K_INDEX, st);
    hipError_t e = ncf::launch_index_build(*s, L, ws, users, items, n, st, false, false, false, index_fold(*s, h));
    prof_end(NCF_K_INDEX, st);
    return hip_check(e, "index build");
}

int ncf_update_rows(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                    int64_t n, int64_t row_begin, int64_t row_count, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (!model || !model->emb) return fail(NCF_EINVAL, "NULL device pointer");
    if (!optim || !optim->step || (h->optimizer == NCF_OPT_ADAM && (!optim->emb_m || !optim->emb_v)))
        return fail(NCF_EINVAL, "NULL optimizer state");
    if (row_begin < 0 || row_count < 0 || row_begin + row_count > s->num_rows)
        return fail(NCF_EINVAL, "invalid row range");
    // the per-sample rows, list and offsets sit where the layout of the preceding batch n put them
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    const int64_t off = row_begin * s->row_width;
    prof_begin(NCF_K_EMB_UPDATE, st);
    hipError_t e = ncf::launch_emb_update(*s, L, ws, model->emb + off, optim->emb_m ? optim->emb_m + off : nullptr,
                                          optim->emb_v ? optim->emb_v + off : nullptr, optim->step, *h, nullptr,
                                          row_count, st, nullptr, row_begin);
    prof_end(NCF_K_EMB_UPDATE, st);
    return hip_check(e, "local row update");
}

int ncf_evaluate(const ncf_shape_t* s, const ncf_model_t* model, const ncf_hyper_t* h, const int32_t* users,
                 const int32_t* items, const float* labels, int64_t n, double* stats, float* probs_out, void* ws,
                 size_t ws_bytes, void* stream) {
    if (int r = check_train_args(s, model, h, users, items, labels, n)) return r;
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    float* probs = ncf::at<float>(ws, L.probs);
    int nbce = 0;
    hipError_t e = launch_predict(*s, h, L, ws, model->emb, model->mlp, users, items, labels, n, probs,
                                  ncf::table_ids(*s), &nbce, st);
    if (e != hipSuccess) return hip_check(e, "forward");
    const int64_t ng = n / h->group;
    int nmet = 0;
    e = ncf::launch_group_metrics(probs, labels, ng, h->group, h->k, nullptr, nullptr, ncf::at<float>(ws, L.part_hit),
                                  ncf::at<float>(ws, L.part_dcg), &nmet, st);
    if (e != hipSuccess) return hip_check(e, "metrics");
    float* summary = ncf::at<float>(ws, L.summary);
    int nreg_emb = 0, nreg_mlp = 0;
    if (h->l2[0] != 0.0f) {
        e = ncf::launch_emb_reg(*s, L, ws, model->emb, s->num_rows, h->l2[0], st);
        if (e != hipSuccess) return hip_check(e, "embedding l2");
        nreg_emb = ncf::kUpdateGrid;
    }
    e = ncf::launch_mlp_update(*s, L, ws, model->mlp, nullptr, nullptr, nullptr, *h, 0, model->mlp, nullptr, false,
                               &nreg_mlp, st, true);
    if (e != hipSuccess) return hip_check(e, "dense l2");
    e = ncf::launch_summary(L, ws, nbce, nmet, (float)ng, nreg_emb, nreg_mlp, summary, st);
    if (e != hipSuccess) return hip_check(e, "summary");
    if (probs_out) {
        e = hipMemcpyAsync(probs_out, probs, (size_t)n * 4, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return hip_check(e, "probs copy");
    }
    e = ncf::launch_stats(L, ws, summary, 0, 0, h->inv_batch, stats, nullptr, false, st);
    return hip_check(e, "stats");
}

int ncf_apply_update(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                     int64_t row_begin, int64_t row_count, const float* emb_grad, const float* mlp_grad,
                     const float* summary, double* stats, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (!model || !model->emb || !model->mlp || !mlp_grad || !summary || (row_count > 0 && !emb_grad))
        return fail(NCF_EINVAL, "NULL device pointer");
    if (!optim || !optim->step || (h->optimizer == NCF_OPT_ADAM &&
                                   (!optim->emb_m || !optim->emb_v || !optim->mlp_m || !optim->mlp_v)))
        return fail(NCF_EINVAL, "NULL optimizer state");
    if (row_begin < 0 || row_count < 0 || row_begin > s->num_rows) return fail(NCF_EINVAL, "invalid row range");
    if (row_begin + row_count > s->num_rows) row_count = s->num_rows - row_begin;
    ncf::WsLayout L;
    if (int r = check_ws(*s, 1, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    if (row_count > 0 && side_stream_mode() == 0 && h->l2[0] == 0.0f && ncf::part_tail_foldable(*s, *h, 1 << 30)) {
        // L2 off, one stream: the dense layers' step runs in extra workgroups of the row update
        prof_begin(NCF_K_EMB_UPDATE, st);
        hipError_t e = ncf::launch_apply_fused(*s, model->emb + row_begin * s->row_width, optim->emb_m, optim->emb_v,
                                               emb_grad, row_count, model->mlp, optim->mlp_m, optim->mlp_v, mlp_grad,
                                               optim->step, *h, st);
        prof_end(NCF_K_EMB_UPDATE, st);
        if (e != hipSuccess) return hip_check(e, "embedding + dense update");
        e = ncf::launch_stats(L, ws, summary, 0, 0, h->inv_batch, stats, optim->step, true, st);
        return hip_check(e, "stats");
    }
    SideStream* ss = nullptr;
    hipStream_t st2 = fork_side(st, &ss);
    int nreg_mlp = 0;
    prof_begin(NCF_K_MLP_UPDATE, st2);
    hipError_t e = ncf::launch_mlp_update(*s, L, ws, model->mlp, optim->mlp_m, optim->mlp_v, optim->step, *h, 0,
                                          mlp_grad, nullptr, true, &nreg_mlp, st2);
    prof_end(NCF_K_MLP_UPDATE, st2);
    if (e != hipSuccess) return hip_check(e, "dense update");
    if (row_count > 0) {
        prof_begin(NCF_K_EMB_UPDATE, st);
        e = ncf::launch_emb_update(*s, L, ws, model->emb + row_begin * s->row_width, optim->emb_m, optim->emb_v,
                                   optim->step, *h, emb_grad, row_count, st);
        prof_end(NCF_K_EMB_UPDATE, st);
        if (e != hipSuccess) return hip_check(e, "embedding update");
    }
    e = join_side(st, ss);
    if (e != hipSuccess) return hip_check(e, "side-stream join");
    // the L2 loss of the pre-update weights arrives in summary[NCF_SUM_REG]
    e = ncf::launch_stats(L, ws, summary, 0, 0, h->inv_batch, stats, optim->step, true, st);
    return hip_check(e, "stats");
}

// ------------------------------------------------------------ row-sharded data parallelism

int ncf_shard_rows(const ncf_shape_t* s, int32_t world, int64_t* rows) {
    if (int r = check_shape(s)) return r;
    if (int r = check_world(world)) return r;
    if (!rows) return fail(NCF_EINVAL, "rows is NULL");
    *rows = ncf::shard_rows_of(s->num_rows, world);
    return 0;
}

int ncf_shard_workspace_size(const ncf_shape_t* s, int64_t max_batch, int32_t world, size_t* bytes) {
    if (int r = check_shape(s)) return r;
    if (int r = check_world(world)) return r;
    if (!bytes) return fail(NCF_EINVAL, "bytes is NULL");
    if (max_batch <= 0 || max_batch > ncf::kMaxBatch)
        return fail(NCF_EINVAL, "max_batch must be in [1, %lld]", (long long)ncf::kMaxBatch);
    *bytes = ncf::make_layout(*s, max_batch, world).total;
    return 0;
}

int ncf_shard_workspace_init(const ncf_shape_t* s, int64_t max_batch, int32_t world, void* ws, size_t ws_bytes,
                             void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_world(world)) return r;
    ncf::WsLayout L = ncf::make_layout(*s, max_batch, world);
    if (!ws || ws_bytes < L.total) return fail(NCF_EINVAL, "workspace too small");
    return hip_check(hipMemsetAsync(ws, 0, L.persistent_end, (hipStream_t)stream), "hipMemsetAsync");
}

int ncf_shard_plan(const ncf_shape_t* s, const ncf_hyper_t* h, int32_t world, const int32_t* users,
                   const int32_t* items, int64_t n, int32_t* uniq_rows, int32_t* send_counts, void* ws, size_t ws_bytes,
                   void* stream) {
    if (int r = check_shape(s)) return r;
    if (h)
        if (int r = check_hyper(h)) return r;
    if (int r = check_world(world)) return r;
    if (!users || !items || !uniq_rows || !send_counts) return fail(NCF_EINVAL, "NULL device pointer");
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L, world)) return r;
    hipStream_t st = (hipStream_t)stream;
    prof_begin(NCF_K_INDEX, st);
    hipError_t e = ncf::launch_shard_plan(*s, L, ws, users, items, n, uniq_rows, send_counts, st, index_fold(*s, h));
    prof_end(NCF_K_INDEX, st);
    return hip_check(e, "shard plan");
}

int ncf_gather_rows(const ncf_shape_t* s, const float* table, int64_t table_rows, const int32_t* rows, int64_t m,
                    float* out, void* stream) {
    if (int r = check_shape(s)) return r;
    if (m < 0 || table_rows < 0) return fail(NCF_EINVAL, "negative row count");
    if (m > 0 && (!table || !rows || !out)) return fail(NCF_EINVAL, "NULL device pointer");
    return hip_check(ncf::launch_gather_rows(*s, table, table_rows, rows, m, out, (hipStream_t)stream),
                     "gather rows");
}

// The shard as a table of its own: S rows, every one under deferred decay (lazy_rows 0)
static ncf_shape_t shard_shape(const ncf_shape_t& s, int world) {
    ncf_shape_t o = s;
    o.num_rows = ncf::shard_rows_of(s.num_rows, world);
    return o;
}

static int check_shard_lazy(const ncf_shape_t* s, const ncf_model_t* model, const ncf_optim_t* optim,
                            const ncf_hyper_t* h, int world) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (int r = check_world(world)) return r;
    if (!model || !model->emb) return fail(NCF_EINVAL, "NULL device pointer");
    if (!optim || !optim->step || !optim->row_step || (h->optimizer == NCF_OPT_ADAM && (!optim->emb_m || !optim->emb_v)))
        return fail(NCF_EINVAL, "deferred decay needs the optimizer state and row_step");
    if (h->l2[0] != 0.0f)
        return fail(NCF_EINVAL, "deferred decay (row_step) needs the embedding L2 off: the loss sums the whole table");
    return 0;
}

int ncf_shard_serve_rows(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                         int32_t world, const int32_t* rows, int64_t m, float* out, void* ws, size_t ws_bytes,
                         void* stream) {
    if (int r = check_shard_lazy(s, model, optim, h, world)) return r;
    const int64_t S = ncf::shard_rows_of(s->num_rows, world);
    if (m < 0 || m > (int64_t)world * S)
        return fail(NCF_EINVAL, "served row count %lld outside [0, world * shard_rows]", (long long)m);
    if (m > 0 && (!rows || !out)) return fail(NCF_EINVAL, "NULL device pointer");
    ncf::WsLayout L;
    if (int r = check_ws(*s, 1, ws, ws_bytes, &L, world)) return r;
    hipStream_t st = (hipStream_t)stream;
    const ncf::WsLayout O = ncf::owner_view(L, m);
    const ncf_shape_t ss = shard_shape(*s, world);
    ncf_hyper_t hs = *h;
    hs.lazy_rows = 0;
    // the owner index of the served rows (ascending entry = ascending source rank): the served
    // rows' list for the catch-up now, the per-row entry lists for ncf_shard_apply_update later
    prof_begin(NCF_K_INDEX, st);
    hipError_t e = ncf::launch_owner_touched_index(L, ws, rows, m, st);
    prof_end(NCF_K_INDEX, st);
    if (e != hipSuccess) return hip_check(e, "owner index");
    if (h->optimizer == NCF_OPT_ADAM) {
        // the served rows' missed zero-gradient steps (p only: the update re-derives m, v)
        prof_begin(NCF_K_CATCHUP, st);
        e = ncf::launch_emb_catchup(ss, O, ws, model->emb, optim->emb_m, optim->emb_v, optim->row_step, optim->step,
                                    hs, false, st);
        prof_end(NCF_K_CATCHUP, st);
        if (e != hipSuccess) return hip_check(e, "served-row catch-up");
    }
    return hip_check(ncf::launch_gather_rows(*s, model->emb, S, rows, m, out, st), "gather rows");
}

int ncf_shard_flush(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                    int32_t world, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shard_lazy(s, model, optim, h, world)) return r;
    ncf::WsLayout L;
    if (int r = check_ws(*s, 1, ws, ws_bytes, &L, world)) return r;
    hipStream_t st = (hipStream_t)stream;
    const ncf_shape_t ss = shard_shape(*s, world);
    ncf_hyper_t hs = *h;
    hs.lazy_rows = 0;
    hipError_t e = ncf::launch_emb_catchup(ss, ncf::owner_view(L, 1), ws, model->emb, optim->emb_m, optim->emb_v,
                                           optim->row_step, optim->step, hs, true, st);
    if (e != hipSuccess) return hip_check(e, "shard flush");
    return hip_check(ncf::launch_row_step_fill(optim->row_step, ss.num_rows, optim->step, st), "row-step fill");
}

int ncf_shard_forward_backward(const ncf_shape_t* s, const ncf_model_t* model, const ncf_hyper_t* h, int32_t world,
                               const float* labels, int64_t n, float* uniq_grad, float* mlp_grad, float* summary,
                               float* probs_out, const float* reg_table, int64_t reg_rows,
                               int32_t include_dense_reg, void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (int r = check_world(world)) return r;
    if (!model || !model->emb || !model->mlp || !labels) return fail(NCF_EINVAL, "NULL device pointer");
    if (!uniq_grad || !mlp_grad || !summary) return fail(NCF_EINVAL, "NULL gradient output");
    if (n % h->group)
        return fail(NCF_EINVAL, "Batch size must be divisible by (num_negs_per_pos + 1). Found: batch_size=%lld, "
                    "group=%d", (long long)n, h->group);
    if (reg_rows < 0 || (h->l2[0] != 0.0f && reg_rows > 0 && !reg_table))
        return fail(NCF_EINVAL, "invalid regulariser rows");
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L, world)) return r;
    hipStream_t st = (hipStream_t)stream;
    FbOut fb;
    if (int r = run_fb(*s, L, model, h, nullptr, nullptr, labels, n, ws, probs_out, &fb, st, true)) return r;
    SideStream* ss = nullptr;
    hipStream_t st2 = fork_side(st, &ss);
    int nreg_mlp = 0, nreg_emb = 0;
    hipError_t e = ncf::launch_mlp_update(*s, L, ws, model->mlp, nullptr, nullptr, nullptr, *h, fb.nslab, nullptr,
                                          mlp_grad, false, &nreg_mlp, st2, include_dense_reg != 0);
    if (e != hipSuccess) return hip_check(e, "dense-layer gradient");
    if (h->l2[0] != 0.0f && reg_rows > 0) {
        e = ncf::launch_emb_reg(*s, L, ws, reg_table, reg_rows, h->l2[0], st2);
        if (e != hipSuccess) return hip_check(e, "embedding l2");
        nreg_emb = ncf::kUpdateGrid;
    }
    e = ncf::launch_summary(L, ws, fb.nbce, fb.nmet, fb.n_groups, nreg_emb, nreg_mlp, summary, st2);
    if (e != hipSuccess) return hip_check(e, "summary");
    e = ncf::launch_uniq_grad(*s, L, ws, n, uniq_grad, st);
    if (e != hipSuccess) return hip_check(e, "compact embedding gradient");
    return hip_check(join_side(st, ss), "side-stream join");
}

int ncf_shard_apply_update(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h,
                           int32_t world, const int32_t* recv_rows, const float* recv_grad, int64_t m,
                           const float* mlp_grad, const float* summary, double* stats, void* ws, size_t ws_bytes,
                           void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (int r = check_world(world)) return r;
    if (!model || !model->emb || !model->mlp || !mlp_grad || !summary || (m > 0 && (!recv_rows || !recv_grad)))
        return fail(NCF_EINVAL, "NULL device pointer");
    if (!optim || !optim->step || (h->optimizer == NCF_OPT_ADAM &&
                                   (!optim->emb_m || !optim->emb_v || !optim->mlp_m || !optim->mlp_v)))
        return fail(NCF_EINVAL, "NULL optimizer state");
    const int64_t S = ncf::shard_rows_of(s->num_rows, world);
    if (m < 0 || m > (int64_t)world * S)
        return fail(NCF_EINVAL, "received row count %lld outside [0, world * shard_rows]", (long long)m);
    if (optim->row_step) {
        // deferred decay: the served rows only, through the owner index ncf_shard_serve_rows built
        // for these m entries (their gradients arrive in the same order as their ids did)
        if (int r = check_shard_lazy(s, model, optim, h, world)) return r;
        ncf::WsLayout L;
        if (int r = check_ws(*s, 1, ws, ws_bytes, &L, world)) return r;
        hipStream_t st = (hipStream_t)stream;
        const ncf::WsLayout O = ncf::owner_view(L, m);
        const ncf_shape_t ss = shard_shape(*s, world);
        ncf_hyper_t hs = *h;
        hs.lazy_rows = 0;
        int nreg_mlp = 0;
        prof_begin(NCF_K_MLP_UPDATE, st);
        hipError_t e = ncf::launch_mlp_update(*s, L, ws, model->mlp, optim->mlp_m, optim->mlp_v, optim->step, *h, 0,
                                              mlp_grad, nullptr, true, &nreg_mlp, st);
        prof_end(NCF_K_MLP_UPDATE, st);
        if (e != hipSuccess) return hip_check(e, "dense update");
        if (m > 0) {
            prof_begin(NCF_K_EMB_UPDATE, st);
            e = ncf::launch_emb_update_touched(ss, O, ws, model->emb, optim->emb_m, optim->emb_v, optim->row_step,
                                               optim->step, hs, st, nullptr, nullptr, 0, nullptr, 0, nullptr,
                                               recv_grad);
            prof_end(NCF_K_EMB_UPDATE, st);
            if (e != hipSuccess) return hip_check(e, "served-row update");
        }
        e = ncf::launch_stats(L, ws, summary, 0, 0, h->inv_batch, stats, optim->step, true, st);
        return hip_check(e, "stats");
    }
    // smallest batch whose layout holds m received rows (the workspace was sized for a larger one)
    int64_t nb = (m + 2 * world - 1) / (2 * world);
    if (nb < 1) nb = 1;
    ncf::WsLayout L;
    if (int r = check_ws(*s, nb, ws, ws_bytes, &L, world)) return r;
    hipStream_t st = (hipStream_t)stream;
    prof_begin(NCF_K_INDEX, st);
    hipError_t e = ncf::launch_owner_index(L, ws, recv_rows, m, st);
    prof_end(NCF_K_INDEX, st);
    if (e != hipSuccess) return hip_check(e, "owner index");
    SideStream* ss = nullptr;
    hipStream_t st2 = fork_side(st, &ss);
    int nreg_mlp = 0;
    prof_begin(NCF_K_MLP_UPDATE, st2);
    e = ncf::launch_mlp_update(*s, L, ws, model->mlp, optim->mlp_m, optim->mlp_v, optim->step, *h, 0, mlp_grad,
                               nullptr, true, &nreg_mlp, st2);
    prof_end(NCF_K_MLP_UPDATE, st2);
    if (e != hipSuccess) return hip_check(e, "dense update");
    prof_begin(NCF_K_EMB_UPDATE, st);
    e = ncf::launch_emb_update(*s, L, ws, model->emb, optim->emb_m, optim->emb_v, optim->step, *h, nullptr, S, st,
                               recv_grad);
    prof_end(NCF_K_EMB_UPDATE, st);
    if (e != hipSuccess) return hip_check(e, "embedding update");
    e = join_side(st, ss);
    if (e != hipSuccess) return hip_check(e, "side-stream join");
    e = ncf::launch_stats(L, ws, summary, 0, 0, h->inv_batch, stats, optim->step, true, st);
    return hip_check(e, "stats");
}

int ncf_shard_predict(const ncf_shape_t* s, const ncf_model_t* model, int32_t world, int64_t n, float* probs,
                      void* ws, size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_world(world)) return r;
    if (!model || !model->emb || !model->mlp || !probs) return fail(NCF_EINVAL, "NULL device pointer");
    ncf::WsLayout L;
    if (int r = check_ws(*s, n, ws, ws_bytes, &L, world)) return r;
    int nbce = 0;
    return hip_check(ncf::launch_predict_generic(*s, L, ws, model->emb, model->mlp, ncf::at<int32_t>(ws, L.cid_u),
                                                 ncf::at<int32_t>(ws, L.cid_i), nullptr, n, probs,
                                                 ncf::compact_ids(n), &nbce, (hipStream_t)stream),
                     "shard predict");
}

// ------------------------------------------------------------ deferred exact decay

int ncf_lazy_flush(const ncf_shape_t* s, ncf_model_t* model, ncf_optim_t* optim, const ncf_hyper_t* h, void* ws,
                   size_t ws_bytes, void* stream) {
    if (int r = check_shape(s)) return r;
    if (int r = check_hyper(h)) return r;
    if (!model || !model->emb || !optim || !optim->step || !optim->row_step)
        return fail(NCF_EINVAL, "NULL device pointer");
    if (h->optimizer == NCF_OPT_ADAM && (!optim->emb_m || !optim->emb_v)) return fail(NCF_EINVAL, "NULL Adam state");
    ncf::WsLayout L;
    if (int r = check_ws(*s, 1, ws, ws_bytes, &L)) return r;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = ncf::launch_emb_catchup(*s, L, ws, model->emb, optim->emb_m, optim->emb_v, optim->row_step,
                                           optim->step, *h, true, st);
    if (e != hipSuccess) return hip_check(e, "flush");
    return hip_check(ncf::launch_row_step_fill(optim->row_step, ncf::lazy_bound(*s, *h), optim->step, st),
                     "row-step fill");
}

// ------------------------------------------------------------ negative sampling

int ncf_sample_batch(const ncf_sampler_data_t* d, const int32_t* order, int64_t first, int32_t n_pos, int32_t negs,
                     uint64_t seed, uint64_t stream_id, int32_t* x_user, int32_t* x_item, float* labels, int32_t* err,
                     void* stream) {
    if (!d || !d->pos_users || !d->pos_items || !d->excl_ptr || !d->excl_items || !order || !x_user || !x_item ||
        !labels || !err)
        return fail(NCF_EINVAL, "NULL pointer");
    if (negs <= 0) return fail(NCF_EINVAL, "negatives_per_positive must be > 0, found %d", negs);
    if (d->num_users <= 0 || d->num_items <= 0) return fail(NCF_EINVAL, "num_users and num_items must be > 0");
    if (n_pos < 0 || first < 0 || first + n_pos > d->num_pos)
        return fail(NCF_EINVAL, "positives [%lld, %lld) outside the epoch order of %lld", (long long)first,
                    (long long)(first + n_pos), (long long)d->num_pos);
    hipStream_t st = (hipStream_t)stream;
    prof_begin(NCF_K_SAMPLE, st);
    hipError_t e = ncf::launch_sample_batch(d->pos_users, d->pos_items, d->excl_ptr, d->excl_items, d->num_users,
                                            d->num_items, order, first, n_pos, negs, seed, stream_id, x_user, x_item,
                                            labels, err, st);
    prof_end(NCF_K_SAMPLE, st);
    return hip_check(e, "sample batch");
}

// ------------------------------------------------------------ all-item scoring + top-k

int ncf_score_supported(const ncf_shape_t* s, int32_t precision) {
    if (check_shape(s)) return 0;
    if (precision == NCF_SCORE_FP32) return 1;
    if (precision == NCF_SCORE_FP16) return ncf::score_fast_supported(*s) ? 1 : 0;
    return 0;
}

int ncf_score_workspace_size(const ncf_shape_t* s, int64_t max_users, size_t* bytes) {
    if (int r = check_shape(s)) return r;
    if (!bytes) return fail(NCF_EINVAL, "bytes is NULL");
    if (max_users <= 0 || max_users > ((int64_t)1 << 26))
        return fail(NCF_EINVAL, "max_users must be in [1, 2^26], got %lld", (long long)max_users);
    *bytes = ncf::make_score_layout(*s, max_users).total;
    return 0;
}

int ncf_score_topk(const ncf_shape_t* s, const ncf_model_t* model, const int32_t* users, int64_t n, int32_t k,
                   int32_t precision, int32_t* top_items, float* top_scores, void* ws, size_t ws_bytes,
                   void* stream) {
    if (int r = check_shape(s)) return r;
    if (!model || !model->emb || !model->mlp || !users || !top_items || !top_scores || !ws)
        return fail(NCF_EINVAL, "NULL device pointer");
    if (k < 1 || k > NCF_SCORE_MAX_K) return fail(NCF_EINVAL, "k must be in [1, %d], got %d", NCF_SCORE_MAX_K, k);
    if (n <= 0) return 0;
    if (precision != NCF_SCORE_FP16 && precision != NCF_SCORE_FP32)
        return fail(NCF_EINVAL, "unknown scoring precision %d", precision);
    if (precision == NCF_SCORE_FP16 && !ncf::score_fast_supported(*s))
        return fail(NCF_EINVAL, "the fp16 MFMA scorer needs a 4-layer model with layers[1] <= 64, layers[2] <= 32, "
                    "layers[3] <= 32, gmf_dim <= 64 (use NCF_SCORE_FP32)");
    // nothing persists between calls: the layout for n users fits any workspace sized for >= n
    const ncf::ScoreLayout L = ncf::make_score_layout(*s, n);
    if (ws_bytes < L.total)
        return fail(NCF_EINVAL, "score workspace too small: %zu bytes for %lld users (need %zu)", ws_bytes,
                    (long long)n, L.total);
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    if (precision == NCF_SCORE_FP16) {
        e = ncf::launch_score_prep(*s, L, ws, model->emb, model->mlp, users, n, st);
        if (e != hipSuccess) return hip_check(e, "score preparation");
        prof_begin(NCF_K_SCORE, st);
        e = ncf::launch_score_main(*s, L, ws, n, k, top_items, top_scores, st);
        prof_end(NCF_K_SCORE, st);
        return hip_check(e, "score top-k");
    }
    const int I = s->num_items;
    if (I > ncf::kMaxBatch)
        return fail(NCF_EINVAL, "the fp32 scorer handles catalogues of up to %lld items", (long long)ncf::kMaxBatch);
    void* pws = ncf::at<char>(ws, L.pred_ws);
    ncf::WsLayout PL = ncf::make_layout(*s, L.chunk * I > ncf::kMaxBatch ? ncf::kMaxBatch : L.chunk * I);
    for (int64_t q0 = 0; q0 < n; q0 += L.chunk) {
        const int64_t nq = n - q0 < L.chunk ? n - q0 : L.chunk;
        int32_t* pu = ncf::at<int32_t>(ws, L.pu);
        int32_t* pi = ncf::at<int32_t>(ws, L.pi);
        float* probs = ncf::at<float>(ws, L.probs);
        e = ncf::launch_score_pairs(users + q0, nq, I, pu, pi, st);
        if (e != hipSuccess) return hip_check(e, "score pairs");
        int nbce = 0;
        e = launch_predict(*s, nullptr, PL, pws, model->emb, model->mlp, pu, pi, nullptr, nq * I, probs,
                           ncf::table_ids(*s), &nbce, st);
        if (e != hipSuccess) return hip_check(e, "score forward");
        e = ncf::launch_topk_rows(probs, nq, I, k, top_items + q0 * k, top_scores + q0 * k, st);
        if (e != hipSuccess) return hip_check(e, "score top-k");
    }
    return 0;
}

int ncf_profile_enable(int32_t kernel_mask, int32_t capacity) {
    g_prof.mask = kernel_mask < 0 ? 0u : (uint32_t)kernel_mask;
    g_prof.select = ~0u;
    g_prof.paused = false;
    for (int k = 0; k < 16; ++k) {
        ProfSlot& p = g_prof.slot[k];
        p.used = 0;
        if (!(g_prof.mask >> k & 1u)) continue;
        if (capacity < 1) return fail(NCF_EINVAL, "capacity must be >= 1");
        while ((int)p.start.size() < capacity) {
            hipEvent_t a, b;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)
                return fail(NCF_EHIP, "hipEventCreate failed");
            p.start.push_back(a);
            p.stop.push_back(b);
        }
    }
    return 0;
}

int ncf_profile_pause(int32_t paused) {
    g_prof.paused = paused != 0;
    return 0;
}

int ncf_profile_select(int32_t kernel_mask) {
    g_prof.select = (uint32_t)kernel_mask;
    return 0;
}

int ncf_profile_read(int32_t kernel_id, double* total_ms, int64_t* launches) {
    if (!total_ms || !launches || kernel_id < 0 || kernel_id > 15) return fail(NCF_EINVAL, "invalid argument");
    ProfSlot& p = g_prof.slot[kernel_id];
    double tot = 0.0;
    if (p.used > 0) {
        hipError_t e = hipEventSynchronize(p.stop[p.used - 1]);
        if (e != hipSuccess) return hip_check(e, "hipEventSynchronize");
    }
    for (size_t i = 0; i < p.used; ++i) {
        float ms = 0.f;
        hipError_t e = hipEventElapsedTime(&ms, p.start[i], p.stop[i]);
        if (e != hipSuccess) return hip_check(e, "hipEventElapsedTime");
        tot += ms;
    }
    *total_ms = tot;
    *launches = (int64_t)p.used;
    p.used = 0;
    return 0;
}

}  // extern "C"
