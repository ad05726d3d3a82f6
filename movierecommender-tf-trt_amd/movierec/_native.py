"""ctypes binding of the C ABI in ``include/movierec_ncf.h``.

The shared library is ``movierec/_lib/libmovierec_ncf.so`` (built in-tree by
``csrc/build.py`` / ``__graft_entry__.build()``).  There is no fallback: if
the library is missing or cannot be loaded, :func:`lib` raises — the HIP path
is the product.

``torch`` is imported first on purpose: the library's NEEDED
``libamdhip64.so.7`` then resolves to the HIP runtime PyTorch already loaded,
so torch streams and device pointers are valid inside the library.
"""

import ctypes
import os

import torch  # noqa: F401  (must precede the library load, see module doc)

NCF_MAX_LAYERS = 8
NCF_EINVAL = -1
NCF_EHIP = -2
NCF_OPT_ADAM = 0
NCF_OPT_SGD = 1
NCF_NUM_STATS = 8
NCF_NUM_SUMMARY = 8
NCF_WSERR_ID_RANGE, NCF_WSERR_STALE_COUNT, NCF_WSERR_FOLD = 1, 4, 8
NCF_ROW_PRISTINE = 0x7fffffff   # row_step mark of a row whose Adam moments are exactly +0
FB_KERNELS = {0: "generic", 2: "fused-mfma-tile", 3: "fused-mfma-unit", 4: "fused-mfma-wave",
              5: "layered-mfma"}
SUM_BCE, SUM_HIT, SUM_DCG, SUM_GROUPS, SUM_REG = range(5)
STAT_LOSS_SUM, STAT_HR_SUM, STAT_DCG_SUM, STAT_STEPS, STAT_LAST_LOSS, STAT_LAST_HR, STAT_LAST_DCG, STAT_BCE_SUM = \
    range(8)

LIB_PATH = os.environ.get("NCF_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                      "libmovierec_ncf.so")

_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_vp = ctypes.c_void_p


class NcfShape(ctypes.Structure):
    _fields_ = [("num_users", _i32), ("num_items", _i32), ("num_layers", _i32), ("gmf_dim", _i32),
                ("layers", _i32 * NCF_MAX_LAYERS),
                ("du", _i32), ("di", _i32), ("gmf_stride", _i32), ("row_width", _i32),
                ("num_rows", _i64), ("out_features", _i32), ("mlp_params", _i32),
                ("layer_off", _i32 * NCF_MAX_LAYERS), ("fast_path", _i32), ("reserved", _i32 * 7)]


class NcfModel(ctypes.Structure):
    _fields_ = [("emb", _vp), ("mlp", _vp)]


class NcfOptim(ctypes.Structure):
    _fields_ = [("emb_m", _vp), ("emb_v", _vp), ("mlp_m", _vp), ("mlp_v", _vp), ("step", _vp), ("row_step", _vp)]


class NcfHyper(ctypes.Structure):
    _fields_ = [("optimizer", _i32), ("lr", _f32), ("beta_1", _f32), ("beta_2", _f32), ("epsilon", _f32),
                ("l2", _f32 * NCF_MAX_LAYERS), ("group", _i32), ("k", _i32), ("inv_batch", _f32),
                ("force_generic", _i32), ("index_ready", _i32), ("mlp_bf16", _i32), ("lazy_rows", _i32),
                ("reserved", _i32 * 3)]


class NcfSamplerData(ctypes.Structure):
    _fields_ = [("pos_users", _vp), ("pos_items", _vp), ("num_pos", _i64), ("excl_ptr", _vp), ("excl_items", _vp),
                ("num_users", _i32), ("num_items", _i32)]


_P = ctypes.POINTER
_SIGNATURES = {
    "ncf_abi_version": (ctypes.c_int, []),
    "ncf_last_error": (ctypes.c_char_p, []),
    "ncf_build_info": (ctypes.c_char_p, []),
    "ncf_shape_init": (ctypes.c_int, [_P(NcfShape), _i32, _i32, _P(_i32), _i32, _i32]),
    "ncf_workspace_size": (ctypes.c_int, [_P(NcfShape), _i64, _P(ctypes.c_size_t)]),
    "ncf_workspace_init": (ctypes.c_int, [_P(NcfShape), _i64, _vp, ctypes.c_size_t, _vp]),
    "ncf_workspace_flags": (ctypes.c_int, [_P(NcfShape), _i64, _vp, ctypes.c_size_t, _vp, _vp]),
    "ncf_shard_workspace_flags": (ctypes.c_int, [_P(NcfShape), _i64, _i32, _vp, ctypes.c_size_t, _vp, _vp]),
    "ncf_workspace_discard_counts": (ctypes.c_int, [_P(NcfShape), _i64, _vp, ctypes.c_size_t, _vp]),
    "ncf_predict": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _vp, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_rank": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp]),
    "ncf_group_metrics": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp]),
    "ncf_train_step": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _vp, _vp, _vp, _i64,
                                      _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_train_step_ahead": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _vp, _vp, _vp,
                                            _i64, _vp, _vp, _i64, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_evaluate": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfHyper), _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                    ctypes.c_size_t, _vp]),
    "ncf_forward_backward": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfHyper), _vp, _vp, _vp, _i64, _vp, _vp,
                                            _vp, _vp, _i64, _i64, _i32, _vp, ctypes.c_size_t, _vp]),
    "ncf_forward_backward_part": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfHyper), _vp, _vp, _vp, _i64,
                                                 _i64, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp, ctypes.c_size_t,
                                                 _vp]),
    "ncf_update_rows": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _i64, _i64, _i64, _vp,
                                       ctypes.c_size_t, _vp]),
    "ncf_fb_kernel": (ctypes.c_int, [_P(NcfShape), _P(NcfHyper), _i64]),
    "ncf_build_index": (ctypes.c_int, [_P(NcfShape), _P(NcfHyper), _vp, _vp, _i64, _vp, ctypes.c_size_t, _vp]),
    "ncf_forward_backward_part_lazy": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _vp,
                                                      _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _vp, ctypes.c_size_t,
                                                      _vp]),
    "ncf_update_rows_lazy": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _i64, _vp, _vp,
                                            _i64, _vp, ctypes.c_size_t, _vp]),
    "ncf_comm_unique_id": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "ncf_comm_init": (ctypes.c_int, [_i32, _i32, _vp, ctypes.c_size_t, _P(_vp)]),
    "ncf_comm_destroy": (ctypes.c_int, [_vp]),
    "ncf_comm_allreduce": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "ncf_comm_timing": (ctypes.c_int, [_vp, _i32]),
    "ncf_comm_timing_read": (ctypes.c_int, [_vp, _vp, _P(_i64)]),
    "ncf_user_dp_step": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _vp, _vp, _vp, _i64,
                                        _vp, _vp, _i64, _vp, _i32, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_user_dp_step_split": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _vp, _vp, _vp,
                                              _i64, _vp, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp,
                                              ctypes.c_size_t, _vp]),
    "ncf_lazy_flush": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _vp, ctypes.c_size_t,
                                      _vp]),
    "ncf_apply_update": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _i64, _i64, _vp, _vp,
                                        _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_shard_rows": (ctypes.c_int, [_P(NcfShape), _i32, _P(_i64)]),
    "ncf_shard_workspace_size": (ctypes.c_int, [_P(NcfShape), _i64, _i32, _P(ctypes.c_size_t)]),
    "ncf_shard_workspace_init": (ctypes.c_int, [_P(NcfShape), _i64, _i32, _vp, ctypes.c_size_t, _vp]),
    "ncf_shard_plan": (ctypes.c_int, [_P(NcfShape), _P(NcfHyper), _i32, _vp, _vp, _i64, _vp, _vp, _vp,
                                      ctypes.c_size_t, _vp]),
    "ncf_gather_rows": (ctypes.c_int, [_P(NcfShape), _vp, _i64, _vp, _i64, _vp, _vp]),
    "ncf_shard_forward_backward": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfHyper), _i32, _vp, _i64, _vp,
                                                  _vp, _vp, _vp, _vp, _i64, _i32, _vp, ctypes.c_size_t, _vp]),
    "ncf_shard_apply_update": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _i32, _vp,
                                              _vp, _i64, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_shard_serve_rows": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _i32, _vp,
                                            _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_shard_flush": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _P(NcfOptim), _P(NcfHyper), _i32, _vp,
                                       ctypes.c_size_t, _vp]),
    "ncf_shard_predict": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _i32, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "ncf_sample_batch": (ctypes.c_int, [_P(NcfSamplerData), _vp, _i64, _i32, _i32, ctypes.c_uint64, ctypes.c_uint64,
                                        _vp, _vp, _vp, _vp, _vp]),
    "ncf_score_supported": (ctypes.c_int, [_P(NcfShape), _i32]),
    "ncf_score_workspace_size": (ctypes.c_int, [_P(NcfShape), _i64, _P(ctypes.c_size_t)]),
    "ncf_score_topk": (ctypes.c_int, [_P(NcfShape), _P(NcfModel), _vp, _i64, _i32, _i32, _vp, _vp, _vp,
                                      ctypes.c_size_t, _vp]),
    "ncf_profile_enable": (ctypes.c_int, [_i32, _i32]),
    "ncf_profile_read": (ctypes.c_int, [_i32, _P(ctypes.c_double), _P(_i64)]),
    "ncf_profile_pause": (ctypes.c_int, [_i32]),
    "ncf_profile_select": (ctypes.c_int, [_i32]),
}
EXPORTED = sorted(_SIGNATURES)
K_INDEX, K_FWD_BWD, K_EMB_UPDATE, K_MLP_UPDATE, K_METRICS, K_SCORE, K_SAMPLE, K_CATCHUP = 1, 2, 3, 4, 5, 6, 7, 8
NCF_SCORE_FP16, NCF_SCORE_FP32, NCF_SCORE_MAX_K = 0, 1, 32


def profile_enable(kernels, capacity):
    """Time the given launch groups (K_* ids) with HIP events on their streams."""
    mask = 0
    for k in kernels:
        mask |= 1 << k
    check(lib().ncf_profile_enable(mask, int(capacity)))


def profile_pause(paused):
    """Stop (True) / resume (False) attaching events to the enabled launch groups."""
    check(lib().ncf_profile_pause(1 if paused else 0))


def profile_select(kernels):
    """Of the enabled launch groups, attach events to these only (until the next call)."""
    mask = 0
    for k in kernels:
        mask |= 1 << k
    check(lib().ncf_profile_select(mask))


def profile_read(kernel):
    """(summed device ms, launches) of one launch group since profile_enable."""
    ms, n = ctypes.c_double(), ctypes.c_int64()
    check(lib().ncf_profile_read(int(kernel), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value

_lib = None
ABI_VERSION = 11  # include/movierec_ncf.h ncf_abi_version()


def lib():
    """Load (once) and return the library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libmovierec_ncf.so not found at %s — run __graft_entry__.build() "
                               "(there is no CPU fallback)" % LIB_PATH)
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        got = handle.ncf_abi_version()
        if got != ABI_VERSION:
            raise RuntimeError("libmovierec_ncf.so at %s has ABI %d, this binding expects %d: rebuild it "
                               "(__graft_entry__.build())" % (LIB_PATH, got, ABI_VERSION))
        _lib = handle
    return _lib


def build_info():
    """The loaded library's provenance (ncf_build_info): source SHA-256, -D defines, arch, ABI."""
    import json
    return json.loads(lib().ncf_build_info().decode("utf-8", "replace"))


def check_value(rc):
    """A call that returns a non-negative value or a negative status."""
    if rc < 0:
        check(rc)
    return rc


def check(rc):
    if rc == 0:
        return
    msg = lib().ncf_last_error().decode("utf-8", "replace")
    if rc == NCF_EINVAL:
        if msg.startswith("Optimizer") and "not implemented" in msg:
            raise NotImplementedError(msg)
        raise ValueError(msg)
    raise RuntimeError("HIP error in movierec native library: %s" % msg)


def ptr(t):
    """A tensor's device address for a ``c_void_p`` parameter (every entry point has its argtypes
    set, so the int converts in C); None passes NULL."""
    return t.data_ptr() if t is not None else None


# the current stream as a raw handle without building a torch Stream object (host issue cost of
# the small-batch step); torch.cuda.current_stream where the private call is absent
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device=None):
    """The current HIP stream of ``device`` (None, an index or a torch.device) as an int address."""
    if _RAW_STREAM is not None:
        if isinstance(device, int):
            return _RAW_STREAM(device)
        if device is None or torch.device(device).index is None:
            return _RAW_STREAM(torch.cuda.current_device())
        return _RAW_STREAM(torch.device(device).index)
    return torch.cuda.current_stream(device).cuda_stream
