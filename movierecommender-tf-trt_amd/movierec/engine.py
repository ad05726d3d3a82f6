"""Device-resident NCF/NeuMF state and the calls into the HIP library.

``NCFEngine`` owns the model and optimizer tensors on one GPU (fp32, layouts
described in ``include/movierec_ncf.h``) and exposes the hot path:
``train_step`` (Keras ``train_on_batch``), ``evaluate`` (validation batch),
``predict`` (``predict_on_batch`` output[0]), ``rank`` (``RankLayer``),
``group_metrics`` (``hit_rate`` / ``discounted_cumulative_gain``), and the
data-parallel split ``forward_backward`` + ``apply_update``.

PyTorch provides device memory, the stream and torch.distributed; every
arithmetic step of the path runs in the library's HIP kernels.
"""

import ctypes

import numpy as np
import torch

from . import _native as N
from .layout import Layout

KERAS_EPSILON = 1e-7


def keras_weight_names(layers, gmf_dim):
    names = ["user_embedding", "item_embedding"] if len(layers) else []
    if gmf_dim > 0:
        names += ["user_gmf_embedding", "item_gmf_embedding"]
    for l in range(1, len(layers)):
        names += ["hidden_%d/kernel" % l, "hidden_%d/bias" % l]
    return names + ["output/kernel", "output/bias"]


def _same_ids(held, u, i, n, group):
    """An index prepared for (users, items) tensors ``held`` = (u, i, n, u_version, i_version,
    group) applies to this call's ids: same tensors (storage), same size, not modified in place
    since, and the same sample group (the index folds a group's user rows, ncf_internal.h)."""
    hu, hi, hn, vu, vi, hg = held
    return (hu.data_ptr() == u.data_ptr() and hi.data_ptr() == i.data_ptr() and hn == n and
            hu._version == vu and hi._version == vi and hg == group)


def raise_ws_flags(f):
    """Raise for the sticky workspace flags ``f`` (ncf_workspace_flags / ncf_shard_workspace_flags)."""
    if f & N.NCF_WSERR_FOLD:
        raise RuntimeError("an index built ahead (build_index / plan) used another sample group than the step")
    if f & N.NCF_WSERR_STALE_COUNT:
        raise RuntimeError("a batch counted ahead (train_step next_batch=) changed its ids before its step: "
                           "that step's embedding update used a stale index")
    if f & N.NCF_WSERR_ID_RANGE:
        raise ValueError("an id outside the embedding table reached the device (those samples were masked)")


def pristine_marks(m, v, rows, step):
    """row_step of rows [0, rows) whose Adam state was just set: NCF_ROW_PRISTINE where a row's
    moments are all bitwise +0 (the zero-gradient step's fixed point), else ``step``."""
    mi = m[:rows].view(torch.int32)
    vi = v[:rows].view(torch.int32)
    zero = ((mi == 0) & (vi == 0)).all(dim=1)
    out = torch.full((rows,), int(step), dtype=torch.int32, device=m.device)
    out[zero] = N.NCF_ROW_PRISTINE
    return out


class NCFEngine(object):
    """Model + optimizer state of one replica on one device."""

    def __init__(self, num_users, num_items, layers_sizes, gmf_dim=0, max_batch=65536, device=None,
                 optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=None,
                 force_generic=False, force_layered=False, lazy_adam=False, fb_kernel=None, precision="fp32",
                 lazy_rows=None):
        """``lazy_adam``: deferred exact decay (``ncf_optim_t.row_step``) — a training step updates
        only the batch's rows, the others catch up on their missed zero-gradient steps when next
        touched or read; bitwise the dense Keras sweep (F5).  Needs layers_l2reg[0] == 0; the
        table is flushed before every read (predict, evaluate, scoring, weights export).
        ``lazy_rows``: only rows [0, lazy_rows) are deferred (user-partitioned data parallelism:
        the rank's own users; the replicated item rows are swept every step)."""
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("NCFEngine needs a HIP device (got %s); there is no CPU path" % self.device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._dev_idx = self.device.index
        L = N.lib()
        self.layers = [int(x) for x in layers_sizes]
        self.gmf_dim = int(gmf_dim)
        self.shape = N.NcfShape()
        arr = (ctypes.c_int32 * max(len(self.layers), 1))(*self.layers)
        N.check(L.ncf_shape_init(ctypes.byref(self.shape), int(num_users), int(num_items), arr, len(self.layers),
                                 self.gmf_dim))
        s = self.shape
        self.layout = Layout(num_users, num_items, self.layers, self.gmf_dim)
        assert (self.layout.row_width, self.layout.mlp_params) == (s.row_width, s.mlp_params)
        self.num_users, self.num_items = int(num_users), int(num_items)
        self.row_width = s.row_width
        self.num_rows = s.num_rows
        self.mlp_params = s.mlp_params
        dev = self.device
        with torch.cuda.device(dev):
            self.emb = torch.zeros(s.num_rows, s.row_width, dtype=torch.float32, device=dev)
            self.mlp = torch.zeros(s.mlp_params, dtype=torch.float32, device=dev)
            self.emb_m = torch.zeros_like(self.emb)
            self.emb_v = torch.zeros_like(self.emb)
            self.mlp_m = torch.zeros_like(self.mlp)
            self.mlp_v = torch.zeros_like(self.mlp)
            self.step = torch.zeros(1, dtype=torch.int32, device=dev)
            self.lazy_rows = None if lazy_rows is None else int(lazy_rows)
            if self.lazy_rows is not None and not 0 < self.lazy_rows <= s.num_rows:
                raise ValueError("lazy_rows must be in [1, %d]" % s.num_rows)
            nlazy = s.num_rows if self.lazy_rows is None else self.lazy_rows
            # fresh moments are +0: every row starts pristine (a fixed point of the zero-gradient
            # step, so it owes no replay until its first gradient)
            self.row_step = (torch.full((nlazy,), N.NCF_ROW_PRISTINE, dtype=torch.int32, device=dev)
                             if lazy_adam else None)
            self._dirty = False
            self.stats = torch.zeros(N.NCF_NUM_STATS, dtype=torch.float64, device=dev)
            self.val_stats = torch.zeros(N.NCF_NUM_STATS, dtype=torch.float64, device=dev)
            self.max_batch = 0
            self.ws = None
            self._prebuilt = None   # (users, items, n) of an index built ahead by build_index
            self._counted = None    # (users, items, n) whose index counts ncf_train_step_ahead took
            self._ensure_ws(int(max_batch))
        self.model_s = N.NcfModel(self.emb.data_ptr(), self.mlp.data_ptr())
        self.hyper = N.NcfHyper()
        self.hyper.lazy_rows = self.lazy_rows or 0
        self._bind_optim()
        self.set_hyper(optimizer, lr, beta_1, beta_2, layers_l2reg or [0.0] * len(self.layers))
        if fb_kernel not in (None, "tile", "unit", "wave", "wave1"):
            raise ValueError("fb_kernel must be None, 'tile', 'unit', 'wave' or 'wave1'")
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        self.hyper.force_generic = (1 if force_generic else 2 if force_layered else
                                    {None: 0, "tile": 3, "unit": 4, "wave": 5, "wave1": 6}[fb_kernel])
        # bf16 MLP operands (fp32 accumulation, master weights and Adam): BASELINE config B
        self.precision = precision
        self.hyper.mlp_bf16 = 1 if precision == "bf16" else 0
        if precision == "bf16" and self.kernel_for(max(self.max_batch, 1)) != "fused-mfma-unit":
            raise ValueError("precision='bf16' needs a model shape the fused unit kernel holds")

    # ------------------------------------------------------------------ setup
    @property
    def fast_path(self):
        return bool(self.shape.fast_path) and self.hyper.force_generic not in (1, 2)

    def kernel_for(self, n):
        """Forward/backward kernel a training call with n samples runs (ncf_fb_kernel):
        "fused-mfma-unit", "fused-mfma-wave", "fused-mfma-tile", "layered-mfma" (every layer hand-written MFMA),
        "layered-rocblas" (some layers on rocBLAS) or "generic"."""
        k = N.check_value(N.lib().ncf_fb_kernel(ctypes.byref(self.shape), ctypes.byref(self.hyper), int(n)))
        return N.FB_KERNELS[k]

    @property
    def kernel_path(self):
        """Forward/backward path at the engine's batch capacity (see kernel_for)."""
        return self.kernel_for(max(self.max_batch, 1))

    def _bind_optim(self):
        self.optim_s = N.NcfOptim(self.emb_m.data_ptr(), self.emb_v.data_ptr(), self.mlp_m.data_ptr(),
                                  self.mlp_v.data_ptr(), self.step.data_ptr(),
                                  self.row_step.data_ptr() if self.row_step is not None else None)

    @property
    def lazy(self):
        return self.row_step is not None

    def flush(self):
        """Deferred decay: bring every row up to the current step (a no-op in dense mode)."""
        if self.row_step is not None and self._dirty:
            N.check(N.lib().ncf_lazy_flush(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                           ctypes.byref(self.optim_s), ctypes.byref(self.hyper), N.ptr(self.ws),
                                           self.ws_bytes, N.stream_handle(self.device)))
        self._dirty = False

    def disable_lazy(self):
        """Flush and return to the dense sweep (data-parallel paths update every row)."""
        self.flush()
        self.row_step = None
        self.lazy_rows = None
        self.hyper.lazy_rows = 0
        self._bind_optim()

    def set_hyper(self, optimizer, lr, beta_1=0.9, beta_2=0.999, layers_l2reg=None, group=None, k=None):
        if getattr(self, "row_step", None) is not None:
            self.flush()  # pending decay is owed under the previous hyper-parameters
            if layers_l2reg is not None and len(layers_l2reg) and float(layers_l2reg[0]) != 0.0:
                self.disable_lazy()
        h = self.hyper
        opt = {"adam": N.NCF_OPT_ADAM, "sgd": N.NCF_OPT_SGD}.get(optimizer)
        if opt is None:
            raise NotImplementedError("Optimizer {} is not implemented.".format(optimizer))
        h.optimizer = opt
        h.lr, h.beta_1, h.beta_2, h.epsilon = float(lr), float(beta_1), float(beta_2), KERAS_EPSILON
        if layers_l2reg is not None:
            for i in range(N.NCF_MAX_LAYERS):
                h.l2[i] = float(layers_l2reg[i]) if i < len(layers_l2reg) else 0.0
        if group is not None:
            h.group = int(group)
        if k is not None:
            h.k = int(k)

    def _ensure_ws(self, n):
        if n <= self.max_batch:
            return
        self._discard_counted()  # (a new workspace starts with zero counters)
        L = N.lib()
        nbytes = ctypes.c_size_t()
        N.check(L.ncf_workspace_size(ctypes.byref(self.shape), int(n), ctypes.byref(nbytes)))
        self.ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=self.device)
        self._prebuilt = None
        self._counted = None
        self.ws_bytes = int(nbytes.value)
        N.check(L.ncf_workspace_init(ctypes.byref(self.shape), int(n), N.ptr(self.ws), self.ws_bytes,
                                     N.stream_handle(self.device)))
        self.max_batch = int(n)

    # --------------------------------------------------- weights marshalling
    def set_keras_weights(self, w):
        """Load a dict of Keras-layout arrays (names as ``keras_weight_names``)."""
        self.flush()
        emb, flat = self.layout.to_device(w)
        self.emb[:self.num_rows].copy_(torch.from_numpy(emb))
        self.mlp.copy_(torch.from_numpy(flat))

    def keras_weights(self, emb=None, mlp=None):
        """Current weights (or the given device tensors in this layout) as a Keras-layout dict."""
        self.flush()
        e = (self.emb if emb is None else emb)[:self.num_rows].detach().cpu().numpy()
        f = (self.mlp if mlp is None else mlp).detach().cpu().numpy()
        return self.layout.from_device(e, f)

    def optimizer_state(self):
        """Adam moments as Keras-layout dicts (m, v) and the iteration count."""
        return (self.keras_weights(self.emb_m, self.mlp_m), self.keras_weights(self.emb_v, self.mlp_v),
                int(self.step.item()))

    def set_optimizer_state(self, m, v, step):
        self.flush()
        saved = (self.emb.clone(), self.mlp.clone())
        self.set_keras_weights(m)
        self.emb_m.copy_(self.emb)
        self.mlp_m.copy_(self.mlp)
        self.set_keras_weights(v)
        self.emb_v.copy_(self.emb)
        self.mlp_v.copy_(self.mlp)
        self.emb.copy_(saved[0])
        self.mlp.copy_(saved[1])
        self.step.fill_(int(step))
        if self.row_step is not None:
            self.row_step.copy_(pristine_marks(self.emb_m, self.emb_v, self.row_step.numel(), int(step)))

    # ------------------------------------------------------------- hot path
    def _ids(self, x):
        # fast path (the step's host issue cost): a 1-D contiguous int32 tensor on this device as is
        if (type(x) is torch.Tensor and x.dtype is torch.int32 and x.is_cuda and x.dim() == 1 and
                x.is_contiguous() and x.get_device() == self._dev_idx):
            return x
        if not torch.is_tensor(x):
            x = torch.from_numpy(np.ascontiguousarray(np.asarray(x).reshape(-1), dtype=np.int32))
        if x.dtype != torch.int32:
            x = x.to(torch.int32)
        return x.reshape(-1).to(self.device, non_blocking=True).contiguous()

    def _labels(self, y):
        if (type(y) is torch.Tensor and y.dtype is torch.float32 and y.is_cuda and y.dim() == 1 and
                y.is_contiguous() and y.get_device() == self._dev_idx):
            return y
        if not torch.is_tensor(y):
            y = torch.from_numpy(np.ascontiguousarray(np.asarray(y).reshape(-1), dtype=np.float32))
        return y.reshape(-1).to(device=self.device, dtype=torch.float32, non_blocking=True).contiguous()

    def check_ids(self, users, items):
        """Host-side range check (TF's gather raises on out-of-range ids).  Batches already on
        the device (DeviceMovieLensDataGenerator) were range-checked by the sampler."""
        if torch.is_tensor(users) and users.is_cuda:
            return
        u = np.asarray(users)
        i = np.asarray(items)
        if u.size and (u.min() < 0 or u.max() >= self.num_users):
            raise ValueError("user id out of range [0, %d)" % self.num_users)
        if i.size and (i.min() < 0 or i.max() >= self.num_items):
            raise ValueError("item id out of range [0, %d)" % self.num_items)

    def train_step(self, users, items, labels, group, k, inv_batch=None, probs_out=None, next_batch=None):
        """Keras ``train_on_batch``.  ``next_batch`` = (users, items) device int32 tensors of the
        following call (deferred-decay Adam): their index counts are taken inside this step's
        touched-row update, and the next call skips its count kernel if it passes exactly these
        tensors (identity-checked; their contents must not change in between)."""
        if self.lazy_rows is not None and self.lazy_rows < self.num_rows:
            raise ValueError("this engine defers the decay of its first %d rows only (user-partitioned data "
                             "parallelism): train it through forward_backward_part / update_rows / apply_update"
                             % self.lazy_rows)
        u, i, y = self._ids(users), self._ids(items), self._labels(labels)
        n = u.numel()
        self._ensure_ws(n)
        h = self.hyper
        h.group, h.k = int(group), int(k)
        h.inv_batch = 1.0 / n if inv_batch is None else float(inv_batch)
        pc = self._counted
        ready = pc is not None and _same_ids(pc, u, i, n, h.group)
        if pc is not None and not ready:
            self._discard_counted()
        nu = ni = None
        if next_batch is not None and self.row_step is not None and h.optimizer == N.NCF_OPT_ADAM:
            nu, ni = next_batch
            if not (torch.is_tensor(nu) and torch.is_tensor(ni) and nu.is_cuda and ni.is_cuda and
                    nu.dtype == torch.int32 and ni.dtype == torch.int32 and nu.is_contiguous() and
                    ni.is_contiguous() and nu.numel() == ni.numel() == n):
                nu = ni = None
        h.index_ready = 2 if ready else 0
        self._counted = None
        try:
            if nu is not None:
                N.check(N.lib().ncf_train_step_ahead(
                    ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(self.optim_s), ctypes.byref(h),
                    N.ptr(u), N.ptr(i), N.ptr(y), n, N.ptr(nu), N.ptr(ni), nu.numel(), N.ptr(self.stats),
                    N.ptr(probs_out), N.ptr(self.ws), self.ws_bytes, N.stream_handle(self._dev_idx)))
                # holds the tensors (their memory stays theirs) and their versions: an in-place
                # refill through torch (copy_, fill_, index assignment) bumps _version and the next
                # call rebuilds the index; writes that bypass torch's version counter are caught on
                # the device (NCF_WSERR_STALE_COUNT, check_errors)
                self._counted = (nu, ni, nu.numel(), nu._version, ni._version, h.group)
            else:
                N.check(N.lib().ncf_train_step(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                               ctypes.byref(self.optim_s), ctypes.byref(h), N.ptr(u), N.ptr(i),
                                               N.ptr(y), n, N.ptr(self.stats), N.ptr(probs_out), N.ptr(self.ws),
                                               self.ws_bytes, N.stream_handle(self._dev_idx)))
        finally:
            h.index_ready = 0
        self._dirty = self.row_step is not None

    def check_errors(self):
        """Raise if an index build since the last call met an id outside the table (ValueError,
        like TF's gather) or a counted-ahead batch whose ids changed after they were counted
        (RuntimeError: that step's embedding update is wrong).  Synchronises the stream."""
        if self.ws is None:
            return
        flags = torch.zeros(1, dtype=torch.int32, device=self.device)
        N.check(N.lib().ncf_workspace_flags(ctypes.byref(self.shape), self.max_batch, N.ptr(self.ws), self.ws_bytes,
                                            N.ptr(flags), N.stream_handle(self.device)))
        raise_ws_flags(int(flags.item()))

    def _discard_counted(self):
        """Clear the index counters holding a next batch's counts (ncf_train_step_ahead) before any
        other index build uses them."""
        if self._counted is not None:
            # the counted batch's stale rows were caught up ahead with p only (P-ahead rows,
            # ncf_update.hip): settle them before the batch is given up
            self.flush()
            # counters only: the sticky error flags stay for check_errors
            N.check(N.lib().ncf_workspace_discard_counts(ctypes.byref(self.shape), self.max_batch, N.ptr(self.ws),
                                                         self.ws_bytes, N.stream_handle(self.device)))
            self._counted = None

    def evaluate(self, users, items, labels, group, k, stats=None, probs_out=None):
        u, i, y = self._ids(users), self._ids(items), self._labels(labels)
        n = u.numel()
        self._ensure_ws(n)
        h = self.hyper
        h.group, h.k = int(group), int(k)
        h.inv_batch = 1.0 / n
        self.flush()
        st = self.val_stats if stats is None else stats
        N.check(N.lib().ncf_evaluate(ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(h),
                                     N.ptr(u), N.ptr(i), N.ptr(y), n, N.ptr(st), N.ptr(probs_out), N.ptr(self.ws),
                                     self.ws_bytes, N.stream_handle(self.device)))

    def predict(self, users, items):
        self.flush()
        u, i = self._ids(users), self._ids(items)
        n = u.numel()
        self._ensure_ws(n)
        out = torch.empty(n, dtype=torch.float32, device=self.device)
        N.check(N.lib().ncf_predict(ctypes.byref(self.shape), ctypes.byref(self.model_s), N.ptr(u), N.ptr(i), n,
                                    N.ptr(out), N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        return out

    def rank(self, probs, group):
        probs = probs.reshape(-1).contiguous()
        if probs.numel() % group:   # RankLayer's reshape (-1, n+1) fails the same way in TF
            raise ValueError("cannot rank %d predictions in groups of %d" % (probs.numel(), group))
        ng = probs.numel() // group
        if ng == 0:
            return torch.empty(0, group, dtype=torch.int32, device=self.device)
        out = torch.empty(ng, group, dtype=torch.int32, device=self.device)
        N.check(N.lib().ncf_rank(N.ptr(probs), ng, int(group), N.ptr(out), N.stream_handle(self.device)))
        return out

    def group_metrics(self, probs, labels, group, k):
        probs = probs.reshape(-1).contiguous()
        y = self._labels(labels)
        ng = probs.numel() // group
        hit = torch.empty(ng, dtype=torch.float32, device=self.device)
        dcg = torch.empty(ng, dtype=torch.float32, device=self.device)
        N.check(N.lib().ncf_group_metrics(N.ptr(probs), N.ptr(y), ng, int(group), int(k), N.ptr(hit), N.ptr(dcg),
                                          N.stream_handle(self.device)))
        return hit, dcg

    # ---------------------------------------------- all-item scoring + top-k
    def score_topk(self, users, k=10, precision="fp16"):
        """For each user id: the k items with the highest score over the whole catalogue, best
        first (ties: lower item id), and their sigmoid outputs — BASELINE config E, the
        workload of trt_client.py:43-57 batched over users.  precision "fp16": MFMA scorer
        (fp16 operands, fp32 accumulation); "fp32": the generic fp32 forward, any shape."""
        prec = {"fp16": N.NCF_SCORE_FP16, "fp32": N.NCF_SCORE_FP32}.get(precision)
        if prec is None:
            raise ValueError("precision must be 'fp16' or 'fp32', got %r" % (precision,))
        L = N.lib()
        if not L.ncf_score_supported(ctypes.byref(self.shape), prec):
            raise ValueError("model shape not supported by the %s scorer" % precision)
        self.flush()
        u = self._ids(users)
        n = u.numel()
        items = torch.empty(n, int(k), dtype=torch.int32, device=self.device)
        scores = torch.empty(n, int(k), dtype=torch.float32, device=self.device)
        if n == 0:
            return items, scores
        nbytes = ctypes.c_size_t()
        N.check(L.ncf_score_workspace_size(ctypes.byref(self.shape), n, ctypes.byref(nbytes)))
        if getattr(self, "_score_ws", None) is None or self._score_ws.numel() < nbytes.value:
            self._score_ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=self.device)
        N.check(L.ncf_score_topk(ctypes.byref(self.shape), ctypes.byref(self.model_s), N.ptr(u), n, int(k), prec,
                                 N.ptr(items), N.ptr(scores), N.ptr(self._score_ws), self._score_ws.numel(),
                                 N.stream_handle(self.device)))
        return items, scores

    # ------------------------------------------------- data-parallel split
    def alloc_grads(self, rows=None):
        """(dense embedding grad [rows x row_width], dense-layer grad, summary); ``rows`` >=
        num_rows pads the embedding gradient (zero rows) for an equal-shard reduce-scatter."""
        rows = self.num_rows if rows is None else int(rows)
        eg = torch.zeros(rows, self.row_width, dtype=torch.float32, device=self.device)
        return (eg, torch.empty_like(self.mlp),
                torch.zeros(N.NCF_NUM_SUMMARY, dtype=torch.float32, device=self.device))

    def forward_backward(self, users, items, labels, group, k, inv_batch, grads, probs_out=None,
                         reg_rows=None, include_dense_reg=True):
        """This replica's gradients (BCE mean over ``inv_batch``); ``reg_rows`` = (begin, count)
        of the embedding rows whose L2 loss this replica reports (default: all)."""
        self._discard_counted()
        if self.row_step is not None:
            self.disable_lazy()   # data-parallel updates sweep every row
        u, i, y = self._ids(users), self._ids(items), self._labels(labels)
        n = u.numel()
        self._ensure_ws(n)
        h = self.hyper
        h.group, h.k, h.inv_batch = int(group), int(k), float(inv_batch)
        eg, mg, sm = grads
        r0, rc = (0, self.num_rows) if reg_rows is None else reg_rows
        N.check(N.lib().ncf_forward_backward(ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(h),
                                             N.ptr(u), N.ptr(i), N.ptr(y), n, N.ptr(eg), N.ptr(mg), N.ptr(sm),
                                             N.ptr(probs_out), int(r0), int(rc), 1 if include_dense_reg else 0,
                                             N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))

    def forward_backward_part(self, users, items, labels, group, k, inv_batch, shared_row_begin, grads,
                              probs_out=None, reg_rows=None, include_dense_reg=True):
        """``forward_backward`` with the dense embedding gradient written for the replicated rows
        [shared_row_begin, num_rows) only (``grads[0]`` indexed from that row); the own rows are
        updated from the per-sample gradients by ``update_rows`` (user-partitioned DP).  With
        ``lazy_rows == shared_row_begin`` the own rows are under deferred decay: the batch's are
        caught up first (or were, ahead, by the previous ``update_rows(..., next_batch=)``)."""
        if self.row_step is not None and self.lazy_rows == int(shared_row_begin):
            return self._forward_backward_part_lazy(users, items, labels, group, k, inv_batch, grads, probs_out,
                                                    include_dense_reg)
        self._discard_counted()
        if self.row_step is not None:
            self.disable_lazy()
        u, i, y = self._ids(users), self._ids(items), self._labels(labels)
        n = u.numel()
        self._ensure_ws(n)
        h = self.hyper
        h.group, h.k, h.inv_batch = int(group), int(k), float(inv_batch)
        # an index prebuilt by build_index is used only for the very tensors it was built from
        pb = self._prebuilt
        ready = pb is not None and _same_ids(pb, u, i, n, h.group)
        h.index_ready = 1 if ready else 0
        eg, mg, sm = grads
        r0, rc = (0, self.num_rows) if reg_rows is None else reg_rows
        try:
            N.check(N.lib().ncf_forward_backward_part(
                ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(h), N.ptr(u), N.ptr(i), N.ptr(y),
                n, int(shared_row_begin), N.ptr(eg), N.ptr(mg), N.ptr(sm), N.ptr(probs_out), int(r0), int(rc),
                1 if include_dense_reg else 0, N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        finally:
            h.index_ready = 0
            self._prebuilt = None
        self._part_n = n

    def _forward_backward_part_lazy(self, users, items, labels, group, k, inv_batch, grads, probs_out,
                                    include_dense_reg):
        u, i, y = self._ids(users), self._ids(items), self._labels(labels)
        n = u.numel()
        self._ensure_ws(n)
        h = self.hyper
        h.group, h.k, h.inv_batch = int(group), int(k), float(inv_batch)
        pc = self._counted
        ready = pc is not None and _same_ids(pc, u, i, n, h.group)
        if pc is not None and not ready:
            self._discard_counted()
        self._counted = None
        h.index_ready = 2 if ready else 0
        eg, mg, sm = grads
        try:
            N.check(N.lib().ncf_forward_backward_part_lazy(
                ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(self.optim_s), ctypes.byref(h),
                N.ptr(u), N.ptr(i), N.ptr(y), n, N.ptr(eg), N.ptr(mg), N.ptr(sm), N.ptr(probs_out),
                1 if include_dense_reg else 0, N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        finally:
            h.index_ready = 0
        self._part_n = n
        self._dirty = True

    def user_dp_step(self, users, items, labels, group, k, inv_batch, shared, comm, next_batch=None,
                     include_dense_reg=True, split=None):
        """The whole user-partitioned step with deferred decay in one library call
        (ncf_user_dp_step): forward/backward, the RCCL all-reduce of ``shared`` = [item-row grad |
        dense-layer grad | summary] on the native communicator ``comm`` beside the own-user update
        (and the next batch counted ahead), then the item rows, dense layers and stats."""
        u, i, y = self._ids(users), self._ids(items), self._labels(labels)
        n = u.numel()
        self._ensure_ws(n)
        h = self.hyper
        h.group, h.k, h.inv_batch = int(group), int(k), float(inv_batch)
        pc = self._counted
        # the previous step counted this batch AND built its index (ncf_user_dp_step): index_ready 3
        ready = pc is not None and _same_ids(pc, u, i, n, h.group)
        if pc is not None and not ready:
            self._discard_counted()
        self._counted = None
        nu = ni = None
        if next_batch is not None and h.optimizer == N.NCF_OPT_ADAM:
            nu, ni = next_batch
            if not (torch.is_tensor(nu) and torch.is_tensor(ni) and nu.is_cuda and ni.is_cuda and
                    nu.dtype == torch.int32 and ni.dtype == torch.int32 and nu.is_contiguous() and
                    ni.is_contiguous() and nu.numel() == ni.numel() == n):
                nu = ni = None
        h.index_ready = 3 if ready else 0
        try:
            if split is not None:
                # (item_world, item_rank, slice_grad): the item rows' Adam split across the ranks
                iw, ir, sg = split
                N.check(N.lib().ncf_user_dp_step_split(
                    ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(self.optim_s),
                    ctypes.byref(h), N.ptr(u), N.ptr(i), N.ptr(y), n, N.ptr(nu), N.ptr(ni),
                    n if nu is not None else 0, N.ptr(shared), N.ptr(sg), int(iw), int(ir),
                    1 if include_dense_reg else 0, comm, N.ptr(self.stats), N.ptr(self.ws), self.ws_bytes,
                    N.stream_handle(self.device)))
            else:
                N.check(N.lib().ncf_user_dp_step(
                    ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(self.optim_s),
                    ctypes.byref(h), N.ptr(u), N.ptr(i), N.ptr(y), n, N.ptr(nu), N.ptr(ni),
                    n if nu is not None else 0, N.ptr(shared), 1 if include_dense_reg else 0, comm,
                    N.ptr(self.stats), N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        finally:
            h.index_ready = 0
        if nu is not None:
            self._counted = (nu, ni, n, nu._version, ni._version, h.group)
        self._part_n = n
        self._dirty = True

    def build_index(self, users, items, group):
        """Build the contribution index of the NEXT ``forward_backward_part`` batch now (e.g. under
        the current step's all-reduce); call after this step's ``update_rows``.  That call must
        pass the same id tensors and ``group`` (checked, else the index is rebuilt), and the ids'
        contents must not change in between (a sampler that refills one buffer in place must not
        use this)."""
        self._discard_counted()
        self._prebuilt = None
        if not (torch.is_tensor(users) and torch.is_tensor(items) and users.is_cuda and items.is_cuda):
            return   # host ids get converted per call: nothing stable to key the index on
        u, i = self._ids(users), self._ids(items)
        n = u.numel()
        if n > self.max_batch or u.data_ptr() != users.data_ptr() or i.data_ptr() != items.data_ptr():
            return
        h = self.hyper
        h.group = int(group)
        N.check(N.lib().ncf_build_index(ctypes.byref(self.shape), ctypes.byref(h), N.ptr(u), N.ptr(i), n,
                                        N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        # holds the tensors: their memory stays theirs
        self._prebuilt = (u, i, n, u._version, i._version, h.group)

    def update_rows(self, row_begin, row_count, inv_batch, next_batch=None):
        """Optimizer step of rows [row_begin, row_begin + row_count) from the per-sample gradient
        rows of the last ``forward_backward_part`` (step counter not advanced).  Deferred decay
        (``lazy_rows == row_count``, ``row_begin == 0``): the batch's touched own rows only, and
        ``next_batch`` = (users, items) device int32 tensors of the next step, whose index is counted
        and whose own rows are caught up in the same launch (pass the same tensors next step)."""
        n = getattr(self, "_part_n", None)
        if n is None:
            raise RuntimeError("update_rows needs a preceding forward_backward_part")
        self.hyper.inv_batch = float(inv_batch)
        if self.row_step is not None and self.lazy_rows == int(row_count) and int(row_begin) == 0:
            nu = ni = None
            if next_batch is not None and self.hyper.optimizer == N.NCF_OPT_ADAM:
                nu, ni = next_batch
                if not (torch.is_tensor(nu) and torch.is_tensor(ni) and nu.is_cuda and ni.is_cuda and
                        nu.dtype == torch.int32 and ni.dtype == torch.int32 and nu.is_contiguous() and
                        ni.is_contiguous() and nu.numel() == ni.numel() == n):
                    nu = ni = None
            N.check(N.lib().ncf_update_rows_lazy(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                                 ctypes.byref(self.optim_s), ctypes.byref(self.hyper), int(n),
                                                 N.ptr(nu), N.ptr(ni), n if nu is not None else 0, N.ptr(self.ws),
                                                 self.ws_bytes, N.stream_handle(self.device)))
            if nu is not None:
                self._counted = (nu, ni, n, nu._version, ni._version, self.hyper.group)
            return
        N.check(N.lib().ncf_update_rows(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                        ctypes.byref(self.optim_s), ctypes.byref(self.hyper), int(n), int(row_begin),
                                        int(row_count), N.ptr(self.ws), self.ws_bytes,
                                        N.stream_handle(self.device)))

    def apply_update(self, grads, inv_batch, rows=None, emb_grad=None, moments_by_row=False):
        """Optimizer step: embedding rows ``rows`` = (begin, count) (default: all) from
        ``emb_grad`` (default grads[0]; indexed from ``begin``), every dense parameter.
        ``moments_by_row``: the Adam moments cover the whole table (indexed by row), not just
        the range (user-partitioned DP)."""
        eg, mg, sm = grads
        eg = eg if emb_grad is None else emb_grad
        r0, rc = (0, self.num_rows) if rows is None else rows
        if self.row_step is not None and not (self.lazy_rows is not None and r0 >= self.lazy_rows):
            self.disable_lazy()   # a dense update of deferred rows: settle them first
        self.hyper.inv_batch = float(inv_batch)
        optim = self.optim_s
        if moments_by_row and r0:
            optim = N.NcfOptim(self.emb_m[r0:].data_ptr(), self.emb_v[r0:].data_ptr(), self.mlp_m.data_ptr(),
                               self.mlp_v.data_ptr(), self.step.data_ptr(), None)
        N.check(N.lib().ncf_apply_update(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                         ctypes.byref(optim), ctypes.byref(self.hyper), int(r0), int(rc),
                                         N.ptr(eg), N.ptr(mg), N.ptr(sm), N.ptr(self.stats), N.ptr(self.ws),
                                         self.ws_bytes, N.stream_handle(self.device)))

    def shard_optimizer_state(self, row_begin, row_count, capacity_rows):
        """Replicated data parallelism: keep Adam moments only for this rank's embedding shard
        and pad the table to ``capacity_rows`` (= world * shard rows) for the all-gather."""
        if self.row_step is not None:
            self.disable_lazy()
        rows = int(capacity_rows)
        if rows > self.emb.shape[0]:
            emb = torch.zeros(rows, self.row_width, dtype=torch.float32, device=self.device)
            emb[:self.num_rows].copy_(self.emb[:self.num_rows])
            self.emb = emb
        self.emb_m = self.emb_m[row_begin:row_begin + row_count].clone()
        self.emb_v = self.emb_v[row_begin:row_begin + row_count].clone()
        self.model_s = N.NcfModel(self.emb.data_ptr(), self.mlp.data_ptr())
        self._bind_optim()

    # ------------------------------------------------------------- stats
    @staticmethod
    def read_stats(t):
        s = t.detach().cpu().numpy()
        steps = max(s[N.STAT_STEPS], 1.0)
        return dict(loss=s[N.STAT_LOSS_SUM] / steps, hr=s[N.STAT_HR_SUM] / steps, dcg=s[N.STAT_DCG_SUM] / steps,
                    steps=int(s[N.STAT_STEPS]), bce=s[N.STAT_BCE_SUM] / steps)
