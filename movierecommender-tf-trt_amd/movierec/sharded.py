"""One rank's state for row-sharded data parallelism.

Rank ``r`` of ``world`` owns the combined-table rows ``g`` (users ``0..U-1``,
items ``U..U+I-1``) with ``g % world == r``, stored at local row ``g // world``
of a ``(shard_rows x row_width)`` shard, together with their Adam moments.  The
dense parameters are replicated.  ``ShardedNCFEngine`` holds that state and
wraps the library's ``ncf_shard_*`` calls; ``movierec.distributed.
RowShardedDataParallel`` runs the exchanges between them.

The reference trains on one CPU; sharding is new.  It computes
the same step as ``NCFEngine.train_step`` on the concatenated global batch (dense
Keras Adam over every row, F5), up to fp32 summation order.
"""

import ctypes

import numpy as np
import torch

from . import _native as N
from .engine import KERAS_EPSILON
from .layout import Layout


class ShardedNCFEngine(object):
    """Embedding shard + replicated dense layers of one rank, on one device."""

    def __init__(self, num_users, num_items, layers_sizes, gmf_dim=0, world=1, rank=0, max_batch=65536,
                 device=None, optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=None,
                 force_generic=False, force_layered=False, lazy_adam=False):
        """``lazy_adam``: deferred exact decay of the shard (``row_step``, as ``NCFEngine``): the owner
        replays a served row's missed zero-gradient steps when a rank requests it and updates only
        the served rows; bitwise the dense shard sweep.  Needs layers_l2reg[0] == 0."""
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("ShardedNCFEngine needs a HIP device (got %s); there is no CPU path" % self.device)
        L = N.lib()
        self.layers = [int(x) for x in layers_sizes]
        self.gmf_dim = int(gmf_dim)
        self.world, self.rank = int(world), int(rank)
        if not 0 <= self.rank < self.world:
            raise ValueError("rank %d outside world %d" % (self.rank, self.world))
        self.shape = N.NcfShape()
        arr = (ctypes.c_int32 * max(len(self.layers), 1))(*self.layers)
        N.check(L.ncf_shape_init(ctypes.byref(self.shape), int(num_users), int(num_items), arr, len(self.layers),
                                 self.gmf_dim))
        s = self.shape
        rows = ctypes.c_int64()
        N.check(L.ncf_shard_rows(ctypes.byref(s), self.world, ctypes.byref(rows)))
        self.shard_rows = int(rows.value)
        self.layout = Layout(num_users, num_items, self.layers, self.gmf_dim)
        self.num_users, self.num_items = int(num_users), int(num_items)
        self.num_rows, self.row_width, self.mlp_params = int(s.num_rows), int(s.row_width), int(s.mlp_params)
        dev = self.device
        with torch.cuda.device(dev):
            self.emb = torch.zeros(self.shard_rows, self.row_width, dtype=torch.float32, device=dev)
            self.emb_m = torch.zeros_like(self.emb)
            self.emb_v = torch.zeros_like(self.emb)
            self.mlp = torch.zeros(self.mlp_params, dtype=torch.float32, device=dev)
            self.mlp_m = torch.zeros_like(self.mlp)
            self.mlp_v = torch.zeros_like(self.mlp)
            self.step = torch.zeros(1, dtype=torch.int32, device=dev)
            self.stats = torch.zeros(N.NCF_NUM_STATS, dtype=torch.float64, device=dev)
            # dense-layer gradient and summary side by side: one all-reduce
            self.dense_buf = torch.zeros(self.mlp_params + N.NCF_NUM_SUMMARY, dtype=torch.float32, device=dev)
            self.mlp_grad = self.dense_buf[:self.mlp_params]
            self.summary = self.dense_buf[self.mlp_params:]
            self.send_counts = torch.zeros(self.world, dtype=torch.int32, device=dev)
            l2 = layers_l2reg or [0.0]
            if lazy_adam and float(l2[0]) != 0.0:
                raise ValueError("lazy_adam needs layers_l2reg[0] == 0 (the L2 loss sums the whole table)")
            # fresh moments are +0: every shard row starts pristine (include/movierec_ncf.h)
            self.row_step = (torch.full((self.shard_rows,), N.NCF_ROW_PRISTINE, dtype=torch.int32, device=dev)
                             if lazy_adam else None)
        self._dirty = False
        self.max_batch = 0
        self._ensure_ws(int(max_batch))
        self.model_s = N.NcfModel(self.emb.data_ptr(), self.mlp.data_ptr())
        self.optim_s = N.NcfOptim(self.emb_m.data_ptr(), self.emb_v.data_ptr(), self.mlp_m.data_ptr(),
                                  self.mlp_v.data_ptr(), self.step.data_ptr(),
                                  self.row_step.data_ptr() if self.row_step is not None else None)
        self.hyper = N.NcfHyper()
        self.set_hyper(optimizer, lr, beta_1, beta_2, layers_l2reg or [0.0] * len(self.layers))
        self.hyper.force_generic = 1 if force_generic else (2 if force_layered else 0)

    # ------------------------------------------------------------------ setup
    @property
    def fast_path(self):
        return bool(self.shape.fast_path) and self.hyper.force_generic not in (1, 2)

    def kernel_for(self, n):
        """Forward/backward kernel a call with n samples runs (ncf_fb_kernel)."""
        k = N.check_value(N.lib().ncf_fb_kernel(ctypes.byref(self.shape), ctypes.byref(self.hyper), int(n)))
        return N.FB_KERNELS[k]

    def set_hyper(self, optimizer, lr, beta_1=0.9, beta_2=0.999, layers_l2reg=None):
        if getattr(self, "row_step", None) is not None:
            # pending zero-gradient steps are owed under the previous hyper-parameters
            self.flush()
            if layers_l2reg is not None and len(layers_l2reg) and float(layers_l2reg[0]) != 0.0:
                raise ValueError("lazy_adam needs layers_l2reg[0] == 0 (the L2 loss sums the whole table)")
        h = self.hyper
        opt = {"adam": N.NCF_OPT_ADAM, "sgd": N.NCF_OPT_SGD}.get(optimizer)
        if opt is None:
            raise NotImplementedError("Optimizer {} is not implemented.".format(optimizer))
        h.optimizer = opt
        h.lr, h.beta_1, h.beta_2, h.epsilon = float(lr), float(beta_1), float(beta_2), KERAS_EPSILON
        if layers_l2reg is not None:
            for i in range(N.NCF_MAX_LAYERS):
                h.l2[i] = float(layers_l2reg[i]) if i < len(layers_l2reg) else 0.0

    def _ensure_ws(self, n):
        if n <= self.max_batch:
            return
        L = N.lib()
        nbytes = ctypes.c_size_t()
        N.check(L.ncf_shard_workspace_size(ctypes.byref(self.shape), int(n), self.world, ctypes.byref(nbytes)))
        dev = self.device
        self.ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)
        self.ws_bytes = int(nbytes.value)
        N.check(L.ncf_shard_workspace_init(ctypes.byref(self.shape), int(n), self.world, N.ptr(self.ws),
                                           self.ws_bytes, N.stream_handle(dev)))
        cap = 2 * int(n)
        recv_cap = self.world * min(cap, self.shard_rows)
        W = self.row_width
        self.uniq = torch.zeros(cap, dtype=torch.int32, device=dev)
        self.uniq_vals = torch.zeros(cap, W, dtype=torch.float32, device=dev)
        self.uniq_grad = torch.zeros(cap, W, dtype=torch.float32, device=dev)
        self.recv_rows = torch.zeros(recv_cap, dtype=torch.int32, device=dev)
        self.recv_vals = torch.zeros(recv_cap, W, dtype=torch.float32, device=dev)
        self.recv_grad = torch.zeros(recv_cap, W, dtype=torch.float32, device=dev)
        self.max_batch = int(n)

    def check_errors(self):
        """Raise for the workspace's sticky flags (an id outside the table, a plan whose fold
        differs from the step that used it); synchronises the stream."""
        from .engine import raise_ws_flags
        flags = torch.zeros(1, dtype=torch.int32, device=self.device)
        N.check(N.lib().ncf_shard_workspace_flags(ctypes.byref(self.shape), self.max_batch, self.world,
                                                  N.ptr(self.ws), self.ws_bytes, N.ptr(flags),
                                                  N.stream_handle(self.device)))
        raise_ws_flags(int(flags.item()))

    # --------------------------------------------------- weights marshalling
    def owned_rows(self):
        """Global table rows of this shard's local rows (-1 for padding rows)."""
        g = np.arange(self.shard_rows, dtype=np.int64) * self.world + self.rank
        g[g >= self.num_rows] = -1
        return g

    @property
    def lazy(self):
        return self.row_step is not None

    def flush(self):
        """Deferred decay: bring every shard row up to the current step (no-op in dense mode)."""
        if self.row_step is not None and self._dirty:
            N.check(N.lib().ncf_shard_flush(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                            ctypes.byref(self.optim_s), ctypes.byref(self.hyper), self.world,
                                            N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        self._dirty = False

    def set_keras_weights(self, w):
        """Load this rank's rows (and the dense layers) from a full Keras-layout dict."""
        self.flush()
        emb, flat = self.layout.to_device(w)
        g = self.owned_rows()
        shard = np.zeros((self.shard_rows, self.row_width), dtype=np.float32)
        shard[g >= 0] = emb[g[g >= 0]]
        self.emb.copy_(torch.from_numpy(shard))
        self.mlp.copy_(torch.from_numpy(flat))

    # ------------------------------------------------------------- hot path
    def _ids(self, x):
        if not torch.is_tensor(x):
            x = torch.from_numpy(np.ascontiguousarray(np.asarray(x).reshape(-1), dtype=np.int32))
        if x.dtype != torch.int32:
            x = x.to(torch.int32)
        return x.reshape(-1).to(self.device, non_blocking=True).contiguous()

    def _labels(self, y):
        if not torch.is_tensor(y):
            y = torch.from_numpy(np.ascontiguousarray(np.asarray(y).reshape(-1), dtype=np.float32))
        return y.reshape(-1).to(device=self.device, dtype=torch.float32, non_blocking=True).contiguous()

    def plan(self, users, items, group=None):
        """Unique rows of the batch grouped by owner: (uniq local-row ids, send_counts) on device.
        ``group``: the sample group of the ``forward_backward`` that follows (its index folds a
        group's user rows); None for a plan that only feeds ``predict_planned``."""
        u, i = self._ids(users), self._ids(items)
        n = u.numel()
        if i.numel() != n:
            raise ValueError("users and items differ in length")
        self._ensure_ws(n)
        self._n = n
        h = None
        if group is not None:
            h = self.hyper
            h.group = int(group)
        self._plan_group = None if group is None else int(group)
        N.check(N.lib().ncf_shard_plan(ctypes.byref(self.shape), ctypes.byref(h) if h is not None else None,
                                       self.world, N.ptr(u), N.ptr(i), n, N.ptr(self.uniq), N.ptr(self.send_counts),
                                       N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        return self.uniq, self.send_counts

    def gather_rows(self, rows, m, out=None):
        """Owner side: this shard's rows ``rows[:m]`` (local ids, each source's rows once, sources
        in rank order) into ``out`` (default ``recv_vals``).  Under deferred decay the rows are
        served (ncf_shard_serve_rows): caught up first, and indexed for this step's
        ``apply_update``, which must follow with their gradients in the same order."""
        out = self.recv_vals if out is None else out
        if self.row_step is not None:
            self._dirty = True
            N.check(N.lib().ncf_shard_serve_rows(ctypes.byref(self.shape), ctypes.byref(self.model_s),
                                                 ctypes.byref(self.optim_s), ctypes.byref(self.hyper), self.world,
                                                 N.ptr(rows), int(m), N.ptr(out), N.ptr(self.ws), self.ws_bytes,
                                                 N.stream_handle(self.device)))
        else:
            N.check(N.lib().ncf_gather_rows(ctypes.byref(self.shape), N.ptr(self.emb), self.shard_rows, N.ptr(rows),
                                            int(m), N.ptr(out), N.stream_handle(self.device)))
        return out[:m]

    def forward_backward(self, labels, group, k, inv_batch, include_dense_reg=True, probs_out=None):
        """Forward/backward of the planned batch on ``uniq_vals`` (the fetched unique rows):
        ``uniq_grad`` (per unique row), ``mlp_grad`` and ``summary`` (this rank's part)."""
        y = self._labels(labels)
        if y.numel() != self._n:
            raise ValueError("labels do not match the planned batch")
        if getattr(self, "_plan_group", None) != int(group):
            raise ValueError("the batch was planned for group %r, not %d: pass group= to plan()"
                             % (getattr(self, "_plan_group", None), int(group)))
        h = self.hyper
        h.group, h.k, h.inv_batch = int(group), int(k), float(inv_batch)
        model = N.NcfModel(self.uniq_vals.data_ptr(), self.mlp.data_ptr())
        N.check(N.lib().ncf_shard_forward_backward(
            ctypes.byref(self.shape), ctypes.byref(model), ctypes.byref(h), self.world, N.ptr(y), self._n,
            N.ptr(self.uniq_grad), N.ptr(self.mlp_grad), N.ptr(self.summary), N.ptr(probs_out), N.ptr(self.emb),
            self.shard_rows, 1 if include_dense_reg else 0, N.ptr(self.ws), self.ws_bytes,
            N.stream_handle(self.device)))

    def apply_update(self, recv_rows, recv_grad, m, inv_batch):
        """Owner side: optimizer step of the whole shard (deferred decay: of the rows served this
        step) from ``m`` received row gradients, and of the dense layers from the (already
        reduced) ``mlp_grad`` / ``summary``."""
        self.hyper.inv_batch = float(inv_batch)
        self._dirty = self._dirty or self.row_step is not None
        N.check(N.lib().ncf_shard_apply_update(
            ctypes.byref(self.shape), ctypes.byref(self.model_s), ctypes.byref(self.optim_s), ctypes.byref(self.hyper),
            self.world, N.ptr(recv_rows), N.ptr(recv_grad), int(m), N.ptr(self.mlp_grad), N.ptr(self.summary),
            N.ptr(self.stats), N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))

    def predict_planned(self):
        """Predictions of the planned batch from ``uniq_vals``."""
        out = torch.empty(self._n, dtype=torch.float32, device=self.device)
        model = N.NcfModel(self.uniq_vals.data_ptr(), self.mlp.data_ptr())
        N.check(N.lib().ncf_shard_predict(ctypes.byref(self.shape), ctypes.byref(model), self.world, self._n,
                                          N.ptr(out), N.ptr(self.ws), self.ws_bytes, N.stream_handle(self.device)))
        return out

    def group_metrics(self, probs, labels, group, k):
        """Per-group hit@k / dcg@k of device probabilities (RankLayer order)."""
        probs = probs.reshape(-1).contiguous()
        y = self._labels(labels)
        ng = probs.numel() // group
        hit = torch.empty(ng, dtype=torch.float32, device=self.device)
        dcg = torch.empty(ng, dtype=torch.float32, device=self.device)
        N.check(N.lib().ncf_group_metrics(N.ptr(probs), N.ptr(y), ng, int(group), int(k), N.ptr(hit), N.ptr(dcg),
                                          N.stream_handle(self.device)))
        return hit, dcg
