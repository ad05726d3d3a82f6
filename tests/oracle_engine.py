"""Test helper: an NCFEngine look-alike on the CPU, computed by the oracle.

It exposes exactly the engine surface that movierec.distributed uses
(forward_backward / apply_update / shard_optimizer_state / alloc_grads, and
the ``emb`` / ``mlp`` tensors in the device layout), so the data-parallel
orchestration can be tested with the gloo backend on CPU.  Test-only: it
lives under tests/ and imports the oracle.
"""

import numpy as np
import torch

from movierec.layout import Layout
from oracle import ncf_oracle as O


class OracleEngine(object):
    def __init__(self, shape, w, lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=None):
        self.shape = shape
        self.layout = Layout(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim)
        self.num_rows = self.layout.num_rows
        self.row_width = self.layout.row_width
        self.num_users, self.num_items = shape.num_users, shape.num_items
        emb, flat = self.layout.to_device(w, dtype=np.float64)
        self.emb = torch.from_numpy(emb)
        self.mlp = torch.from_numpy(flat)
        self.emb_m = torch.zeros_like(self.emb)
        self.emb_v = torch.zeros_like(self.emb)
        self.mlp_m = torch.zeros_like(self.mlp)
        self.mlp_v = torch.zeros_like(self.mlp)
        self.t = 0
        self.lr, self.b1, self.b2 = lr, beta_1, beta_2
        self.l2 = list(layers_l2reg or [0.0] * len(shape.layers))
        # per-parameter L2 factor of the flat dense vector (hidden kernels only)
        lam = np.zeros(self.layout.mlp_params)
        off = 0
        for l in range(1, len(shape.layers)):
            a, b = shape.layers[l - 1], shape.layers[l]
            lam[off:off + a * b] = self.l2[l]
            off += a * b + b
        self.mlp_lam = torch.from_numpy(lam)

    def weights(self):
        return self.layout.from_device(self.emb[:self.num_rows].numpy(), self.mlp.numpy())

    def alloc_grads(self, rows=None):
        rows = self.num_rows if rows is None else rows
        return (torch.zeros(rows, self.row_width, dtype=torch.float64),
                torch.zeros(self.layout.mlp_params, dtype=torch.float64), torch.zeros(8, dtype=torch.float64))

    def forward_backward(self, users, items, labels, group, k, inv_batch, grads, reg_rows=None,
                         include_dense_reg=True, probs_out=None):
        w = self.weights()
        zero_l2 = [0.0] * len(self.shape.layers)
        _, g, p = O.loss_and_grads(self.shape, w, users, items, labels, zero_l2, batch_norm=1.0 / inv_batch)
        eg, mg = self.layout.to_device(g, dtype=np.float64)
        grads[0].zero_()
        grads[0][:self.num_rows] = torch.from_numpy(eg)
        grads[1][:] = torch.from_numpy(mg)
        y = np.asarray(labels, dtype=np.float64)
        ng = len(y) // group
        hr, dcg = O.group_metrics(p, y, group, k)
        r0, rc = (0, self.num_rows) if reg_rows is None else reg_rows
        reg = self.l2[0] * float((self.emb[r0:r0 + rc] ** 2).sum())
        if include_dense_reg:
            reg += float((self.mlp_lam * self.mlp ** 2).sum())
        sm = grads[2]
        sm.zero_()
        sm[0] = float(O.bce_per_sample(p, y).sum())
        sm[1], sm[2], sm[3], sm[4] = hr * ng, dcg * ng, ng, reg

    def shard_optimizer_state(self, row_begin, row_count, capacity_rows):
        if capacity_rows > self.emb.shape[0]:
            emb = torch.zeros(capacity_rows, self.row_width, dtype=torch.float64)
            emb[:self.num_rows] = self.emb[:self.num_rows]
            self.emb = emb
        self.emb_m = self.emb_m[row_begin:row_begin + row_count].clone()
        self.emb_v = self.emb_v[row_begin:row_begin + row_count].clone()

    def _adam(self, p, g, m, v):
        m.mul_(self.b1).add_((1 - self.b1) * g)
        v.mul_(self.b2).add_((1 - self.b2) * g * g)
        lr_t = O.adam_lr_t(self.lr, self.b1, self.b2, self.t)
        p.sub_(lr_t * m / (v.sqrt() + O.KERAS_EPSILON))

    def forward_backward_part(self, users, items, labels, group, k, inv_batch, shared_row_begin, grads,
                              probs_out=None, reg_rows=None, include_dense_reg=True):
        full = self.alloc_grads()
        self.forward_backward(users, items, labels, group, k, inv_batch, full, reg_rows=reg_rows,
                              include_dense_reg=include_dense_reg)
        self._local_grad = full[0]
        grads[0].zero_()   # padding rows past the items (split item optimizer) stay zero
        grads[0][:self.num_rows - shared_row_begin] = full[0][shared_row_begin:self.num_rows]
        grads[1][:] = full[1]
        grads[2][:] = full[2]

    def update_rows(self, row_begin, row_count, inv_batch):
        t, self.t = self.t, self.t + 1     # this step's t, not advanced
        sl = slice(row_begin, row_begin + row_count)
        p = self.emb[sl]
        self._adam(p, self._local_grad[sl] + 2.0 * self.l2[0] * p, self.emb_m[sl], self.emb_v[sl])
        self.t = t

    def apply_update(self, grads, inv_batch, rows=None, emb_grad=None, moments_by_row=False):
        self.t += 1
        eg = grads[0] if emb_grad is None else emb_grad
        r0, rc = (0, self.num_rows) if rows is None else rows
        p = self.emb[r0:r0 + rc]
        mo = r0 if moments_by_row else 0
        self._adam(p, eg[:rc] + 2.0 * self.l2[0] * p, self.emb_m[mo:mo + rc], self.emb_v[mo:mo + rc])
        self._adam(self.mlp, grads[1] + 2.0 * self.mlp_lam * self.mlp, self.mlp_m, self.mlp_v)


class OracleShardedEngine(object):
    """CPU look-alike of movierec.sharded.ShardedNCFEngine (float64, oracle arithmetic): the
    same plan / gather_rows / forward_backward / apply_update surface and buffers, so that
    RowShardedDataParallel's exchanges can be tested with gloo on CPU."""

    def __init__(self, shape, w, world, rank, lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=None):
        self.shape = shape
        self.world, self.rank = int(world), int(rank)
        self.layout = Layout(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim)
        self.num_rows = self.layout.num_rows
        self.row_width = self.layout.row_width
        self.shard_rows = -(-self.num_rows // self.world)
        emb, flat = self.layout.to_device(w, dtype=np.float64)
        g = self.owned_rows()
        shard = np.zeros((self.shard_rows, self.row_width))
        shard[g >= 0] = emb[g[g >= 0]]
        self.emb = torch.from_numpy(shard)
        self.mlp = torch.from_numpy(flat)
        self.emb_m = torch.zeros_like(self.emb)
        self.emb_v = torch.zeros_like(self.emb)
        self.mlp_m = torch.zeros_like(self.mlp)
        self.mlp_v = torch.zeros_like(self.mlp)
        P = self.layout.mlp_params
        self.dense_buf = torch.zeros(P + 8, dtype=torch.float64)
        self.mlp_grad = self.dense_buf[:P]
        self.summary = self.dense_buf[P:]
        self.send_counts = torch.zeros(self.world, dtype=torch.int32)
        # RowShardedDataParallel plans the next batch ahead only for a deferred-decay shard whose
        # workspace holds it (the device's dense owner index shares the plan's regions); this
        # look-alike's buffers grow as needed and its update reads no index: it takes that path
        self.lazy = True
        self.max_batch = 1 << 30
        self.t = 0
        self.lr, self.b1, self.b2 = lr, beta_1, beta_2
        self.l2 = list(layers_l2reg or [0.0] * len(shape.layers))
        lam = np.zeros(P)
        off = 0
        for l in range(1, len(shape.layers)):
            a, b = shape.layers[l - 1], shape.layers[l]
            lam[off:off + a * b] = self.l2[l]
            off += a * b + b
        self.mlp_lam = torch.from_numpy(lam)

    def owned_rows(self):
        g = np.arange(self.shard_rows, dtype=np.int64) * self.world + self.rank
        g[g >= self.num_rows] = -1
        return g

    def plan(self, users, items, group=None):
        u = np.asarray(users, dtype=np.int64)
        v = np.asarray(items, dtype=np.int64)
        rows = np.stack([u, self.shape.num_users + v], 1).reshape(-1)   # c = 2i + side
        keys = (rows % self.world) * self.shard_rows + rows // self.world
        ukeys = np.unique(keys)
        self._users, self._items = u, v
        self._ukeys = ukeys
        self.send_counts = torch.from_numpy(np.bincount(ukeys // self.shard_rows, minlength=self.world)
                                            .astype(np.int32))
        n2 = rows.size
        if getattr(self, "_cap", 0) < n2:
            # fixed-capacity buffers, as the device engine's: a plan made ahead (the next batch's)
            # must not move the current step's unique-row gradients
            self._cap = n2
            cap = self.world * min(n2, self.shard_rows)
            self.uniq = torch.zeros(n2, dtype=torch.int32)
            self.uniq_vals = torch.zeros(n2, self.row_width, dtype=torch.float64)
            self.uniq_grad = torch.zeros(n2, self.row_width, dtype=torch.float64)
            self.recv_rows = torch.zeros(cap, dtype=torch.int32)
            self.recv_vals = torch.zeros(cap, self.row_width, dtype=torch.float64)
            self.recv_grad = torch.zeros(cap, self.row_width, dtype=torch.float64)
        self.uniq[:ukeys.size] = torch.from_numpy((ukeys % self.shard_rows).astype(np.int32))
        return self.uniq, self.send_counts

    def _ids(self, x):
        return x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(np.asarray(x).reshape(-1)))

    def flush(self):
        pass

    def gather_rows(self, rows, m, out=None):
        out = self.recv_vals if out is None else out
        out[:m] = self.emb[rows[:m].long()]
        return out[:m]

    def _global_of_uniq(self):
        owner = self._ukeys // self.shard_rows
        local = self._ukeys % self.shard_rows
        return local * self.world + owner

    def forward_backward(self, labels, group, k, inv_batch, include_dense_reg=True, probs_out=None):
        g = self._global_of_uniq()
        full = np.zeros((self.num_rows, self.row_width))
        full[g] = self.uniq_vals[:len(g)].numpy()
        w = self.layout.from_device(full, self.mlp.numpy())
        zero_l2 = [0.0] * len(self.shape.layers)
        _, grads, p = O.loss_and_grads(self.shape, w, self._users, self._items, labels, zero_l2,
                                       batch_norm=1.0 / inv_batch)
        eg, mg = self.layout.to_device(grads, dtype=np.float64)
        self.uniq_grad[:len(g)] = torch.from_numpy(eg[g])
        self.mlp_grad[:] = torch.from_numpy(mg)
        y = np.asarray(labels, dtype=np.float64)
        ng = len(y) // group
        hr, dcg = O.group_metrics(p, y, group, k)
        reg = self.l2[0] * float((self.emb ** 2).sum())
        if include_dense_reg:
            reg += float((self.mlp_lam * self.mlp ** 2).sum())
        sm = self.summary
        sm.zero_()
        sm[0] = float(O.bce_per_sample(p, y).sum())
        sm[1], sm[2], sm[3], sm[4] = hr * ng, dcg * ng, ng, reg

    def _adam(self, p, g, m, v):
        m.mul_(self.b1).add_((1 - self.b1) * g)
        v.mul_(self.b2).add_((1 - self.b2) * g * g)
        lr_t = O.adam_lr_t(self.lr, self.b1, self.b2, self.t)
        p.sub_(lr_t * m / (v.sqrt() + O.KERAS_EPSILON))

    def apply_update(self, recv_rows, recv_grad, m, inv_batch):
        self.t += 1
        G = torch.zeros_like(self.emb)
        rows = recv_rows[:m].long()
        for j in range(int(m)):                    # ascending source order
            G[rows[j]] += recv_grad[j]
        self._adam(self.emb, G + 2.0 * self.l2[0] * self.emb, self.emb_m, self.emb_v)
        self._adam(self.mlp, self.mlp_grad + 2.0 * self.mlp_lam * self.mlp, self.mlp_m, self.mlp_v)
