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
        return self.layout.from_device(self.emb.numpy(), self.mlp.numpy())

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

    def apply_update(self, grads, inv_batch, rows=None, emb_grad=None):
        self.t += 1
        eg = grads[0] if emb_grad is None else emb_grad
        r0, rc = (0, self.num_rows) if rows is None else rows
        p = self.emb[r0:r0 + rc]
        self._adam(p, eg[:rc] + 2.0 * self.l2[0] * p, self.emb_m[:rc], self.emb_v[:rc])
        self._adam(self.mlp, grads[1] + 2.0 * self.mlp_lam * self.mlp, self.mlp_m, self.mlp_v)
