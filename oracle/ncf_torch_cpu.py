"""CPU baseline trainer: the reference's Keras training step restated on torch-CPU (fp32).

TEST / BASELINE INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): ``bench.py``'s
``cpu_baseline`` leg times it on the GPU box's host cores; nothing in the product path
imports it.  It stands in for "the reference TF-CPU trainer.py timed on the same box"
(BASELINE.json north_star), which cannot run there: TensorFlow is absent and the reference
never travels to the GPU box.  Like TF-CPU it is a framework trainer on the
host's BLAS threads — autograd graph, dense gradients, dense optimizer — not a hand-tuned
kernel:

* graph (``movierec/model.py:154-194``): user/item ``Embedding`` gathers (``:161-170``),
  concatenation (``:171-172``), ``Dense(relu)`` per hidden layer (``:175-181``), the NeuMF
  GMF product when ``gmf_dim > 0``, ``Dense(1, sigmoid)`` (``:184-188``);
* loss (``:213-214``): Keras ``binary_crossentropy`` — clip to ``[1e-7, 1-1e-7]``, logit,
  sigmoid cross-entropy, batch mean; autograd through the clip gives TF's zero gradient
  outside the range;
* optimizer (``:199-202``): Keras v1 Adam on EVERY element (the embedding gradient is the
  densified IndexedSlices): ``lr_t = lr*sqrt(1-b2^t)/(1-b1^t)``,
  ``p -= lr_t*m/(sqrt(v)+1e-7)``.
"""

import math
import os
import time

import numpy as np
import torch

KERAS_EPSILON = 1e-7


def host_threads():
    """Threads the baseline uses: the cores this process may run on, capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box's per-GPU CPU share)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


class TorchCPUTrainer(object):
    def __init__(self, num_users, num_items, layers, gmf_dim, lr=0.001, beta_1=0.9, beta_2=0.999, seed=0):
        g = torch.Generator().manual_seed(seed)
        L = [int(x) for x in layers]

        def glorot(r, c):
            lim = math.sqrt(6.0 / (r + c))
            return ((torch.rand(r, c, generator=g) * 2 - 1) * lim).requires_grad_()

        self.params = {}
        if L:   # layers == []: the GMF-only model (BASELINE config A)
            du, di = L[0] // 2, L[0] - L[0] // 2
            self.params["user_embedding"] = glorot(num_users, du)
            self.params["item_embedding"] = glorot(num_items, di)
        if gmf_dim > 0:
            self.params["user_gmf_embedding"] = glorot(num_users, gmf_dim)
            self.params["item_gmf_embedding"] = glorot(num_items, gmf_dim)
        self.hidden = []
        for l in range(1, len(L)):
            k = glorot(L[l - 1], L[l])
            b = torch.zeros(L[l], requires_grad=True)
            self.params["hidden_%d/kernel" % l], self.params["hidden_%d/bias" % l] = k, b
            self.hidden.append((k, b))
        f = gmf_dim + (L[-1] if L else 0)
        self.has_mlp = bool(L)
        lim = math.sqrt(3.0 / f)
        self.params["output/kernel"] = ((torch.rand(f, 1, generator=g) * 2 - 1) * lim).requires_grad_()
        self.params["output/bias"] = torch.zeros(1, requires_grad=True)
        self.gmf_dim = gmf_dim
        self.m = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.t = 0
        self.lr, self.b1, self.b2 = lr, beta_1, beta_2

    def train_step(self, users, items, labels):
        P = self.params
        if self.has_mlp:
            h = torch.cat([P["user_embedding"][users], P["item_embedding"][items]], dim=1)
            for k, b in self.hidden:
                h = torch.relu(h @ k + b)
        else:
            h = torch.zeros(len(users), 0)
        if self.gmf_dim > 0:
            h = torch.cat([P["user_gmf_embedding"][users] * P["item_gmf_embedding"][items], h], dim=1)
        p = torch.sigmoid(h @ P["output/kernel"] + P["output/bias"]).reshape(-1)
        pc = p.clamp(KERAS_EPSILON, 1.0 - KERAS_EPSILON)
        logit = torch.log(pc / (1.0 - pc))
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, labels)
        for x in P.values():
            x.grad = None
        loss.backward()
        self.t += 1
        lr_t = self.lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        with torch.no_grad():
            for name, x in P.items():
                gr, m, v = x.grad, self.m[name], self.v[name]
                m.mul_(self.b1).add_(gr, alpha=1.0 - self.b1)
                v.mul_(self.b2).addcmul_(gr, gr, value=1.0 - self.b2)
                x.addcdiv_(m, v.sqrt().add_(KERAS_EPSILON), value=-lr_t)
        return float(loss.detach())


def time_protocol(num_users, num_items, layers, gmf_dim, batch, negs, warmup, steps, repeats, budget_s=None):
    """BASELINE.md's CPU protocol: `warmup` untimed steps, then `repeats` runs of `steps` timed
    steps on fresh synthetic batches; returns (median samples/s, per-run samples/s, threads).
    ``budget_s`` bounds the whole timing (the step count of each run shrinks to fit)."""
    threads = host_threads()
    torch.set_num_threads(threads)
    tr = TorchCPUTrainer(num_users, num_items, layers, gmf_dim)
    g = negs + 1
    rng = np.random.RandomState(1)

    def batch_of():
        users = torch.from_numpy(rng.randint(0, num_users, batch // g).repeat(g).astype(np.int64))
        items = torch.from_numpy(rng.randint(0, num_items, batch).astype(np.int64))
        y = torch.from_numpy(np.tile([0.0] * (g - 1) + [1.0], batch // g).astype(np.float32))
        return users, items, y

    t0 = time.perf_counter()
    for _ in range(warmup):
        tr.train_step(*batch_of())
    per_step = (time.perf_counter() - t0) / max(warmup, 1)
    if budget_s is not None and per_step > 0:
        steps = int(max(1, min(steps, budget_s / (repeats * per_step))))
    rates = []
    for _ in range(repeats):
        bs = [batch_of() for _ in range(steps)]
        t0 = time.perf_counter()
        for b in bs:
            tr.train_step(*b)
        rates.append(steps * batch / (time.perf_counter() - t0))
    return float(np.median(rates)), rates, threads, steps
