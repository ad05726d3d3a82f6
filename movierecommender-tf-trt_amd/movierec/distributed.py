"""Data-parallel NCF training over torch.distributed (RCCL over xGMI on MI355X).

One process per GPU.  The reference trains on one CPU (no parallelism of any
kind); this module adds the data-parallel step of BASELINE.json's
north star: minibatches shard across ranks and the dense-layer gradient is
all-reduced.  Two table layouts:

``ReplicatedDataParallel`` — every rank holds the whole table (the north star's
layout at MovieLens scale).

``RowShardedDataParallel`` — rank r owns the rows g % world == r and their Adam
state (SURVEY §8e, config D and the recommended layout for config C's scaling
run).  Per step only the batch's unique rows move: row ids and row values
between requester and owner, then the unique-row gradients back
(``all_to_all``), and the dense Adam sweep of the table is split N ways.

Replicated tables with dense (Keras) Adam need every rank to apply the same
update to every row.  Instead of an all-reduce of the 85 MB dense embedding
gradient followed by N identical full-table Adam sweeps, the all-reduce is
split into its two halves with the optimizer between them (the same bytes on
the wire; 1/N of the sweep per rank, 1/N of the Adam moments in HBM):

  1. ncf_forward_backward on the local batch; BCE mean over the GLOBAL batch
     (inv_batch = 1 / (local batch * world)); the L2 loss of this rank's row
     shard (+ dense kernels on rank 0) goes into the summary
  2. reduce_scatter(dense embedding gradient) -> this rank's row shard;
     all_reduce(dense-layer gradient, summary)
  3. ncf_apply_update: Adam on the own shard rows, and on every dense
     parameter (identical on all ranks)
  4. all_gather(table shards) -> replicated table

The result equals a single-device step on the concatenated global batch (up
to fp32 summation order of the cross-rank gradient sum).
"""

import torch
import torch.distributed as dist


def _reduce_scatter(out, inp, group):
    try:
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)
    except (RuntimeError, NotImplementedError, AttributeError, ValueError):
        # backends without reduce_scatter (gloo): all-reduce, keep the own slice
        full = inp.clone()
        dist.all_reduce(full, group=group)
        rank = dist.get_rank(group)
        out.copy_(full.view(-1, *out.shape)[rank] if out.dim() else full)


def _all_gather_inplace(table, shard_rows, group):
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    mine = table[rank * shard_rows:(rank + 1) * shard_rows]
    try:
        dist.all_gather_into_tensor(table, mine, group=group)
    except (RuntimeError, NotImplementedError, AttributeError, ValueError):
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine.contiguous(), group=group)
        table.copy_(torch.cat(parts, 0))


def _all_to_all(out, inp, out_splits, in_splits, group):
    """``all_to_all_single`` along dim 0 with uneven splits; gloo (tests) moves host tensors only,
    so device tensors are staged through the host there."""
    if out.is_cuda and dist.get_backend(group) == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _all_reduce(t, group):
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)


class RowShardedDataParallel(object):
    """Drives one rank's ``ShardedNCFEngine`` (or a look-alike) through the row-sharded step:

      1. plan: unique rows of the local batch, grouped by owner (device)
      2. all_to_all of the per-owner counts; one host read of the counts (split sizes)
      3. all_to_all of the row ids to their owners; owners gather the rows; all_to_all back
      4. forward/backward on the fetched unique rows (per-unique-row gradients)
      5. all_to_all of the gradients to their owners; all_reduce of dense grad + summary
      6. owner: per-row sum of the received gradients (ascending source rank), dense Adam over
         the shard; Adam on the replicated dense layers
    """

    def __init__(self, engine, group=None):
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if (engine.world, engine.rank) != (self.world, self.rank):
            raise ValueError("engine built for rank %d of %d, process group has rank %d of %d"
                             % (engine.rank, engine.world, self.rank, self.world))
        self.recv_counts = torch.zeros_like(engine.send_counts)
        self.last_exchange = None

    def broadcast_parameters(self, src=0):
        """Make every rank's dense layers equal to rank ``src``'s (shards are per rank)."""
        if self.eng.mlp.is_cuda and dist.get_backend(self.group) == "gloo":
            h = self.eng.mlp.cpu()
            dist.broadcast(h, src, group=self.group)
            self.eng.mlp.copy_(h)
        else:
            dist.broadcast(self.eng.mlp, src, group=self.group)

    def _fetch_rows(self, users, items):
        eng = self.eng
        uniq, send_counts = eng.plan(users, items)
        _all_to_all(self.recv_counts, send_counts, None, None, self.group)
        counts = torch.cat([send_counts, self.recv_counts]).cpu().tolist()
        send, recv = counts[:self.world], counts[self.world:]
        nu, m = sum(send), sum(recv)
        _all_to_all(eng.recv_rows[:m], uniq[:nu], recv, send, self.group)
        vals = eng.gather_rows(eng.recv_rows, m)
        _all_to_all(eng.uniq_vals[:nu], vals, send, recv, self.group)
        self.last_exchange = (nu, m)
        return send, recv, nu, m

    def train_step(self, users, items, labels, group, k, global_batch=None):
        n = len(users)
        gb = n * self.world if global_batch is None else int(global_batch)
        inv = 1.0 / gb
        eng = self.eng
        send, recv, nu, m = self._fetch_rows(users, items)
        eng.forward_backward(labels, group=group, k=k, inv_batch=inv, include_dense_reg=self.rank == 0)
        _all_to_all(eng.recv_grad[:m], eng.uniq_grad[:nu], recv, send, self.group)
        _all_reduce(eng.dense_buf, self.group)
        eng.apply_update(eng.recv_rows, eng.recv_grad, m, inv)

    def predict(self, users, items):
        """Predictions for this rank's (users, items); every rank must call it (exchanges)."""
        self._fetch_rows(users, items)
        return self.eng.predict_planned()

    def full_table(self):
        """The whole embedding table [num_rows x row_width] assembled from every shard."""
        eng = self.eng
        parts = [torch.empty_like(eng.emb) for _ in range(self.world)]
        if eng.emb.is_cuda and dist.get_backend(self.group) == "gloo":
            hp = [p.cpu() for p in parts]
            dist.all_gather(hp, eng.emb.cpu().contiguous(), group=self.group)
            parts = hp
        else:
            dist.all_gather(parts, eng.emb.contiguous(), group=self.group)
        full = torch.stack(parts, 1).reshape(-1, eng.row_width)  # row g = local * world + owner
        return full[:eng.num_rows]

    def keras_weights(self):
        """Full Keras-layout weights (collective: every rank must call it)."""
        full = self.full_table().cpu().numpy()
        return self.eng.layout.from_device(full, self.eng.mlp.detach().cpu().numpy())


class ReplicatedDataParallel(object):
    """Wraps an NCFEngine (one per rank) for replicated-table data parallelism."""

    def __init__(self, engine, group=None):
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        R = int(engine.num_rows)
        self.shard_rows = -(-R // self.world)
        self.capacity = self.shard_rows * self.world
        self.row_begin = self.rank * self.shard_rows
        self.row_count = max(0, min(self.shard_rows, R - self.row_begin))
        engine.shard_optimizer_state(self.row_begin, self.row_count, self.capacity)
        self.grads = engine.alloc_grads(rows=self.capacity)
        self.grad_shard = torch.zeros(self.shard_rows, engine.row_width, dtype=self.grads[0].dtype,
                                      device=self.grads[0].device)

    def broadcast_parameters(self, src=0):
        """Make every replica start from rank ``src``'s weights."""
        dist.broadcast(self.eng.emb, src, group=self.group)
        dist.broadcast(self.eng.mlp, src, group=self.group)

    def train_step(self, users, items, labels, group, k, global_batch=None):
        n = len(users)
        gb = n * self.world if global_batch is None else int(global_batch)
        inv = 1.0 / gb
        eng = self.eng
        eng.forward_backward(users, items, labels, group=group, k=k, inv_batch=inv, grads=self.grads,
                             reg_rows=(self.row_begin, self.row_count), include_dense_reg=self.rank == 0)
        eg, mg, sm = self.grads
        _reduce_scatter(self.grad_shard, eg, self.group)
        dist.all_reduce(mg, group=self.group)
        dist.all_reduce(sm, group=self.group)
        eng.apply_update(self.grads, inv, rows=(self.row_begin, self.row_count), emb_grad=self.grad_shard)
        _all_gather_inplace(eng.emb, self.shard_rows, self.group)
