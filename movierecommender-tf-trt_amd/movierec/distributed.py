"""Data-parallel NCF training over torch.distributed (RCCL over xGMI on MI355X).

One process per GPU.  The reference trains on one CPU (no parallelism of any
kind); this module adds the data-parallel step of BASELINE.json's
north star: minibatches shard across ranks, embedding tables are replicated
(MovieLens scale), the dense-layer gradient is all-reduced.

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
