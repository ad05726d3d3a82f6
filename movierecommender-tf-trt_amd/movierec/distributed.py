"""Data-parallel NCF training over torch.distributed (RCCL over xGMI on MI355X).

One process per GPU.  The reference trains on one CPU (no parallelism of any
kind); this module adds the data-parallel step of BASELINE.json's
north star: minibatches shard across ranks and the dense-layer gradient is
all-reduced.  Two table layouts:

``ReplicatedDataParallel`` — every rank holds the whole table (the north star's
layout at MovieLens scale).

``UserPartitionedDataParallel`` — the training ratings are partitioned by user
(rank r trains the users u % world == r and alone holds their rows and Adam
state); the item table is replicated and its dense gradient is all-reduced in
the same RCCL call as the dense-layer gradient.  One collective per step, no
host synchronisation; the default multi-GPU layout for MovieLens-sized tables.

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

import numpy as np
import torch
import torch.distributed as dist


def ensure_process_group(world_size, backend=None):
    """The process group of a ``world_size``-rank run (``MovierecModel`` params ``world_size``):
    the one already initialised, or one formed from torchrun's environment (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Backend: ``nccl`` (RCCL over xGMI) when the GPUs are visible,
    else ``gloo``; each rank drives GPU LOCAL_RANK.  Returns this process's rank."""
    import os
    if not dist.is_initialized():
        env_world = int(os.environ.get("WORLD_SIZE", "1"))
        if env_world != world_size:
            raise ValueError("world_size %d but WORLD_SIZE=%d: launch one process per GPU, e.g. "
                             "python -m torch.distributed.run --nproc-per-node %d ..." % (world_size, env_world,
                                                                                        world_size))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if torch.cuda.is_available():
            torch.cuda.set_device(local if backend == "nccl" else 0)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if dist.get_world_size() != world_size:
        raise ValueError("world_size %d but the process group has %d ranks" % (world_size, dist.get_world_size()))
    return dist.get_rank()


def all_reduce_min(x, group=None):
    """min over ranks of a host int (the number of steps every rank can run)."""
    t = torch.tensor([int(x)], dtype=torch.int64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


def all_reduce_sum_(t, group=None):
    """In-place sum over ranks of a (device) tensor."""
    _all_reduce(t, group)


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


def _broadcast(t, src, group):
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.broadcast(h, src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src, group=group)


def _all_reduce_async(t, group):
    """Start an all-reduce; returns the work handle (None if it already completed)."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        _all_reduce(t, group)
        return None
    return dist.all_reduce(t, group=group, async_op=True)


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

    def _fetch_rows(self, users, items, group=None):
        eng = self.eng
        uniq, send_counts = eng.plan(users, items, group)
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
        send, recv, nu, m = self._fetch_rows(users, items, group)
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


class NativeComm(object):
    """The library's RCCL communicator (ncf_comm_init) for this rank; destroyed with the object."""

    def __init__(self, handle):
        self.handle = handle

    def close(self):
        if self.handle:
            from . import _native as N
            N.check(N.lib().ncf_comm_destroy(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _native_comm(rank, world, group=None):
    """Form the library's RCCL communicator over the ranks of ``group``: rank 0's unique id goes
    to every rank through the process group, then every rank joins (a collective)."""
    import ctypes
    from . import _native as N
    L = N.lib()
    uid = (ctypes.c_char * 128)()
    if rank == 0:
        N.check(L.ncf_comm_unique_id(uid, 128))
    box = [bytes(uid)]
    dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    uid = (ctypes.c_char * 128).from_buffer_copy(box[0])
    handle = ctypes.c_void_p()
    N.check(L.ncf_comm_init(world, rank, uid, 128, ctypes.byref(handle)))
    return NativeComm(handle)


def partition_keras_weights(w, world, rank):
    """Keras-layout weights of rank ``rank``'s local model under user partitioning: the user
    rows u % world == rank (local row u // world), every item row, the dense layers."""
    out = dict(w)
    for name in ("user_embedding", "user_gmf_embedding"):
        if name in w:
            out[name] = w[name][rank::world]
    return out


class UserPartitionedDataParallel(object):
    """Data parallelism with the training data partitioned by user.

    The reference samples each batch user by user (``data_pipeline.py:115-150``); here rank r
    is given the ratings of the users u with u % world == r, so a user's embedding row is read
    and written by one rank only.  Each rank's ``engine`` is an ordinary single-device engine
    built for ``num_users = ceil((U - r) / world)`` local users (user u at local row u // world)
    and every item; the item rows and the dense layers are replicated.

    One step:

      1. ``forward_backward_part`` on the local batch (user ids already local), BCE mean over
         the GLOBAL batch: dense gradient of the item rows, dense-layer gradient and summary,
         laid out back to back in one buffer; per-sample gradient rows stay in the workspace
      2. ONE asynchronous ``all_reduce`` of [item-row gradient | dense-layer gradient | summary]
         (RCCL, on its own stream) ...
      3. ... while the compute stream applies the fused scatter-add + Adam to the own user rows
         (``update_rows``), which needs nothing from the other ranks
      4. wait; ``apply_update``: Adam over the item rows (identical on every rank), the dense
         layers, stats, step counter

    The own-user gradient never leaves the rank, so each step moves the item table's gradient
    (ml-20m: 27,278 x 512 B = 14 MB) instead of the whole table's.  The result equals one
    device stepping on the concatenated global batch, up to fp32 order of the cross-rank sum.
    """

    def __init__(self, engine, group=None, native=None):
        """``native``: drive the step through ``ncf_user_dp_step`` with the library's own RCCL
        communicator (one host call per step, the all-reduce on its side stream); default: when the
        process group is RCCL (``nccl``) and the engine defers its users' decay.  Otherwise the
        step's calls and the torch.distributed all-reduce are issued one by one (gloo: ranks that
        share one GPU in the tests)."""
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        U, R, W = int(engine.num_users), int(engine.num_rows), int(engine.row_width)
        lazy = getattr(engine, "lazy_rows", None)
        if getattr(engine, "row_step", None) is not None and lazy != U:
            raise ValueError("a deferred-decay engine for user-partitioned training needs lazy_rows = its %d users "
                             "(the replicated item rows are swept every step)" % U)
        if native is None:
            native = (dist.get_backend(group) == "nccl" and getattr(engine, "row_step", None) is not None and
                      hasattr(engine, "user_dp_step"))
        self.comm = _native_comm(self.rank, self.world, group) if native else None
        _, mg0, sm0 = engine.alloc_grads(rows=0)
        P, S = mg0.numel(), sm0.numel()
        dev = engine.emb.device
        self.flat = torch.zeros((R - U) * W + P + S, dtype=engine.emb.dtype, device=dev)
        self.grads = (self.flat[:(R - U) * W].view(R - U, W), self.flat[(R - U) * W:(R - U) * W + P],
                      self.flat[(R - U) * W + P:])
        self.shared = self.flat                  # item rows | dense-layer grad | summary
        self.num_local_users = U
        # the L2 loss of the replicated item rows is reported by rank 0 only
        self.reg_rows = (0, R) if self.rank == 0 else (0, U)

    def broadcast_parameters(self, src=0):
        """Make the replicated part (item rows, dense layers) equal to rank ``src``'s."""
        U = self.num_local_users
        items = self.eng.emb[U:self.eng.num_rows]
        buf = items.contiguous()
        _broadcast(buf, src, self.group)
        items.copy_(buf)
        _broadcast(self.eng.mlp, src, self.group)

    def train_step(self, users, items, labels, group, k, global_batch=None, next_batch=None):
        """``users``: LOCAL user ids (u // world of users owned by this rank).  ``next_batch`` =
        (users, items) device tensors of the following step: its index is built under this step's
        all-reduce (pass the same tensors to the next call)."""
        n = len(users)
        gb = n * self.world if global_batch is None else int(global_batch)
        inv = 1.0 / gb
        eng = self.eng
        U, R = self.num_local_users, int(eng.num_rows)
        if self.comm is not None and eng.row_step is not None:
            eng.user_dp_step(users, items, labels, group=group, k=k, inv_batch=inv, shared=self.shared,
                             comm=self.comm.handle, next_batch=next_batch, include_dense_reg=self.rank == 0)
            return
        eng.forward_backward_part(users, items, labels, group=group, k=k, inv_batch=inv, shared_row_begin=U,
                                  grads=self.grads, reg_rows=self.reg_rows, include_dense_reg=self.rank == 0)
        work = _all_reduce_async(self.shared, self.group)
        if getattr(eng, "lazy_rows", None) == U and eng.row_step is not None:
            # deferred decay of the own users: the touched ones' update, and the next batch's index
            # counted + its own rows caught up ahead, in one launch under the all-reduce
            eng.update_rows(0, U, inv, next_batch=next_batch)
        else:
            eng.update_rows(0, U, inv)               # own users: overlaps the all-reduce
            if next_batch is not None and hasattr(eng, "build_index"):
                eng.build_index(*next_batch, group)  # so does the next step's index
        if work is not None:
            work.wait()
        eng.apply_update(self.grads, inv, rows=(U, R - U), moments_by_row=True)

    def keras_weights(self):
        """Full Keras-layout weights (collective: every rank must call it): user rows gathered
        from their owners, items and dense layers from this rank."""
        eng = self.eng
        local = eng.keras_weights() if hasattr(eng, "keras_weights") else eng.weights()
        out = dict(local)
        for name in ("user_embedding", "user_gmf_embedding"):
            if name not in local:
                continue
            mine = torch.from_numpy(np.ascontiguousarray(local[name]))
            rows = [None] * self.world
            dist.all_gather_object(rows, mine.numpy(), group=self.group)
            total = sum(r.shape[0] for r in rows)
            full = np.empty((total,) + mine.shape[1:], dtype=mine.numpy().dtype)
            for r in range(self.world):
                full[r::self.world] = rows[r]
            out[name] = full
        return out
