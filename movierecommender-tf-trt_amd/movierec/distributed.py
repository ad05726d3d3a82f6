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

import warnings
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


def _batch_token(users, items):
    """What a caller announced as next_batch: tensors by storage, size, dtype, device and version
    counter (an in-place write through torch bumps it); anything else by a copy of its contents."""
    def one(x):
        if torch.is_tensor(x):
            return ("t", x.data_ptr(), x.numel(), x.dtype, str(x.device), x._version)
        return ("h", np.array(x, copy=True))
    return one(users), one(items)


def _same_batch(token, users, items):
    """True when (users, items) are the batch _batch_token recorded, unmodified."""
    for t, x in zip(token, (users, items)):
        if t[0] == "t":
            if not (torch.is_tensor(x) and ("t", x.data_ptr(), x.numel(), x.dtype, str(x.device), x._version) == t):
                return False
        elif torch.is_tensor(x) or not np.array_equal(np.asarray(x), t[1]):
            return False
    return True


class RowShardedDataParallel(object):
    """Drives one rank's ``ShardedNCFEngine`` (or a look-alike) through the row-sharded step:

      1. plan: unique rows of the local batch, grouped by owner (device)
      2. all_to_all of the per-owner counts; their host copy gives the split sizes
      3. all_to_all of the row ids to their owners; owners serve the rows (deferred decay: caught
         up first and indexed for step 6); all_to_all back
      4. forward/backward on the fetched unique rows (per-unique-row gradients)
      5. all_to_all of the gradients to their owners; all_reduce of dense grad + summary
      6. owner: per-row sum of the received gradients (ascending source rank), Adam on the served
         rows (deferred decay) or a dense sweep of the shard; Adam on the replicated dense layers

    ``train_step(..., next_batch=(users, items))`` plans the next batch right after this step's
    forward/backward and exchanges its counts there, copying them to pinned host memory
    asynchronously: the next step reads them with its event long done, so no step waits for
    the device (the host stays up to a step ahead).  Pass exactly those tensors next step.

    ``emulate=True`` (one process, engine built as rank ``engine.rank`` of ``engine.world``):
    every row of the batches must be owned by this rank (the bench draws them so); the exchanges
    become this rank's own buffers, so the step is the per-rank compute of the ``world``-rank step
    without its collectives (a diagnostic of one rank's work, not a scaling result).
    """

    def __init__(self, engine, group=None, emulate=False):
        self.eng = engine
        self.group = group
        self.emulate = bool(emulate)
        if self.emulate:
            self.world, self.rank = engine.world, engine.rank
        else:
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        if (engine.world, engine.rank) != (self.world, self.rank):
            raise ValueError("engine built for rank %d of %d, process group has rank %d of %d"
                             % (engine.rank, engine.world, self.rank, self.world))
        self.recv_counts = torch.zeros_like(engine.send_counts)
        self.last_exchange = None
        self._ahead = None       # (users, items, n, versions, group) planned ahead, counts in flight
        dev = engine.send_counts.device
        pin = dev.type == "cuda"
        self._counts_host = torch.zeros(2 * self.world, dtype=torch.int32, pin_memory=pin)
        self._counts_event = torch.cuda.Event() if pin else None

    def broadcast_parameters(self, src=0):
        """Make every rank's dense layers equal to rank ``src``'s (shards are per rank)."""
        if self.emulate:
            return
        if self.eng.mlp.is_cuda and dist.get_backend(self.group) == "gloo":
            h = self.eng.mlp.cpu()
            dist.broadcast(h, src, group=self.group)
            self.eng.mlp.copy_(h)
        else:
            dist.broadcast(self.eng.mlp, src, group=self.group)

    def _plan_and_count(self, users, items, group, ahead):
        """Plan a batch and exchange its per-owner counts; ``ahead``: the counts' host copy is
        left in flight (read by _counts() of the next step), else read now."""
        eng = self.eng
        eng.plan(users, items, group)
        cat = self._counts_dev = getattr(self, "_counts_dev", None)
        if cat is None or cat.device != eng.send_counts.device:
            cat = self._counts_dev = torch.zeros(2 * self.world, dtype=torch.int32, device=eng.send_counts.device)
        if self.emulate:
            cat[:self.world].copy_(eng.send_counts)
            cat[self.world:].copy_(eng.send_counts)   # the only source is this rank
        else:
            _all_to_all(self.recv_counts, eng.send_counts, None, None, self.group)
            cat[:self.world].copy_(eng.send_counts)
            cat[self.world:].copy_(self.recv_counts)
        if self._counts_event is not None:
            self._counts_host.copy_(cat, non_blocking=True)
            self._counts_event.record()
        else:
            self._counts_host.copy_(cat)
        if not ahead and self._counts_event is not None:
            self._counts_event.synchronize()

    def _counts(self):
        if self._counts_event is not None:
            self._counts_event.synchronize()   # recorded a step ago when planned ahead
        c = self._counts_host.tolist()
        return c[:self.world], c[self.world:]

    def _fetch_rows(self, users, items, group=None):
        eng = self.eng
        held = self._ahead
        self._ahead = None
        ready = held is not None and group is not None and held[4] == int(group) and _same_batch(held[3], users, items)
        if held is not None and group is not None and not ready:
            # re-planning here would issue a counts exchange the ranks whose held plan matches do
            # not issue: the collectives would no longer pair up.  Every rank holds a plan for the
            # batch it announced, so a different batch (or ids refilled in place) is an error
            raise RuntimeError("train_step got another batch than the next_batch= announced in the previous "
                               "step (or its ids changed since): pass exactly those tensors, unmodified")
        if ready:
            eng._n = held[2]   # the plan ahead's batch (the engine planned it last), its normalised ids
        else:
            u, i = eng._ids(users), eng._ids(items)
            self._plan_and_count(u, i, group, ahead=False)
        send, recv = self._counts()
        nu, m = sum(send), sum(recv)
        if self.emulate:
            # every row is this rank's own: its unique rows are the served rows (the id copy stands
            # for the id exchange: the next batch's plan reuses uniq before this step's update)
            eng.recv_rows[:nu].copy_(eng.uniq[:nu])
            vals = eng.gather_rows(eng.recv_rows, nu, out=eng.uniq_vals)
            self._rows_in, self._grad_in = eng.recv_rows, eng.uniq_grad
        else:
            _all_to_all(eng.recv_rows[:m], eng.uniq[:nu], recv, send, self.group)
            vals = eng.gather_rows(eng.recv_rows, m)
            _all_to_all(eng.uniq_vals[:nu], vals, send, recv, self.group)
            self._rows_in, self._grad_in = eng.recv_rows, eng.recv_grad
        self.last_exchange = (nu, m)
        return send, recv, nu, m

    def train_step(self, users, items, labels, group, k, global_batch=None, next_batch=None):
        n = len(users)
        gb = n * self.world if global_batch is None else int(global_batch)
        inv = 1.0 / gb
        eng = self.eng
        send, recv, nu, m = self._fetch_rows(users, items, group)
        eng.forward_backward(labels, group=group, k=k, inv_batch=inv, include_dense_reg=self.rank == 0)
        # The next batch is planned here only under deferred decay: the dense shard update
        # (ncf_shard_apply_update without row_step) builds its owner index in per-batch workspace
        # regions that a plan of the next batch would overwrite, and a next batch larger than the
        # workspace would reallocate it under this step's pending update.  Every rank decides
        # alike — the engines share the layout, the batches their size, and the decision reads
        # nothing of how a rank holds its ids: host, int64 or off-device ids are normalised
        # (eng._ids) and planned like device int32 tensors, the announced objects remembered by
        # identity (tensors: storage, size and version counter; host arrays: a copy of the
        # contents) for the next step's check.  (a rank whose ids _ids copied used to
        # skip the plan while the others planned, so the next step's counts exchange did not pair.)
        if next_batch is not None and eng.lazy and len(next_batch[0]) <= eng.max_batch:
            # the forward/backward and its compact gradient were the last readers of this step's plan
            nu_, ni_ = eng._ids(next_batch[0]), eng._ids(next_batch[1])
            self._plan_and_count(nu_, ni_, group, ahead=True)
            self._ahead = (nu_, ni_, nu_.numel(), _batch_token(next_batch[0], next_batch[1]), int(group))
        if not self.emulate:
            _all_to_all(eng.recv_grad[:m], eng.uniq_grad[:nu], recv, send, self.group)
            _all_reduce(eng.dense_buf, self.group)
        eng.apply_update(self._rows_in, self._grad_in, m, inv)

    def predict(self, users, items):
        """Predictions for this rank's (users, items); every rank must call it (exchanges)."""
        self.eng.flush()
        self._fetch_rows(users, items)
        return self.eng.predict_planned()

    def flush(self):
        self.eng.flush()

    def full_table(self):
        """The whole embedding table [num_rows x row_width] assembled from every shard."""
        eng = self.eng
        eng.flush()
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


_NATIVE_CHECKS = {}


def native_step_check(layers, gmf_dim, group_size, split, group=None, steps=5, per=2048):
    """The library's one-call user-partitioned step (``ncf_user_dp_step`` / ``_split``: its own RCCL
    communicator, the collectives on a side stream beside the own-user update and the next
    batch's index) against the same step issued call by call with torch.distributed's
    collectives, from identical state, on a model of these shapes with small tables (4,000 users x
    3,000 items), ``steps`` steps of ``per`` samples per rank.  Every rank compares its weights,
    Adam moments and stats; returns the max difference over the ranks and whether it is within
    fp32 order of the cross-rank sums (``ok``: <= 1e-5).  A collective: every rank of ``group``
    calls it."""
    from .engine import NCFEngine
    from .model import initial_weights
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    U, I, g = 4000, 3000, int(group_size)
    per = per // g * g
    w = initial_weights(U, I, list(layers), int(gmf_dim), seed=7)
    n_loc = (U - rank + world - 1) // world
    gen = torch.Generator(device="cuda").manual_seed(99 + rank)
    batches = []
    for _ in range(steps):
        u = torch.randint(0, n_loc, (per // g,), generator=gen, device="cuda", dtype=torch.int32).repeat_interleave(g)
        it = torch.randint(0, I, (per,), generator=gen, device="cuda", dtype=torch.int32)
        y = torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(per // g)
        batches.append((u.contiguous(), it, y))
    states = []
    for native in (True, False):
        eng = NCFEngine(n_loc, I, list(layers), int(gmf_dim), max_batch=per, lazy_adam=True, lazy_rows=n_loc)
        eng.set_keras_weights(partition_keras_weights(w, world, rank))
        dp = UserPartitionedDataParallel(eng, group=group, native=native, split_items=split)
        for s_, (u, it, y) in enumerate(batches):
            nxt = batches[s_ + 1][:2] if s_ + 1 < steps else None
            dp.train_step(u, it, y, group=g, k=min(10, g - 1), next_batch=nxt)
        eng.flush()
        R = eng.num_rows
        states.append(torch.cat([eng.emb[:R].flatten(), eng.emb_m[:R].flatten(), eng.emb_v[:R].flatten(), eng.mlp,
                                 eng.mlp_m, eng.mlp_v, eng.stats.float()]))
        if dp.comm is not None:
            dp.comm.close()
    d = (states[0] - states[1]).abs().max().double().reshape(1)
    same = torch.tensor([0.0 if torch.equal(states[0], states[1]) else 1.0], dtype=torch.float64, device="cuda")
    t = torch.cat([d, same])
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    torch.cuda.synchronize()
    return {"max_abs_diff": float(t[0]), "bitwise": bool(t[1] == 0), "steps": steps, "per_rank_batch": per,
            "tables": "%d x %d" % (U, I), "ok": float(t[0]) <= 1e-5}


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

    def __init__(self, engine, group=None, native=None, split_items=False, emulate_world=None):
        """``native``: drive the step through ``ncf_user_dp_step`` with the library's own RCCL
        communicator (one host call per step, the all-reduce on its side stream); default: when the
        process group is RCCL (``nccl``) and the engine defers its users' decay.  Otherwise the
        step's calls and the torch.distributed collectives are issued one by one (gloo: ranks that
        share one GPU in the tests).

        ``split_items``: the item rows' Adam split across the ranks (``ncf_user_dp_step_split``):
        a reduce-scatter of the item-row gradient (rank r gets item rows [r Ic, r Ic + Ic), Ic =
        ceil(items / world)) with the all-reduce of [dense-layer gradient | summary], Adam on the
        rank's item slice, an all-gather of the updated item rows.  The same bytes on the links
        as the all-reduce; the item Adam and its moment traffic per rank are 1/world.  The table
        is padded to world * Ic item rows for the in-place all-gather.

        ``emulate_world`` (one-rank process group): rank 0's compute of a step of that many ranks
        (its item slice only, no exchange) — the bench's per-rank diagnostic.

        Construction is a COLLECTIVE over ``group`` when the one-call step is considered at world
        > 1: every rank must construct its instance together (the first construction per model
        shape runs ``native_step_check``, 2 x 5 training steps with their collectives, and the
        library communicator's rendezvous).  A failed check logs a warning and falls back to the
        call-by-call step (``self.native_check`` holds its numbers)."""
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        U, R, W = int(engine.num_users), int(engine.num_rows), int(engine.row_width)
        lazy = getattr(engine, "lazy_rows", None)
        if getattr(engine, "row_step", None) is not None and lazy != U:
            raise ValueError("a deferred-decay engine for user-partitioned training needs lazy_rows = its %d users "
                             "(the replicated item rows are swept every step)" % U)
        self.native_check = None
        if native is None:
            native = (dist.get_backend(group) == "nccl" and getattr(engine, "row_step", None) is not None and
                      hasattr(engine, "user_dp_step"))
            if native and self.world > 1:
                # a world > 1 run uses the one-call step only after it matched the call-by-call step
                # on this process group (once per model shape)
                key = (tuple(engine.layers), int(engine.gmf_dim), bool(split_items), id(group))
                if key not in _NATIVE_CHECKS:
                    _NATIVE_CHECKS[key] = native_step_check(engine.layers, engine.gmf_dim, 4, bool(split_items), group)
                self.native_check = _NATIVE_CHECKS[key]
                native = self.native_check["ok"]
                if not native:
                    warnings.warn("the one-call RCCL user step differs from the call-by-call step on this process "
                                  "group (%r): falling back to the call-by-call step" % (self.native_check,),
                                  RuntimeWarning, stacklevel=2)
        self.comm = _native_comm(self.rank, self.world, group) if native else None
        iw = self.world
        if emulate_world is not None and int(emulate_world) > 1:
            if self.world != 1:
                raise ValueError("emulate_world needs a one-rank process group")
            iw = int(emulate_world)
        self.split = bool(split_items)
        self.item_world, self.item_rank = (iw, self.rank) if self.split else (1, 0)
        I = R - U
        self.Ic = -(-I // self.item_world)
        rows_g = self.item_world * self.Ic if self.split else I
        if self.split and U + rows_g > engine.emb.shape[0]:
            # zero padding rows past the items: the in-place all-gather writes item_world * Ic rows
            emb = torch.zeros(U + rows_g, W, dtype=engine.emb.dtype, device=engine.emb.device)
            emb[:R].copy_(engine.emb[:R])
            engine.emb = emb
            from . import _native as N
            engine.model_s = N.NcfModel(engine.emb.data_ptr(), engine.mlp.data_ptr())
        _, mg0, sm0 = engine.alloc_grads(rows=0)
        P, S = mg0.numel(), sm0.numel()
        dev = engine.emb.device
        self.flat = torch.zeros(rows_g * W + P + S, dtype=engine.emb.dtype, device=dev)
        self.grads = (self.flat[:rows_g * W].view(rows_g, W), self.flat[rows_g * W:rows_g * W + P],
                      self.flat[rows_g * W + P:])
        self.shared = self.flat                  # item rows | dense-layer grad | summary
        self.slice_grad = (torch.zeros(self.Ic, W, dtype=engine.emb.dtype, device=dev)
                           if self.split else None)
        self.num_local_users = U
        # the L2 loss of the replicated item rows is reported by rank 0 only
        self.reg_rows = (0, R) if self.rank == 0 else (0, U)
        self._t_every, self._t_calls, self._t_sets = 0, 0, []

    # ---- exchange timing (bench.py's in-step diagnostic at N > 1) ----
    def exchange_timing(self, every):
        """Every ``every``-th step from now on (0: none) records how long its collectives run and
        how long the compute stream waits for them: HIP events on the library communicator's side
        stream and around its join waits (one-call step, ``ncf_comm_timing``), or CUDA events on the
        compute stream around the collective calls and waits (call-by-call step)."""
        self._t_every, self._t_calls, self._t_sets = int(every), 0, []
        if self.comm is not None:
            from . import _native as N
            N.check(N.lib().ncf_comm_timing(self.comm.handle, int(every)))

    def read_exchange_timing(self):
        """Mean ms per sampled step since ``exchange_timing``: ``rs_ar_ms`` / ``ag_ms`` (the
        reduce-scatter + all-reduce group, or the all-reduce, and the all-gather on the
        communicator's stream; None when not observable — torch's collectives run on streams of
        their own), ``rs_ar_exposed_ms`` / ``ag_exposed_ms`` (the compute stream's waits), the
        sampled ``steps`` and the ``path``."""
        if self.comm is not None:
            import ctypes
            from . import _native as N
            out = (ctypes.c_double * 4)()
            k = ctypes.c_int64()
            N.check(N.lib().ncf_comm_timing_read(self.comm.handle, out, ctypes.byref(k)))
            k = int(k.value)
            mean = [v / k if k else None for v in out]
            return {"steps": k, "rs_ar_ms": mean[0], "ag_ms": mean[1] if self.split and self.world > 1 else None,
                    "rs_ar_exposed_ms": mean[2], "ag_exposed_ms": mean[3] if self.split and self.world > 1 else None,
                    "path": "one-call step (ncf_user_dp_step%s, library RCCL communicator)" % ("_split" if self.split else "")}
        torch.cuda.synchronize()
        k = len(self._t_sets)
        acc = [0.0, 0.0]
        for ev in self._t_sets:
            for j, pair in enumerate(ev):
                for a, b in pair:
                    acc[j] += a.elapsed_time(b)
        self._t_sets = []
        gather = self.split and self.world > 1
        return {"steps": k, "rs_ar_ms": None, "ag_ms": None,
                "rs_ar_exposed_ms": acc[0] / k if k else None, "ag_exposed_ms": acc[1] / k if k and gather else None,
                "path": "call by call (torch.distributed %s collectives)" % dist.get_backend(self.group)}

    def _t_begin(self):
        """The call-by-call step's event lists ([waits for the reduce-scatter/all-reduce], [for the
        all-gather]) when this step is sampled, else None."""
        if self._t_every <= 0:
            return None
        self._t_calls += 1
        if (self._t_calls - 1) % self._t_every:
            return None
        ev = ([], [])
        self._t_sets.append(ev)
        return ev

    @staticmethod
    def _t_span(ev, j, fn):
        """fn() bracketed by CUDA events on the current stream when ev is set."""
        if ev is None:
            return fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        r = fn()
        b.record()
        ev[j].append((a, b))
        return r

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
                             comm=self.comm.handle, next_batch=next_batch, include_dense_reg=self.rank == 0,
                             split=(self.item_world, self.item_rank, self.slice_grad) if self.split else None)
            return
        eng.forward_backward_part(users, items, labels, group=group, k=k, inv_batch=inv, shared_row_begin=U,
                                  grads=self.grads, reg_rows=self.reg_rows, include_dense_reg=self.rank == 0)
        ev = self._t_begin()
        if self.split:
            return self._split_tail(U, R, inv, group, next_batch, ev)
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
            self._t_span(ev, 0, work.wait)
        eng.apply_update(self.grads, inv, rows=(U, R - U), moments_by_row=True)

    def _split_tail(self, U, R, inv, group, next_batch, ev=None):
        """The split-items step after the forward/backward, call by call (ncf_user_dp_step_split's
        sequence): reduce-scatter of the item gradient + all-reduce of the dense part, the own
        users' update and the next index meanwhile, the item slice's Adam, the all-gather."""
        eng = self.eng
        eg, mg, sm = self.grads
        r0 = self.item_rank * self.Ic
        cnt = max(0, min(self.Ic, (R - U) - r0))
        dense = self.flat[eg.numel():]
        exchange = self.world > 1
        if exchange:
            self._t_span(ev, 0, lambda: _reduce_scatter(self.slice_grad, eg, self.group))
            work = _all_reduce_async(dense, self.group)
            slice_grad = self.slice_grad
        else:
            work = None
            slice_grad = eg[r0:r0 + self.Ic]
        if getattr(eng, "lazy_rows", None) == U and eng.row_step is not None:
            eng.update_rows(0, U, inv, next_batch=next_batch)
        else:
            eng.update_rows(0, U, inv)
            if next_batch is not None and hasattr(eng, "build_index"):
                eng.build_index(*next_batch, group)
        if work is not None:
            self._t_span(ev, 0, work.wait)
        eng.apply_update((slice_grad, mg, sm), inv, rows=(U + (r0 if cnt else R - U), cnt), moments_by_row=True)
        if exchange:
            items = eng.emb[U:U + self.item_world * self.Ic]
            self._t_span(ev, 1, lambda: _all_gather_inplace(items, self.Ic, self.group))

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
