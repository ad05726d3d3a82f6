"""Data-parallel orchestration (movierec.distributed) with world_size 2 and 3.

CPU part (gloo, no GPU): ranks drive the oracle-backed OracleEngine /
OracleShardedEngine through ReplicatedDataParallel / RowShardedDataParallel;
after several steps every rank's weights must equal a single-process run on the
concatenated global batch (float64, so only the cross-rank summation order
differs).

GPU part (-m gpu): processes share the one GPU of the box with the gloo backend
and drive the real HIP library (NCFEngine / ShardedNCFEngine); compared against
a single-process NCFEngine run on the global batch at the fp32 tolerance.  The
row-sharded path with world 1 must be bitwise identical to ncf_train_step.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import gpu_available
from oracle import ncf_oracle as O

SHAPE = (23, 17, [8, 6, 4], 4)
L2 = [0.01, 0.02, 0.0]
STEPS = 3
B = 48          # global batch
GROUP = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


SHAPE_D = (40, 30, [256, 128, 64, 32], 128)   # config D's model (layered path), small tables


def _weights(dims=SHAPE):
    shape = O.NCFShape(*dims)
    w = O.init_weights(shape, seed=4)
    scale = 3 if dims == SHAPE else 1
    return shape, {k: (v * scale).astype(np.float32).astype(np.float64) for k, v in w.items()}


def _l2(dims):
    return L2 if dims == SHAPE else [0.0] * len(dims[2])


def _batches(dims=SHAPE):
    shape = O.NCFShape(*dims)
    rng = np.random.RandomState(7)
    out = []
    for _ in range(STEPS):
        users = rng.randint(0, shape.num_users, B // GROUP).repeat(GROUP).astype(np.int32)
        items = rng.randint(0, shape.num_items, B).astype(np.int32)
        y = np.tile([0] * (GROUP - 1) + [1], B // GROUP).astype(np.float32)
        out.append((users, items, y))
    return out


def _cpu_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from oracle_engine import OracleEngine
    from movierec.distributed import ReplicatedDataParallel
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights()
    eng = OracleEngine(shape, w, layers_l2reg=L2)
    dp = ReplicatedDataParallel(eng)
    summaries = []
    per = B // world
    for users, items, y in _batches():
        sl = slice(rank * per, (rank + 1) * per)
        dp.train_step(users[sl], items[sl], y[sl], group=GROUP, k=2)
        summaries.append(dp.grads[2].clone().numpy())
    q.put((rank, eng.emb[:eng.num_rows].numpy().copy(), eng.mlp.numpy().copy(), summaries))
    dist.barrier()
    dist.destroy_process_group()


def test_replicated_dp_matches_single_process_cpu():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_engine import OracleEngine
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, emb, mlp, summ = q.get(timeout=120)
        res[r] = (emb, mlp, summ)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference on the global batch
    shape, w = _weights()
    ref = OracleEngine(shape, w, layers_l2reg=L2)
    grads = ref.alloc_grads()
    ref_summ = []
    for users, items, y in _batches():
        ref.forward_backward(users, items, y, group=GROUP, k=2, inv_batch=1.0 / B, grads=grads)
        ref_summ.append(grads[2].clone().numpy())
        ref.apply_update(grads, 1.0 / B)
    for r in range(world):
        emb, mlp, summ = res[r]
        np.testing.assert_allclose(emb, ref.emb[:ref.num_rows].numpy(), rtol=0, atol=1e-12)
        np.testing.assert_allclose(mlp, ref.mlp.numpy(), rtol=0, atol=1e-12)
        for a, b in zip(summ, ref_summ):
            np.testing.assert_allclose(a[:5], b[:5], rtol=1e-6, atol=1e-9)


def _cpu_sharded_worker(rank, world, port, q, ahead=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from oracle_engine import OracleShardedEngine
    from movierec.distributed import RowShardedDataParallel
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights()
    eng = OracleShardedEngine(shape, w, world, rank, layers_l2reg=L2)
    dp = RowShardedDataParallel(eng)
    summaries, probs = [], []
    per = B // world
    sl = slice(rank * per, (rank + 1) * per)
    mine = [tuple(torch.from_numpy(np.ascontiguousarray(a[sl])) for a in b) for b in _batches()]
    if ahead == "mixed" and rank == 0:
        # this rank holds host int64 arrays (the engine's _ids copies them), the others int32 tensors:
        # every rank must still plan ahead alike, or the counts exchanges do not pair up
        mine = [(u.numpy().astype(np.int64), i.numpy().astype(np.int64), y) for u, i, y in mine]
    for s, (users, items, y) in enumerate(mine):
        # ahead: the next batch planned (and its counts exchanged) inside this step
        nxt = mine[s + 1][:2] if ahead and s + 1 < len(mine) else None
        dp.train_step(users, items, y.numpy(), group=GROUP, k=2, global_batch=B, next_batch=nxt)
        summaries.append(eng.summary.clone().numpy())
    full = dp.full_table().numpy().copy()
    q.put((rank, full, eng.mlp.numpy().copy(), summaries))
    dist.barrier()
    dist.destroy_process_group()


def _run_cpu(worker, world, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, emb, mlp, summ = q.get(timeout=120)
        res[r] = (emb, mlp, summ)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,ahead", [(2, False), (3, False), (2, True), (2, "mixed"), (3, "mixed")])
def test_row_sharded_dp_matches_single_process_cpu(world, ahead):
    """Row-sharded exchanges (plan, all_to_all of ids/rows/grads, owner update) reproduce the
    single-process step; world 3 leaves padding rows in the last shard (40 rows); ahead: each step
    plans the next batch and exchanges its counts (the next step reads them, no replan); mixed:
    rank 0 passes host int64 ids, the others int32 tensors — the plan-ahead decision must not
    depend on how a rank holds its ids."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_engine import OracleEngine
    assert B % (world * GROUP) == 0
    res = _run_cpu(_cpu_sharded_worker, world, ahead)
    shape, w = _weights()
    ref = OracleEngine(shape, w, layers_l2reg=L2)
    grads = ref.alloc_grads()
    ref_summ = []
    for users, items, y in _batches():
        ref.forward_backward(users, items, y, group=GROUP, k=2, inv_batch=1.0 / B, grads=grads)
        ref_summ.append(grads[2].clone().numpy())
        ref.apply_update(grads, 1.0 / B)
    for r in range(world):
        emb, mlp, summ = res[r]
        np.testing.assert_allclose(emb, ref.emb[:ref.num_rows].numpy(), rtol=0, atol=1e-12)
        np.testing.assert_allclose(mlp, ref.mlp.numpy(), rtol=0, atol=1e-12)
        for a, b in zip(summ, ref_summ):
            np.testing.assert_allclose(a[:5], b[:5], rtol=1e-6, atol=1e-9)


def _user_part_batches(world):
    """Per-step, per-rank batches with the users partitioned by rank (u % world == r); global
    user ids, ranks' parts concatenated in rank order = the global batch."""
    shape = O.NCFShape(*SHAPE)
    rng = np.random.RandomState(11)
    per = B // world
    out = []
    for _ in range(STEPS):
        parts = []
        for r in range(world):
            n_loc = (shape.num_users - r + world - 1) // world
            users = (rng.randint(0, n_loc, per // GROUP) * world + r).repeat(GROUP).astype(np.int32)
            items = rng.randint(0, shape.num_items, per).astype(np.int32)
            y = np.tile([0] * (GROUP - 1) + [1], per // GROUP).astype(np.float32)
            parts.append((users, items, y))
        out.append(parts)
    return out


def _cpu_user_part_worker(rank, world, port, q, split=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from oracle_engine import OracleEngine
    from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights()
    n_loc = (shape.num_users - rank + world - 1) // world
    local = O.NCFShape(n_loc, shape.num_items, shape.layers, shape.gmf_dim)
    eng = OracleEngine(local, partition_keras_weights(w, world, rank), layers_l2reg=L2)
    dp = UserPartitionedDataParallel(eng, split_items=split)
    dp.broadcast_parameters()
    summaries = []
    for parts in _user_part_batches(world):
        users, items, y = parts[rank]
        dp.train_step(users // world, items, y, group=GROUP, k=2, global_batch=B)
        summaries.append(dp.grads[2].clone().numpy())
    q.put((rank, dp.keras_weights(), None, summaries))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,split", [(2, False), (3, False), (2, True), (3, True)])
def test_user_partitioned_dp_matches_single_process_cpu(world, split):
    """User-partitioned data + replicated items reproduce the single-process step on the
    concatenated global batch, with the item rows' Adam on every rank (one all-reduce per step) or
    split across the ranks (reduce-scatter, Adam on the rank's item slice, all-gather); world 3
    gives unequal user shards and, split, a short last item slice (17 items = 6 + 6 + 5)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_engine import OracleEngine
    res = _run_cpu(_cpu_user_part_worker, world, split)
    shape, w = _weights()
    ref = OracleEngine(shape, w, layers_l2reg=L2)
    grads = ref.alloc_grads()
    ref_summ = []
    for parts in _user_part_batches(world):
        users, items, y = (np.concatenate(x) for x in zip(*parts))
        ref.forward_backward(users, items, y, group=GROUP, k=2, inv_batch=1.0 / B, grads=grads)
        ref_summ.append(grads[2].clone().numpy())
        ref.apply_update(grads, 1.0 / B)
    rw = ref.weights()
    for r in range(world):
        wts, _, summ = res[r]
        for name in rw:
            np.testing.assert_allclose(wts[name], rw[name], rtol=0, atol=1e-12, err_msg=name)
        for a, b in zip(summ, ref_summ):
            np.testing.assert_allclose(a[:5], b[:5], rtol=1e-6, atol=1e-9)


# ---------------------------------------------------------------- GPU (HIP)

def _gpu_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.engine import NCFEngine
    from movierec.distributed import ReplicatedDataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights()
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B,
                    layers_l2reg=L2)
    eng.set_keras_weights(w)
    dp = ReplicatedDataParallel(eng)
    per = B // world
    for users, items, y in _batches():
        sl = slice(rank * per, (rank + 1) * per)
        dp.train_step(users[sl], items[sl], y[sl], group=GROUP, k=2)
    torch.cuda.synchronize()
    q.put((rank, eng.keras_weights(), NCFEngine.read_stats(eng.stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_replicated_dp_matches_single_process_gpu():
    from movierec.engine import NCFEngine
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, wts, st = q.get(timeout=300)
        res[r] = (wts, st)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    shape, w = _weights()
    ref = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, layers_l2reg=L2)
    ref.set_keras_weights(w)
    for users, items, y in _batches():
        ref.train_step(users, items, y, group=GROUP, k=2)
    rw = ref.keras_weights()
    rst = NCFEngine.read_stats(ref.stats)
    for r in range(world):
        wts, st = res[r]
        for name in rw:
            np.testing.assert_allclose(wts[name], rw[name], rtol=0, atol=1e-5, err_msg=name)
        assert st["loss"] == pytest.approx(rst["loss"], rel=1e-5)
        assert st["hr"] == pytest.approx(rst["hr"], abs=1e-6)
    assert gpu_available()


def _gpu_sharded_worker(rank, world, port, q, dims=SHAPE):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.sharded import ShardedNCFEngine
    from movierec.distributed import RowShardedDataParallel
    from movierec.engine import NCFEngine
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights(dims)
    eng = ShardedNCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, world=world, rank=rank,
                           max_batch=B, layers_l2reg=_l2(dims))
    eng.set_keras_weights(w)
    dp = RowShardedDataParallel(eng)
    per = B // world
    probs = []
    for users, items, y in _batches(dims):
        sl = slice(rank * per, (rank + 1) * per)
        dp.train_step(users[sl], items[sl], y[sl], group=GROUP, k=2, global_batch=B)
        probs.append(dp.predict(users[sl], items[sl]).cpu().numpy())
    torch.cuda.synchronize()
    q.put((rank, dp.keras_weights(), NCFEngine.read_stats(eng.stats), probs))
    dist.barrier()
    dist.destroy_process_group()


def _gpu_reference(dims=SHAPE):
    from movierec.engine import NCFEngine
    shape, w = _weights(dims)
    ref = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B,
                    layers_l2reg=_l2(dims))
    ref.set_keras_weights(w)
    probs = []
    for users, items, y in _batches(dims):
        ref.train_step(users, items, y, group=GROUP, k=2)
        probs.append(ref.predict(users, items).cpu().numpy())
    return ref.keras_weights(), NCFEngine.read_stats(ref.stats), probs


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_row_sharded_dp_matches_single_process_gpu(world):
    """HIP row-sharded path (gloo between processes sharing the GPU) vs ncf_train_step on the
    global batch: bitwise at world 1, fp32 tolerance at world 2."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, wts, st, pr = q.get(timeout=300)
        res[r] = (wts, st, pr)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rw, rst, rprobs = _gpu_reference()
    per = B // world
    for r in range(world):
        wts, st, pr = res[r]
        for name in rw:
            if world == 1:
                np.testing.assert_array_equal(wts[name], rw[name], err_msg=name)
            else:
                np.testing.assert_allclose(wts[name], rw[name], rtol=0, atol=1e-5, err_msg=name)
        assert st["loss"] == pytest.approx(rst["loss"], rel=1e-5)
        assert st["hr"] == pytest.approx(rst["hr"], abs=1e-6)
        for a, b in zip(pr, rprobs):
            np.testing.assert_allclose(a, b[r * per:(r + 1) * per], rtol=0, atol=2e-6)
    assert gpu_available()


def _gpu_user_part_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.engine import NCFEngine
    from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights()
    n_loc = (shape.num_users - rank + world - 1) // world
    eng = NCFEngine(n_loc, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, layers_l2reg=L2)
    eng.set_keras_weights(partition_keras_weights(w, world, rank))
    dp = UserPartitionedDataParallel(eng)
    dp.broadcast_parameters()
    for parts in _user_part_batches(world):
        users, items, y = parts[rank]
        dp.train_step(users // world, items, y, group=GROUP, k=2, global_batch=B)
    torch.cuda.synchronize()
    q.put((rank, dp.keras_weights(), NCFEngine.read_stats(eng.stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_user_partitioned_dp_matches_single_process_gpu(world):
    """HIP user-partitioned path (gloo between processes sharing the GPU) vs ncf_train_step on
    the concatenated global batch, at the fp32 tolerance."""
    from movierec.engine import NCFEngine
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_user_part_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, wts, st = q.get(timeout=300)
        res[r] = (wts, st)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    shape, w = _weights()
    ref = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, layers_l2reg=L2)
    ref.set_keras_weights(w)
    for parts in _user_part_batches(world):
        users, items, y = (np.concatenate(x) for x in zip(*parts))
        ref.train_step(users, items, y, group=GROUP, k=2)
    rw = ref.keras_weights()
    rst = NCFEngine.read_stats(ref.stats)
    for r in range(world):
        wts, st = res[r]
        for name in rw:
            np.testing.assert_allclose(wts[name], rw[name], rtol=0, atol=1e-5, err_msg=name)
        assert st["loss"] == pytest.approx(rst["loss"], rel=1e-5)
        assert st["hr"] == pytest.approx(rst["hr"], abs=1e-6)
    assert gpu_available()


@pytest.mark.gpu
def test_row_sharded_dp_config_d_model_gpu():
    """Config D's model (MLP [256,128,64,32] + GMF 128: the layered GEMM path on compact row
    ids) through the row-sharded exchanges at world 2 vs one process on the global batch."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_sharded_worker, args=(r, world, port, q, SHAPE_D)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, wts, st, pr = q.get(timeout=300)
        res[r] = (wts, st, pr)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rw, rst, rprobs = _gpu_reference(SHAPE_D)
    per = B // world
    for r in range(world):
        wts, st, pr = res[r]
        for name in rw:
            np.testing.assert_allclose(wts[name], rw[name], rtol=0, atol=1e-5, err_msg=name)
        assert st["loss"] == pytest.approx(rst["loss"], rel=1e-5)
        for a, b in zip(pr, rprobs):
            np.testing.assert_allclose(a, b[r * per:(r + 1) * per], rtol=0, atol=2e-6)
    assert gpu_available()


# ------------------------------------------- user-partitioned, deferred decay (GPU)

SHAPE_C = (200, 150, [128, 64, 32, 16], 64)   # config C's model, small tables (fused kernels)


def _reporting(body, rank, world, port, q):
    """Run a worker body; an exception goes to the parent through the queue (a worker that died
    silently would leave the parent waiting for its result)."""
    import traceback
    try:
        body(rank, world, port, q)
    except BaseException:
        q.put((rank, "worker failed:\n" + traceback.format_exc()))
        raise


def _get(q, n, timeout=150):
    res = {}
    for _ in range(n):
        item = q.get(timeout=timeout)
        if isinstance(item[1], str) and item[1].startswith("worker failed"):
            pytest.fail(item[1])
        res[item[0]] = item[1:] if len(item) > 2 else item[1]
    return res


def _user_part_device_batches(dims, world, per, steps, seed):
    shape = O.NCFShape(*dims)
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(steps):
        parts = []
        for r in range(world):
            n_loc = (shape.num_users - r + world - 1) // world
            users = (rng.randint(0, n_loc, per // GROUP) * world + r).repeat(GROUP).astype(np.int32)
            items = rng.randint(0, shape.num_items, per).astype(np.int32)
            y = np.tile([0] * (GROUP - 1) + [1], per // GROUP).astype(np.float32)
            parts.append((users, items, y))
        out.append(parts)
    return out


def _gpu_user_lazy_worker(rank, world, port, q):
    _reporting(_gpu_user_lazy_worker_body, rank, world, port, q)


def _gpu_user_lazy_worker_body(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.engine import NCFEngine
    from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shape, w = _weights(SHAPE_C)
    n_loc = (shape.num_users - rank + world - 1) // world
    per = 256
    out = []
    for lazy in (False, True):
        eng = NCFEngine(n_loc, shape.num_items, shape.layers, shape.gmf_dim, max_batch=per, lazy_adam=lazy,
                        lazy_rows=n_loc if lazy else None)
        eng.set_keras_weights(partition_keras_weights(w, world, rank))
        dp = UserPartitionedDataParallel(eng)
        dp.broadcast_parameters()
        batches = _user_part_device_batches(SHAPE_C, world, per, 12, 21)
        dev = [tuple(torch.from_numpy(x).cuda() for x in (p[rank][0] // world, p[rank][1], p[rank][2]))
               for p in batches]
        for s, (u, it, y) in enumerate(dev):
            nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < len(dev) and s != 5 else None   # step 6: not counted
            dp.train_step(u, it, y, group=GROUP, k=2, global_batch=per * world, next_batch=nxt)
        eng.check_errors()
        eng.flush()
        torch.cuda.synchronize()
        m, v, t = eng.optimizer_state()
        out.append((dp.keras_weights(), m, v, t, NCFEngine.read_stats(eng.stats)))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_user_partitioned_deferred_decay_bitwise_dense_gpu(world):
    """The user-partitioned step with deferred decay of the own users (touched-row update, the next
    batch counted and its rows caught up ahead under the all-reduce, one step not counted) against
    the same layout's dense sweep of every own user row: bitwise equal weights, Adam moments,
    iteration count and metrics after 12 steps (the item rows are swept every step in both)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_user_lazy_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = _get(q, world)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        (wd, md, vd, td, sd), (wl, ml, vl, tl, sl) = res[r]
        for name in wd:
            np.testing.assert_array_equal(wl[name], wd[name], err_msg=name)
        for name in md:
            np.testing.assert_array_equal(ml[name], md[name], err_msg="m " + name)
            np.testing.assert_array_equal(vl[name], vd[name], err_msg="v " + name)
        assert tl == td == 12
        assert sl == sd
    assert gpu_available()


def _gpu_user_full_worker(rank, world, port, q, per=65536, split=False):
    _reporting(lambda *a: _gpu_user_full_worker_body(*a, per=per, split=split), rank, world, port, q)


def _gpu_user_full_worker_body(rank, world, port, q, per=65536, split=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.engine import NCFEngine
    from movierec.model import initial_weights
    from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    U, I, layers, gmf = 138493, 27278, [128, 64, 32, 16], 64
    n_loc = (U - rank + world - 1) // world
    w = initial_weights(U, I, layers, gmf, seed=3)
    eng = NCFEngine(n_loc, I, layers, gmf, max_batch=per, lazy_adam=True, lazy_rows=n_loc)
    eng.set_keras_weights(partition_keras_weights(w, world, rank))
    dp = UserPartitionedDataParallel(eng, split_items=split)
    batches = _user_part_device_batches((U, I, layers, gmf), world, per, 3, 31)
    dev = [tuple(torch.from_numpy(x).cuda() for x in (p[rank][0] // world, p[rank][1], p[rank][2]))
           for p in batches]
    for s, (u, it, y) in enumerate(dev):
        nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < len(dev) else None
        dp.train_step(u, it, y, group=GROUP, k=2, global_batch=per * world, next_batch=nxt)
    eng.check_errors()
    q.put((rank, eng.keras_weights(), NCFEngine.read_stats(eng.stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("per,split", [(65536, False), (8192, True)], ids=["65536-replicated-items",
                                                                          "8192-split-items"])
def test_user_partitioned_full_config_c_tables_gpu(per, split):
    """The user layout at config C's full tables (138,493 x 27,278) at world 2, deferred decay with
    counting ahead, 3 steps, against ncf_train_step on the concatenated 2 x per batches: 65,536
    samples per rank with the item rows' Adam replicated (one all-reduce), and 8,192 per rank
    (config C's BASELINE global batch over 8 GPUs, the strong-scaling shape) with it split across
    the ranks (reduce-scatter + all-gather).  The step is the same arithmetic up to fp32 summation
    order of the item-row and dense-layer gradients; from step 2 on that order can move a sample
    across a ReLU kink (a pre-activation within ~1e-9 of 0), which changes its rows by up to two
    Adam steps.  So: dense layers within 1e-5; embedding rows beyond 1e-5 fewer than 0.1 % of the
    table and every element within 3e-3 (two Adam steps of lr 1e-3); loss rel 1e-5."""
    from movierec.engine import NCFEngine
    from movierec.model import initial_weights
    from movierec.distributed import partition_keras_weights
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_user_full_worker, args=(r, world, port, q, per, split)) for r in range(world)]
    for p in procs:
        p.start()
    res = _get(q, world)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    U, I, layers, gmf = 138493, 27278, [128, 64, 32, 16], 64
    # the reference step on the ranks' forward/backward kernel (below 16,384 samples the ranks run
    # the unit kernel, the concatenated batch would take the wave kernel's group-user form): the
    # comparison is then of the exchange, not of two kernels' fp32 orders
    ref = NCFEngine(U, I, layers, gmf, max_batch=2 * per, lazy_adam=True, fb_kernel="unit" if per < 16384 else None)
    ref.set_keras_weights(initial_weights(U, I, layers, gmf, seed=3))
    batches = _user_part_device_batches((U, I, layers, gmf), world, per, 3, 31)
    dev = [tuple(torch.from_numpy(np.concatenate(x)).cuda() for x in zip(*parts)) for parts in batches]
    for s, (u, it, y) in enumerate(dev):
        nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < len(dev) else None
        ref.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
    rw = ref.keras_weights()
    rst = NCFEngine.read_stats(ref.stats)
    for r in range(world):
        wts, st = res[r]
        loc = partition_keras_weights(rw, world, r)
        for name in loc:
            d = np.abs(np.asarray(wts[name], np.float64) - loc[name])
            if name.endswith("embedding"):
                rows_off = (d > 1e-5).any(axis=1).mean()
                assert rows_off < 1e-3, "%s: %.4f of the rows beyond 1e-5" % (name, rows_off)
                assert d.max() <= 3e-3, "%s: max err %g" % (name, d.max())
            else:
                assert d.max() <= 1e-5, "%s: max err %g" % (name, d.max())
        assert st["loss"] == pytest.approx(rst["loss"], rel=1e-5)
        assert st["steps"] == rst["steps"] == 3
    assert gpu_available()


def _gpu_native_comm_worker(rank, world, port, q, per=256):
    _reporting(lambda *a: _gpu_native_comm_worker_body(*a, per=per), rank, world, port, q)


def _gpu_native_comm_worker_body(rank, world, port, q, per=256):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "movierecommender-tf-trt_amd")]
    from movierec.engine import NCFEngine
    from movierec.distributed import UserPartitionedDataParallel, partition_keras_weights
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
    shape, w = _weights(SHAPE_C)
    out = []
    for native, split in ((True, False), (False, False), (True, True), (False, True)):
        eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=per, lazy_adam=True,
                        lazy_rows=shape.num_users)
        eng.set_keras_weights(partition_keras_weights(w, world, rank))
        dp = UserPartitionedDataParallel(eng, native=native, split_items=split)
        assert (dp.comm is not None) == native
        batches = _user_part_device_batches(SHAPE_C, world, per, 10, 41)
        dev = [tuple(torch.from_numpy(x).cuda() for x in p[rank]) for p in batches]
        for s, (u, it, y) in enumerate(dev):
            nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < len(dev) and s != 4 else None
            dp.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
        eng.check_errors()
        eng.flush()
        torch.cuda.synchronize()
        m, v, t = eng.optimizer_state()
        out.append((eng.keras_weights(), m, v, t, NCFEngine.read_stats(eng.stats)))
        if dp.comm is not None:
            dp.comm.close()
    # an emulated rank 0 of 8 with the split item optimizer (its item slice only, no exchange): one
    # step, natively and call by call, against the replicated-item step of the same local table
    emu = []
    for native, split in ((True, True), (False, True), (True, False)):
        eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=per, lazy_adam=True,
                        lazy_rows=shape.num_users)
        eng.set_keras_weights(partition_keras_weights(w, world, rank))
        dp = UserPartitionedDataParallel(eng, native=native, split_items=split, emulate_world=8)
        u, it, y = (torch.from_numpy(x).cuda() for x in _user_part_device_batches(SHAPE_C, world, per, 1, 43)[0][rank])
        dp.train_step(u, it, y, group=GROUP, k=2, global_batch=8 * per)
        eng.flush()
        torch.cuda.synchronize()
        emu.append((eng.emb[:eng.num_rows].cpu().numpy(), eng.mlp.cpu().numpy(), dp.Ic))
        if dp.comm is not None:
            dp.comm.close()
    q.put((rank, out, emu, eng.num_users, partition_keras_weights(w, world, rank)))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("per", [256, 4096])
def test_user_partitioned_native_comm_step_bitwise_gpu(per):
    """ncf_user_dp_step (one library call per step, the all-reduce on the library's own RCCL
    communicator and side stream) against the same step issued call by call from Python with
    torch.distributed's all-reduce: one rank over RCCL (the box has one GPU), 10 steps with the next
    batch counted ahead (one step not), bitwise equal weights, moments, iteration count, metrics.
    At 4,096 samples the one-call step fills its index inside the forward/backward launch and
    orders the unsorted lists in the gradient tail and the own-user update (round 6); the call-by-
    call step builds and sorts it with launches of its own: same sums in the same order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    p = ctx.Process(target=_gpu_native_comm_worker, args=(0, 1, port, q, per))
    p.start()
    out, emu, U, w0 = _get(q, 1)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    (wa, ma, va, ta, sa) = out[0]
    # native / call by call, replicated / split item optimizer: all bitwise at one rank
    for (wb, mb, vb, tb, sb) in out[1:]:
        for name in wa:
            np.testing.assert_array_equal(wa[name], wb[name], err_msg=name)
            np.testing.assert_array_equal(ma[name], mb[name], err_msg="m " + name)
            np.testing.assert_array_equal(va[name], vb[name], err_msg="v " + name)
        assert ta == tb == 10 and sa == sb
    # emulated rank 0 of 8, split: its user rows, its item slice and the dense layers are those of
    # the replicated step; the other item rows keep their values (no all-gather)
    (es, ms, ic), (ep, mp_, _), (er, mr, _) = emu
    np.testing.assert_array_equal(es, ep)
    np.testing.assert_array_equal(ms, mp_)
    np.testing.assert_array_equal(ms, mr)
    np.testing.assert_array_equal(es[:U + ic], er[:U + ic])
    assert not np.array_equal(es[U + ic:], er[U + ic:])
    from movierec.layout import Layout
    shape, _ = _weights(SHAPE_C)
    e0, _ = Layout(U, shape.num_items, shape.layers, shape.gmf_dim).to_device(w0)
    np.testing.assert_array_equal(es[U + ic:], e0[U + ic:])
    assert gpu_available()
