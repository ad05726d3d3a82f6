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


def _cpu_sharded_worker(rank, world, port, q):
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
    for users, items, y in _batches():
        sl = slice(rank * per, (rank + 1) * per)
        dp.train_step(users[sl], items[sl], y[sl], group=GROUP, k=2, global_batch=B)
        summaries.append(eng.summary.clone().numpy())
    full = dp.full_table().numpy().copy()
    q.put((rank, full, eng.mlp.numpy().copy(), summaries))
    dist.barrier()
    dist.destroy_process_group()


def _run_cpu(worker, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
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


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_dp_matches_single_process_cpu(world):
    """Row-sharded exchanges (plan, all_to_all of ids/rows/grads, owner update) reproduce the
    single-process step; world 3 leaves padding rows in the last shard (40 rows)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_engine import OracleEngine
    assert B % (world * GROUP) == 0
    res = _run_cpu(_cpu_sharded_worker, world)
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


def _cpu_user_part_worker(rank, world, port, q):
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
    dp = UserPartitionedDataParallel(eng)
    dp.broadcast_parameters()
    summaries = []
    for parts in _user_part_batches(world):
        users, items, y = parts[rank]
        dp.train_step(users // world, items, y, group=GROUP, k=2, global_batch=B)
        summaries.append(dp.grads[2].clone().numpy())
    q.put((rank, dp.keras_weights(), None, summaries))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_user_partitioned_dp_matches_single_process_cpu(world):
    """User-partitioned data + replicated items (one all-reduce per step) reproduce the
    single-process step on the concatenated global batch; world 3 gives unequal user shards."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_engine import OracleEngine
    res = _run_cpu(_cpu_user_part_worker, world)
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
