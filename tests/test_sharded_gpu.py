"""Row-sharded tables under deferred exact decay (BASELINE config D's layout: "embedding tables
row-sharded across 8 GPUs"; reference movierec/model.py:161-170 gather, 199-202 Adam).

The owner of a shard serves the rows other ranks request (ncf_shard_serve_rows: the served rows'
missed zero-gradient Adam steps replayed, an owner index built) and updates only those rows
(ncf_shard_apply_update with row_step).  Keras' dense Adam moves every row every
step; the deferred form must be bitwise that dense sweep:

  * world 1 (the one-rank shard, emulated exchanges): lazy == dense shard == ncf_train_step,
    bitwise, with and without the next batch planned ahead;
  * an emulated rank 3 of 8 (batches drawn from its own rows) == the single table on the same
    batches, bitwise on its rows and the dense layers;
  * world 2 (gloo, two processes sharing the GPU) at config D's full 10 M x 1 M tables against
    the compacted oracle (tests/test_config_d_gpu.py's construction; fp32 tolerances there).
"""

import os

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec import _native as N
    from movierec.engine import NCFEngine
    from movierec.sharded import ShardedNCFEngine
    from movierec.distributed import RowShardedDataParallel

GROUP = 4


def _weights(shape, seed):
    w = O.init_weights(shape, seed=seed)
    rng = np.random.RandomState(seed + 100)
    for k in w:
        if k.endswith("embedding"):
            w[k] = rng.uniform(-0.5, 0.5, size=w[k].shape)
        elif k.endswith("bias"):
            w[k] = rng.uniform(-0.1, 0.1, size=w[k].shape)
        else:
            w[k] = w[k] * 3.0
    return {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}


def _dev_batches(shape, B, steps, seed, users=None, items=None):
    """Device batches of B samples (groups of GROUP sharing a user); ids drawn from the given
    candidate arrays (default: the whole tables)."""
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(steps):
        u = rng.randint(0, shape.num_users, B // GROUP) if users is None else rng.choice(users, B // GROUP)
        it = rng.randint(0, shape.num_items, B) if items is None else rng.choice(items, B)
        y = np.tile([0.0] * (GROUP - 1) + [1.0], B // GROUP)
        out.append(tuple(torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).cuda()
                         for a, dt in ((u.repeat(GROUP), np.int32), (it, np.int32), (y, np.float32))))
    return out


@pytest.mark.parametrize("dims", [(200, 150, [128, 64, 32, 16], 64), (40, 30, [256, 128, 64, 32], 128)],
                         ids=["configC", "configD"])
@pytest.mark.parametrize("ahead", [False, True], ids=["plain", "planned-ahead"])
def test_sharded_deferred_decay_bitwise_dense_world1(dims, ahead):
    """The deferred-decay shard (one rank: every row) against the dense shard sweep and against
    ncf_train_step: bitwise weights, moments and stats after steps whose small batches leave most
    rows untouched for several steps, a predict in the middle (a read: flush first)."""
    shape = O.NCFShape(*dims)
    w = _weights(shape, 3)
    B, steps = 32, 7
    batches = _dev_batches(shape, B, steps, 11)
    lazy = ShardedNCFEngine(*dims, world=1, rank=0, max_batch=B, lazy_adam=True)
    dense = ShardedNCFEngine(*dims, world=1, rank=0, max_batch=B)
    single = NCFEngine(*dims, max_batch=B)
    for e in (lazy, dense, single):
        e.set_keras_weights(w)
    assert lazy.lazy and not dense.lazy
    dl, dd = RowShardedDataParallel(lazy, emulate=True), RowShardedDataParallel(dense, emulate=True)
    for s, (u, it, y) in enumerate(batches):
        nxt = (batches[s + 1][0], batches[s + 1][1]) if ahead and s + 1 < steps else None
        dl.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
        dd.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
        single.train_step(u, it, y, group=GROUP, k=2)
        if s == 3:
            assert torch.equal(dl.predict(u, it), dd.predict(u, it))
    lazy.flush()
    torch.cuda.synchronize()
    R = single.num_rows
    assert torch.equal(lazy.emb[:R], dense.emb[:R]) and torch.equal(lazy.emb[:R], single.emb)
    assert torch.equal(lazy.emb_m[:R], single.emb_m) and torch.equal(lazy.emb_v[:R], single.emb_v)
    assert torch.equal(dense.emb_m[:R], single.emb_m)
    assert torch.equal(lazy.mlp, single.mlp) and torch.equal(lazy.mlp_m, single.mlp_m)
    assert torch.equal(lazy.stats, single.stats)
    rs = lazy.row_step
    assert int((rs == N.NCF_ROW_PRISTINE).sum()) > 0            # rows no batch touched stay pristine
    assert int(rs[rs != N.NCF_ROW_PRISTINE].min()) == steps


def test_sharded_emulated_rank_equals_single_table():
    """``RowShardedDataParallel(emulate=True)``: rank 3 of 8 stepping batches drawn from its own
    rows (users u = 3 mod 8, items whose table row U + i = 3 mod 8) — the bench's per-rank compute
    of the 8-rank step — equals the single table stepping the same batches, bitwise on the rows it
    owns, the dense layers and the stats."""
    dims = (203, 157, [128, 64, 32, 16], 64)
    shape = O.NCFShape(*dims)
    U, I = dims[0], dims[1]
    world, rank = 8, 3
    w = _weights(shape, 5)
    users = np.arange(rank, U, world)
    items = np.array([i for i in range(I) if (U + i) % world == rank])
    B, steps = 64, 5
    batches = _dev_batches(shape, B, steps, 13, users=users, items=items)
    shard = ShardedNCFEngine(*dims, world=world, rank=rank, max_batch=B, lazy_adam=True)
    shard.set_keras_weights(w)
    single = NCFEngine(*dims, max_batch=B, lazy_adam=True)
    single.set_keras_weights(w)
    dp = RowShardedDataParallel(shard, emulate=True)
    for s, (u, it, y) in enumerate(batches):
        nxt = (batches[s + 1][0], batches[s + 1][1]) if s + 1 < steps else None
        dp.train_step(u, it, y, group=GROUP, k=2, global_batch=B, next_batch=nxt)
        single.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
    assert dp.last_exchange[0] == dp.last_exchange[1]      # every unique row served by this rank
    shard.flush()
    single.flush()
    torch.cuda.synchronize()
    g = torch.from_numpy(shard.owned_rows()).cuda()
    own = g >= 0
    gl = g[own].long()
    assert torch.equal(shard.emb[own], single.emb[gl])
    assert torch.equal(shard.emb_m[own], single.emb_m[gl]) and torch.equal(shard.emb_v[own], single.emb_v[gl])
    assert torch.equal(shard.mlp, single.mlp) and torch.equal(shard.mlp_v, single.mlp_v)
    assert torch.equal(shard.stats, single.stats)


# --------------------------------------------- config D's full tables, world 2 (gloo, one GPU)

DU, DI, D_LAYERS, D_GMF = 10_000_000, 1_000_000, [256, 128, 64, 32], 128
D_HYPER = dict(optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=[0.0] * 4)


def _formula_rows(g, W):
    """Initial table row g (int64 array / tensor of global rows): a counter hash to U(-0.5, 0.5),
    the same in numpy (the oracle's compacted rows) and on the device (each rank's shard)."""
    if torch.is_tensor(g):
        c = torch.arange(W, device=g.device, dtype=torch.int64)
        h = (g.unsqueeze(1) * 2654435761 + c.unsqueeze(0) * 40503 + 12345) % (1 << 32)
        return (h.double() / float(1 << 32) - 0.5).float()
    c = np.arange(W, dtype=np.int64)
    h = (g[:, None] * 2654435761 + c[None, :] * 40503 + 12345) % (1 << 32)
    return (h.astype(np.float64) / float(1 << 32) - 0.5).astype(np.float32)


def _d_world2_worker(rank, world, port, q, flat, batches, want_rows):
    import traceback
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        eng = ShardedNCFEngine(DU, DI, D_LAYERS, D_GMF, world=world, rank=rank, max_batch=len(batches[0][0]),
                               lazy_adam=True)
        gl = torch.arange(eng.shard_rows, device="cuda", dtype=torch.int64) * world + rank
        for r0 in range(0, eng.shard_rows, 1 << 20):
            r1 = min(eng.shard_rows, r0 + (1 << 20))
            rows = _formula_rows(gl[r0:r1], eng.row_width)
            rows[gl[r0:r1] >= eng.num_rows] = 0
            eng.emb[r0:r1].copy_(rows)
        eng.mlp.copy_(torch.from_numpy(flat))
        dp = RowShardedDataParallel(eng)
        dev = [tuple(torch.from_numpy(a).cuda() for a in b) for b in batches]
        for s, (u, it, y) in enumerate(dev):
            nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < len(dev) else None
            dp.train_step(u, it, y, group=GROUP, k=2, global_batch=world * len(u), next_batch=nxt)
        eng.check_errors()
        eng.flush()
        torch.cuda.synchronize()
        mine = want_rows[want_rows % world == rank]
        loc = torch.from_numpy(mine // world).cuda()
        q.put((rank, NCFEngine.read_stats(eng.stats), eng.mlp.cpu().numpy(), mine,
               eng.emb[loc].cpu().numpy(), (eng.emb_m[loc] != 0).any(dim=1).cpu().numpy(),
               int((eng.row_step != N.NCF_ROW_PRISTINE).sum()),
               int(((eng.emb_m != 0).any(dim=1) | (eng.emb_v != 0).any(dim=1)).sum())))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        q.put((rank, "worker failed:\n" + traceback.format_exc()))
        raise


def test_config_d_row_sharded_world2_matches_compacted_oracle():
    """Config D as BASELINE names it — 10 M x 1 M tables row-sharded across ranks — at world 2:
    two processes (gloo, sharing the GPU), each holding a 5.5 M-row shard with its Adam state under
    deferred decay, 32,768 samples per rank per step, the next batch planned ahead.  Against the
    oracle on the compacted model of the global 65,536-sample batches (test_config_d_gpu.py's
    construction, its tolerances): every compacted row (fetched from its owner), the dense layers
    and the loss; each shard's non-pristine rows are exactly the rows the batches touched."""
    import socket
    import torch.multiprocessing as mp
    from test_config_d_gpu import _dense_weights, _off_kinks
    from movierec.layout import Layout
    world, per, steps = 2, 32768, 3
    B = world * per
    ngroups = B // GROUP
    rng = np.random.RandomState(50)
    cand = []
    for s in range(steps):
        n = ngroups + ngroups // 8
        cu, ci = rng.randint(0, DU, n), rng.randint(0, DI, (n, GROUP))
        if s == 0:
            cu[:3] = [0, DU - 1, 8_388_608]
            ci[:3, -1] = [0, DI - 1, DI // 2]
        cand.append((cu, ci))
    users = np.unique(np.concatenate([c[0] for c in cand]))
    items = np.unique(np.concatenate([c[1].reshape(-1) for c in cand]))
    W = Layout(DU, DI, D_LAYERS, D_GMF).row_width
    urows = _formula_rows(users.astype(np.int64), W).astype(np.float64)
    irows = _formula_rows(items.astype(np.int64) + DU, W).astype(np.float64)
    g4 = D_GMF
    du = di = D_LAYERS[0] // 2
    w = dict(_dense_weights(52))
    w["user_gmf_embedding"], w["item_gmf_embedding"] = urows[:, :D_GMF], irows[:, :D_GMF]
    w["user_embedding"], w["item_embedding"] = urows[:, g4:g4 + du], irows[:, g4:g4 + di]
    shape = O.NCFShape(len(users), len(items), D_LAYERS, D_GMF)

    def cids(u, i):
        return np.searchsorted(users, u).astype(np.int32), np.searchsorted(items, i).astype(np.int32)
    u0, i0 = cids(cand[0][0][:512].repeat(GROUP), cand[0][1][:512].reshape(-1))
    _, c = O.forward(shape, w, u0, i0)
    f = 6.0 / max(np.max(np.abs(c["z"])), 1e-6)
    w["output/kernel"], w["output/bias"] = w["output/kernel"] * f, w["output/bias"] * f
    w = {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}
    flat = Layout(1, 1, D_LAYERS, D_GMF).to_device({**w, "user_embedding": np.zeros((1, du)),
                                                     "item_embedding": np.zeros((1, di)),
                                                     "user_gmf_embedding": np.zeros((1, D_GMF)),
                                                     "item_gmf_embedding": np.zeros((1, D_GMF))})[1]
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    rank_batches = [[] for _ in range(world)]
    losses, touched = [], []
    for s in range(steps):
        cu, ci = cand[s]
        lu, li = cids(cu.repeat(GROUP), ci.reshape(-1))
        ok = _off_kinks(ref, lu, li).reshape(-1, GROUP).all(axis=1)
        if s == 0:
            ok[:3] = True
        keep = np.flatnonzero(ok)[:ngroups]
        assert len(keep) == ngroups, "too many kink groups: %d" % int((~ok).sum())
        gu = cu[keep].repeat(GROUP).astype(np.int32)
        gi = ci[keep].reshape(-1).astype(np.int32)
        y = np.tile([0.0] * (GROUP - 1) + [1.0], ngroups).astype(np.float32)
        lu, li = cids(gu, gi)
        losses.append(O.train_step(shape, ref, st, lu, li, y, D_HYPER)[0])
        for r in range(world):
            sl = slice(r * per, (r + 1) * per)
            rank_batches[r].append((gu[sl], gi[sl], y[sl]))
        touched.append(np.concatenate([gu.astype(np.int64), gi.astype(np.int64) + DU]))
    touched = np.unique(np.concatenate(touched))
    want = np.concatenate([users.astype(np.int64), items.astype(np.int64) + DU])

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_d_world2_worker, args=(r, world, port, q, flat, rank_batches[r], want))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=600)
        if isinstance(item[1], str):
            pytest.fail(item[1])
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0

    got = np.zeros((len(want), W))
    pos = {int(g): j for j, g in enumerate(want)}
    for r in range(world):
        stats, mlp, mine, vals, nz, n_live, n_moments = res[r]
        assert stats["steps"] == steps
        assert stats["loss"] == pytest.approx(np.mean(losses), rel=2e-5)
        got[[pos[int(g)] for g in mine]] = vals
        # the shard's rows that left the pristine state / carry moments: exactly its touched rows
        own_touched = int((touched % world == r).sum())
        assert n_live == own_touched and n_moments == own_touched, (r, n_live, n_moments, own_touched)
        dense_got = Layout(1, 1, D_LAYERS, D_GMF).from_device(np.zeros((2, W), np.float32), mlp)
        for name in ref:
            if not name.endswith("embedding"):
                tol = steps * 2e-6 + 2e-6 * float(np.max(np.abs(ref[name])))
                e = float(np.max(np.abs(dense_got[name] - ref[name])))
                assert e <= tol, "rank %d %s: %g > %g" % (r, name, e, tol)
    nu = len(users)
    emb_got = {"user_gmf_embedding": got[:nu, :D_GMF], "item_gmf_embedding": got[nu:, :D_GMF],
               "user_embedding": got[:nu, g4:g4 + du], "item_embedding": got[nu:, g4:g4 + di]}
    for name, g in emb_got.items():
        tol = steps * 2e-6 + 2e-6 * float(np.max(np.abs(ref[name])))
        d = np.abs(g - ref[name])
        assert float(d.max()) <= tol, "%s: max err %g > %g (%d rows beyond)" % (
            name, float(d.max()), tol, int((d > tol).any(axis=1).sum()))


# ------------------------------- dense shard, next batch announced, K >> batch, world 2 (gloo)

def _dense_world2_worker(rank, world, port, q, dims, w, batches):
    import traceback
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        eng = ShardedNCFEngine(*dims, world=world, rank=rank, max_batch=len(batches[0][0]))
        eng.set_keras_weights(w)
        dp = RowShardedDataParallel(eng)
        dev = [tuple(torch.from_numpy(a).cuda() for a in b) for b in batches]
        for s, (u, it, y) in enumerate(dev):
            nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < len(dev) else None
            dp.train_step(u, it, y, group=GROUP, k=2, global_batch=world * len(u), next_batch=nxt)
        eng.check_errors()
        full = dp.full_table().cpu().numpy()
        q.put((rank, full, eng.mlp.cpu().numpy(), NCFEngine.read_stats(eng.stats)))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        q.put((rank, "worker failed:\n" + traceback.format_exc()))
        raise


def test_dense_shard_next_batch_large_table_world2():
    """a DENSE shard (no deferred decay) with next_batch passed, a key space far
    larger than the batch (400,000 x 300,000 rows, 256 samples per rank) — the layout where the
    dense update's owner index would overlap a plan of the next batch.  The row-sharded step does
    not plan ahead for a dense shard; two gloo ranks sharing the GPU must equal one table stepping
    the concatenated batches (fp32 order of the cross-rank sums)."""
    import socket
    import torch.multiprocessing as mp
    dims = (400_000, 300_000, [128, 64, 32, 16], 64)
    shape = O.NCFShape(*dims)
    world, per, steps = 2, 256, 4
    rng = np.random.RandomState(7)
    w = O.init_weights(shape, seed=8)
    w = {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}
    rank_batches = [[] for _ in range(world)]
    glob = []
    for s in range(steps):
        u = rng.randint(0, dims[0], world * per // GROUP).repeat(GROUP).astype(np.int32)
        it = rng.randint(0, dims[1], world * per).astype(np.int32)
        y = np.tile([0.0] * (GROUP - 1) + [1.0], world * per // GROUP).astype(np.float32)
        glob.append((u, it, y))
        for r in range(world):
            sl = slice(r * per, (r + 1) * per)
            rank_batches[r].append((u[sl], it[sl], y[sl]))
    single = NCFEngine(*dims, max_batch=world * per)
    single.set_keras_weights(w)
    for u, it, y in glob:
        single.train_step(u, it, y, group=GROUP, k=2)
    want_emb = single.emb.cpu().numpy()
    want_mlp = single.mlp.cpu().numpy()
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dense_world2_worker, args=(r, world, port, q, dims, w, rank_batches[r]))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=600)
        if isinstance(item[1], str):
            pytest.fail(item[1])
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        full, mlp, stats = res[r]
        assert stats["steps"] == steps
        assert float(np.max(np.abs(full - want_emb))) <= 1e-6
        assert float(np.max(np.abs(mlp - want_mlp))) <= 1e-6
