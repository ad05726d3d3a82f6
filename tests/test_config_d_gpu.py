"""BASELINE config D at its real size: 10,000,000 users x 1,000,000 items, NeuMF gmf 128 + MLP
[256, 128, 64, 32] (reference ``movierec/model.py:154-215`` plus the GMF branch), one GPU.

The combined table has 11,000,000 rows of 256 floats (2.8 G floats, 11.3 GB; with the Adam moments
34 GB): element offsets past 2^31 are reached by every item row and by users from 8,388,608 on,
so this test is what proves no 32-bit element offset survives on the path the bench runs
(deferred-decay Adam, the next batch counted ahead, the layer-by-layer forward/backward).

The oracle cannot hold 11 M rows in float64, and does not need to: under Keras' dense Adam (F5) a
row only interacts with the others through the batches that read it.  A row no batch touches has
g = 0 at every step, and with zero moments that step leaves it unchanged (m = v = 0, the update
is 0).  So the oracle runs on the COMPACTED model — the union of the rows any step reads (plus
every candidate row the batch draw looked at), ids remapped — and every touched row of the device
table is compared with it after the steps; every untouched row must still equal its initial
value, bit for bit, with zero moments.

Tolerances (fp32 device vs float64 oracle): weights after k steps |dw| <= k * 2e-6 + 2e-6 * max|w|
and loss rel 2e-5, as tests/test_headline_parity_gpu.py; probabilities |dp| <= 2e-6 on the initial
weights and <= 2e-6 * (1 + s) after s optimizer steps — the weights may drift by the tolerance
above each step, and config D's 256-wide first layer (O(1) activations here) sums that drift over
twice the inputs of config C's.
Batches are drawn off the ReLU kinks (every hidden |z| beyond 64 fp32 ulps of its accumulation's
magnitude under the oracle's weights of that step; config D's O(1) activations over 256 inputs
put that near 1e-4), as the headline test does; tests/test_headline_parity_gpu.py also covers
unfiltered batches.
"""

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec import _native as N
    from movierec.engine import NCFEngine

U, I, LAYERS, GMF = 10_000_000, 1_000_000, [256, 128, 64, 32], 128
GROUP = 4
HYPER = dict(optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=[0.0] * 4)


def _dense_weights(seed):
    """Dense layers: Keras initialisation of the config-D layers, scaled like the small-shape
    tests so activations stay O(1) with O(1) embeddings; the output layer rescaled later."""
    small = O.NCFShape(2, 2, LAYERS, GMF)
    w = O.init_weights(small, seed=seed)
    rng = np.random.RandomState(seed + 1)
    out = {}
    for k, v in w.items():
        if k.endswith("embedding"):
            continue
        out[k] = rng.uniform(-0.1, 0.1, size=v.shape) if k.endswith("bias") else v * 4.0
    return out


def _device_tables(eng, seed):
    """Uniform(-0.5, 0.5) embedding tables drawn on the device (deterministic generator)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    chunk = 1 << 20
    for r0 in range(0, eng.num_rows, chunk):
        r1 = min(eng.num_rows, r0 + chunk)
        eng.emb[r0:r1].copy_(torch.rand(r1 - r0, eng.row_width, generator=g, device="cuda") - 0.5)
    torch.cuda.synchronize()


class Compact(object):
    """The compacted oracle model: rows gathered from the device's initial table."""

    def __init__(self, emb0, dense, users, items, gstride, du, di):
        self.users = np.unique(users)
        self.items = np.unique(items)
        ur = torch.from_numpy(self.users.astype(np.int64)).cuda()
        ir = torch.from_numpy(self.items.astype(np.int64) + U).cuda()
        urows = emb0[ur].double().cpu().numpy()
        irows = emb0[ir].double().cpu().numpy()
        self.w = dict(dense)
        self.w["user_gmf_embedding"] = urows[:, :GMF]
        self.w["item_gmf_embedding"] = irows[:, :GMF]
        self.w["user_embedding"] = urows[:, gstride:gstride + du]
        self.w["item_embedding"] = irows[:, gstride:gstride + di]
        self.shape = O.NCFShape(len(self.users), len(self.items), LAYERS, GMF)

    def ids(self, users, items):
        return (np.searchsorted(self.users, users).astype(np.int32),
                np.searchsorted(self.items, items).astype(np.int32))


def _off_kinks(w, users, items, ulps=64):
    """Samples whose every hidden pre-activation is more than ``ulps`` fp32 rounding units of its
    accumulation's magnitude sum away from 0 (tests/test_headline_parity_gpu.py kink_samples):
    fp32 and float64 then take the same side of every ReLU."""
    h = np.concatenate([w["user_embedding"][users], w["item_embedding"][items]], axis=1)
    ok = np.ones(len(users), bool)
    eps = float(np.finfo(np.float32).eps)
    for l in range(1, len(LAYERS)):
        W, b = w["hidden_%d/kernel" % l], w["hidden_%d/bias" % l]
        z = h @ W + b
        ok &= (np.abs(z) > ulps * eps * (np.abs(h) @ np.abs(W) + np.abs(b))).all(axis=1)
        h = np.maximum(z, 0)
    return ok


def test_config_d_full_size_matches_compacted_oracle():
    B = 65536
    steps = 3
    rng = np.random.RandomState(40)
    ngroups = B // GROUP
    # candidate groups, 1/8 spare for the kink filter; the first groups pin the table's corners
    cand = []
    for s in range(steps):
        n = ngroups + ngroups // 8
        cu = rng.randint(0, U, n)
        ci = rng.randint(0, I, (n, GROUP))
        if s == 0:
            cu[:3] = [0, U - 1, 8_388_608]        # first user, last user, first past 2^31 / 256
            ci[:3, -1] = [0, I - 1, I // 2]
        cand.append((cu, ci))

    eng = NCFEngine(U, I, LAYERS, GMF, max_batch=B, lazy_adam=True)
    assert eng.kernel_for(B) == "layered-mfma", eng.kernel_for(B)   # no vendor GEMM on the step
    gstride, du, di = eng.shape.gmf_stride, eng.shape.du, eng.shape.di
    assert eng.row_width * eng.num_rows > (1 << 31)
    _device_tables(eng, seed=41)
    emb0 = eng.emb.clone()
    dense = _dense_weights(42)
    all_u = np.concatenate([c[0] for c in cand])
    all_i = np.concatenate([c[1].reshape(-1) for c in cand])
    cm = Compact(emb0, dense, all_u, all_i, gstride, du, di)
    # output layer: keep logits well inside the BCE clip range on the first candidates
    u0, i0 = cm.ids(cand[0][0][:512].repeat(GROUP), cand[0][1][:512].reshape(-1))
    _, c = O.forward(cm.shape, cm.w, u0, i0)
    f = 6.0 / max(np.max(np.abs(c["z"])), 1e-6)
    cm.w["output/kernel"] = cm.w["output/kernel"] * f
    cm.w["output/bias"] = cm.w["output/bias"] * f
    cm.w = {k: v.astype(np.float32).astype(np.float64) for k, v in cm.w.items()}
    from movierec.layout import Layout
    flat = Layout(1, 1, LAYERS, GMF).to_device({**cm.w, "user_embedding": np.zeros((1, du)),
                                                 "item_embedding": np.zeros((1, di)),
                                                 "user_gmf_embedding": np.zeros((1, GMF)),
                                                 "item_gmf_embedding": np.zeros((1, GMF))})[1]
    eng.mlp.copy_(torch.from_numpy(flat))

    # the oracle runs first: each step's batch is drawn off the kinks of the weights it meets
    ref = {k: v.copy() for k, v in cm.w.items()}
    st = O.new_opt_state(ref)
    batches, outs = [], []
    for s in range(steps):
        cu, ci = cand[s]
        users = cu.repeat(GROUP)
        items = ci.reshape(-1)
        lu, li = cm.ids(users, items)
        ok = _off_kinks(ref, lu, li).reshape(-1, GROUP).all(axis=1)
        if s == 0:
            ok[:3] = True                        # the corner groups stay (checked below)
        keep = np.flatnonzero(ok)[:ngroups]
        assert len(keep) == ngroups, "too many kink groups: %d" % int((~ok).sum())
        gu = cu[keep].repeat(GROUP).astype(np.int32)
        gi = ci[keep].reshape(-1).astype(np.int32)
        y = np.tile([0.0] * (GROUP - 1) + [1.0], ngroups).astype(np.float32)
        lu, li = cm.ids(gu, gi)
        outs.append(O.train_step(cm.shape, ref, st, lu, li, y, HYPER))
        batches.append((gu, gi, y))
    assert batches[0][0][GROUP] == U - 1 and batches[0][1][3 * GROUP - 1] == I // 2

    dev = [tuple(torch.from_numpy(a).cuda() for a in b) for b in batches]
    for s, (u, it, y) in enumerate(dev):
        probs = torch.empty(B, dtype=torch.float32, device="cuda")
        nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < steps else None
        eng.train_step(u, it, y, group=GROUP, k=2, probs_out=probs, next_batch=nxt)
        err = float(np.max(np.abs(probs.cpu().numpy() - outs[s][1])))
        assert err <= 2e-6 * (1 + s), "step %d probs: max err %g" % (s, err)
    eng.check_errors()
    stats = NCFEngine.read_stats(eng.stats)
    assert stats["steps"] == steps
    assert stats["loss"] == pytest.approx(np.mean([o[0] for o in outs]), rel=2e-5)
    eng.flush()
    torch.cuda.synchronize()
    rs = eng.row_step[eng.row_step != N.NCF_ROW_PRISTINE]
    assert int(rs.min()) == int(rs.max()) == steps == int(eng.step.item())
    # only the rows some batch touched lost the pristine mark (the flush skipped the others)
    assert rs.numel() <= 2 * B * steps

    # every row of the compacted model (touched or not) against the oracle
    ur = torch.from_numpy(cm.users.astype(np.int64)).cuda()
    ir = torch.from_numpy(cm.items.astype(np.int64) + U).cuda()
    got = {}
    urows, irows = eng.emb[ur].double().cpu().numpy(), eng.emb[ir].double().cpu().numpy()
    got["user_gmf_embedding"], got["item_gmf_embedding"] = urows[:, :GMF], irows[:, :GMF]
    got["user_embedding"] = urows[:, gstride:gstride + du]
    got["item_embedding"] = irows[:, gstride:gstride + di]
    dense_got = Layout(1, 1, LAYERS, GMF).from_device(np.zeros((2, eng.row_width), np.float32),
                                                      eng.mlp.cpu().numpy())
    for name in O.weight_names(cm.shape):
        g = got[name] if name.endswith("embedding") else dense_got[name]
        tol = steps * 2e-6 + 2e-6 * float(np.max(np.abs(ref[name])))
        d = np.abs(np.asarray(g, np.float64) - ref[name])
        e = float(np.max(d))
        assert e <= tol, "%s: max err %g > %g (%d elements in %d rows beyond)" % (
            name, e, tol, int((d > tol).sum()), int((d > tol).reshape(len(d), -1).any(axis=1).sum()))

    # untouched rows: bitwise their initial values, zero moments
    touched = torch.zeros(eng.num_rows, dtype=torch.bool, device="cuda")
    for u, it, _ in dev:
        touched[u.long()] = True
        touched[it.long() + U] = True
    n_touched = int(touched.sum())
    chunk = 1 << 20
    for r0 in range(0, eng.num_rows, chunk):
        r1 = min(eng.num_rows, r0 + chunk)
        cold = ~touched[r0:r1]
        moved = (eng.emb[r0:r1] != emb0[r0:r1]).any(dim=1)
        assert not bool((moved & cold).any()), "untouched rows moved in [%d, %d)" % (r0, r1)
        nz = (eng.emb_m[r0:r1] != 0).any(dim=1) | (eng.emb_v[r0:r1] != 0).any(dim=1)
        assert not bool((nz & cold).any()), "untouched rows got moments in [%d, %d)" % (r0, r1)
        assert bool((nz | ~touched[r0:r1]).all()), "a touched row kept zero moments in [%d, %d)" % (r0, r1)
    assert 0 < n_touched < eng.num_rows


@pytest.mark.parametrize("lazy", [True, False], ids=["deferred", "dense"])
def test_large_key_space_index_matches_compacted_table(lazy):
    """Tables past 256 scan blocks (524,288 rows) build their index with k_prefix + k_fill_big
    (one workgroup per scan block) instead of k_fill.  Training steps on a 600,000 x 500 table
    equal, bit for bit, the same steps on the compacted table (the rows the batches read, ids
    remapped: built by k_fill) — rows interact only through the batches, and with zero initial
    moments an untouched row does not move under dense Adam either."""
    Ub, Ib, layers, gmf = 600_000, 500, [64, 32, 16, 8], 8
    B, steps = 4096, 3
    rng = np.random.RandomState(7)
    bt = []
    for s in range(steps):
        u = rng.randint(0, Ub, B // GROUP)
        if s == 0:
            u[:2] = [0, Ub - 1]
        bt.append((u.repeat(GROUP).astype(np.int32), rng.randint(0, Ib, B).astype(np.int32),
                   np.tile([0.0] * (GROUP - 1) + [1.0], B // GROUP).astype(np.float32)))
    uu = np.unique(np.concatenate([b[0] for b in bt]))
    ii = np.unique(np.concatenate([b[1] for b in bt]))
    big = NCFEngine(Ub, Ib, layers, gmf, max_batch=B, lazy_adam=lazy)
    assert big.num_rows + 1 > 256 * 2048   # more than 256 scan blocks of 2,048 keys
    _device_tables(big, seed=8)
    small = NCFEngine(len(uu), len(ii), layers, gmf, max_batch=B, lazy_adam=lazy)
    small.emb[:len(uu)].copy_(big.emb[torch.from_numpy(uu.astype(np.int64)).cuda()])
    small.emb[len(uu):].copy_(big.emb[torch.from_numpy(ii.astype(np.int64) + Ub).cuda()])
    small.mlp.copy_(big.mlp)
    dev_b = [tuple(torch.from_numpy(a).cuda() for a in b) for b in bt]
    dev_s = [(torch.from_numpy(np.searchsorted(uu, b[0]).astype(np.int32)).cuda(),
              torch.from_numpy(np.searchsorted(ii, b[1]).astype(np.int32)).cuda(), d[2]) for b, d in zip(bt, dev_b)]
    for eng, dev in ((big, dev_b), (small, dev_s)):
        for s, (u, it, y) in enumerate(dev):
            nxt = (dev[s + 1][0], dev[s + 1][1]) if lazy and s + 1 < steps else None
            eng.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
        eng.check_errors()
        eng.flush() if lazy else None
    torch.cuda.synchronize()
    rows = torch.from_numpy(np.concatenate([uu, ii + Ub]).astype(np.int64)).cuda()
    assert torch.equal(big.emb[rows], small.emb)
    assert torch.equal(big.emb_m[rows], small.emb_m) and torch.equal(big.emb_v[rows], small.emb_v)
    assert torch.equal(big.mlp, small.mlp) and torch.equal(big.stats, small.stats)


def test_layered_sparse_index_mixed_groups_matches_compacted_table():
    """Config D's widths on a table past 256 scan blocks (600,000 x 500 rows): the layered path with
    the sparse counted index (k_fill_touched, seen tags), user-row folding and layer 1's user half
    once per group (k_lay_l1f_gu, k_lay_dw1<4>), on batches that mix folded groups, groups with
    another user and masked-free samples, equals bit for bit the same steps on the compacted table
    (the rows the batches read, ids remapped: the dense index of a small key space).  Both engines
    run the same kernels on the same samples, so only the index paths differ."""
    Ub, Ib = 600_000, 500
    B, steps = 4096, 3
    rng = np.random.RandomState(17)
    bt = []
    for s in range(steps):
        users = rng.randint(0, Ub, B // GROUP).repeat(GROUP)
        pos = np.arange(B) % GROUP
        swap = (pos != 0) & (rng.rand(B) < 0.05)          # a few samples with another user
        users[swap] = rng.randint(0, Ub, int(swap.sum()))
        if s == 0:
            users[:GROUP] = 0
            users[GROUP:2 * GROUP] = Ub - 1
        bt.append((users.astype(np.int32), rng.randint(0, Ib, B).astype(np.int32),
                   np.tile([0.0] * (GROUP - 1) + [1.0], B // GROUP).astype(np.float32)))
    uu = np.unique(np.concatenate([b[0] for b in bt]))
    ii = np.unique(np.concatenate([b[1] for b in bt]))
    big = NCFEngine(Ub, Ib, LAYERS, GMF, max_batch=B, lazy_adam=True)
    assert big.kernel_for(B) == "layered-mfma" and big.num_rows + 1 > 256 * 2048
    _device_tables(big, seed=18)
    small = NCFEngine(len(uu), len(ii), LAYERS, GMF, max_batch=B, lazy_adam=True)
    small.emb[:len(uu)].copy_(big.emb[torch.from_numpy(uu.astype(np.int64)).cuda()])
    small.emb[len(uu):].copy_(big.emb[torch.from_numpy(ii.astype(np.int64) + Ub).cuda()])
    dense = _dense_weights(19)
    from movierec.layout import Layout
    flat = Layout(1, 1, LAYERS, GMF).to_device({**dense, "user_embedding": np.zeros((1, 128)),
                                                 "item_embedding": np.zeros((1, 128)),
                                                 "user_gmf_embedding": np.zeros((1, GMF)),
                                                 "item_gmf_embedding": np.zeros((1, GMF))})[1]
    big.mlp.copy_(torch.from_numpy(flat))
    small.mlp.copy_(big.mlp)
    dev_b = [tuple(torch.from_numpy(a).cuda() for a in b) for b in bt]
    dev_s = [(torch.from_numpy(np.searchsorted(uu, b[0]).astype(np.int32)).cuda(),
              torch.from_numpy(np.searchsorted(ii, b[1]).astype(np.int32)).cuda(), d[2]) for b, d in zip(bt, dev_b)]
    for eng, dev in ((big, dev_b), (small, dev_s)):
        for s, (u, it, y) in enumerate(dev):
            nxt = (dev[s + 1][0], dev[s + 1][1]) if s + 1 < steps else None
            eng.train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
        eng.check_errors()
        eng.flush()
    torch.cuda.synchronize()
    rows = torch.from_numpy(np.concatenate([uu, ii + Ub]).astype(np.int64)).cuda()
    assert torch.equal(big.emb[rows], small.emb)
    assert torch.equal(big.emb_m[rows], small.emb_m) and torch.equal(big.emb_v[rows], small.emb_v)
    assert torch.equal(big.mlp, small.mlp) and torch.equal(big.stats, small.stats)
