"""HIP path vs the CPU oracle, through the C ABI (ctypes → libmovierec_ncf.so).

Tolerances (fp32 device arithmetic vs float64 oracle; stated per north_star
"within a stated fp32 tolerance"):
  * probabilities: |dp| <= 2e-6
  * loss: relative 1e-5
  * gradients: |dg| <= 1e-5 * max|g| (+1e-9)
  * weights after k optimizer steps: |dw| <= k * 2e-6 (Adam moves each element
    by at most ~lr per step; fp32 rounding of m/sqrt(v) bounds the drift)
  * hr/dcg, ranking: exact.
"""

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec import _native as N
    from movierec.engine import NCFEngine, pristine_marks


SHAPES = [
    # (num_users, num_items, layers, gmf_dim)
    (5, 10, [6, 4], 0),                 # reference test model (test/test_model.py:8-26)
    (37, 53, [8, 6, 4], 4),
    (120, 90, [64, 32, 16, 8], 8),      # config B shape (ml-1m NeuMF) at small row counts
    (200, 150, [128, 64, 32, 16], 64),  # config C shape (ml-20m NeuMF)
    (31, 17, [7, 5], 3),                # odd widths: du != di, gmf not a multiple of 4
    (40, 30, [256, 128, 64, 32], 128),  # config D shape: weights outgrow LDS -> layered GEMM path
    (943, 1682, [], 8),                 # config A: ml-100k GMF-only (no MLP; generic kernel)
]


def _weights(shape, seed, scale=4.0):
    w = O.init_weights(shape, seed=seed)
    rng = np.random.RandomState(seed + 100)
    for k in w:
        if k.endswith("embedding"):
            w[k] = rng.uniform(-0.5, 0.5, size=w[k].shape)
        else:
            w[k] = w[k] * scale
            if k.endswith("bias"):
                w[k] = rng.uniform(-0.1, 0.1, size=w[k].shape)
    # keep logits well inside the BCE clip range (|z| <~ 6): near the clip
    # boundary fp32 vs fp64 rounding may legitimately flip the clip mask
    users = rng.randint(0, shape.num_users, 512)
    items = rng.randint(0, shape.num_items, 512)
    _, c = O.forward(shape, w, users, items)
    f = 6.0 / max(np.max(np.abs(c["z"])), 1e-6)
    w["output/kernel"] = w["output/kernel"] * f
    w["output/bias"] = w["output/bias"] * f
    # round to fp32 so both sides start from identical values
    return {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}


def _batch(shape, B, group, seed, dup_items=None):
    rng = np.random.RandomState(seed)
    users = rng.randint(0, shape.num_users, B // group).repeat(group)
    hi = shape.num_items if dup_items is None else dup_items
    items = rng.randint(0, hi, B)
    y = np.tile([0] * (group - 1) + [1], B // group)
    return users.astype(np.int32), items.astype(np.int32), y.astype(np.float32)


def _engine(shape, w, max_batch=4096, **kw):
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=max_batch, **kw)
    eng.set_keras_weights(w)
    return eng


def _close(a, b, atol, name=""):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    err = np.max(np.abs(a - b)) if a.size else 0.0
    assert err <= atol, "%s: max err %g > %g" % (name, err, atol)


@pytest.mark.parametrize("dims", SHAPES, ids=[str(s[2]) + "g" + str(s[3]) for s in SHAPES])
def test_predict_matches_oracle(dims):
    shape = O.NCFShape(*dims)
    w = _weights(shape, 1)
    users, items, _ = _batch(shape, 200, 4, 2)
    eng = _engine(shape, w)
    p = eng.predict(users, items).cpu().numpy()
    ref, _ = O.forward(shape, w, users, items)
    _close(p, ref, 2e-6, "probs")


@pytest.mark.parametrize("dims", SHAPES, ids=[str(s[2]) + "g" + str(s[3]) for s in SHAPES])
@pytest.mark.parametrize("path", ["auto", "generic", "layered"])
def test_forward_backward_grads_match_oracle(dims, path):
    """Every forward/backward kernel path (fused MFMA / layered MFMA where the shape has it, else the
    per-sample generic kernel — no vendor GEMM anywhere) against the oracle's gradients."""
    shape = O.NCFShape(*dims)
    w = _weights(shape, 3)
    users, items, y = _batch(shape, 256, 4, 4, dup_items=min(shape.num_items, 7))  # heavy duplicate rows
    eng = _engine(shape, w, force_generic=path == "generic", force_layered=path == "layered")
    grads = eng.alloc_grads()
    eng.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / 256, grads=grads)
    l2 = [0.0] * len(shape.layers)
    loss, g, _ = O.loss_and_grads(shape, w, users, items, y, l2)
    got = eng.keras_weights(grads[0], grads[1])
    for name in O.weight_names(shape):
        scale = np.max(np.abs(g[name])) + 1e-12
        _close(got[name], g[name], 1e-5 * scale + 1e-9, name)
    summ = grads[2].cpu().numpy()
    bce = O.bce_per_sample(O.forward(shape, w, users, items)[0], y).sum()
    assert summ[0] == pytest.approx(bce, rel=1e-5)
    hr, dcg = O.group_metrics(O.forward(shape, w, users, items)[0], y, 4, 2)
    assert summ[1] / summ[3] == pytest.approx(hr, abs=1e-6)
    assert summ[2] / summ[3] == pytest.approx(dcg, abs=1e-6)


@pytest.mark.parametrize("dims", SHAPES, ids=[str(s[2]) + "g" + str(s[3]) for s in SHAPES])
@pytest.mark.parametrize("opt,l2", [("adam", 0.0), ("adam", 0.01), ("sgd", 0.01)])
def test_train_steps_match_oracle(dims, opt, l2):
    shape = O.NCFShape(*dims)
    w = _weights(shape, 5)
    l2s = [l2] * len(shape.layers)
    lr = 0.001 if opt == "adam" else 0.05
    eng = _engine(shape, w, optimizer=opt, lr=lr, layers_l2reg=l2s)
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    hyper = dict(optimizer=opt, lr=lr, beta_1=0.9, beta_2=0.999, layers_l2reg=l2s)
    steps = 3
    losses = []
    for s in range(steps):
        users, items, y = _batch(shape, 120, 6, 10 + s, dup_items=min(shape.num_items, 9) if s == 1 else None)
        eng.train_step(users, items, y, group=6, k=3)
        loss, _ = O.train_step(shape, ref, st, users, items, y, hyper)
        losses.append(loss)
    got = eng.keras_weights()
    for name in O.weight_names(shape):
        _close(got[name], ref[name], steps * 2e-6 + 2e-6 * np.max(np.abs(ref[name])), name)
    stats = NCFEngine.read_stats(eng.stats)
    assert stats["steps"] == steps
    assert stats["loss"] == pytest.approx(np.mean(losses), rel=2e-5)
    assert int(eng.step.item()) == (steps if True else 0)


def test_clipped_samples_have_zero_gradient():
    """Keras BCE clips p to [eps, 1-eps]; TF's clip_by_value gradient is zero
    outside the range, so saturated samples contribute no gradient."""
    shape = O.NCFShape(40, 30, [8, 4], 4)
    w = _weights(shape, 2)
    w["output/bias"] = np.array([40.0])   # sigmoid saturates to 1 for every sample
    eng = _engine(shape, w)
    users, items, y = _batch(shape, 64, 4, 1)
    grads = eng.alloc_grads()
    eng.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / 64, grads=grads)
    assert float(grads[0].abs().max()) == 0.0 and float(grads[1].abs().max()) == 0.0
    p, _ = O.forward(shape, w, users, items)
    assert grads[2][0].item() == pytest.approx(O.bce_per_sample(p, y).sum(), rel=1e-5)


@pytest.mark.parametrize("batch", [512, 8192])
def test_apply_update_equals_train_step(batch):
    """forward_backward + apply_update (the data-parallel split of a step) is bitwise the fused
    train_step.  At batch 8192 the fused kernel writes more than 2 x kSlabSplit slabs, so the
    folded tails run (slab partials + summary, dense embedding gradient + dense-layer gradient
    in one launch; row update + dense-layer Adam in one launch)."""
    shape = O.NCFShape(200, 150, [128, 64, 32, 16], 64)
    w = _weights(shape, 7)
    a = _engine(shape, w, max_batch=batch)
    b = _engine(shape, w, max_batch=batch)
    users, items, y = _batch(shape, batch, 4, 8)
    a.train_step(users, items, y, group=4, k=2)
    grads = b.alloc_grads()
    b.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / batch, grads=grads)
    b.apply_update(grads, inv_batch=1.0 / batch)
    sa, sb = NCFEngine.read_stats(a.stats), NCFEngine.read_stats(b.stats)
    assert sa["loss"] == sb["loss"] and sa["hr"] == sb["hr"] and sa["steps"] == sb["steps"]
    assert torch.equal(a.emb, b.emb) and torch.equal(a.mlp, b.mlp)
    assert torch.equal(a.emb_m, b.emb_m) and torch.equal(a.emb_v, b.emb_v)


def test_user_partitioned_split_equals_train_step():
    """The user-partitioned step at world 1 (forward_backward_part -> update_rows of the user rows
    -> apply_update of the item rows and dense layers), at a batch where every folded tail
    runs, is bitwise the single-device train_step."""
    shape = O.NCFShape(3000, 700, [128, 64, 32, 16], 64)
    w = _weights(shape, 9)
    B, U = 8192, shape.num_users
    a = _engine(shape, w, max_batch=B)
    b = _engine(shape, w, max_batch=B)
    grads = (torch.zeros(shape.num_items, b.row_width, device="cuda"), torch.zeros(b.mlp_params, device="cuda"),
             torch.zeros(8, device="cuda"))
    for s in range(3):
        users, items, y = _batch(shape, B, 4, 60 + s)
        a.train_step(users, items, y, group=4, k=2)
        u, it, yy = (torch.from_numpy(x).cuda() for x in (users, items, y))
        b.forward_backward_part(u, it, yy, group=4, k=2, inv_batch=1.0 / B, shared_row_begin=U, grads=grads)
        b.update_rows(0, U, 1.0 / B)
        b.apply_update(grads, 1.0 / B, rows=(U, shape.num_items), moments_by_row=True)
    torch.cuda.synchronize()
    for x, z in ((a.emb, b.emb), (a.mlp, b.mlp), (a.emb_m, b.emb_m), (a.emb_v, b.emb_v), (a.mlp_v, b.mlp_v)):
        assert torch.equal(x, z)


def test_rank_and_metrics_kats():
    """test/test_model.py:94-190 known answers, on the device."""
    shape = O.NCFShape(5, 10, [6, 4], 0)
    eng = _engine(shape, _weights(shape, 0))
    dev = eng.device
    p = torch.tensor([0.9, 0.8, 0.7, 0.7, 0.8, 0.9], device=dev)
    np.testing.assert_equal(eng.rank(p, 3).cpu().numpy(), [[0, 1, 2], [2, 1, 0]])
    p = torch.tensor([0.9, 0.8, 0.7, 0.6, 0.5, 0.9, 0.9, 0.9], device=dev)
    np.testing.assert_equal(eng.rank(p, 4).cpu().numpy(), [[0, 1, 2, 3], [1, 2, 3, 0]])
    y = np.array([0, 0, 0, 1, 0, 0, 0, 1], np.float32)
    p = torch.tensor([0.1, 0.2, 0.9, 0.5, 0.9, 0.8, 0.7, 0.6], device=dev)
    for k, exp_hr in {0: 0.0, 1: 0.0, 2: 0.5, 3: 0.5, 4: 1.0}.items():
        hit, dcg = eng.group_metrics(p, y, 4, k)
        assert hit.mean().item() == pytest.approx(exp_hr)
        ref = O.discounted_cumulative_gain(y.reshape(2, 4), k, O.rank_layer(p.cpu().numpy(), 4))
        assert dcg.mean().item() == pytest.approx(ref, rel=1e-6)
    p = torch.tensor([0.9, 0.55, 0.55, 0.55], device=dev)   # ties: positive ranked last
    for k in (0, 1, 2, 3):
        hit, dcg = eng.group_metrics(p, y[:4], 4, k)
        assert hit.item() == 0.0 and dcg.item() == 0.0
    hit, _ = eng.group_metrics(p, y[:4], 4, 4)
    assert hit.item() == 1.0


def test_rank_random_matches_oracle():
    shape = O.NCFShape(5, 10, [6, 4], 0)
    eng = _engine(shape, _weights(shape, 0))
    rng = np.random.RandomState(0)
    p = np.round(rng.rand(100 * 37), 2).astype(np.float32)  # many ties
    got = eng.rank(torch.from_numpy(p).to(eng.device), 100).cpu().numpy()
    np.testing.assert_array_equal(got, O.rank_layer(p, 100))


def test_evaluate_matches_oracle():
    shape = O.NCFShape(120, 90, [64, 32, 16, 8], 8)
    w = _weights(shape, 9)
    l2s = [0.01, 0.02, 0.0, 0.01]
    eng = _engine(shape, w, layers_l2reg=l2s)
    users, items, y = _batch(shape, 400, 100, 3)
    eng.evaluate(users, items, y, group=100, k=10)
    p, _ = O.forward(shape, w, users, items)
    loss = O.bce_per_sample(p, y).mean() + O.reg_loss(shape, w, l2s)
    hr, dcg = O.group_metrics(p, y, 100, 10)
    st = NCFEngine.read_stats(eng.val_stats)
    assert st["loss"] == pytest.approx(loss, rel=1e-5)
    assert st["hr"] == pytest.approx(hr, abs=1e-7)
    assert st["dcg"] == pytest.approx(dcg, abs=1e-6)


def test_deterministic_bitwise():
    shape = O.NCFShape(1000, 300, [128, 64, 32, 16], 64)
    w = _weights(shape, 11)
    runs = []
    for _ in range(2):
        eng = _engine(shape, w)
        for s in range(3):
            users, items, y = _batch(shape, 4096, 4, 20 + s, dup_items=50)
            eng.train_step(users, items, y, group=4, k=2)
        runs.append((eng.emb.clone(), eng.mlp.clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


def test_invalid_params_raise():
    with pytest.raises(ValueError):
        NCFEngine(10, 10, [], 0)
    shape = O.NCFShape(10, 10, [6, 4], 0)
    eng = _engine(shape, _weights(shape, 0))
    u, i, y = _batch(shape, 12, 4, 0)
    with pytest.raises(ValueError):
        eng.train_step(u, i, y, group=5, k=2)  # batch not divisible by group


@pytest.mark.parametrize("opt", ["adam", "sgd"])
@pytest.mark.parametrize("dims", [SHAPES[3], SHAPES[1], SHAPES[5]], ids=["configC", "small", "configD"])
def test_lazy_decay_bitwise_equals_dense_sweep(dims, opt):
    """Deferred exact decay (ncf_optim_t.row_step): rows untouched for several steps replay
    their zero-gradient Adam steps when next touched or flushed — bitwise the dense sweep."""
    shape = O.NCFShape(*dims)
    w = _weights(shape, 12)
    lr = 0.001 if opt == "adam" else 0.05
    dense = _engine(shape, w, optimizer=opt, lr=lr)
    lazy = _engine(shape, w, optimizer=opt, lr=lr, lazy_adam=True)
    assert lazy.lazy and not dense.lazy
    for s in range(7):
        # small batches over a larger table: most rows stay untouched for several steps
        users, items, y = _batch(shape, 24, 4, 40 + s, dup_items=min(shape.num_items, 11) if s % 3 == 0 else None)
        dense.train_step(users, items, y, group=4, k=2)
        lazy.train_step(users, items, y, group=4, k=2)
        if s in (2, 6):
            lazy.flush()
            assert torch.equal(dense.emb, lazy.emb) and torch.equal(dense.mlp, lazy.mlp)
            if opt == "adam":
                assert torch.equal(dense.emb_m, lazy.emb_m) and torch.equal(dense.emb_v, lazy.emb_v)
            rs = lazy.row_step[lazy.row_step != N.NCF_ROW_PRISTINE]
            if opt == "adam":
                assert int(rs.min()) == int(lazy.step.item()) == s + 1
            else:   # SGD leaves no moments: every row stays pristine (current at any step)
                assert rs.numel() == 0 and int(lazy.step.item()) == s + 1
    # reads flush implicitly
    users, items, y = _batch(shape, 40, 4, 99)
    dense.train_step(users, items, y, group=4, k=2)
    lazy.train_step(users, items, y, group=4, k=2)
    assert torch.equal(dense.predict(users, items), lazy.predict(users, items))
    assert torch.equal(dense.emb, lazy.emb)
    np.testing.assert_array_equal(dense.keras_weights()["item_embedding"], lazy.keras_weights()["item_embedding"])
    assert NCFEngine.read_stats(dense.stats) == NCFEngine.read_stats(lazy.stats)


@pytest.mark.parametrize("dims", [SHAPES[3], SHAPES[5]], ids=["configC", "configD"])
def test_pristine_rows_after_set_optimizer_state_bitwise(dims):
    """Pristine rows (row_step == NCF_ROW_PRISTINE: Adam moments exactly +0) skip every replay
    and the flush; set_optimizer_state marks exactly the rows whose moments are all +0 (a -0
    moment is not +0: the zero-gradient step would flip a -0 weight's sign).  The run continues
    bitwise the dense sweep, with and without counting ahead."""
    shape = O.NCFShape(*dims)
    w = _weights(shape, 21)
    dense = _engine(shape, w)
    lazy = _engine(shape, w, lazy_adam=True)
    ahead = _engine(shape, w, lazy_adam=True)
    R = int(dense.num_rows)
    assert int((lazy.row_step == N.NCF_ROW_PRISTINE).sum()) == R   # fresh moments: every row pristine
    # a saved optimizer state: moments on the even rows (one of them only a -0 entry), +0 elsewhere
    rng = np.random.RandomState(5)
    m, v, _ = dense.optimizer_state()
    for name in m:
        if name.endswith("embedding"):
            mm = np.zeros_like(m[name])
            vv = np.zeros_like(v[name])
            mm[::2] = rng.uniform(-1e-3, 1e-3, size=mm[::2].shape)
            vv[::2] = rng.uniform(0, 1e-6, size=vv[::2].shape)
            m[name], v[name] = mm, vv
        else:
            m[name] = rng.uniform(-1e-3, 1e-3, size=m[name].shape)
            v[name] = rng.uniform(0, 1e-6, size=v[name].shape)
    for e in (dense, lazy, ahead):
        e.set_optimizer_state(m, v, 9)
    for e in (lazy, ahead):
        e.emb_m[1, 0] = -0.0
        e.row_step.copy_(pristine_marks(e.emb_m, e.emb_v, R, 9))
    dense.emb_m[1, 0] = -0.0
    marks = lazy.row_step.cpu().numpy()
    assert marks[1] == 9 and (marks[3::2] == N.NCF_ROW_PRISTINE).all() and (marks[0::2] == 9).all()
    batches = [tuple(torch.from_numpy(a).cuda() for a in _batch(shape, 24, 4, 70 + s)) for s in range(6)]
    for s, (u, it, y) in enumerate(batches):
        dense.train_step(u, it, y, group=4, k=2)
        lazy.train_step(u, it, y, group=4, k=2)
        nxt = (batches[s + 1][0], batches[s + 1][1]) if s + 1 < len(batches) else None
        ahead.train_step(u, it, y, group=4, k=2, next_batch=nxt)
    for e in (lazy, ahead):
        e.flush()
        assert torch.equal(dense.emb, e.emb) and torch.equal(dense.mlp, e.mlp)
        assert torch.equal(dense.emb_m, e.emb_m) and torch.equal(dense.emb_v, e.emb_v)
        assert (e.row_step == N.NCF_ROW_PRISTINE).any()


@pytest.mark.parametrize("dims", [SHAPES[3], SHAPES[1], SHAPES[5]], ids=["configC", "small", "configD"])
@pytest.mark.parametrize("path", ["auto", "generic", "layered"])
def test_out_of_range_ids_are_masked(dims, path):
    """Device semantics for ids outside the table (the Python layer rejects them first, like
    TF's gather; a device batch can still carry them): such a sample predicts NaN and
    contributes no gradient, loss or metric; the rest of the batch is untouched — the
    gradients equal the oracle's on the valid samples with the same 1/B normalisation."""
    shape = O.NCFShape(*dims)
    w = _weights(shape, 21)
    users, items, y = _batch(shape, 128, 4, 22)
    bad = np.zeros(128, bool)
    bad[[3, 50, 77]] = True
    users[3], items[50], users[77], items[77] = shape.num_users, -1, -5, shape.num_items + 9
    eng = _engine(shape, w, force_generic=path == "generic", force_layered=path == "layered")
    grads = eng.alloc_grads()
    probs = torch.empty(128, dtype=torch.float32, device="cuda")
    eng.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / 128, grads=grads, probs_out=probs)
    p = probs.cpu().numpy()
    assert np.isnan(p[bad]).all() and np.isfinite(p[~bad]).all()
    ok = ~bad
    _, g, _ = O.loss_and_grads(shape, w, users[ok], items[ok], y[ok], [0.0] * len(shape.layers), batch_norm=128)
    got = eng.keras_weights(grads[0], grads[1])
    for name in O.weight_names(shape):
        scale = np.max(np.abs(g[name])) + 1e-12
        _close(got[name], g[name], 1e-5 * scale + 1e-9, name)
    pref, _ = O.forward(shape, w, users[ok], items[ok])
    _close(p[ok], pref, 2e-6, "probs")
    bce = O.bce_per_sample(pref, y[ok]).sum()
    assert grads[2][0].item() == pytest.approx(bce, rel=1e-5)


def test_model_rejects_out_of_range_ids():
    """MovierecModel raises ValueError before the device sees an id outside the table."""
    from movierec.model import MovierecModel
    params = dict(num_users=20, num_items=30, layers_sizes=[8, 4], layers_l2reg=[0, 0], optimizer="adam",
                  lr=0.001, beta_1=0.9, beta_2=0.999, batch_size=8, num_negs_per_pos=3, batch_size_eval=8,
                  num_negs_per_pos_eval=3, k=2)
    m = MovierecModel(params, output_dir="/tmp/movierec_models", verbose=0)
    with pytest.raises(ValueError):
        m.model.predict_on_batch([np.array([0, 20], np.int32), np.array([1, 2], np.int32)])
    with pytest.raises(ValueError):
        m.model.predict_on_batch([np.array([0, 1], np.int32), np.array([1, 30], np.int32)])


@pytest.mark.parametrize("group", [5, 100])
def test_single_group_batch(group):
    """Smallest batch: one user group (group does not divide 32 -> metrics outside the fused
    kernel; 100 = the evaluation group)."""
    shape = O.NCFShape(*SHAPES[3])
    w = _weights(shape, 30)
    users, items, y = _batch(shape, group, group, 31)
    eng = _engine(shape, w)
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    eng.train_step(users, items, y, group=group, k=2)
    loss, _ = O.train_step(shape, ref, st, users, items, y, dict(optimizer="adam", lr=0.001, beta_1=0.9,
                                                                  beta_2=0.999, layers_l2reg=[0.0] * 4))
    got = eng.keras_weights()
    for name in O.weight_names(shape):
        _close(got[name], ref[name], 2e-6 + 2e-6 * np.max(np.abs(ref[name])), name)
    assert NCFEngine.read_stats(eng.stats)["loss"] == pytest.approx(loss, rel=2e-5)


def test_prebuilt_index_equals_inline_build():
    """User-partitioned step with the next batch's index built ahead (ncf_build_index under the
    all-reduce, hyper.index_ready) is bitwise the step that builds its own index."""
    shape = O.NCFShape(*SHAPES[3])
    w = _weights(shape, 40)
    U = shape.num_users
    batches = []
    for s in range(4):
        users, items, y = _batch(shape, 256, 4, 41 + s)
        batches.append((torch.from_numpy(users).cuda(), torch.from_numpy(items).cuda(), torch.from_numpy(y).cuda()))
    engines = [_engine(shape, w), _engine(shape, w)]
    outs = []
    for e, ahead in zip(engines, (False, True)):
        grads = (torch.zeros(shape.num_items, e.row_width, device="cuda"), torch.zeros(e.mlp_params, device="cuda"),
                 torch.zeros(8, device="cuda"))
        for s, (u, it, y) in enumerate(batches):
            e.forward_backward_part(u, it, y, group=4, k=2, inv_batch=1.0 / 256, shared_row_begin=U, grads=grads)
            e.update_rows(0, U, 1.0 / 256)
            if ahead and s + 1 < len(batches):
                e.build_index(batches[s + 1][0], batches[s + 1][1], 4)
                assert e._prebuilt is not None
            e.apply_update(grads, 1.0 / 256, rows=(U, shape.num_items), moments_by_row=True)
        torch.cuda.synchronize()
        outs.append((e.emb.clone(), e.mlp.clone(), e.emb_m.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_count_ahead_equals_plain_steps():
    """ncf_train_step_ahead (the next batch's index counts taken inside this step's touched-row
    update, hyper.index_ready = 2 on the next call) is bitwise the plain step sequence, including
    a call whose batch differs from the counted one (counters discarded) and reads in between."""
    shape = O.NCFShape(*SHAPES[3])
    w = _weights(shape, 50)
    bt = []
    for s in range(6):
        users, items, y = _batch(shape, 256, 4, 51 + s)
        bt.append((torch.from_numpy(users).cuda(), torch.from_numpy(items).cuda(), torch.from_numpy(y).cuda()))
    a = _engine(shape, w, lazy_adam=True)
    b = _engine(shape, w, lazy_adam=True)
    order = [0, 1, 2, 4, 5]           # the step after 2 was announced as 3 but 4 comes
    announced = [1, 2, 3, 5, None]
    for s, j in enumerate(order):
        nxt = announced[s]
        a.train_step(*bt[j], group=4, k=2, next_batch=None if nxt is None else (bt[nxt][0], bt[nxt][1]))
        if s == 1:
            a.predict(bt[0][0], bt[0][1])   # a read (flush) between counted steps
        b.train_step(*bt[j], group=4, k=2)
        if s == 1:
            b.predict(bt[0][0], bt[0][1])
    a.flush()
    b.flush()
    torch.cuda.synchronize()
    for x, y in ((a.emb, b.emb), (a.emb_m, b.emb_m), (a.emb_v, b.emb_v), (a.mlp, b.mlp), (a.stats, b.stats)):
        assert torch.equal(x, y)


def test_counted_ahead_ids_changed_in_place():
    """A counted-ahead batch refilled in place before its step (a staging pattern): through torch
    (version bump) the engine rebuilds the index — bitwise the plain steps; behind torch's back
    (.data writes, or a kernel writing the pointer) the device guard keeps every list write inside
    its key's slots, clears the counters and reports NCF_WSERR_STALE_COUNT (check_errors raises);
    the engine keeps working afterwards."""
    shape = O.NCFShape(*SHAPES[3])
    w = _weights(shape, 60)
    bt = []
    for s in range(4):
        users, items, y = _batch(shape, 256, 4, 61 + s)
        bt.append((torch.from_numpy(users).cuda(), torch.from_numpy(items).cuda(), torch.from_numpy(y).cuda()))
    a = _engine(shape, w, lazy_adam=True)
    b = _engine(shape, w, lazy_adam=True)
    stage = (bt[1][0].clone(), bt[1][1].clone())
    a.train_step(*bt[0], group=4, k=2, next_batch=stage)
    stage[1].copy_(bt[2][1])             # refill through torch: _version moves
    stage[0].copy_(bt[2][0])
    a.train_step(stage[0], stage[1], bt[2][2], group=4, k=2)
    b.train_step(*bt[0], group=4, k=2)
    b.train_step(*bt[2], group=4, k=2)
    a.check_errors()                     # nothing flagged
    a.flush()
    b.flush()
    assert torch.equal(a.emb, b.emb) and torch.equal(a.emb_m, b.emb_m) and torch.equal(a.mlp, b.mlp)
    # behind torch's back: the version counter does not move
    stage2 = (bt[3][0].clone(), bt[3][1].clone())
    a.train_step(*bt[1], group=4, k=2, next_batch=stage2)
    v = stage2[1]._version
    stage2[1].data.copy_(bt[0][1])
    assert stage2[1]._version == v
    a.train_step(stage2[0], stage2[1], bt[3][2], group=4, k=2)
    with pytest.raises(RuntimeError):
        a.check_errors()
    a.check_errors()                     # cleared by the read
    for s in range(2):                   # counters were cleared on the device: later builds are sound
        a.train_step(*bt[s], group=4, k=2)
    a.check_errors()
    assert torch.isfinite(a.emb).all()


def test_stale_count_step_keeps_the_dense_decay_state():
    """A counted-ahead batch whose item ids change behind torch's back (NCF_WSERR_STALE_COUNT):
    the rows it reads that the counted set missed owe their deferred decay.  The step must leave
    the table in a consistent deferred-decay state either way — the in-kernel fill drops the step
    (nothing of it applied), the index launches replay the missed rows before the forward pass —
    so an engine that flushes (every row current) right before the same stale step ends bitwise
    equal after the final flush; a stale p read and then applied would differ."""
    shape = O.NCFShape(*SHAPES[3])
    w = _weights(shape, 70)
    bt = []
    for s in range(4):
        users, items, y = _batch(shape, 256, 4, 71 + s)
        bt.append((torch.from_numpy(users).cuda(), torch.from_numpy(items).cuda(), torch.from_numpy(y).cuda()))
    # items of bt[3] restricted to 0..74, the stale ids 75..149: every stale item row is missed by
    # the counted set, and rows idle since step 0 owe several zero-gradient steps
    it3 = (bt[3][1] % 75).contiguous()
    stale_items = (75 + bt[0][1] % 75).contiguous()
    engines = []
    for flush_first in (False, True):
        e = _engine(shape, w, lazy_adam=True)
        for s in range(3):
            e.train_step(*bt[s], group=4, k=2)
        stage = (bt[3][0].clone(), it3.clone())
        e.train_step(*bt[2], group=4, k=2, next_batch=stage)
        stage[1].data.copy_(stale_items)     # behind torch's back: counted ids no longer match
        if flush_first:
            e.flush()                        # every row current: no replay owed
            e._dirty = True
        e.train_step(stage[0], stage[1], bt[3][2], group=4, k=2)
        with pytest.raises(RuntimeError):
            e.check_errors()
        e.flush()
        engines.append(e)
    torch.cuda.synchronize()
    a, d = engines
    assert torch.equal(a.row_step, d.row_step)
    assert torch.equal(a.emb, d.emb) and torch.equal(a.emb_m, d.emb_m) and torch.equal(a.emb_v, d.emb_v)
    assert torch.equal(a.mlp, d.mlp)


def test_discarded_counts_keep_sticky_flags():
    """Dropping a counted-ahead batch (the next step passes other ids) clears only the index
    counters: an id-range flag raised before stays for check_errors."""
    shape = O.NCFShape(*SHAPES[3])
    w = _weights(shape, 80)
    b0 = [torch.from_numpy(x).cuda() for x in _batch(shape, 256, 4, 81)]
    b1 = [torch.from_numpy(x).cuda() for x in _batch(shape, 256, 4, 82)]
    b2 = [torch.from_numpy(x).cuda() for x in _batch(shape, 256, 4, 83)]
    e = _engine(shape, w, lazy_adam=True)
    bad_items = b0[1].clone()
    bad_items[5] = shape.num_items + 3       # outside the table: masked and flagged on the device
    e.train_step(b0[0], bad_items, b0[2], group=4, k=2, next_batch=(b1[0], b1[1]))
    e.train_step(*b2, group=4, k=2)          # not the counted batch: the counts are discarded
    with pytest.raises(ValueError):
        e.check_errors()
    e.check_errors()


def test_sharded_workspace_flags():
    """ShardedNCFEngine.check_errors reads the flags at the row-sharded layout's offset."""
    from movierec.sharded import ShardedNCFEngine
    shape = O.NCFShape(*SHAPES[3])
    e = ShardedNCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, world=3, rank=1,
                         max_batch=256)
    users, items, _ = _batch(shape, 256, 4, 90)
    e.plan(users, items, group=4)
    e.check_errors()
    items[7] = -1
    e.plan(users, items, group=4)
    with pytest.raises(ValueError):
        e.check_errors()
    e.check_errors()


def test_evaluate_full_protocol_fused_forward():
    """ncf_evaluate on a 200,000-sample validation pass (2,000 users x [99 negatives + the
    held-out positive], k = 10) over config C's full tables: the fused MFMA forward against the
    oracle (probabilities |dp| <= 2e-6; HR@10 / NDCG@10 of the device's own probabilities equal
    the oracle's metric functions applied to them, and within the north star's +-0.002 of the
    oracle's fp64 forward)."""
    U, I = 138493, 27278
    shape = O.NCFShape(U, I, [128, 64, 32, 16], 64)
    w = {k: v.astype(np.float32).astype(np.float64) for k, v in O.init_weights(shape, seed=70).items()}
    for k in w:   # spread the logits (Keras init gives ~0.5 everywhere): realistic ranking margins
        if not k.endswith("bias"):
            w[k] = (w[k] * (20.0 if k.endswith("embedding") else 2.0)).astype(np.float32).astype(np.float64)
    rng = np.random.RandomState(71)
    users = rng.choice(U, 2000, replace=False).repeat(100).astype(np.int32)
    items = rng.randint(0, I, 200000).astype(np.int32)
    y = np.tile([0.0] * 99 + [1.0], 2000).astype(np.float32)
    eng = _engine(shape, w, max_batch=200000)
    assert eng.fast_path
    probs = torch.empty(200000, dtype=torch.float32, device="cuda")
    eng.evaluate(users, items, y, group=100, k=10, probs_out=probs)
    st = NCFEngine.read_stats(eng.val_stats)
    p = probs.cpu().numpy()
    pref, _ = O.forward(shape, w, users, items)
    _close(p, pref, 2e-6, "probs")
    hr_dev, dcg_dev = O.group_metrics(p, y, 100, 10)
    assert st["hr"] == pytest.approx(hr_dev, abs=1e-7) and st["dcg"] == pytest.approx(dcg_dev, abs=1e-6)
    hr_ref, dcg_ref = O.group_metrics(pref, y, 100, 10)
    assert abs(st["hr"] - hr_ref) <= 0.002 and abs(st["dcg"] - dcg_ref) <= 0.002
    assert st["loss"] == pytest.approx(O.bce_per_sample(pref, y).mean(), rel=1e-5)
    # predict() takes the same fused forward
    np.testing.assert_array_equal(eng.predict(users[:4096], items[:4096]).cpu().numpy(), p[:4096])


@pytest.mark.parametrize("group", [9, 100, 150])
def test_group_metrics_wide_groups_match_oracle(group):
    """Groups wider than 8 run one wave per group (k_group_metrics_wave, chunks of 64 lanes for
    group > 64): per-group hit and dcg equal the reference's RankLayer + _get_hits_per_user
    restatement (model.py:344-455), label ties (first max wins) and probability ties included."""
    shape = O.NCFShape(5, 10, [6, 4], 0)
    eng = _engine(shape, _weights(shape, 0))
    rng = np.random.RandomState(group)
    ng = 300
    p = np.round(rng.rand(ng, group), 2).astype(np.float32)      # many probability ties
    y = np.zeros((ng, group), np.float32)
    lab = rng.randint(0, group, ng)
    y[np.arange(ng), lab] = 1.0
    y[::7, (lab[::7] + 3) % group] = 1.0                         # two positives: the first counts
    p[::5, (lab[::5] + 1) % group] = p[::5, lab[::5]]             # a negative tied with the positive
    for k in (1, 10, group):
        hit, dcg = eng.group_metrics(torch.from_numpy(p.reshape(-1)).to(eng.device), y.reshape(-1), group, k)
        rank = O.rank_layer(p.reshape(-1), group)
        hits, pos = O.hits_per_user(y, rank, k)
        np.testing.assert_array_equal(hit.cpu().numpy(), hits.astype(np.float32))
        ref_dcg = np.where(hits, np.log(2.0) / np.log(pos + 2.0), 0.0)
        np.testing.assert_allclose(dcg.cpu().numpy(), ref_dcg, rtol=1e-6, atol=0)


@pytest.mark.parametrize("B,group", [(5000, 5), (3000, 3), (100, 5), (4095, 7)])
def test_deferred_decay_step_metrics_in_update_launch(B, group):
    """Deferred decay on one stream: a group the forward/backward kernel does not rank in-kernel
    (not a fold width) has its hr/dcg partials computed by extra blocks of the touched-row update
    launch (the batch summary follows it) — or, when the summary is written before that launch
    (few slabs: the one-level tail), by the separate metrics launch.  Either way the step's stats
    equal the oracle metric of the device probabilities, and the dense-sweep engine (metrics
    always launched on their own) agrees bitwise on the stats."""
    shape = O.NCFShape(*SHAPES[2])
    w = _weights(shape, 70)
    users, items, y = _batch(shape, B, group, 71 + B)
    a = _engine(shape, w, lazy_adam=True, max_batch=B)
    b = _engine(shape, w, lazy_adam=False, max_batch=B)
    probs = torch.empty(B, dtype=torch.float32, device="cuda")
    a.train_step(users, items, y, group=group, k=3, probs_out=probs)
    b.train_step(users, items, y, group=group, k=3)
    torch.cuda.synchronize()
    hr, dcg = O.group_metrics(probs.cpu().numpy().astype(np.float64), y, group, 3)
    r = NCFEngine.read_stats(a.stats)
    assert r["hr"] == pytest.approx(hr, abs=1e-6) and r["dcg"] == pytest.approx(dcg, abs=1e-6)
    rb = NCFEngine.read_stats(b.stats)
    for key in ("hr", "dcg", "loss"):
        assert r[key] == pytest.approx(rb[key], rel=1e-6, abs=1e-9), key
