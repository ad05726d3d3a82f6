"""The MFMA forward/backward kernels of the fused shapes — the sample-unit kernel (ncf_unit.hip,
the default), the wave-chain kernel (ncf_wave.hip, hyper.force_generic 5: its split form with
separate weight-gradient waves where the shape fits, "wave1" = force_generic 6: its one-wave form)
and the 128-sample tile kernel (ncf_fused.hip, hyper.force_generic 3) — each against the oracle (reference
movierec/model.py:154-214 restated) on the same batches, forced per engine (``fb_kernel=``) so
every one runs at every size here.

Tolerances as tests/test_native_gpu.py: gradients |dg| <= 1e-5 max|g|, probabilities 2e-6,
weights after k steps k * 2e-6 + 2e-6 max|w|, BCE sum relative 1e-5, hr/dcg of the device
probabilities exact.
"""

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec.engine import NCFEngine

FUSED_SHAPES = [
    (200, 150, [128, 64, 32, 16], 64),  # config C
    (120, 90, [64, 32, 16, 8], 8),      # config B
    (120, 90, [64, 32, 16, 8], 0),      # reference trainer default (MLP-only)
    (200, 150, [128, 64, 32, 16], 0),
]
IDS = ["configC", "configB", "mlp64", "mlp128"]


def _weights(shape, seed):
    from test_native_gpu import _weights as w
    return w(shape, seed)


def _batch(shape, B, group, seed):
    rng = np.random.RandomState(seed)
    users = rng.randint(0, shape.num_users, -(-B // group)).repeat(group)[:B]
    items = rng.randint(0, shape.num_items, B)
    y = np.tile([0] * (group - 1) + [1], -(-B // group))[:B].astype(np.float32)
    return users.astype(np.int32), items.astype(np.int32), y


def _engine(shape, w, kernel, max_batch=4096, **kw):
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=max_batch,
                    fb_kernel=kernel, **kw)
    eng.set_keras_weights(w)
    return eng


@pytest.mark.parametrize("dims", FUSED_SHAPES, ids=IDS)
@pytest.mark.parametrize("kernel", ["unit", "wave", "wave1", "tile"])
@pytest.mark.parametrize("B,group", [(32, 4), (100, 4), (1000, 5), (2050, 2), (4099, 1)])
def test_grads_match_oracle(dims, kernel, B, group):
    shape = O.NCFShape(*dims)
    w = _weights(shape, 11)
    users, items, y = _batch(shape, B, group, 12 + B)
    eng = _engine(shape, w, kernel)
    assert eng.kernel_for(B) == "fused-mfma-" + kernel.rstrip("1")
    grads = eng.alloc_grads()
    probs = torch.empty(B, dtype=torch.float32, device="cuda")
    eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads, probs_out=probs)
    _, g, _ = O.loss_and_grads(shape, w, users, items, y, [0.0] * len(shape.layers))
    got = eng.keras_weights(grads[0], grads[1])
    for name in O.weight_names(shape):
        scale = np.max(np.abs(g[name])) + 1e-12
        err = np.max(np.abs(got[name] - g[name]))
        assert err <= 1e-5 * scale + 1e-9, (name, err, scale)
    pref, _ = O.forward(shape, w, users, items)
    assert np.max(np.abs(probs.cpu().numpy() - pref)) <= 2e-6
    bce = O.bce_per_sample(pref, y).sum()
    assert grads[2][0].item() == pytest.approx(bce, rel=1e-5)


@pytest.mark.parametrize("dims", FUSED_SHAPES[:2], ids=IDS[:2])
@pytest.mark.parametrize("lazy", [False, True], ids=["dense", "deferred"])
@pytest.mark.parametrize("kernel", ["unit", "wave"])
def test_unit_train_steps_match_oracle(dims, lazy, kernel):
    shape = O.NCFShape(*dims)
    w = _weights(shape, 21)
    eng = _engine(shape, w, kernel, lazy_adam=lazy)
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    hyper = dict(optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=[0.0] * 4)
    for s in range(3):
        users, items, y = _batch(shape, 512, 4, 22 + s)
        eng.train_step(users, items, y, group=4, k=2)
        loss, _ = O.train_step(shape, ref, st, users, items, y, hyper)
    got = eng.keras_weights()
    for name in O.weight_names(shape):
        tol = 3 * 2e-6 + 2e-6 * np.max(np.abs(ref[name]))
        err = np.max(np.abs(got[name] - ref[name]))
        assert err <= tol, (name, err, tol)
    assert NCFEngine.read_stats(eng.stats)["loss"] > 0


@pytest.mark.parametrize("B", [16384 + 100, 20000])
@pytest.mark.parametrize("kernel", ["unit", "wave", "wave1"])
def test_two_group_schedule_matches_oracle(B, kernel):
    """Batches of >= 16384 run two unit groups per workgroup (two waves per SIMD); uneven rounds
    leave the last group of some workgroups on masked samples.  The wave kernel: several units
    per wave, the last ones partly or wholly past n."""
    shape = O.NCFShape(*FUSED_SHAPES[0])
    w = _weights(shape, 51)
    users, items, y = _batch(shape, B, 4, 52)
    eng = _engine(shape, w, kernel, max_batch=B)
    grads = eng.alloc_grads()
    probs = torch.empty(B, dtype=torch.float32, device="cuda")
    eng.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / B, grads=grads, probs_out=probs)
    _, g, _ = O.loss_and_grads(shape, w, users, items, y, [0.0] * 4)
    got = eng.keras_weights(grads[0], grads[1])
    for name in O.weight_names(shape):
        scale = np.max(np.abs(g[name])) + 1e-12
        assert np.max(np.abs(got[name] - g[name])) <= 1e-5 * scale + 1e-9, name
    pref, _ = O.forward(shape, w, users, items)
    assert np.max(np.abs(probs.cpu().numpy() - pref)) <= 2e-6
    assert grads[2][0].item() == pytest.approx(O.bce_per_sample(pref, y).sum(), rel=1e-5)


@pytest.mark.parametrize("kernel", ["unit", "wave", "wave1"])
def test_unit_masked_ids_and_metrics(kernel):
    """Ids outside the table: NaN probability, no gradient; in-kernel hr/dcg (group | 32, wave
    kernel group | 16) equal the metric of the device probabilities."""
    shape = O.NCFShape(*FUSED_SHAPES[0])
    w = _weights(shape, 31)
    users, items, y = _batch(shape, 256, 4, 32)
    bad = np.zeros(256, bool)
    bad[[5, 66, 200]] = True
    users[5], items[66], users[200] = shape.num_users + 3, -2, -1
    eng = _engine(shape, w, kernel)
    grads = eng.alloc_grads()
    probs = torch.empty(256, dtype=torch.float32, device="cuda")
    eng.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / 256, grads=grads, probs_out=probs)
    p = probs.cpu().numpy()
    assert np.isnan(p[bad]).all() and np.isfinite(p[~bad]).all()
    ok = ~bad
    _, g, _ = O.loss_and_grads(shape, w, users[ok], items[ok], y[ok], [0.0] * 4, batch_norm=256)
    got = eng.keras_weights(grads[0], grads[1])
    for name in O.weight_names(shape):
        scale = np.max(np.abs(g[name])) + 1e-12
        assert np.max(np.abs(got[name] - g[name])) <= 1e-5 * scale + 1e-9, name
    # metrics: a clean batch through train_step, stats vs the oracle metric of the device probs
    users, items, y = _batch(shape, 512, 4, 33)
    eng2 = _engine(shape, w, kernel)
    probs = torch.empty(512, dtype=torch.float32, device="cuda")
    eng2.train_step(users, items, y, group=4, k=2, probs_out=probs)
    hr, dcg = O.group_metrics(probs.cpu().numpy().astype(np.float64), y, 4, 2)
    r = NCFEngine.read_stats(eng2.stats)
    assert r["hr"] == pytest.approx(hr, abs=1e-6) and r["dcg"] == pytest.approx(dcg, abs=1e-6)


def test_unit_deterministic_and_close_to_tile():
    shape = O.NCFShape(*FUSED_SHAPES[0])
    w = _weights(shape, 41)
    users, items, y = _batch(shape, 4096, 4, 42)
    outs = {}
    for kernel in ("unit", "unit", "wave", "wave", "tile"):
        eng = _engine(shape, w, kernel)
        for _ in range(2):
            eng.train_step(users, items, y, group=4, k=2)
        torch.cuda.synchronize()
        outs.setdefault(kernel, []).append((eng.emb.clone(), eng.mlp.clone()))
    t = outs["tile"][0]
    for kernel in ("unit", "wave"):
        a, b = outs[kernel]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        assert torch.max(torch.abs(a[0] - t[0])).item() <= 1e-6
        assert torch.max(torch.abs(a[1] - t[1])).item() <= 1e-6


@pytest.mark.parametrize("dims", FUSED_SHAPES, ids=IDS)
@pytest.mark.parametrize("B,group", [(64, 4), (4096 + 48, 4), (16384 * 4 + 16, 4), (65536, 4), (20000, 8),
                                     (12000, 2), (3000, 1), (131072 + 32, 4)])
def test_wave_split_form_bitwise_one_wave(dims, B, group):
    """The split form (chain waves + weight-gradient waves, one barrier per unit) issues the same
    MFMAs on the same operands in the same order as the one-wave form: every output bitwise equal,
    including workgroups whose waves run different unit counts (tails) and the in-kernel metric
    variants.  With user-row folding (group 2, 4, 8) the split form computes the user half of
    layer 1 and of dX once per group (group-user form): the same sums reassociated, so there the
    two forms agree within fp32 rounding — sample 7 (an out-of-range user, not its group head's)
    takes the group-user form's per-sample branch."""
    shape = O.NCFShape(*dims)
    w = _weights(shape, 61)
    users, items, y = _batch(shape, B, group, 62 + B)
    users[7] = shape.num_users + 1       # masked samples: row 0 read, zero gradient
    items[B - 3] = -5
    outs = []
    for kernel in ("wave", "wave1"):
        eng = _engine(shape, w, kernel, max_batch=B)
        grads = eng.alloc_grads()
        probs = torch.empty(B, dtype=torch.float32, device="cuda")
        eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads, probs_out=probs)
        eng2 = _engine(shape, w, kernel, max_batch=B)
        users2 = users.copy()
        users2[7] = 0
        items2 = items.copy()
        items2[B - 3] = 0
        eng2.train_step(users2, items2, y, group=group, k=min(2, group))
        torch.cuda.synchronize()
        outs.append([grads[0].clone(), grads[1].clone(), grads[2].clone(), probs.clone(), eng2.emb.clone(),
                     eng2.mlp.clone(), eng2.stats.clone()])
    if group == 1:
        for a, b in zip(*outs):
            assert torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))
        return
    (ge, gm, gsum, p, emb, mlp, st), (re_, rm, rsum, rp, remb, rmlp, rst) = outs
    assert torch.equal(torch.isnan(p), torch.isnan(rp))
    assert torch.max(torch.abs(p.nan_to_num(0.0) - rp.nan_to_num(0.0))).item() <= 2e-6
    for a, b in ((ge, re_), (gm, rm)):
        assert torch.max(torch.abs(a - b)).item() <= 1e-5 * max(torch.max(torch.abs(b)).item(), 1e-30)
    assert torch.max(torch.abs(emb - remb)).item() <= 1e-6 and torch.max(torch.abs(mlp - rmlp)).item() <= 1e-6
    # summary / stats: the loss and the counts; hit / dcg rank probabilities that may tie (or
    # saturate at 1) within rounding, so they are compared through the oracle in other tests
    ia, ib = NCFEngine.read_stats(st), NCFEngine.read_stats(rst)
    assert ia["loss"] == pytest.approx(ib["loss"], rel=1e-5)
    assert gsum[0].item() == pytest.approx(rsum[0].item(), rel=1e-5)


def test_kernel_selection_by_batch():
    shape = O.NCFShape(*FUSED_SHAPES[0])
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256)
    assert eng.kernel_for(8192) == "fused-mfma-unit"
    assert eng.kernel_for(16384) == "fused-mfma-wave"
    assert eng.kernel_for(65536) == "fused-mfma-wave"
    # bf16 operands: the unit kernel at every size
    assert NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256,
                     precision="bf16").kernel_for(65536) == "fused-mfma-unit"
    assert NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256,
                     fb_kernel="tile").kernel_for(65536) == "fused-mfma-tile"
    assert NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256,
                     fb_kernel="wave").kernel_for(65536) == "fused-mfma-wave"
    # bf16 operands are the unit kernel's: a forced wave kernel falls back to it
    assert NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256,
                     fb_kernel="wave", precision="bf16").kernel_for(65536) == "fused-mfma-unit"
    assert NCFEngine(5, 10, [6, 4], 0, max_batch=64).kernel_for(64) == "generic"
    assert gpu_available()
