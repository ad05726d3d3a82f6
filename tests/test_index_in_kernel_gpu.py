"""The step's index built inside the forward/backward launch (ncf_capi.hip fill_in_kernel).

A deferred-decay step whose batch was counted ahead by the previous step (``train_step(...,
next_batch=)``, as bench.py and fit_generator run it) skips the index fill and list-sort
launches: from 16,384 samples the wave kernel's weight-gradient waves fill the index while their
chain waves run the first unit (``fill_wave``, ncf_internal.h); below, spare workgroups of the
unit kernel's launch do, where its grid leaves CUs idle (else a fill launch of its own).  The
touched-row update orders each row's contribution list itself — across the lanes of the row's
group, or block-wide for rows longer than a row group (heavy rows).  The embedding update must still sum every row's
contributions in ascending order, so these tests hold that path BITWISE against the dense Keras
sweep (every row, sorted lists) and against deferred decay with the fill and sort launches
(reference semantics: movierec/model.py:199-202, Keras v1 Adam over the densified IndexedSlices).
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

LAYERS, GMF = [128, 64, 32, 16], 64     # config C's model: the wave kernel's split form
GROUP = 4


def _weights(shape, seed):
    w = O.init_weights(shape, seed=seed)
    rng = np.random.RandomState(seed + 1)
    for k in w:
        if k.endswith("embedding"):
            w[k] = rng.uniform(-0.05, 0.05, size=w[k].shape)
    return {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}


def _batch(U, I, B, seed, hot_items=3, hot_frac=0.05, mixed_frac=0.1):
    """Groups of GROUP samples sharing a user, except a fraction of groups whose samples have
    different users (the fill's per-sample user rows); a few hot items and one hot user, so some
    rows get far more contributions than a row group has lanes (heavy rows)."""
    rng = np.random.RandomState(seed)
    ng = B // GROUP
    users = rng.randint(0, U, ng).repeat(GROUP)
    users[:ng // 8 * GROUP] = 7                       # hot user: ng / 8 groups
    mixed = np.flatnonzero(rng.uniform(size=ng) < mixed_frac)
    for g in mixed:
        users[g * GROUP + 1:(g + 1) * GROUP] = rng.randint(0, U, GROUP - 1)
    items = rng.randint(0, I, B)
    hot = rng.uniform(size=B) < hot_frac
    items[hot] = rng.randint(0, hot_items, int(hot.sum()))
    y = np.tile([0.0] * (GROUP - 1) + [1.0], ng)
    return [torch.from_numpy(a).cuda().contiguous() for a in
            (users.astype(np.int32), items.astype(np.int32), y.astype(np.float32))]


@pytest.mark.parametrize("B,prec", [(16384, "fp32"), (20480, "fp32"), (4096, "fp32"), (12288, "fp32"),
                                    (12288, "bf16"), (4096, "bf16")])
def test_in_kernel_index_bitwise_dense_sweep(B, prec):
    """12,288 samples: the unit kernel (fp32 below 16,384, bf16 at every size) needs 384 unit
    workgroups, so its grid is clamped to 256 and every workgroup runs two rounds while fill
    workgroups sit past the unit grid — the units' stride must be the unit grid's, not gridDim's
    (units [256, 256 + nfill) of each round were skipped)."""
    U, I = 3000, 2000
    shape = O.NCFShape(U, I, LAYERS, GMF)
    w = _weights(shape, 5)
    engines = {}
    for name, kw in (("dense", {}), ("lazy", dict(lazy_adam=True)), ("ahead", dict(lazy_adam=True))):
        e = NCFEngine(U, I, LAYERS, GMF, max_batch=B, precision=prec, **kw)
        e.set_keras_weights(w)
        engines[name] = e
    # 16,384 and up: the wave kernel's weight-gradient waves fill; below (and bf16): the unit kernel's
    # grid leaves CUs idle and spare workgroups of its launch fill
    assert engines["ahead"].kernel_for(B) == ("fused-mfma-wave" if B >= 16384 and prec == "fp32"
                                              else "fused-mfma-unit")
    batches = [_batch(U, I, B, 40 + s) for s in range(6)]
    for s, (u, it, y) in enumerate(batches):
        nxt = (batches[s + 1][0], batches[s + 1][1]) if s + 1 < len(batches) else None
        engines["dense"].train_step(u, it, y, group=GROUP, k=2)
        engines["lazy"].train_step(u, it, y, group=GROUP, k=2)
        engines["ahead"].train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
        if s == 2:
            engines["ahead"].predict(u, it)           # a read (flush) between counted steps
    for e in engines.values():
        e.check_errors()
        e.flush()
    torch.cuda.synchronize()
    d = engines["dense"]
    for name in ("lazy", "ahead"):
        e = engines[name]
        assert torch.equal(d.emb, e.emb), name
        assert torch.equal(d.emb_m, e.emb_m) and torch.equal(d.emb_v, e.emb_v), name
        assert torch.equal(d.mlp, e.mlp) and torch.equal(d.mlp_m, e.mlp_m), name
        assert NCFEngine.read_stats(d.stats) == NCFEngine.read_stats(e.stats), name
    assert torch.equal(engines["lazy"].row_step, engines["ahead"].row_step)


def test_in_kernel_index_matches_oracle():
    """Two counted-ahead steps of 16,384 samples with heavy rows against the float64 oracle
    (test_native_gpu.py's tolerances)."""
    U, I, B = 1500, 900, 16384
    shape = O.NCFShape(U, I, LAYERS, GMF)
    w = _weights(shape, 9)
    eng = NCFEngine(U, I, LAYERS, GMF, max_batch=B, lazy_adam=True)
    eng.set_keras_weights(w)
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    hyper = dict(optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=[0.0] * 4)
    batches = [_batch(U, I, B, 60 + s, mixed_frac=0.0) for s in range(3)]
    for s, (u, it, y) in enumerate(batches):
        nxt = (batches[s + 1][0], batches[s + 1][1]) if s + 1 < len(batches) else None
        probs = torch.empty(B, dtype=torch.float32, device="cuda")
        eng.train_step(u, it, y, group=GROUP, k=2, probs_out=probs, next_batch=nxt)
        _, p_ref = O.train_step(shape, ref, st, u.cpu().numpy(), it.cpu().numpy(), y.cpu().numpy(), hyper)
        assert float(np.max(np.abs(probs.cpu().numpy() - p_ref))) <= 2e-6, s
    got = eng.keras_weights()
    for name in O.weight_names(shape):
        tol = 3 * 2e-6 + 2e-6 * float(np.max(np.abs(ref[name])))
        err = float(np.max(np.abs(np.asarray(got[name], np.float64) - ref[name])))
        assert err <= tol, "%s: max err %g > %g" % (name, err, tol)


def test_in_kernel_index_flags_stale_and_range():
    """A counted batch whose ids change behind torch's back is flagged (RuntimeError), an id
    outside the table is flagged (ValueError); the counters are cleared, so later counted steps
    are sound (bitwise a fresh engine's from the same state)."""
    U, I, B = 3000, 2000, 16384
    shape = O.NCFShape(U, I, LAYERS, GMF)
    w = _weights(shape, 11)
    eng = NCFEngine(U, I, LAYERS, GMF, max_batch=B, lazy_adam=True)
    eng.set_keras_weights(w)
    bt = [_batch(U, I, B, 80 + s) for s in range(6)]
    stage = (bt[1][0].clone(), bt[1][1].clone())
    eng.train_step(*bt[0], group=GROUP, k=2, next_batch=stage)
    stage[1].data.copy_(bt[2][1])                      # behind torch's back
    eng.train_step(stage[0], stage[1], bt[1][2], group=GROUP, k=2)
    with pytest.raises(RuntimeError):
        eng.check_errors()
    bad = bt[3][1].clone()
    bad[123] = I + 5
    eng.train_step(*bt[2], group=GROUP, k=2, next_batch=(bt[3][0], bad))
    eng.train_step(bt[3][0], bad, bt[3][2], group=GROUP, k=2)
    with pytest.raises(ValueError):
        eng.check_errors()
    # from here both engines start from the same state: counted steps must agree bitwise
    eng.flush()
    twin = NCFEngine(U, I, LAYERS, GMF, max_batch=B, lazy_adam=True)
    twin.set_keras_weights(eng.keras_weights())
    m, v, t = eng.optimizer_state()
    twin.set_optimizer_state(m, v, t)
    eng.set_optimizer_state(m, v, t)                  # same pristine marks on both
    for s in (4, 5):
        nxt = (bt[5][0], bt[5][1]) if s == 4 else None
        eng.train_step(*bt[s], group=GROUP, k=2, next_batch=nxt)
        twin.train_step(*bt[s], group=GROUP, k=2)
    eng.check_errors()
    eng.flush()
    twin.flush()
    assert torch.equal(eng.emb, twin.emb) and torch.equal(eng.emb_m, twin.emb_m)
    assert torch.equal(eng.mlp, twin.mlp)
    assert torch.isfinite(eng.emb).all()
    assert N.NCF_ROW_PRISTINE > 0


def _short_count(users):
    """Ids changed so that fewer contributions are valid than were counted, with no counted row
    overflowing: the mixed groups' users set to their group head's, so those samples' user rows fold
    into the head's (no contribution of their own) while no key gains one — counted slots are left
    unfilled and nothing overflows (such a step was applied, not dropped)."""
    u = users.cpu().numpy().reshape(-1, GROUP).copy()
    mixed = (u != u[:, :1]).any(axis=1)
    assert mixed.any()
    u[mixed] = u[mixed, :1]
    return torch.from_numpy(u.reshape(-1)).cuda()


@pytest.mark.parametrize("B,mode", [(16384, "moved"), (1024, "moved"), (16384, "short"), (4096, "short"),
                                    (1024, "short")])
def test_stale_counted_step_is_dropped(B, mode):
    """A counted batch whose ids change behind torch's back (the in-kernel fill: the wave kernel's
    at 16,384 samples, the unit launch's fill workgroups at 4,096, the fill launch's at 1,024).
    "moved": a changed id reaches a row that was not counted (the forward pass may have read it at
    its deferred step): the step is dropped — nothing applied, bitwise the engine that never ran it.
    "short": the changes only leave counted rows with fewer contributions (mixed groups' users set to
    their head's: they now fold) — no row outside the counted set is read, so the step is applied
    exactly: the unfilled list slots are skipped, bitwise the engine that runs the same ids without
    counting ahead (those slots were summed as contributions).  Either way the error is
    raised.  The stale step counts the next batch ahead itself, and two counted steps run before any
    flush: the counted rows the previous step caught up ahead (P-ahead: p current, m and v owed) must
    be settled by a dropped launch, or a row absent from the next batch keeps its mark past the next
    bump."""
    U, I = 3000, 2000
    shape = O.NCFShape(U, I, LAYERS, GMF)
    w = _weights(shape, 13)
    bt = [_batch(U, I, B, 90 + s) for s in range(6)]
    short_users = _short_count(bt[1][0])
    engines = []
    for stale in (True, False):
        e = NCFEngine(U, I, LAYERS, GMF, max_batch=B, lazy_adam=True)
        e.set_keras_weights(w)
        e.train_step(*bt[0], group=GROUP, k=2)
        stage = (bt[1][0].clone(), bt[1][1].clone())
        e.train_step(*bt[0], group=GROUP, k=2, next_batch=stage)
        if stale:
            if mode == "moved":
                stage[1].data.copy_(bt[2][1])             # behind torch's back
            else:
                stage[0].data.copy_(short_users)
            e.train_step(stage[0], stage[1], bt[1][2], group=GROUP, k=2, next_batch=(bt[3][0], bt[3][1]))
            with pytest.raises(RuntimeError):
                e.check_errors()
        elif mode == "short":
            # the same ids, not counted ahead (the engine gives up its counted batch: flushed)
            e.train_step(short_users.clone(), bt[1][1].clone(), bt[1][2], group=GROUP, k=2,
                         next_batch=(bt[3][0], bt[3][1]))
        # two counted steps before any flush
        e.train_step(*bt[3], group=GROUP, k=2, next_batch=(bt[4][0], bt[4][1]))
        e.train_step(*bt[4], group=GROUP, k=2)
        e.check_errors()
        e.flush()
        engines.append(e)
    a, d = engines
    torch.cuda.synchronize()
    assert torch.equal(a.emb, d.emb) and torch.equal(a.emb_m, d.emb_m) and torch.equal(a.emb_v, d.emb_v)
    assert torch.equal(a.mlp, d.mlp) and torch.equal(a.mlp_m, d.mlp_m) and torch.equal(a.mlp_v, d.mlp_v)
    assert NCFEngine.read_stats(a.stats) == NCFEngine.read_stats(d.stats)
    assert int(a.step.item()) == int(d.step.item())
    # afterwards both train the same counted steps to the same bits
    for s in (5, 0):
        for e in engines:
            e.train_step(*bt[s], group=GROUP, k=2, next_batch=(bt[0][0], bt[0][1]) if s == 5 else None)
    for e in engines:
        e.check_errors()
        e.flush()
    assert torch.equal(a.emb, d.emb) and torch.equal(a.mlp, d.mlp)
