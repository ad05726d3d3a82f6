"""bf16 MLP mode (include/movierec_ncf.h ``mlp_bf16``; BASELINE config B "bf16"): the MLP tower's
matrix products take bf16 operands (RNE) with fp32 accumulation; embeddings, GMF, the output
layer, loss, master weights and Adam stay fp32.

1. One step's gradients against the oracle with the same operand rounding (oracle ``mm_round =
   bf16_round`` on both operands of every hidden-layer product, forward and backward).  Tolerance
   2e-3 max|g|: the device rounds fp32 values and the oracle fp64 ones, so an operand within
   ~1e-7 of a bf16 rounding midpoint may land one bf16 ulp (2^-8) apart.  The fp32 oracle is
   further away (checked), so the bf16 path is really the one that ran.
2. Training on an ml-1m-shaped synthetic catalogue (6040 users x 3706 items, config B: NeuMF gmf 8
   + MLP [64,32,16,8], 4 negatives, batch 4095, Adam): HR@10 / NDCG@10 of the bf16 path within
   +-0.002 of the fp32 path, and the fp32 path within +-0.002 of the oracle trained on
   the same batches (the north star's bar at ml-1m's shape).  Evaluation: every user's held-out
   positive + 99 sampled negatives, k = 10, fp32 forward of the trained master weights (ncf_predict),
   the metric of the device probabilities computed by the oracle's RankLayer restatement.
"""

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec.engine import NCFEngine


@pytest.mark.parametrize("dims", [(120, 90, [64, 32, 16, 8], 8), (200, 150, [128, 64, 32, 16], 64)],
                         ids=["configB", "configC"])
def test_bf16_grads_match_rounded_oracle(dims):
    from test_native_gpu import _weights
    shape = O.NCFShape(*dims)
    w = _weights(shape, 61)
    rng = np.random.RandomState(62)
    B, group = 1000, 5
    users = rng.randint(0, shape.num_users, B // group).repeat(group).astype(np.int32)
    items = rng.randint(0, shape.num_items, B).astype(np.int32)
    y = np.tile([0.0] * (group - 1) + [1.0], B // group).astype(np.float32)
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, precision="bf16")
    eng.set_keras_weights(w)
    grads = eng.alloc_grads()
    probs = torch.empty(B, dtype=torch.float32, device="cuda")
    eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads, probs_out=probs)
    got = eng.keras_weights(grads[0], grads[1])
    _, gb, pb = O.loss_and_grads(shape, w, users, items, y, [0.0] * 4, mm_round=O.bf16_round)
    _, g32, _ = O.loss_and_grads(shape, w, users, items, y, [0.0] * 4)
    far = 0
    for name in O.weight_names(shape):
        scale = np.max(np.abs(gb[name])) + 1e-12
        err = np.max(np.abs(got[name] - gb[name]))
        assert err <= 2e-3 * scale + 1e-9, (name, err / scale)
        far += np.max(np.abs(got[name] - g32[name])) > 1e-5 * (np.max(np.abs(g32[name])) + 1e-12)
    assert far > 0, "bf16 gradients indistinguishable from fp32: the bf16 path did not run"
    assert np.max(np.abs(probs.cpu().numpy() - pb)) <= 1e-4


U, I, LAYERS, GMF = 6040, 3706, [64, 32, 16, 8], 8
NEGS, GROUP, BATCH, EPOCHS = 4, 5, 4095, 2
EVAL_CHUNK = 200000   # evaluation samples per predict call (2000 users x 100)


def _dataset(seed=0):
    rng = np.random.RandomState(seed)
    fu, fi = rng.normal(size=(U, 8)), rng.normal(size=(I, 8))
    aff = fu @ fi.T + 0.5 * rng.normal(size=(U, I))
    top = np.argsort(-aff, axis=1)[:, :16]   # each user's 16 favourite items; [0] is held out
    return top[:, 1:], top[:, 0], rng


def _negatives(rng, pos, k):
    """k items per row outside that row's positives (rejection sampling, vectorised)."""
    n = pos.shape[0]
    out = rng.randint(0, I, (n, k))
    for _ in range(50):
        bad = (out[:, :, None] == pos[:, None, :]).any(axis=2)
        if not bad.any():
            break
        out[bad] = rng.randint(0, I, int(bad.sum()))
    return out


def _batches(train, top, rng):
    pu = np.repeat(np.arange(U), train.shape[1])
    pi = train.reshape(-1)
    per = BATCH // GROUP
    out = []
    for _ in range(EPOCHS):
        order = rng.permutation(len(pu))
        for b in range(len(order) // per):
            sel = order[b * per:(b + 1) * per]
            u = pu[sel]
            negs = _negatives(rng, top[u], NEGS)
            items = np.concatenate([negs, pi[sel][:, None]], axis=1).reshape(-1)
            users = np.repeat(u, GROUP)
            y = np.tile([0.0] * NEGS + [1.0], per).astype(np.float32)
            out.append((users.astype(np.int32), items.astype(np.int32), y))
    return out


def _eval_set(held, top, rng):
    negs = _negatives(rng, top, 99)
    items = np.concatenate([negs, held[:, None]], axis=1).reshape(-1)
    users = np.repeat(np.arange(U), 100)
    y = np.tile([0.0] * 99 + [1.0], U).astype(np.float32)
    return users.astype(np.int32), items.astype(np.int32), y


def test_bf16_and_fp32_hr_at_ml1m_shape():
    from movierec.model import initial_weights
    train, held, rng = _dataset()
    top = np.concatenate([held[:, None], train], axis=1)
    batches = _batches(train, top, rng)
    eu, ei, ey = _eval_set(held, top, rng)
    w0 = initial_weights(U, I, LAYERS, GMF, seed=5)
    hyper = dict(optimizer="adam", lr=0.002, beta_1=0.9, beta_2=0.999, layers_l2reg=[0.0] * 4)

    res = {}
    for prec in ("fp32", "bf16"):
        eng = NCFEngine(U, I, LAYERS, GMF, max_batch=EVAL_CHUNK, lr=hyper["lr"], precision=prec)
        eng.set_keras_weights(w0)
        dev = [tuple(torch.from_numpy(x).cuda() for x in b) for b in batches]
        for u, it, yy in dev:
            eng.train_step(u, it, yy, group=GROUP, k=10)
        probs = []
        for c in range(0, len(eu), EVAL_CHUNK):
            probs.append(eng.predict(eu[c:c + EVAL_CHUNK], ei[c:c + EVAL_CHUNK]).cpu().numpy())
        res[prec] = O.group_metrics(np.concatenate(probs).astype(np.float64), ey, 100, 10)

    shape = O.NCFShape(U, I, LAYERS, GMF)
    w = {k: v.astype(np.float64) for k, v in w0.items()}
    opt = O.new_opt_state(w)
    for u, it, yy in batches:
        O.train_step(shape, w, opt, u, it, yy, hyper)
    p, _ = O.forward(shape, w, eu, ei)
    res["oracle"] = O.group_metrics(p, ey, 100, 10)

    print("HR/NDCG@10", {k: tuple(round(float(x), 4) for x in v) for k, v in res.items()})
    assert res["fp32"][0] > 0.3, "training must lift HR@10 well above a random ranking (0.10)"
    for a, b in (("bf16", "fp32"), ("fp32", "oracle")):
        assert abs(res[a][0] - res[b][0]) <= 0.002, (a, b, res)
        assert abs(res[a][1] - res[b][1]) <= 0.002, (a, b, res)
