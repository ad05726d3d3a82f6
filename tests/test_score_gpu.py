"""All-item scoring + top-k (BASELINE config E) vs the CPU oracle, through the C ABI.

Checks, per user row (z = the oracle's float64 logit of every item):
  * position-wise optimality: the r-th returned item's oracle logit is within
    ``tol_z`` of the r-th best oracle logit (an approximate top-k is correct to
    within the scorer's own error);
  * scores: the returned sigmoid outputs match sigmoid(z) of the returned items;
  * exact lists wherever the oracle's top-(k+1) logits are separated by more than
    the scorer's error.

Tolerances: fp32 path |dz| <= 1e-5 (fp32 forward, ranked by probability);
fp16 MFMA path |dz| <= 5e-3 (fp16 operands — 11-bit mantissa — fp32 accumulation;
logits of the test models stay within |z| < 8).
"""

import numpy as np
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec.engine import NCFEngine

TOL_Z = {"fp32": 1e-5, "fp16": 5e-3}


def _weights(shape, seed):
    w = O.init_weights(shape, seed=seed)
    rng = np.random.RandomState(seed + 7)
    for k in w:
        if k.endswith("embedding"):
            w[k] = rng.uniform(-0.5, 0.5, size=w[k].shape)
        elif k.endswith("bias"):
            w[k] = rng.uniform(-0.1, 0.1, size=w[k].shape)
        else:
            w[k] = w[k] * 3.0
    users = rng.randint(0, shape.num_users, 64)
    z = O.score_all_items(shape, w, users)
    f = 5.0 / max(np.max(np.abs(z)), 1e-6)   # keep |z| <~ 5: sigmoid well resolved in fp32
    w["output/kernel"] = w["output/kernel"] * f
    w["output/bias"] = w["output/bias"] * f
    return {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}


def _engine(shape, w):
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=1024)
    eng.set_keras_weights(w)
    return eng


def _check(items, scores, z, k, tol_z, exact_gap=None):
    items = np.asarray(items)
    scores = np.asarray(scores, dtype=np.float64)
    ref_items, ref_z = O.top_k_items(z, k)
    kk = min(k, z.shape[1])
    assert np.all(items[:, :kk] >= 0) and np.all(items[:, :kk] < z.shape[1])
    got_z = np.take_along_axis(z, items[:, :kk].astype(np.int64), axis=1)
    assert np.max(ref_z[:, :kk] - got_z) <= 2 * tol_z, "returned items are not a top-k"
    for row in items:
        assert len(set(row[:kk].tolist())) == kk, "duplicate items in a top-k list"
    p_ref = 1.0 / (1.0 + np.exp(-got_z))
    assert np.max(np.abs(scores[:, :kk] - p_ref)) <= tol_z, "scores"
    if kk < k:
        assert np.all(items[:, kk:] == -1) and np.all(scores[:, kk:] == 0)
    if exact_gap is not None:
        # position r is determined when the oracle's r-th best logit is separated from both
        # neighbours by more than the scorer's error: there the returned item must be exact
        m = min(kk + 1, z.shape[1])
        srt = -np.sort(-z, axis=1)[:, :m]
        up = np.full((len(z), kk), np.inf)
        dn = np.full((len(z), kk), np.inf)
        up[:, 1:] = srt[:, :kk - 1] - srt[:, 1:kk]
        if m > kk:
            dn[:, :] = srt[:, :kk] - srt[:, 1:kk + 1]
        else:
            dn[:, :kk - 1] = srt[:, :kk - 1] - srt[:, 1:kk]
        det = (up > exact_gap) & (dn > exact_gap)
        np.testing.assert_array_equal(items[:, :kk][det], ref_items[:, :kk][det])
        return float(det.mean())
    return 0


SHAPES = [
    # (num_users, num_items, layers, gmf_dim)
    (200, 999, [128, 64, 32, 16], 64),   # ml-20m NeuMF (configs C / E), partial last 32-item tile
    (150, 640, [128, 64, 32, 16], 0),    # its MLP-only form
    (100, 333, [64, 32, 16, 8], 8),      # ml-1m NeuMF (config B)
    (90, 257, [64, 32, 16, 8], 0),       # the trainer default model (trainer.py:8-27)
    (70, 5000, [128, 64, 32, 16], 64),   # 157 item tiles: 3 item ranges per user block + merge
]


@pytest.mark.parametrize("dims", SHAPES, ids=[str(s[2]) + "g" + str(s[3]) for s in SHAPES])
@pytest.mark.parametrize("precision", ["fp16", "fp32"])
def test_score_topk_matches_oracle(dims, precision):
    shape = O.NCFShape(*dims)
    w = _weights(shape, 3)
    eng = _engine(shape, w)
    rng = np.random.RandomState(5)
    users = rng.randint(0, shape.num_users, 77).astype(np.int32)  # not a multiple of 32, duplicates
    users[:3] = [0, shape.num_users - 1, 0]
    k = 10
    items, scores = eng.score_topk(users, k=k, precision=precision)
    z = O.score_all_items(shape, w, users)
    tol = TOL_Z[precision]
    covered = _check(items.cpu().numpy(), scores.cpu().numpy(), z, k, tol, exact_gap=2 * tol)
    assert covered >= 0.5   # the exact-position check covered most positions


@pytest.mark.parametrize("precision", ["fp16", "fp32"])
def test_score_topk_full_ml20m_catalogue(precision):
    """BASELINE config E at its real size: the ml-20m NeuMF model (config C's) over the full
    138,493 x 27,278 tables; 77 users (not a multiple of 32, with duplicates, the first and the
    last user) scored against every one of the 27,278 items (853 item tiles: every item range of
    a user block and the merge), top-10 compared with the oracle's full catalogue scores."""
    shape = O.NCFShape(138493, 27278, [128, 64, 32, 16], 64)
    w = _weights(shape, 11)
    eng = _engine(shape, w)
    rng = np.random.RandomState(12)
    users = rng.randint(0, shape.num_users, 77).astype(np.int32)
    users[:4] = [0, shape.num_users - 1, 0, users[10]]
    items, scores = eng.score_topk(users, k=10, precision=precision)
    z = O.score_all_items(shape, w, users)
    tol = TOL_Z[precision]
    covered = _check(items.cpu().numpy(), scores.cpu().numpy(), z, 10, tol, exact_gap=2 * tol)
    assert covered >= 0.5
    # duplicate users get identical lists
    it = items.cpu().numpy()
    np.testing.assert_array_equal(it[0], it[2])
    np.testing.assert_array_equal(it[3], it[10])


@pytest.mark.parametrize("k", [1, 5, 32])
def test_score_topk_k_values(k):
    shape = O.NCFShape(120, 300, [128, 64, 32, 16], 64)
    w = _weights(shape, 4)
    eng = _engine(shape, w)
    users = np.arange(0, 120, 3, dtype=np.int32)
    z = O.score_all_items(shape, w, users)
    for precision in ("fp16", "fp32"):
        items, scores = eng.score_topk(users, k=k, precision=precision)
        _check(items.cpu().numpy(), scores.cpu().numpy(), z, k, TOL_Z[precision])


def test_score_topk_catalogue_smaller_than_k():
    shape = O.NCFShape(40, 6, [64, 32, 16, 8], 8)
    w = _weights(shape, 5)
    eng = _engine(shape, w)
    users = np.arange(40, dtype=np.int32)
    z = O.score_all_items(shape, w, users)
    for precision in ("fp16", "fp32"):
        items, scores = eng.score_topk(users, k=10, precision=precision)
        _check(items.cpu().numpy(), scores.cpu().numpy(), z, 10, TOL_Z[precision])


def test_score_topk_fp32_any_shape_and_unsupported_fp16():
    shape = O.NCFShape(31, 17, [7, 5], 3)   # odd widths, 2 layers: fp32 scorer only
    w = _weights(shape, 6)
    eng = _engine(shape, w)
    users = np.arange(31, dtype=np.int32)
    items, scores = eng.score_topk(users, k=4, precision="fp32")
    _check(items.cpu().numpy(), scores.cpu().numpy(), O.score_all_items(shape, w, users), 4, 1e-5, exact_gap=2e-5)
    with pytest.raises(ValueError):
        eng.score_topk(users, k=4, precision="fp16")
    with pytest.raises(ValueError):
        eng.score_topk(users, k=33, precision="fp32")


def test_score_topk_ties_prefer_lower_item():
    """Identical item rows score identically: the lower item id ranks first."""
    shape = O.NCFShape(32, 64, [64, 32, 16, 8], 8)
    w = _weights(shape, 8)
    for name in ("item_embedding", "item_gmf_embedding"):
        w[name][:] = w[name][5]   # every item identical
    eng = _engine(shape, w)
    users = np.arange(32, dtype=np.int32)
    for precision in ("fp16", "fp32"):
        items, _ = eng.score_topk(users, k=10, precision=precision)
        np.testing.assert_array_equal(items.cpu().numpy(), np.tile(np.arange(10), (32, 1)))


def test_model_recommend_api():
    from movierec.model import MovierecModel
    params = dict(num_users=50, num_items=120, layers_sizes=[64, 32, 16, 8], layers_l2reg=[0, 0, 0, 0],
                  optimizer="adam", lr=0.001, batch_size=100, num_negs_per_pos=9, batch_size_eval=200,
                  num_negs_per_pos_eval=99, k=5, seed=1, gmf_dim=8)
    import tempfile
    m = MovierecModel(params, "t", tempfile.mkdtemp(), verbose=0)
    items, scores = m.recommend([0, 7, 49], k=10)
    assert items.shape == (3, 10) and scores.shape == (3, 10)
    assert np.all(np.diff(scores, axis=1) <= 1e-3)
    with pytest.raises(ValueError):
        m.recommend([50])
