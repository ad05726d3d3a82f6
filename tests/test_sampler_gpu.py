"""On-device negative sampler (ncf_sample_batch) vs its numpy restatement (bit-exact) and
the reference generator's invariants (data_pipeline.py:99-150, pinned by
test/test_data_pipeline.py:42-133: batch layout, negatives never positives of data or extra,
no replacement when enough candidates)."""

import numpy as np
import pandas as pd
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from movierec.sampler import DeviceMovieLensDataGenerator, excluded_csr

U, I = 943, 1682   # ml-100k constants (movielens_utils.py NUM_USERS / NUM_ITEMS)


def _frame(seed, n=3000, dense_user=None):
    rng = np.random.RandomState(seed)
    u = rng.randint(0, 60, n)
    i = rng.randint(0, I, n)
    if dense_user is not None:   # a user who rated all but 3 items: fewer candidates than negatives
        keep = np.setdiff1d(np.arange(I), [7, 500, 1600])
        u = np.concatenate([u, np.full(len(keep), dense_user)])
        i = np.concatenate([i, keep])
    return pd.DataFrame({"userId": u, "itemId": i, "rating": np.ones(len(u))})


def _excluded_dict(gen):
    ptr, items = excluded_csr(gen.num_users, [gen.data, gen.extra_data])
    return {u: items[ptr[u]:ptr[u + 1]] for u in range(gen.num_users) if ptr[u + 1] > ptr[u]}


@pytest.mark.parametrize("negs", [4, 9])
def test_device_batches_match_restatement(negs):
    data = _frame(1, n=800, dense_user=59)
    extra = _frame(2, n=200)
    gen = DeviceMovieLensDataGenerator("ml-100k", data, (negs + 1) * 40, negs, extra_data_df=extra, seed=1234)
    ex = _excluded_dict(gen)
    order = gen._order.cpu().numpy()   # the epoch's positive order (a device permutation)
    for idx in (0, 3, len(gen) - 1):
        (xu, xi), y = gen[idx]
        ru, ri, ry = O.sample_batch(gen._users, gen._items, ex, I, order, idx * 40, 40, negs, 1234,
                                    (gen.epoch << 32) | idx)
        np.testing.assert_array_equal(xu.cpu().numpy(), ru)
        np.testing.assert_array_equal(xi.cpu().numpy(), ri)
        np.testing.assert_array_equal(y.cpu().numpy(), ry)
    gen.check_errors()


def test_device_batches_invariants():
    data = _frame(3, n=5000, dense_user=59)
    extra = _frame(4, n=1000)
    negs = 9
    gen = DeviceMovieLensDataGenerator("ml-100k", data, 10 * 100, negs, extra_data_df=extra, seed=7)
    ex = _excluded_dict(gen)
    assert len(gen) == len(data) // 1000   # data_pipeline.py:97 quirk kept
    order = gen._order.cpu().numpy()
    assert np.array_equal(np.sort(order), np.arange(len(data)))   # a permutation of the positives
    for idx in range(len(gen)):
        (xu, xi), y = gen[idx]
        xu, xi, y = xu.cpu().numpy().reshape(-1, negs + 1), xi.cpu().numpy().reshape(-1, negs + 1), y.cpu().numpy()
        np.testing.assert_array_equal(y, np.tile([0] * negs + [1], 100))
        assert (xu == xu[:, :1]).all()
        pos = order[idx * 100:(idx + 1) * 100]
        np.testing.assert_array_equal(xi[:, -1], gen._items[pos])
        for row_u, row_i in zip(xu[:, 0], xi):
            negatives = row_i[:-1]
            exc = ex.get(row_u, np.zeros(0, int))
            cand = I - len(exc)
            assert not np.isin(negatives, exc).any()
            assert ((negatives >= 0) & (negatives < I)).all()
            if cand >= negs:
                assert len(set(negatives.tolist())) == negs
            else:
                assert set(negatives.tolist()) <= {7, 500, 1600}
    gen.check_errors()


def test_device_batches_reproducible_and_epoch_dependent():
    data = _frame(5)
    a = DeviceMovieLensDataGenerator("ml-100k", data, 500, 4, seed=11, shuffle=False)
    b = DeviceMovieLensDataGenerator("ml-100k", data, 500, 4, seed=11, shuffle=False)
    (_, xa), _ = a[2]
    (_, xb), _ = b[2]
    assert torch.equal(xa, xb)
    a.on_epoch_end()
    (_, xc), _ = a[2]
    assert not torch.equal(xa, xc)


def test_device_negatives_uniform():
    """One user with 10 excluded items: 20000 draws spread uniformly over the other 1672
    (chi-square, p > 1e-4)."""
    rng = np.random.RandomState(0)
    excl = np.sort(rng.choice(I, 10, replace=False))
    data = pd.DataFrame({"userId": np.zeros(5000, int), "itemId": np.resize(excl, 5000), "rating": 1.0})
    gen = DeviceMovieLensDataGenerator("ml-100k", data, 5 * 1000, 4, seed=3, shuffle=False)
    draws = np.concatenate([gen[i][0][1].cpu().numpy().reshape(-1, 5)[:, :4].ravel() for i in range(len(gen))])
    counts = np.bincount(draws, minlength=I)
    assert counts[excl].sum() == 0
    cand = np.setdiff1d(np.arange(I), excl)
    from scipy.stats import chisquare
    assert chisquare(counts[cand]).pvalue > 1e-4


def test_fit_generator_with_device_batches():
    from movierec.model import MovierecModel
    import tempfile
    data = _frame(6, n=4000)
    val = _frame(7, n=60)
    params = dict(num_users=U, num_items=I, layers_sizes=[64, 32, 16, 8], layers_l2reg=[0, 0, 0, 0],
                  optimizer="adam", lr=0.001, batch_size=500, num_negs_per_pos=4, batch_size_eval=100,
                  num_negs_per_pos_eval=99, k=5, seed=1, gmf_dim=8)
    m = MovierecModel(params, "t", tempfile.mkdtemp(), verbose=0)
    tr = DeviceMovieLensDataGenerator("ml-100k", data, 500, 4, seed=1)
    va = DeviceMovieLensDataGenerator("ml-100k", val, 100, 99, extra_data_df=data, shuffle=False, seed=2)
    hist = m.fit_generator(tr, va, epochs=3)
    assert len(hist.history["loss"]) >= 1
    assert hist.history["loss"][-1] < hist.history["loss"][0]
