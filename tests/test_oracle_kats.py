"""Pin the CPU oracle: the reference's known-answer tests for ranking/metrics
(``test/test_model.py:69-190``) and a finite-difference check of the
restated loss gradients (loss/grad semantics are parity-unpinned by reference
fixtures)."""

import math

import numpy as np
import pytest

from oracle import ncf_oracle as O


def _dcg_index(i):
    return math.log(2) / math.log(i + 2)


def test_hit_rate_kat():
    y_true = np.array([[0, 0, 0, 1], [0, 0, 0, 1]])
    rank = np.array([[2, 3, 1, 0], [0, 1, 2, 3]], dtype=np.int32)
    for k, exp in {0: 0.0, 1: 0.0, 2: 0.5, 3: 0.5, 4: 1.0}.items():
        assert O.hit_rate(y_true, k, rank) == pytest.approx(exp)


def test_dcg_kat():
    y_true = np.array([[0, 0, 0, 1], [0, 0, 0, 1]])
    y_pred = np.array([[0.1, 0.2, 0.9, 0.5], [0.9, 0.8, 0.7, 0.6]], dtype=np.float32)
    rank = O.rank_layer(y_pred, 4)
    d0, d1 = _dcg_index(1), _dcg_index(3)
    for k, exp in {0: 0.0, 1: 0.0, 2: d0 / 2, 3: d0 / 2, 4: (d0 + d1) / 2}.items():
        assert O.discounted_cumulative_gain(y_true, k, rank) == pytest.approx(exp, rel=1e-6)


def test_ties_rank_positive_last():
    y_true = np.array([[0, 0, 0, 1]])
    y_pred = np.array([[0.9, 0.55, 0.55, 0.55]], dtype=np.float32)
    rank = O.rank_layer(y_pred, 4)
    for k in (0, 1, 2, 3):
        assert O.hit_rate(y_true, k, rank) == 0.0
        assert O.discounted_cumulative_gain(y_true, k, rank) == 0.0
    assert O.hit_rate(y_true, 4, rank) == pytest.approx(1.0)
    assert O.discounted_cumulative_gain(y_true, 4, rank) == pytest.approx(_dcg_index(3), rel=1e-6)


def test_rank_layer_kat():
    np.testing.assert_equal(O.rank_layer(np.array([0.9, 0.8, 0.7, 0.7, 0.8, 0.9]), 3),
                            np.array([[0, 1, 2], [2, 1, 0]]))
    np.testing.assert_equal(O.rank_layer(np.array([0.9, 0.8, 0.7, 0.6, 0.5, 0.9, 0.9, 0.9]), 4),
                            np.array([[0, 1, 2, 3], [1, 2, 3, 0]]))


@pytest.mark.parametrize("layers,gmf", [([6, 4], 0), ([8, 6, 4], 4), ([5, 3], 2), ([], 8)])
def test_gradients_finite_difference(layers, gmf):
    shape = O.NCFShape(7, 9, layers, gmf)
    w = O.init_weights(shape, seed=1)
    # larger weights so activations are not all tiny
    for k in w:
        w[k] = w[k] * 3.0 + (0.05 if k.endswith("bias") else 0.0)
    rng = np.random.RandomState(0)
    users = rng.randint(0, 7, 12)
    items = rng.randint(0, 9, 12)
    y = rng.randint(0, 2, 12)
    l2 = [0.01] * len(layers)
    loss, g, _ = O.loss_and_grads(shape, w, users, items, y, l2)
    for name in O.weight_names(shape):
        a = w[name]
        flat = a.reshape(-1)
        for idx in rng.choice(flat.size, min(6, flat.size), replace=False):
            old = flat[idx]
            flat[idx] = old + 1e-6
            lp, _, _ = O.loss_and_grads(shape, w, users, items, y, l2)
            flat[idx] = old - 1e-6
            lm, _, _ = O.loss_and_grads(shape, w, users, items, y, l2)
            flat[idx] = old
            fd = (lp - lm) / 2e-6
            assert g[name].reshape(-1)[idx] == pytest.approx(fd, rel=1e-4, abs=1e-8), name


def test_adam_matches_closed_form_first_step():
    w = {"a": np.array([1.0, -2.0])}
    g = {"a": np.array([0.5, -0.25])}
    m = {"a": np.zeros(2)}
    v = {"a": np.zeros(2)}
    O.adam_update(w, g, m, v, 1, 0.001)
    # first step: m/(sqrt(v)) = sign(g) (up to eps); lr_t = lr*sqrt(1-b2)/(1-b1)
    lr_t = 0.001 * math.sqrt(1 - 0.999) / (1 - 0.9)
    exp = np.array([1.0, -2.0]) - lr_t * (0.1 * np.array([0.5, -0.25])) / (
        np.sqrt(0.001 * np.array([0.25, 0.0625])) + 1e-7)
    np.testing.assert_allclose(w["a"], exp, rtol=1e-12)


def test_top_k_items_order_and_ties():
    s = np.array([[0.1, 0.9, 0.5, 0.9, 0.2], [3.0, 3.0, 3.0, 1.0, 4.0]])
    items, vals = O.top_k_items(s, 3)
    np.testing.assert_array_equal(items, [[1, 3, 2], [4, 0, 1]])
    np.testing.assert_allclose(vals, [[0.9, 0.9, 0.5], [4.0, 3.0, 3.0]])


def test_score_all_items_matches_forward():
    shape = O.NCFShape(6, 9, [8, 6, 4], 4)
    w = O.init_weights(shape, seed=2)
    z = O.score_all_items(shape, w, [0, 5])
    _, c = O.forward(shape, w, [5] * 9, np.arange(9))
    np.testing.assert_allclose(z[1], c["z"])


def test_philox_known_answers():
    """Philox4x32-10 known-answer vectors (Random123 kat_vectors, first output word)."""
    assert O.philox_u32(0, 0, 0, 0, 0, 0) == 0x6627e8d5
    m = 0xFFFFFFFF
    assert O.philox_u32(m, m, m, m, m, m) == 0x408f276d
    assert O.philox_u32(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0) == 0xd16cfe09


def test_sampler_restatement_invariants():
    excluded = {0: np.array([1, 2, 3]), 1: np.arange(0, 18)}   # user 1: 2 candidates < 4 negatives
    order = np.array([1, 0, 2])
    xu, xi, y = O.sample_batch(np.array([0, 0, 1]), np.array([1, 2, 5]), excluded, 20, order, 0, 3, 4, 9, 5)
    xi = xi.reshape(3, 5)
    assert list(xi[:, -1]) == [2, 1, 5]
    assert len(set(xi[0, :4])) == 4 and not set(xi[0, :4]) & {1, 2, 3}
    assert set(xi[2, :4]) <= {18, 19}
    np.testing.assert_array_equal(y, np.tile([0, 0, 0, 0, 1], 3))
