"""MovierecModel surface, mirroring the reference's own model tests (test/test_model.py:8-166).

The parameter checks run before any device work, so they are CPU tests; the built model's
structure and output shapes need the HIP engine (-m gpu).
"""

import os
import tempfile

import numpy as np
import pytest

from conftest import gpu_available

# the reference's TEST_PARAMS (test/test_model.py:8-26)
TEST_PARAMS = {
    "num_users": 5, "num_items": 10, "layers_sizes": [6, 4], "layers_l2reg": [0.01, 0.01],
    "optimizer": "adam", "lr": 0.001, "beta_1": 0.9, "beta_2": 0.999,
    "batch_size": 8, "num_negs_per_pos": 3, "batch_size_eval": 10, "num_negs_per_pos_eval": 4, "k": 4,
}


def _model(params, **kw):
    from movierec.model import MovierecModel
    return MovierecModel(params, output_dir=os.path.join(tempfile.gettempdir(), "movierec_test_models"), **kw)


def _params(**changes):
    p = {k: (list(v) if isinstance(v, list) else v) for k, v in TEST_PARAMS.items()}
    p.update(changes)
    return p


def test_wrong_layers():
    """test_model.py:31-35: layers_sizes and layers_l2reg of different lengths -> ValueError."""
    p = _params()
    p["layers_sizes"].append(2)
    with pytest.raises(ValueError):
        _model(p)


def test_missing_param():
    """test_model.py:37-40: a missing key -> KeyError."""
    p = _params()
    del p["num_users"]
    with pytest.raises(KeyError):
        _model(p)


def test_not_implemented_optimizer():
    """test_model.py:57-60: unknown optimizer -> NotImplementedError."""
    with pytest.raises(NotImplementedError):
        _model(_params(optimizer="other"))


@pytest.mark.parametrize("changes", [
    dict(num_negs_per_pos=0),                    # model.py:91-92
    dict(batch_size=9),                          # model.py:94-96 (9 % 4 != 0)
    dict(num_negs_per_pos_eval=0),               # model.py:100-101
    dict(batch_size_eval=12),                    # model.py:103-106 (12 % 5 != 0)
    dict(k=5),                                   # model.py:108-112 (k > negs + 1)
])
def test_invalid_batch_and_k_params(changes):
    with pytest.raises(ValueError):
        _model(_params(**changes))


@pytest.mark.gpu
def test_build_mlp_model():
    """test_model.py:42-55: inputs, layers, outputs and weights of the built model."""
    model = _model(_params(), verbose=0).model
    assert model.input_shape == [(None, 1), (None, 1)]
    assert len(model.inputs) == 2
    assert len(model.layers) == 10   # 2 inputs, 2 embeddings, 2 flatten, 1 concat, 1 hidden, 2 outputs
    assert len(model.outputs) == 2
    assert model.output_shape == [(None, 1), (None, None)]
    assert model.trainable
    assert len(model.trainable_weights) == 6
    assert len(model.trainable_variables) == 6
    assert len(model.non_trainable_weights) == 0
    assert len(model.non_trainable_variables) == 0
    assert gpu_available()


@pytest.mark.gpu
def test_outputs():
    """test_model.py:151-166: predict_on_batch -> [probabilities (10, 1), rank (2, 5)] in the
    evaluation learning phase (groups of num_negs_per_pos_eval + 1)."""
    x_users = np.array([1, 1, 1, 1, 1, 2, 2, 2, 2, 2])
    x_items = np.array([1, 2, 3, 4, 5, 1, 2, 3, 4, 5])
    model = _model(_params(), verbose=0)
    model.log_summary()
    output, rank = model.model.predict_on_batch([x_users, x_items])
    assert output.shape == (10, 1)
    assert rank.shape == (2, 5)
    assert np.all((output > 0) & (output < 1))
    for g in range(2):   # rank = descending order of the group's probabilities (ties: lower index)
        expect = np.argsort(-output[5 * g:5 * g + 5, 0], kind="stable")
        np.testing.assert_array_equal(rank[g], expect)
