"""End to end through the reference's entry point (trainer.py:30-80): a MovieLens ratings
file on disk -> leave-two-out split -> host generators (reference RNG stream) ->
MovierecModel.fit_generator (validation, EarlyStopping / best checkpoints) -> save ->
MovierecModel.load_from_dir, on the HIP path.

The data is an ml-100k-format file (u.data, tab separated, 1-based ids) written here with
ml-100k's table sizes (943 users x 1682 items) and a learnable structure; no download.
"""

import glob
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _write_ml100k(data_dir, seed=0):
    rng = np.random.RandomState(seed)
    U, I = 943, 1682
    fu, fi = rng.normal(size=(U, 4)), rng.normal(size=(I, 4))
    rows = []
    ts = 0
    for u in range(U):
        pref = np.argsort(-(fi @ fu[u] + 0.3 * rng.normal(size=I)))[:8]   # each user's 8 favourites
        for it in pref:
            ts += 1
            rows.append("%d\t%d\t%d\t%d" % (u + 1, it + 1, rng.randint(1, 6), ts))
    os.makedirs(os.path.join(data_dir, "ml-100k"), exist_ok=True)
    with open(os.path.join(data_dir, "ml-100k", "u.data"), "w") as f:
        f.write("\n".join(rows) + "\n")


def test_trainer_end_to_end(tmp_path):
    import random
    from movierec import trainer
    from movierec.model import MovierecModel
    data_dir, out_dir = str(tmp_path / "data"), str(tmp_path / "models")
    _write_ml100k(data_dir)
    np.random.seed(0)
    random.seed(0)
    params = dict(trainer.DEFAULT_PARAMS)
    params.update(layers_sizes=[16, 8], layers_l2reg=[0, 0], batch_size=240, num_negs_per_pos=3,
                  batch_size_eval=200, num_negs_per_pos_eval=99, k=4, epochs=3, gmf_dim=8, seed=1)
    model, history = trainer.train("e2e", "ml-100k", data_dir, out_dir, params, verbose=0)

    h = history.history
    for key in ("loss", "output_hr", "output_dcg", "val_loss", "val_output_hr", "val_output_dcg"):
        assert len(h[key]) >= 1 and all(np.isfinite(h[key])), key
    assert h["loss"][-1] < h["loss"][0]                       # training lowers the loss
    assert os.path.exists(MovierecModel.get_model_weights_path(out_dir, "e2e"))
    assert os.path.exists(MovierecModel.get_params_json_path(out_dir, "e2e"))
    assert glob.glob(os.path.join(out_dir, "e2e-checkpoint-*"))  # best-only checkpoints

    # the saved model reloads to the same predictions
    users = np.arange(20, dtype=np.int32).repeat(5)
    items = np.tile(np.arange(5, dtype=np.int32), 20)
    p0, _ = model.model.predict_on_batch([users, items])
    loaded = MovierecModel.load_from_dir(out_dir, "e2e", verbose=0)
    p1, _ = loaded.model.predict_on_batch([users, items])
    np.testing.assert_array_equal(p0, p1)
    assert gpu_available()


def test_trainer_ml20m_format(tmp_path):
    """trainer.train(..., "ml-20m") on ml-20m-format files whose raw movieIds reach 131262
    (csv with headers, movies.csv in movieId order): the split remaps the items to dense ids
     and training runs to completion over the full 138,493 x 27,278 tables."""
    import random
    from movierec import trainer
    from movierec.model import MovierecModel
    from test_data_pipeline import _write_ml20m
    data_dir, out_dir = str(tmp_path / "data"), str(tmp_path / "models")
    _write_ml20m(data_dir, n_users=300, per_user=12, seed=3)
    np.random.seed(1)
    random.seed(1)
    params = dict(trainer.DEFAULT_PARAMS)
    params.update(batch_size=400, num_negs_per_pos=3, batch_size_eval=200, num_negs_per_pos_eval=99, k=4,
                  epochs=2, gmf_dim=8, seed=2)
    model, history = trainer.train("ml20m", "ml-20m", data_dir, out_dir, params, verbose=0)
    assert params["num_users"] == 138493 and params["num_items"] == 27278
    h = history.history
    assert len(h["loss"]) == 2 and all(np.isfinite(h["loss"])) and all(np.isfinite(h["val_output_hr"]))
    assert os.path.exists(MovierecModel.get_model_weights_path(out_dir, "ml20m"))
    assert gpu_available()


def test_trainer_gmf_only_config_a(tmp_path):
    """BASELINE config A through the reference entry point: ml-100k, GMF-only model
    (layers_sizes == [], gmf_dim 8), batch 256 with 3 negatives per positive."""
    import random
    from movierec import trainer
    from movierec.model import MovierecModel
    data_dir, out_dir = str(tmp_path / "data"), str(tmp_path / "models")
    _write_ml100k(data_dir, seed=4)
    np.random.seed(2)
    random.seed(2)
    params = dict(trainer.DEFAULT_PARAMS)
    params.update(layers_sizes=[], layers_l2reg=[], batch_size=256, num_negs_per_pos=3, batch_size_eval=200,
                  num_negs_per_pos_eval=99, k=4, epochs=3, gmf_dim=8, seed=5, lr=0.01)
    model, history = trainer.train("gmf", "ml-100k", data_dir, out_dir, params, verbose=0)
    h = history.history
    assert h["loss"][-1] < h["loss"][0]
    assert sorted(model.model.get_weights()) == ["item_gmf_embedding", "output/bias", "output/kernel",
                                                 "user_gmf_embedding"]
    loaded = MovierecModel.load_from_dir(out_dir, "gmf", verbose=0)
    users = np.arange(2, dtype=np.int32).repeat(100)     # two evaluation groups of 100
    items = np.tile(np.arange(100, dtype=np.int32), 2)
    np.testing.assert_array_equal(model.model.predict_on_batch([users, items])[0],
                                  loaded.model.predict_on_batch([users, items])[0])
    assert gpu_available()
