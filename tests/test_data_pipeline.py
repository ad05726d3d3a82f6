"""Data pipeline parity: the reference's own unit tests
(``test/test_data_pipeline.py``, ``test/test_movielens_utils.py``) restated
against this package, plus exact-replay golden vectors captured from the
reference pipeline (``tests/golden/make_golden.py``)."""

import os
from unittest.mock import PropertyMock, patch

import numpy as np
import pandas as pd
import pytest

from movierec import data_pipeline as dp
from movierec.data_pipeline import MovieLensDataGenerator, load_ratings_train_test_sets
from movierec.util import movielens_utils as ml
from movierec.util.movielens_utils import load_ratings_data

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---- reference unit tests, restated (test/test_data_pipeline.py:19-145) ----

def test_wrong_database_name_load():
    with pytest.raises(ValueError):
        load_ratings_train_test_sets("wrong db", "/tmp/")


@patch("movierec.data_pipeline.load_ratings_data")
def test_load_ratings_train_test_sets(mock_ml):
    mock_ml.return_value = pd.DataFrame({"userId": pd.Series([0, 0, 0, 0, 1, 1, 1]),
                                         "itemId": pd.Series([110, 122, 199, 332, 100, 221, 299]),
                                         "rating": pd.Series([5., 5., 4., 3., 2., 4., 5.])})
    train, validation, test = load_ratings_train_test_sets("ml-100k", "ml-100k", download=False)
    pd.testing.assert_frame_equal(train, pd.DataFrame({"userId": pd.Series([0, 0, 1]),
                                                       "itemId": pd.Series([110, 122, 100]),
                                                       "rating": pd.Series([5., 5., 2])}))
    pd.testing.assert_frame_equal(validation, pd.DataFrame({"userId": pd.Series([0, 1]),
                                                            "itemId": pd.Series([199, 221]),
                                                            "rating": pd.Series([4., 4.])}))
    pd.testing.assert_frame_equal(test, pd.DataFrame({"userId": pd.Series([0, 1]),
                                                      "itemId": pd.Series([332, 299]),
                                                      "rating": pd.Series([3., 5.])}))


@patch("movierec.data_pipeline.MovieLensDataGenerator.num_items", new_callable=PropertyMock)
def test_generator_get_item(mock_num_items):
    mock_num_items.return_value = 5
    data = pd.DataFrame({"userId": pd.Series([0, 2, 0, 1]), "itemId": pd.Series([0, 0, 2, 3])})
    extra = pd.DataFrame({"userId": pd.Series([0, 0, 1, 2, 2, 2]), "itemId": pd.Series([1, 4, 4, 1, 2, 4])})
    g = MovieLensDataGenerator("ml-100k", data, batch_size=6, negatives_per_positive=2,
                               extra_data_df=extra, shuffle=False)
    for _ in range(10):
        (xu, xi), y = g[0]
        np.testing.assert_equal(xu, np.array([0, 0, 0, 2, 2, 2]))
        np.testing.assert_equal(xi, np.array([3, 3, 0, 3, 3, 0]))
        np.testing.assert_equal(y, np.array([0, 0, 1, 0, 0, 1]))
    for _ in range(10):
        (xu, xi), y = g[1]
        np.testing.assert_equal(xu, np.array([0, 0, 0, 1, 1, 1]))
        np.testing.assert_equal(xi[:3], np.array([3, 3, 2]))
        assert len(np.setdiff1d(np.array([0, 1, 2]), xi[3:5])) == 1
        assert xi[5] == 3
        np.testing.assert_equal(y, np.array([0, 0, 1, 0, 0, 1]))


@patch("movierec.data_pipeline.MovieLensDataGenerator.num_items", new_callable=PropertyMock)
def test_generator_get_item_duplicated_user_batch(mock_num_items):
    mock_num_items.return_value = 6
    data = pd.DataFrame({"userId": pd.Series([0, 0, 0, 1]), "itemId": pd.Series([0, 1, 2, 3]),
                         "rating": pd.Series([5., 5., 4., 3.])})
    g = MovieLensDataGenerator("ml-100k", data, batch_size=6, negatives_per_positive=2,
                               extra_data_df=None, shuffle=False)
    differ_in_batch = differ_between_runs = False
    last = None
    for _ in range(50):
        (xu, xi), y = g[0]
        np.testing.assert_equal(xu, np.zeros(6, dtype=np.int64))
        assert len(np.setdiff1d(np.array([3, 4, 5]), xi[:2])) == 1
        assert len(np.setdiff1d(np.array([3, 4, 5]), xi[3:6])) == 1
        np.testing.assert_equal(y, np.array([0, 0, 1, 0, 0, 1]))
        differ_in_batch |= not np.array_equal(xi[:2], xi[3:6])
        differ_between_runs |= last is not None and not np.array_equal(last, xi[:2])
        last = xi[:2]
    assert differ_between_runs and differ_in_batch


def test_generator_value_errors():
    data = pd.DataFrame({"userId": pd.Series([0, 0, 0, 1]), "itemId": pd.Series([0, 1, 2, 3]),
                         "rating": pd.Series([5., 5., 4., 3.])})
    with pytest.raises(ValueError, match="Invalid dataset name"):
        MovieLensDataGenerator("wrong_name", data, batch_size=6, negatives_per_positive=2)
    with pytest.raises(ValueError, match="negatives_per_positive must be > 0"):
        MovieLensDataGenerator("ml-100k", data, batch_size=6, negatives_per_positive=0)
    with pytest.raises(ValueError, match="Batch size must be divisible by"):
        MovieLensDataGenerator("ml-100k", data, batch_size=10, negatives_per_positive=6)


# ---- test/test_movielens_utils.py:11-47, restated ----

@patch("movierec.util.movielens_utils.os.path.exists")
def test_file_not_found(mock_exists):
    mock_exists.return_value = False
    with pytest.raises(FileNotFoundError):
        load_ratings_data("MOCK TEST PATH", "ml-100k", download=False)


@patch("movierec.util.movielens_utils.download_movielens")
@patch("movierec.util.movielens_utils.pd.read_csv")
@patch("movierec.util.movielens_utils.os.path.exists")
def test_load_ratings_data_download(mock_exists, mock_read_csv, mock_download):
    mock_exists.side_effect = [False, True]
    mock_read_csv.return_value = pd.DataFrame({"userId": pd.Series([1, 1, 1, 2, 2, 2]),
                                               "itemId": pd.Series([100, 111, 200, 222, 300, 100]),
                                               "rating": pd.Series([4., 5., 5., 4., 3., 2.])})
    load_ratings_data("testPath", "ml-100k", download=True)
    mock_download.assert_called_with("ml-100k", "testPath")
    mock_read_csv.assert_called_once()


@patch("movierec.util.movielens_utils.pd.read_csv")
@patch("movierec.util.movielens_utils.os.path.exists")
def test_load_ratings_data(mock_exists, mock_read_csv):
    mock_exists.return_value = True
    mock_read_csv.return_value = pd.DataFrame({"userId": pd.Series([1, 1, 1, 1, 2, 2, 2]),
                                               "itemId": pd.Series([111, 123, 200, 333, 101, 222, 300]),
                                               "rating": pd.Series([5., 5., 4., 3., 2., 4., 5.])})
    ratings = load_ratings_data("test_data", "ml-100k")
    pd.testing.assert_frame_equal(ratings, pd.DataFrame({
        "userId": pd.Series([0, 0, 0, 0, 1, 1, 1]),
        "itemId": pd.Series([110, 122, 199, 332, 100, 221, 299]),
        "rating": pd.Series([5., 5., 4., 3., 2., 4., 5.])}))


# ---- golden replays captured from the reference pipeline ----

def _gold():
    return np.load(os.path.join(GOLD, "pipeline_golden.npz"))


def _split_from_gold(g):
    ratings = pd.DataFrame({"userId": g["split_in_user"], "itemId": g["split_in_item"],
                            "rating": g["split_in_rating"]})
    return ratings, dp.split_leave_two_out(ratings)


def test_split_matches_reference_golden():
    g = _gold()
    _, (train, val, test) = _split_from_gold(g)
    for nm, df in (("train", train), ("val", val), ("test", test)):
        for col in ("userId", "itemId", "rating"):
            ref = g["split_%s_%s" % (nm, col)]
            assert df[col].dtype == ref.dtype
            np.testing.assert_array_equal(df[col].values, ref)


# mirrors make_golden.GEN_CASES
GEN_CASES = [
    ("train_b10_n4_shuffle", "ml-100k", 10, 4, False, True, 7, 6),
    ("train_b100_n9_shuffle", "ml-100k", 100, 9, False, True, 11, 3),
    ("val_b200_n99_extra", "ml-100k", 200, 99, True, False, 13, 2),
    ("train_b6_n2_noshuffle", "ml-100k", 6, 2, False, False, 17, 5),
    ("train_b8_n3_extra_shuffle", "ml-100k", 8, 3, True, True, 19, 5),
]


@pytest.mark.parametrize("case", GEN_CASES, ids=[c[0] for c in GEN_CASES])
def test_generator_replays_reference_rng_stream(case):
    name, ds, bs, negs, use_extra, shuffle, seed, nb = case
    g = _gold()
    _, (train, val, test) = _split_from_gold(g)
    data = val if use_extra and negs == 99 else train
    extra = train if use_extra else None
    if use_extra and negs != 99:
        data, extra = val, test
    np.random.seed(seed)
    gen = MovieLensDataGenerator(ds, data, bs, negs, extra_data_df=extra, shuffle=shuffle)
    assert len(gen) == int(g[name + "/len"][0])          # F4 length quirk preserved
    np.testing.assert_array_equal(gen.indexes, g[name + "/indexes0"])
    for b in range(nb):
        if b == nb // 2:
            gen.on_epoch_end()
            np.testing.assert_array_equal(gen.indexes, g[name + "/indexes1"])
        (xu, xi), y = gen[b % max(1, len(gen))]
        np.testing.assert_array_equal(xu, g[name + "/x_user"][b])
        np.testing.assert_array_equal(xi, g[name + "/x_item"][b])
        np.testing.assert_array_equal(y, g[name + "/y"][b])
        assert [str(xu.dtype), str(xi.dtype), str(y.dtype)] == list(g[name + "/dtypes"])


def test_loader_matches_reference_golden():
    g = np.load(os.path.join(GOLD, "loader_golden.npz"))
    base = os.path.join(GOLD, "movielens_tiny")
    for ds in ("ml-100k", "ml-1m", "ml-20m"):
        df = load_ratings_data(base, ds, download=False)
        for col in ("userId", "itemId", "rating"):
            ref = g["%s/%s" % (ds, col)]
            assert df[col].dtype == ref.dtype
            np.testing.assert_array_equal(df[col].values, ref)


def test_fast_batch_excludes_positives():
    g = _gold()
    _, (train, val, test) = _split_from_gold(g)
    gen = MovieLensDataGenerator("ml-100k", train, 100, 9, shuffle=True)
    rng = np.random.default_rng(0)
    (xu, xi), y = gen.fast_batch(0, rng)
    assert xu.shape == xi.shape == y.shape == (100,)
    pos = set(zip(train["userId"].tolist(), train["itemId"].tolist()))
    for u, i, lab in zip(xu, xi, y):
        assert ((int(u), int(i)) in pos) == bool(lab)


def test_remap_item_ids_dense():
    df = pd.DataFrame({"userId": np.array([0, 0, 1], np.int32), "itemId": np.array([131261, 1, 28], np.int32)})
    out, raw = ml.remap_item_ids(df)
    np.testing.assert_array_equal(out["itemId"].values, np.array([2, 0, 1], np.int32))
    np.testing.assert_array_equal(raw, np.array([1, 28, 131261]))
