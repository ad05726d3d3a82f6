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


def _write_ml20m(base, n_users=60, per_user=8, seed=0):
    """ml-20m-format files (csv with headers; raw movieIds sparse up to 131262, 1-based)."""
    rng = np.random.RandomState(seed)
    movie_ids = np.unique(np.concatenate([rng.choice(np.arange(1, 131263), 300, replace=False), [131262, 1]]))
    d = os.path.join(base, "ml-20m")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "movies.csv"), "w", encoding="utf-8") as f:
        f.write("movieId,title,genres\n")
        for m in movie_ids:
            f.write('%d,Movie %d (1999),Drama\n' % (m, m))
    rows = ["userId,movieId,rating,timestamp"]
    ts = 0
    for u in range(1, n_users + 1):
        for m in rng.choice(movie_ids, per_user, replace=False):
            ts += 1
            rows.append("%d,%d,%.1f,%d" % (u, m, rng.randint(1, 11) / 2.0, ts))
    with open(os.path.join(d, "ratings.csv"), "w") as f:
        f.write("\n".join(rows) + "\n")
    return movie_ids


def test_ml20m_split_has_dense_item_ids(tmp_path):
    """load_ratings_train_test_sets remaps ml-20m's raw movieIds (up to 131262) to dense ids in
    movies.csv order, so every id fits NUM_ITEMS['ml-20m'] = 27278."""
    from movierec.data_pipeline import load_ratings_train_test_sets
    movie_ids = _write_ml20m(str(tmp_path))
    raw = load_ratings_data(str(tmp_path), "ml-20m", download=False)
    assert raw["itemId"].max() == 131261 or raw["itemId"].max() > 27278
    train, val, test = load_ratings_train_test_sets("ml-20m", str(tmp_path), download=False)
    lut = {int(m) - 1: i for i, m in enumerate(movie_ids)}       # 0-based raw -> position in movies.csv
    both = pd.concat([train, val, test])
    assert both["itemId"].max() < ml.NUM_ITEMS["ml-20m"]
    # the split itself is unchanged: same rows, items renamed through the movies order
    tr0, va0, te0 = __import__("movierec.data_pipeline", fromlist=["x"]).split_leave_two_out(raw)
    for a, b in ((train, tr0), (val, va0), (test, te0)):
        np.testing.assert_array_equal(a["userId"].values, b["userId"].values)
        np.testing.assert_array_equal(a["itemId"].values, [lut[int(x)] for x in b["itemId"].values])
    # remap_items=False keeps the reference's raw ids
    tr, _, _ = load_ratings_train_test_sets("ml-20m", str(tmp_path), download=False, remap_items=False)
    np.testing.assert_array_equal(tr["itemId"].values, tr0["itemId"].values)
    # the dense -> raw table travels with the frames (invert the mapping: ids back to movieIds)
    for f in (train, val, test):
        np.testing.assert_array_equal(f.attrs["raw_item_ids"], movie_ids - 1)
    np.testing.assert_array_equal(train.attrs["raw_item_ids"][train["itemId"].values], tr0["itemId"].values)


def test_ml20m_remap_needs_the_movies_file(tmp_path):
    """One numbering only: without ml-20m's movies.csv the default remap refuses instead of
    silently numbering by the rated ids; remap_items='ratings' asks for that numbering."""
    from movierec.data_pipeline import load_ratings_train_test_sets
    _write_ml20m(str(tmp_path))
    os.remove(os.path.join(str(tmp_path), "ml-20m", "movies.csv"))
    with pytest.raises(FileNotFoundError):
        load_ratings_train_test_sets("ml-20m", str(tmp_path), download=False)
    train, val, test = load_ratings_train_test_sets("ml-20m", str(tmp_path), download=False, remap_items="ratings")
    raw = train.attrs["raw_item_ids"]
    assert np.all(np.diff(raw) > 0)
    both = pd.concat([train, val, test])
    assert set(raw[both["itemId"].values].tolist()) == set(raw.tolist())


def test_remap_rejects_unknown_movie():
    df = pd.DataFrame({"userId": np.array([0], np.int32), "itemId": np.array([5], np.int32)})
    movies = pd.DataFrame({"itemId": np.array([1, 2], np.int32)})
    with pytest.raises(ValueError):
        ml.remap_item_ids(df, movies_df=movies)


def test_movie_titles_decoded_latin1(tmp_path):
    """ml-100k u.item and ml-1m movies.dat are latin-1 files; their titles decode (the
    reference's load_movies_data, movielens_utils.py:85-101, reads them as utf-8 and fails)."""
    d = tmp_path / "ml-1m"
    d.mkdir()
    (d / "movies.dat").write_bytes("1::Misérables, Les (1995)::Drama\n2::Señorita (2001)::Comedy\n".encode("latin-1"))
    m = ml.load_movies_data(str(tmp_path), "ml-1m", download=False)
    assert list(m["itemId"]) == [0, 1]
    assert m["movieTitle"][0] == "Misérables, Les (1995)" and m["movieTitle"][1] == "Señorita (2001)"
    d = tmp_path / "ml-100k"
    d.mkdir()
    (d / "u.item").write_bytes("1|Très Bien (1996)|01-Jan-1996||http://x|0|1\n".encode("latin-1"))
    m = ml.load_movies_data(str(tmp_path), "ml-100k", download=False)
    assert m["movieTitle"][0] == "Très Bien (1996)"


def test_eval_batch_per_rank_whole_groups():
    """trainer.eval_batch_per_rank: the global validation batch split over the ranks in whole
    (negs + 1)-groups, at least one group per rank (the reference defaults: 200 with 99 negatives)."""
    from movierec.trainer import eval_batch_per_rank, _per_rank
    assert eval_batch_per_rank(200, 99, 1) == 200
    assert eval_batch_per_rank(200, 99, 2) == 100
    assert eval_batch_per_rank(200, 99, 4) == 100
    assert eval_batch_per_rank(200, 99, 8) == 100
    assert eval_batch_per_rank(1000, 99, 4) == 200
    assert eval_batch_per_rank(400, 3, 3) == 132
    assert _per_rank(120, 9, 4, "batch_size") == 30
    with pytest.raises(ValueError):
        _per_rank(100, 9, 4, "batch_size")
