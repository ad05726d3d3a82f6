"""MovieLens dataset constants and file readers.

Host-side mirror of ``movierec/util/movielens_utils.py`` in the reference
(constants ``:13-55``, path helpers ``:58-82``, ``load_movies_data`` ``:85-101``,
``load_ratings_data`` ``:104-125``, ``download_movielens`` ``:128-170``).
Same names, argument meaning and errors, so callers (and the reference's own
tests, which patch ``os.path.exists`` / ``pd.read_csv`` / ``download_movielens``
in this module) work unchanged.

Additions (documented in DESIGN.md): ``remap_item_ids`` — dense 0-based item
ids for ml-20m, whose raw movieIds are non-contiguous, applied by
``data_pipeline.load_ratings_train_test_sets``; movie titles are decoded with each
file's own encoding (``MOVIES_ENCODING``: the ml-100k ``u.item`` and ml-1m
``movies.dat`` files are latin-1, ml-20m's ``movies.csv`` is utf-8), which the
reference's ``load_movies_data`` (``:85-101``) leaves to pandas' utf-8 default.
"""

import logging
import os
import tempfile
import zipfile
from urllib.request import urlretrieve

import numpy as np
import pandas as pd

MOVIELENS_URL_FORMAT = "http://files.grouplens.org/datasets/movielens/{}.zip"
ZIP_EXTENSION = ".zip"

ML_100K = "ml-100k"
ML_1M = "ml-1m"
ML_20M = "ml-20m"
MOVIELENS_DATASET_NAMES = [ML_100K, ML_1M, ML_20M]

# per-dataset file layout: (ratings file, movies file, separator regex, header?)
_LAYOUT = {
    ML_100K: ("u.data", "u.item", "\t|\\|", False),
    ML_1M: ("ratings.dat", "movies.dat", "::", False),
    ML_20M: ("ratings.csv", "movies.csv", ",", True),
}
RATINGS_FILE_NAME = {name: spec[0] for name, spec in _LAYOUT.items()}
MOVIES_FILE_NAME = {name: spec[1] for name, spec in _LAYOUT.items()}
SEPARATOR = {name: spec[2] for name, spec in _LAYOUT.items()}
HAS_HEADER = {name: spec[3] for name, spec in _LAYOUT.items()}

# Table sizes come from these constants, not from the data (reference
# data_pipeline.py:60-61, trainer.py:72-73).
NUM_USERS = {ML_100K: 943, ML_1M: 6040, ML_20M: 138493}
NUM_ITEMS = {ML_100K: 1682, ML_1M: 3952, ML_20M: 27278}

# text encoding of each dataset's movies file (titles such as "Misérables" in latin-1)
MOVIES_ENCODING = {ML_100K: "latin-1", ML_1M: "latin-1", ML_20M: "utf-8"}


def get_path(data_dir, dataset_name, file_name):
    return os.path.join(data_dir, dataset_name, file_name)


def get_movies_path(data_dir, dataset_name):
    return get_path(data_dir, dataset_name, MOVIES_FILE_NAME[dataset_name])


def get_ratings_path(data_dir, dataset_name):
    return get_path(data_dir, dataset_name, RATINGS_FILE_NAME[dataset_name])


def _resolve_or_fetch(data_dir, dataset_name, file_name, download=True):
    """Return the file path; if it is missing either raise FileNotFoundError
    (download=False) or call ``download_movielens`` once and re-check."""
    path = get_path(data_dir, dataset_name, file_name)
    if os.path.exists(path):
        return path
    if not download:
        raise FileNotFoundError(
            "{} not found. Download the dataset first or set param download=True.".format(path))
    download_movielens(dataset_name, data_dir)
    if not os.path.exists(path):
        raise FileNotFoundError(
            'Unexpected error: {} not found after calling "download_movielens". '.format(path))
    return path


def _read_table(path, dataset_name, names, dtypes, usecols, encoding=None):
    kwargs = dict(filepath_or_buffer=path, sep=SEPARATOR[dataset_name],
                  header=0 if HAS_HEADER[dataset_name] else None,
                  engine="python",  # regex separators
                  usecols=usecols, names=names, dtype=dtypes)
    if encoding is not None:
        kwargs["encoding"] = encoding
    return pd.read_csv(**kwargs)


def load_movies_data(data_dir, dataset_name, col_item_id="itemId", col_movie_title="movieTitle",
                     download=True):
    path = _resolve_or_fetch(data_dir, dataset_name, MOVIES_FILE_NAME[dataset_name], download)
    movies = _read_table(path, dataset_name, (col_item_id, col_movie_title),
                         {col_item_id: np.int32}, (0, 1), encoding=MOVIES_ENCODING[dataset_name])
    movies[col_item_id] = movies[col_item_id] - 1  # 1-based → 0-based
    return movies


def load_ratings_data(data_dir, dataset_name, col_user_id="userId", col_item_id="itemId",
                      col_rating="rating", download=True):
    path = _resolve_or_fetch(data_dir, dataset_name, RATINGS_FILE_NAME[dataset_name], download)
    ratings = _read_table(path, dataset_name, (col_user_id, col_item_id, col_rating),
                          {col_user_id: np.int32, col_item_id: np.int32, col_rating: np.float32},
                          (0, 1, 2), encoding="utf-8")
    # users and items are 1-indexed in the files
    ratings[col_user_id] = ratings[col_user_id] - 1
    ratings[col_item_id] = ratings[col_item_id] - 1
    return ratings


def remap_item_ids(ratings_df, col_item_id="itemId", movies_df=None):
    """Dense 0-based item ids (new).  ml-20m movieIds reach ~131k
    while NUM_ITEMS['ml-20m'] is 27278, so the reference cannot gather them.
    Ids are mapped in the order of ``movies_df`` when given (27278 movies for
    ml-20m), else in ascending raw-id order.  Returns (new_df, raw_ids):
    ``raw_ids[dense] = raw``.  A rating of a movie absent from ``movies_df``
    raises ValueError."""
    raw = (np.asarray(movies_df[col_item_id]) if movies_df is not None
           else np.unique(np.asarray(ratings_df[col_item_id])))
    ids = np.asarray(ratings_df[col_item_id])
    order = np.argsort(raw, kind="stable")
    pos = np.searchsorted(raw[order], ids)
    pos = np.minimum(pos, max(len(raw) - 1, 0))
    dense = order[pos] if len(raw) else pos
    if ids.size and (len(raw) == 0 or not np.array_equal(raw[dense], ids)):
        bad = ids[raw[dense] != ids] if len(raw) else ids
        raise ValueError("item id {} not in the movies list".format(int(bad[0])))
    out = ratings_df.copy()
    out[col_item_id] = dense.astype(ratings_df[col_item_id].dtype)
    return out, raw


def download_movielens(dataset_name, output_dir):
    """Download and extract one MovieLens zip into ``output_dir`` (same contract
    as the reference).  Needs network access; never called by the tests."""
    if dataset_name not in MOVIELENS_DATASET_NAMES:
        raise ValueError("Invalid dataset name {}. Must be one of {}".format(
            dataset_name, ", ".join(MOVIELENS_DATASET_NAMES)))
    with tempfile.TemporaryDirectory() as tmp:
        url = MOVIELENS_URL_FORMAT.format(dataset_name)
        zip_path = os.path.join(tmp, dataset_name + ZIP_EXTENSION)
        logging.info("Downloading Movielens {}".format(url))
        urlretrieve(url, zip_path)
        if not os.path.isdir(output_dir):
            os.makedirs(output_dir)
        with zipfile.ZipFile(zip_path, "r") as zf:
            zf.extractall(output_dir)
        dataset_dir = os.path.join(output_dir, dataset_name)
        logging.info("Dataset extracted to {}".format(dataset_dir))
    return dataset_dir
