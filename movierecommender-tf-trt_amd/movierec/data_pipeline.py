"""MovieLens split and negative-sampling batch generator (host side).

Mirror of the reference ``movierec/data_pipeline.py``:

* ``MovieLensDataGenerator`` (``:17-154``): batches of ``(n+1)``-groups
  ``[neg_1 .. neg_n, pos]`` per positive (``:141-148``); negatives drawn per
  positive from the items the user has in neither ``data`` nor ``extra``
  (``:99-113``), without replacement when possible, with the SAME numpy
  legacy-RNG calls in the SAME order as the reference (``np.random.shuffle``
  at ``:154``, one ``np.random.choice(possible_negs, n, replace)`` per
  positive at ``:112``), so a seeded run yields identical batches
  (pinned by ``tests/golden``).  ``__len__`` keeps the reference's quirk
  ``floor(len(data) / batch_size)`` (``:97``).
* ``load_ratings_train_test_sets`` (``:157-200``): leave-last-two-out per user
  in file order; outputs grouped by user (ascending), indexes reset.

The per-positive cost is what differs: the reference filters the whole
DataFrame for every positive (``:103-105``, O(N) each); this mirror builds a
per-user CSR of positives once and caches each user's candidate array, so a
batch costs O(batch * num_items) only inside ``np.random.choice`` itself.

``fast_batch`` (new) draws negatives with a vectorised rejection sampler —
same distribution family (uniform over the user's non-positives), NOT the
reference's RNG stream; used for throughput runs.  Documented in DESIGN.md.
"""

import logging
import os

import numpy as np

from .util import movielens_utils as ml
from .util.movielens_utils import load_ratings_data

COL_USER_ID = "userId"
COL_ITEM_ID = "itemId"
COL_RATING = "rating"
COL_LABEL = "label"


class Sequence(object):
    """Minimal stand-in for ``keras.utils.Sequence`` (the reference's base,
    ``data_pipeline.py:6``): ``__len__``, ``__getitem__``, ``on_epoch_end``."""

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


def _check_dataset_name(dataset_name):
    if dataset_name not in ml.MOVIELENS_DATASET_NAMES:
        raise ValueError("Invalid dataset name {}. Must be one of {}".format(
            dataset_name, ", ".join(ml.MOVIELENS_DATASET_NAMES)))


class MovieLensDataGenerator(Sequence):

    def __init__(self, dataset_name, data_df, batch_size, negatives_per_positive, extra_data_df=None,
                 shuffle=True):
        _check_dataset_name(dataset_name)
        if negatives_per_positive <= 0:
            raise ValueError("negatives_per_positive must be > 0, found {}".format(negatives_per_positive))
        if batch_size % (negatives_per_positive + 1):
            raise ValueError("Batch size must be divisible by (negatives_per_positive + 1). Found: batch_size={}, "
                             "negatives_per_positive={}".format(batch_size, negatives_per_positive))

        self._dataset_name = dataset_name
        self._num_users = ml.NUM_USERS[dataset_name]
        self._num_items = ml.NUM_ITEMS[dataset_name]
        self.data = data_df
        self.extra_data = extra_data_df
        self.batch_size = batch_size
        self.negatives_per_positive = negatives_per_positive
        self.num_positives_per_batch = batch_size // (negatives_per_positive + 1)
        self.num_negatives_per_batch = batch_size - self.num_positives_per_batch
        self.shuffle = shuffle
        self.indexes = np.arange(len(self.data))

        # column views used by every batch
        self._users = self.data[COL_USER_ID].values
        self._items = self.data[COL_ITEM_ID].values
        self._csr = None          # lazily built (num_items may be patched by tests)
        self._cand_cache = {}

        self.on_epoch_end()
        logging.info("Created generator for {}. Num users={}, num items={}, num_batches={}, batch size={}, "
                     "positives per batch={}, negatives per batch={}".format(
                         dataset_name, self._num_users, self._num_items, len(self), batch_size,
                         self.num_positives_per_batch, self.num_negatives_per_batch))

    @property
    def num_users(self):
        return self._num_users

    @property
    def num_items(self):
        return self._num_items

    @property
    def dataset_name(self):
        return self._dataset_name

    def __len__(self):
        # reference data_pipeline.py:97 — positives / batch_size (F4 quirk kept)
        return int(np.floor(len(self.indexes) / self.batch_size))

    # -- positives per user ------------------------------------------------
    def _build_csr(self):
        frames = [(self._users, self._items)]
        if self.extra_data is not None:
            frames.append((self.extra_data[COL_USER_ID].values, self.extra_data[COL_ITEM_ID].values))
        u = np.concatenate([np.asarray(f[0], dtype=np.int64) for f in frames])
        it = np.concatenate([np.asarray(f[1], dtype=np.int64) for f in frames])
        order = np.argsort(u, kind="stable")
        u, it = u[order], it[order]
        keys, starts = np.unique(u, return_index=True)
        ends = np.append(starts[1:], len(u))
        self._csr = (keys, starts, ends, it)

    def _positives_of(self, user):
        if self._csr is None:
            self._build_csr()
        keys, starts, ends, it = self._csr
        j = np.searchsorted(keys, user)
        if j < len(keys) and keys[j] == user:
            return it[starts[j]:ends[j]]
        return it[:0]

    def candidate_negatives(self, user):
        """Items the user has in neither data nor extra, ascending (the array the
        reference builds with np.setdiff1d at data_pipeline.py:108)."""
        user = int(user)
        cand = self._cand_cache.get(user)
        if cand is None:
            n_items = self.num_items
            taken = np.zeros(n_items, dtype=bool)
            pos = self._positives_of(user)
            pos = pos[(pos >= 0) & (pos < n_items)]
            taken[pos] = True
            cand = np.arange(n_items)[~taken]
            self._cand_cache[user] = cand
        return cand

    # -- batches ------------------------------------------------------------
    def __getitem__(self, idx):
        n = self.negatives_per_positive
        P = self.num_positives_per_batch
        idxs_pos = self.indexes[idx * P:(idx + 1) * P]
        pos_users = self._users[idxs_pos]
        pos_items = self._items[idxs_pos]
        x_user = np.repeat(pos_users, 1 + n)
        x_item = np.empty(len(idxs_pos) * (n + 1), dtype=np.int64)
        for j in range(len(idxs_pos)):
            cand = self.candidate_negatives(pos_users[j])
            replace = len(cand) < n
            x_item[j * (n + 1):j * (n + 1) + n] = np.random.choice(cand, n, replace=replace)
            x_item[j * (n + 1) + n] = int(pos_items[j])
        y = np.tile([0] * n + [1], P)
        return [x_user, x_item], y

    def fast_batch(self, idx, rng):
        """Vectorised negatives (rejection sampling, ``rng`` = np.random.Generator).
        Not the reference RNG stream; uniform over the user's non-positives."""
        n = self.negatives_per_positive
        P = self.num_positives_per_batch
        idxs_pos = self.indexes[idx * P:(idx + 1) * P]
        pos_users = np.asarray(self._users[idxs_pos], dtype=np.int64)
        pos_items = np.asarray(self._items[idxs_pos], dtype=np.int64)
        if self._csr is None:
            self._build_csr()
        negs = rng.integers(0, self.num_items, size=(len(idxs_pos), n))
        bad = self._is_positive(np.repeat(pos_users, n).reshape(-1, n), negs)
        while bad.any():
            negs[bad] = rng.integers(0, self.num_items, size=int(bad.sum()))
            bad = self._is_positive(np.repeat(pos_users, n).reshape(-1, n), negs)
        x_item = np.concatenate([negs, pos_items[:, None]], axis=1).reshape(-1)
        x_user = np.repeat(pos_users, n + 1)
        y = np.tile([0] * n + [1], len(idxs_pos))
        return [x_user, x_item], y

    def _is_positive(self, users, items):
        key = users * np.int64(self.num_items) + items
        if not hasattr(self, "_pos_keys"):
            keys, starts, ends, it = self._csr
            rep = np.repeat(keys, ends - starts)
            self._pos_keys = np.unique(rep * np.int64(self.num_items) + it)
        j = np.searchsorted(self._pos_keys, key)
        j = np.minimum(j, len(self._pos_keys) - 1)
        return self._pos_keys[j] == key

    def on_epoch_end(self):
        if self.shuffle:
            np.random.shuffle(self.indexes)


def split_leave_two_out(ratings_df):
    """Per user, in file order: test = last row, validation = second-last,
    train = the rest (reference data_pipeline.py:190-198).  Outputs are
    grouped by ascending user id with fresh indexes."""
    users = np.asarray(ratings_df[COL_USER_ID])
    order = np.argsort(users, kind="stable")  # group by user, keep file order inside
    su = users[order]
    if len(su) == 0:
        empty = ratings_df.iloc[[]].reset_index(drop=True)
        return empty, empty.copy(), empty.copy()
    last_of_user = np.append(su[1:] != su[:-1], True)
    first_of_user = np.append(True, su[1:] != su[:-1])
    counts = np.diff(np.append(np.flatnonzero(first_of_user), len(su)))
    if (counts < 2).any():
        # the reference's x.iloc[[-2]] raises on a single-rating user
        raise IndexError("positional indexers are out-of-bounds")
    test_pos = order[last_of_user]
    val_pos = order[np.flatnonzero(last_of_user) - 1]
    keep = np.ones(len(su), dtype=bool)
    keep[last_of_user] = False
    keep[np.flatnonzero(last_of_user) - 1] = False
    train_pos = order[keep]
    take = lambda pos: ratings_df.iloc[pos].reset_index(drop=True)
    return take(train_pos), take(val_pos), take(test_pos)


def load_ratings_train_test_sets(dataset_name, data_dir, download=True, remap_items=None):
    """Reference ``data_pipeline.py:157-200``.  ``remap_items`` (new, default: ml-20m only) gives
    the items dense ids before the split (DESIGN deviation 5).  One deterministic
    mapping: the item's position in the dataset's movies file (ml-20m's ``movies.csv``: 27,278
    movies, ascending movieId), which ships in every MovieLens zip; a missing movies file raises
    FileNotFoundError rather than falling back to another numbering.  ``remap_items="ratings"``
    asks for ascending rated ids instead (files without a movies list).  Without a remap ml-20m's
    raw movieIds (up to 131,262) fall outside the 27,278-row item table.  The raw (0-based) id of
    every dense id is kept in ``df.attrs["raw_item_ids"]`` of the three frames, so predictions can
    be mapped back to movieIds and titles (``trainer.train`` saves it next to the model)."""
    _check_dataset_name(dataset_name)
    ratings_df = load_ratings_data(data_dir, dataset_name, COL_USER_ID, COL_ITEM_ID, COL_RATING, download)
    if remap_items is None:
        remap_items = dataset_name == ml.ML_20M
    raw = None
    if remap_items:
        movies_df = None
        if remap_items != "ratings":
            path = ml.get_movies_path(data_dir, dataset_name)
            if not os.path.exists(path):
                raise FileNotFoundError("{} is needed to number {}'s items (or pass remap_items='ratings')"
                                        .format(path, dataset_name))
            movies_df = ml.load_movies_data(data_dir, dataset_name, COL_ITEM_ID, download=False)
        ratings_df, raw = ml.remap_item_ids(ratings_df, COL_ITEM_ID, movies_df)
    frames = split_leave_two_out(ratings_df)
    if raw is not None:
        for f in frames:
            f.attrs["raw_item_ids"] = np.asarray(raw)
    return frames
