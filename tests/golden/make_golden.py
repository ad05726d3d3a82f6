"""Generate golden vectors from the REFERENCE data pipeline (run in the build
container only; ``/root/reference`` does not exist on the GPU box).

The reference's ``movierec/data_pipeline.py`` and ``util/movielens_utils.py``
import with a stub for ``tensorflow.python.keras.utils.Sequence`` (the only TF
symbol they touch) and one pandas-2 shim (``Series.append`` was removed; the
reference uses it at data_pipeline.py:105).  Outputs are plain data
(``.npz`` of int/float arrays, tiny text inputs) — no reference source is
copied.  Usage::

    python tests/golden/make_golden.py   # rewrites tests/golden/*.npz
"""

import os
import sys
import types

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/movierec"


def import_reference():
    tf = types.ModuleType("tensorflow")
    tfp = types.ModuleType("tensorflow.python")
    tfk = types.ModuleType("tensorflow.python.keras")
    tfu = types.ModuleType("tensorflow.python.keras.utils")

    class Sequence(object):
        pass

    tfu.Sequence = Sequence
    for name, mod in (("tensorflow", tf), ("tensorflow.python", tfp),
                      ("tensorflow.python.keras", tfk), ("tensorflow.python.keras.utils", tfu)):
        sys.modules.setdefault(name, mod)
    if not hasattr(pd.Series, "append"):
        pd.Series.append = lambda s, o: pd.concat([s, o])
    sys.path.insert(0, REF)
    import data_pipeline as ref_dp  # noqa: E402
    import util.movielens_utils as ref_ml  # noqa: E402
    return ref_dp, ref_ml


def synthetic_ratings(n_users, n_items, per_user_min, per_user_max, seed):
    """Ratings frame in shuffled file order, with per-user duplicates avoided."""
    rng = np.random.RandomState(seed)
    rows = []
    for u in range(n_users):
        k = rng.randint(per_user_min, per_user_max + 1)
        items = rng.choice(n_items, k, replace=False)
        for it in items:
            rows.append((u, it, float(rng.randint(1, 6))))
    rng.shuffle(rows)
    arr = np.array(rows)
    return pd.DataFrame({"userId": arr[:, 0].astype(np.int32), "itemId": arr[:, 1].astype(np.int32),
                         "rating": arr[:, 2].astype(np.float32)})


# generator scenarios: (name, dataset, batch, negs, use_extra, shuffle, seed, n_batches)
GEN_CASES = [
    ("train_b10_n4_shuffle", "ml-100k", 10, 4, False, True, 7, 6),
    ("train_b100_n9_shuffle", "ml-100k", 100, 9, False, True, 11, 3),
    ("val_b200_n99_extra", "ml-100k", 200, 99, True, False, 13, 2),
    ("train_b6_n2_noshuffle", "ml-100k", 6, 2, False, False, 17, 5),
    ("train_b8_n3_extra_shuffle", "ml-100k", 8, 3, True, True, 19, 5),
]


def make_pipeline_goldens(ref_dp):
    out = {}
    ratings = synthetic_ratings(60, 1682, 3, 40, seed=3)
    out["split_in_user"] = ratings["userId"].values
    out["split_in_item"] = ratings["itemId"].values
    out["split_in_rating"] = ratings["rating"].values
    ref_dp.load_ratings_data = lambda *a, **k: ratings.copy()
    train, val, test = ref_dp.load_ratings_train_test_sets("ml-100k", "unused", download=False)
    for nm, df in (("train", train), ("val", val), ("test", test)):
        for col in ("userId", "itemId", "rating"):
            out["split_%s_%s" % (nm, col)] = df[col].values
    for (name, ds, bs, negs, use_extra, shuffle, seed, nb) in GEN_CASES:
        np.random.seed(seed)
        data = val if use_extra and negs == 99 else train
        extra = train if use_extra else None
        if use_extra and negs != 99:
            data, extra = val, test
        g = ref_dp.MovieLensDataGenerator(ds, data, bs, negs, extra_data_df=extra, shuffle=shuffle)
        out[name + "/len"] = np.array([len(g)])
        out[name + "/indexes0"] = g.indexes.copy()
        users, items, ys = [], [], []
        for b in range(nb):
            if b == nb // 2:
                g.on_epoch_end()
                out[name + "/indexes1"] = g.indexes.copy()
            (xu, xi), y = g[b % max(1, len(g))]
            users.append(xu)
            items.append(xi)
            ys.append(y)
        out[name + "/x_user"] = np.stack(users)
        out[name + "/x_item"] = np.stack(items)
        out[name + "/y"] = np.stack(ys)
        out[name + "/dtypes"] = np.array([str(users[0].dtype), str(items[0].dtype), str(ys[0].dtype)])
    np.savez_compressed(os.path.join(HERE, "pipeline_golden.npz"), **out)
    return out


def make_loader_goldens(ref_ml):
    """Tiny ratings files in the three on-disk formats, loaded by the reference."""
    base = os.path.join(HERE, "movielens_tiny")
    contents = {
        "ml-100k": ("u.data", "1\t10\t5\t881250949\n1\t20\t3\t881250950\n2\t10\t4\t881250951\n"
                              "3\t7\t1\t881250952\n2\t1682\t2\t881250953\n"),
        "ml-1m": ("ratings.dat", "1::1193::5::978300760\n1::661::3::978302109\n2::3952::4::978300275\n"
                                 "6040::1::2::978824291\n"),
        "ml-20m": ("ratings.csv", "userId,movieId,rating,timestamp\n1,2,3.5,1112486027\n1,29,3.5,1112484676\n"
                                  "138493,131262,4.0,1112484819\n"),
    }
    out = {}
    for ds, (fname, text) in contents.items():
        d = os.path.join(base, ds)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, fname), "w") as f:
            f.write(text)
        df = ref_ml.load_ratings_data(base, ds, download=False)
        for col in ("userId", "itemId", "rating"):
            out["%s/%s" % (ds, col)] = df[col].values
    np.savez_compressed(os.path.join(HERE, "loader_golden.npz"), **out)
    return out


if __name__ == "__main__":
    ref_dp, ref_ml = import_reference()
    p = make_pipeline_goldens(ref_dp)
    l = make_loader_goldens(ref_ml)
    print("wrote %d pipeline arrays, %d loader arrays" % (len(p), len(l)))
