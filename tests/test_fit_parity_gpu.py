"""fit_generator parity: the HIP path's training loop against the oracle restatement of
Keras' loop (tests/oracle_fit.py; reference ``movierec/model.py:305-333``) on the same batches.

Both runs draw their batches from the host ``MovieLensDataGenerator`` (the reference's numpy
RNG stream, pinned by tests/golden) with the same seeds, and the epoch order from python
``random`` with the same seed, so they see identical batches in identical order.  Compared:

  * the History dict, key by key and epoch by epoch: losses relative 1e-4; hr / dcg absolute
    0.01 (a tie between fp32 and fp64 probabilities can flip one ranking position);
  * the epochs run, the early-stopping epoch and the best-only checkpoint files (names carry
    the epoch and val_loss);
  * the weights after the loop (restored to the best epoch): relative Frobenius error <= 5e-3
    per tensor (as tests/test_convergence_gpu.py; an element whose gradient is ~0 may take
    Adam's sign(g) step the other way in fp32);
  * on the device, the restored weights equal the best checkpoint file bit for bit.
"""

import glob
import os
import random

import numpy as np
import pandas as pd
import pytest

from conftest import gpu_available
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

LAYERS, GMF, L2 = [16, 8], 8, [0.0, 0.001]   # embedding L2 off (deferred decay), dense L2 on


def _ratings(seed=0, users=300, per_user=12):
    rng = np.random.RandomState(seed)
    I = 1682
    fu, fi = rng.normal(size=(users, 4)), rng.normal(size=(I, 4))
    rows = []
    for u in range(users):
        fav = np.argsort(-(fi @ fu[u] + 0.3 * rng.normal(size=I)))[:per_user]
        rows += [(u, int(i)) for i in fav]
    df = pd.DataFrame(rows, columns=["userId", "itemId"]).astype(np.int32)
    df["rating"] = np.float32(4.0)
    return df


def _generators(train, val, seed):
    from movierec.data_pipeline import MovieLensDataGenerator
    np.random.seed(seed)
    random.seed(seed)
    tg = MovieLensDataGenerator("ml-100k", train, 64, 3, shuffle=True)
    vg = MovieLensDataGenerator("ml-100k", val, 100, 99, extra_data_df=train, shuffle=False)
    return tg, vg


def test_fit_generator_matches_oracle_loop(tmp_path):
    from movierec.data_pipeline import split_leave_two_out
    from movierec.model import MovierecModel, initial_weights, load_tensors
    from oracle_fit import oracle_fit
    train, val, _ = split_leave_two_out(_ratings())
    epochs, patience, k, lr = 12, 2, 4, 0.02
    params = dict(num_users=943, num_items=1682, layers_sizes=LAYERS, layers_l2reg=L2, optimizer="adam", lr=lr,
                  beta_1=0.9, beta_2=0.999, batch_size=64, num_negs_per_pos=3, batch_size_eval=100,
                  num_negs_per_pos_eval=99, k=k, gmf_dim=GMF, seed=3)
    out = str(tmp_path)

    tg, vg = _generators(train, val, 11)
    model = MovierecModel(params, "fit", out, verbose=0)
    hist = model.fit_generator(tg, vg, epochs, patience=patience).history
    got = model.model.get_weights()

    tg, vg = _generators(train, val, 11)
    shape = O.NCFShape(943, 1682, LAYERS, GMF)
    w0 = {n: a.astype(np.float64) for n, a in initial_weights(943, 1682, LAYERS, GMF, seed=3).items()}
    hyper = dict(optimizer="adam", lr=lr, beta_1=0.9, beta_2=0.999, layers_l2reg=L2)
    ref_hist, ref_w, saved, stopped = oracle_fit(shape, w0, hyper, tg, vg, epochs, k, patience)

    print("gpu val_output_dcg", np.round(hist["val_output_dcg"], 4))
    print("ora val_output_dcg", np.round(ref_hist["val_output_dcg"], 4))
    assert sorted(hist) == sorted(ref_hist)
    assert len(hist["loss"]) == len(ref_hist["loss"]), "epochs run"
    assert stopped is not None and len(hist["loss"]) < epochs, "the setup must exercise early stopping"
    for key in hist:
        a, b = np.asarray(hist[key]), np.asarray(ref_hist[key])
        if key.endswith("loss"):
            np.testing.assert_allclose(a, b, rtol=1e-4, err_msg=key)
        else:
            np.testing.assert_allclose(a, b, atol=0.01, err_msg=key)
    assert not np.allclose(hist["loss"], hist["output_loss"])   # dense L2 on: loss = BCE + L2
    files = sorted(os.path.basename(f) for f in glob.glob(os.path.join(out, "fit-checkpoint-*")))
    assert files == sorted("fit-checkpoint-%02d-%.2f.safetensors" % (e, vl) for e, vl in saved)
    for name in O.weight_names(shape):
        rel = np.linalg.norm(got[name] - ref_w[name]) / max(np.linalg.norm(ref_w[name]), 1e-12)
        assert rel <= 5e-3, (name, rel)
    best = max(saved)[0]
    ck = load_tensors(os.path.join(out, "fit-checkpoint-%02d-%.2f.safetensors" % (best, dict(saved)[best])))
    for name in got:
        np.testing.assert_array_equal(got[name].astype(np.float32), ck[name].astype(np.float32), err_msg=name)
    assert gpu_available()
