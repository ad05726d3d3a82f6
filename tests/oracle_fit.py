"""Test helper: the reference's training loop restated on the CPU oracle.

``MovierecModel.fit_generator`` (reference ``movierec/model.py:305-333``) hands the batches
to Keras ``fit_generator`` with two callbacks, in this order:
``EarlyStopping(monitor='val_output_dcg', mode='max', patience=5, restore_best_weights=True)``
and ``ModelCheckpoint(..., monitor='val_output_dcg', save_best_only=True, mode='max')``.
Restated here from the Keras 2.2 / TF 1.13 algorithm (TF is absent, parity unpinned by reference
fixtures):

* per epoch: every batch of the train ``Sequence`` in a shuffled order (``OrderedEnqueuer``
  shuffles the batch indexes with python ``random``), ``train_on_batch``; then
  ``on_epoch_end``; then the validation ``Sequence`` in order (``evaluate_generator``);
* epoch logs: per-batch values averaged over the epoch's batches (weighted by batch size; all
  batches here have one size): ``loss`` (BCE mean + L2 terms), ``output_loss`` (BCE mean),
  ``output_hr``, ``output_dcg`` and their ``val_`` counterparts;
* EarlyStopping: ``current > best`` → best = current, wait = 0, keep the weights; else
  wait += 1 and, when wait >= patience, stop and restore the kept weights (best starts at -inf);
* ModelCheckpoint: save when ``current > best_so_far`` (same ordering), file name
  ``{name}-checkpoint-{epoch+1:02d}-{val_loss:.2f}``.

Test-only: it imports the oracle.
"""

import math
import random

import numpy as np

from oracle import ncf_oracle as O


def oracle_fit(shape, w, hyper, train_gen, val_gen, epochs, k, patience=5):
    """Returns (history dict, final weights, [(epoch, val_loss) of the saved checkpoints],
    stopped epoch or None).  ``w`` is updated in place."""
    st = O.new_opt_state(w)
    l2 = hyper["layers_l2reg"]
    g_t = train_gen.negatives_per_positive + 1
    g_v = val_gen.negatives_per_positive + 1
    hist = {}
    best, wait, best_w = -math.inf, 0, None
    saved, stopped = [], None
    for epoch in range(epochs):
        order = list(range(len(train_gen)))
        random.shuffle(order)
        tl, tb, th, td = [], [], [], []
        for i in order:
            (xu, xi), y = train_gen[i]
            reg = O.reg_loss(shape, w, l2)
            loss, p = O.train_step(shape, w, st, xu, xi, y, hyper)
            hr, dcg = O.group_metrics(p, y, g_t, k)
            tl.append(loss)
            tb.append(loss - reg)
            th.append(hr)
            td.append(dcg)
        train_gen.on_epoch_end()
        vl, vb, vh, vd = [], [], [], []
        for i in range(len(val_gen)):
            (xu, xi), y = val_gen[i]
            p, _ = O.forward(shape, w, xu, xi)
            bce = float(np.mean(O.bce_per_sample(p, y)))
            hr, dcg = O.group_metrics(p, y, g_v, k)
            vl.append(bce + O.reg_loss(shape, w, l2))
            vb.append(bce)
            vh.append(hr)
            vd.append(dcg)
        logs = {"loss": np.mean(tl), "output_loss": np.mean(tb), "output_hr": np.mean(th), "output_dcg": np.mean(td),
                "val_loss": np.mean(vl), "val_output_loss": np.mean(vb), "val_output_hr": np.mean(vh),
                "val_output_dcg": np.mean(vd)}
        for key, val in logs.items():
            hist.setdefault(key, []).append(float(val))
        current = logs["val_output_dcg"]
        if current > best:
            best, wait = current, 0
            best_w = {n: a.copy() for n, a in w.items()}
            saved.append((epoch + 1, logs["val_loss"]))
        else:
            wait += 1
            if wait >= patience:
                stopped = epoch
                for n in w:
                    w[n][...] = best_w[n]
                break
    return hist, w, saved, stopped
