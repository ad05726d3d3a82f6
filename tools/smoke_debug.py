"""Diagnose a smoke() mismatch: per-weight max error after one Adam step, and the oracle
gradient at the worst element (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from oracle import ncf_oracle as O  # noqa: E402

shape = O.NCFShape(50, 40, [64, 32, 16, 8], 8)
w = O.init_weights(shape, seed=0)
w = {k: (v * 3).astype(np.float32).astype(np.float64) for k, v in w.items()}
rng = np.random.RandomState(0)
users = rng.randint(0, 50, 64).astype(np.int32)
items = rng.randint(0, 40, 64).astype(np.int32)
y = np.tile([0, 0, 0, 1], 16).astype(np.float32)
for gen in (False, True):
    eng = NCFEngine(50, 40, shape.layers, shape.gmf_dim, max_batch=64, force_generic=gen)
    eng.set_keras_weights(w)
    grads = eng.alloc_grads()
    eng.forward_backward(users, items, y, group=4, k=2, inv_batch=1.0 / 64, grads=grads)
    _, g, _ = O.loss_and_grads(shape, w, users, items, y, [0] * 4)
    got = eng.keras_weights(grads[0], grads[1])
    for k in O.weight_names(shape):
        e = np.abs(got[k] - g[k])
        i = np.unravel_index(np.argmax(e), e.shape)
        print("generic" if gen else "fused", "grad", k, "maxerr %.3g at %s: got %.6g ref %.6g (max|g| %.3g)" % (
            e[i], i, got[k][i], g[k][i], np.max(np.abs(g[k]))))
    eng2 = NCFEngine(50, 40, shape.layers, shape.gmf_dim, max_batch=64, force_generic=gen)
    eng2.set_keras_weights(w)
    eng2.train_step(users, items, y, group=4, k=2)
    ref = {k: v.copy() for k, v in w.items()}
    st = O.new_opt_state(ref)
    O.train_step(shape, ref, st, users, items, y,
                 dict(optimizer="adam", lr=0.001, beta_1=0.9, beta_2=0.999, layers_l2reg=[0] * 4))
    got = eng2.keras_weights()
    for k in ref:
        e = np.abs(got[k] - ref[k])
        i = np.unravel_index(np.argmax(e), e.shape)
        print("generic" if gen else "fused", "weight", k, "maxerr %.3g at %s grad_ref %.6g" % (e[i], i, g[k][i]))
