"""Per-item logit errors of the fp16 scorer on a 32-item catalogue (every item returned)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from oracle import ncf_oracle as O  # noqa: E402

for dims in [(64, 32, [128, 64, 32, 16], 64), (64, 32, [128, 64, 32, 16], 0), (64, 32, [64, 32, 16, 8], 8),
             (64, 32, [64, 32, 16, 8], 0)]:
    shape = O.NCFShape(*dims)
    w = O.init_weights(shape, seed=1)
    rng = np.random.RandomState(2)
    for k in w:
        if k.endswith("embedding"):
            w[k] = rng.uniform(-0.5, 0.5, size=w[k].shape)
        elif k.endswith("bias"):
            w[k] = rng.uniform(-0.1, 0.1, size=w[k].shape)
    w = {k: v.astype(np.float32).astype(np.float64) for k, v in w.items()}
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=256)
    eng.set_keras_weights(w)
    users = np.arange(64, dtype=np.int32)
    z = O.score_all_items(shape, w, users)
    for prec in ("fp16", "fp32"):
        items, scores = eng.score_topk(users, k=32, precision=prec)
        items = items.cpu().numpy()
        p = scores.cpu().numpy().astype(np.float64)
        zg = np.log(p / (1 - p))
        zt = np.full_like(z, np.nan)
        for q in range(64):
            zt[q, items[q]] = zg[q]
        err = np.abs(zt - z)
        print(dims, prec, "max err %.4g" % np.nanmax(err), "per-user max (first 8):",
              np.round(np.nanmax(err, axis=1)[:8], 4), "per-item max:", np.round(np.nanmax(err, axis=0), 3))
