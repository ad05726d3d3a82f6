# GPU box: group-user form, mixed batch of fold 2: which samples' dX the wrong rows are off by
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "movierecommender-tf-trt_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
from oracle import ncf_oracle as O
from movierec.engine import NCFEngine
from test_user_fold_gpu import _weights, _mixed_batch, CONFIG_C

group = 2
shape = O.NCFShape(*CONFIG_C)
w = _weights(shape, 60 + group)
B = 1024
users, items, y = _mixed_batch(shape, B, group, 61 + group)
eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, fb_kernel="wave")
eng.set_keras_weights(w)
grads = eng.alloc_grads()
eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads)
got = eng.keras_weights(grads[0], grads[1])
_, g, _ = O.loss_and_grads(shape, w, users, items, y, [0.0] * 4)
# per-sample dX (MLP input gradient) as the oracle computes it
p, c = O.forward(shape, w, users, items)
lo, hi = O.clip_bounds()
dz = np.where((c["p"] >= lo) & (c["p"] <= hi), (c["p"] - y) / B, 0.0)
dh = (dz[:, None] * w["output/kernel"][:, 0][None, :])[:, shape.gmf_dim:]
h = c["h"]
for l in range(shape.n - 1, 0, -1):
    dzl = dh * (h[l] > 0)
    dh = dzl @ w["hidden_%d/kernel" % l].T
du = shape.du
for name, ids_, sl in (("user_embedding", users, slice(0, du)), ("item_embedding", items, slice(du, None))):
    d = got[name] - g[name]
    scale = np.max(np.abs(g[name]))
    bad = np.nonzero(np.max(np.abs(d), axis=1) > 1e-5 * scale)[0]
    for r in bad:
        print(name, "row", r, "max|d|", np.max(np.abs(d[r])))
        cand = []
        for s in range(B):
            v = dh[s, sl]
            nv = np.linalg.norm(v)
            if nv == 0:
                continue
            coef = float(d[r] @ v / (nv * nv))
            resid = np.linalg.norm(d[r] - coef * v) / (np.linalg.norm(d[r]) + 1e-30)
            cand.append((resid, s, coef))
        cand.sort()
        for resid, s, coef in cand[:4]:
            print("   sample", s, "pos", s % group, "user", users[s], "head user", users[s - s % group], "item", items[s],
                  "coef %.4f resid %.3g" % (coef, resid))
