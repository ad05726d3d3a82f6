# GPU box: per-sample gradient rows (workspace region gs) of the group-user form vs the one-wave form
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "movierecommender-tf-trt_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
from oracle import ncf_oracle as O
from movierec.engine import NCFEngine
from test_user_fold_gpu import _weights, _mixed_batch, CONFIG_C

def up(x):
    return (x + 255) // 256 * 256
group = int(sys.argv[1]) if len(sys.argv) > 1 else 2
shape = O.NCFShape(*CONFIG_C)
w = _weights(shape, 60 + group)
B = 1024
users, items, y = _mixed_batch(shape, B, group, 61 + group)
K = shape.num_users + shape.num_items
off = up((K + 1) * 4); off = up(off + 4); off = up(off + 4); off = up(off + 4)
probs_off = off
gs_off = up(off + B * 4)
W = 128
rows = {}
for kern in ("wave", "wave1"):
    eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, fb_kernel=kern)
    eng.set_keras_weights(w)
    grads = eng.alloc_grads()
    eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads)
    torch.cuda.synchronize()
    ws = eng.ws.view(torch.uint8)
    rows[kern] = ws[gs_off:gs_off + 2 * B * W * 4].view(torch.float32).view(2 * B, W).cpu().numpy()
a, b = rows["wave"], rows["wave1"]
hd = np.arange(B) & ~(group - 1)
folded = (np.arange(B) != hd) & (users == users[hd])
for s in range(B):
    for part, r in (("user", 2 * s), ("item", 2 * s + 1)):
        if part == "user" and folded[s]:
            continue
        d = np.max(np.abs(a[r] - b[r]))
        sc = np.max(np.abs(b[r])) + 1e-30
        if d > 1e-4 * sc:
            cols = np.nonzero(np.abs(a[r] - b[r]) > 1e-4 * sc)[0]
            print("sample", s, part, "unit", s // 16, "lane", s % 16, "maxdiff %.3g scale %.3g" % (d, sc), "cols", cols.min(), cols.max(), len(cols),
                  "mism" if users[s] != users[hd[s]] else "")
