# GPU box: group-user form vs the one-wave form on test_user_fold_gpu's mixed batches: where the
# dense embedding / dense-layer gradients differ
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "movierecommender-tf-trt_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
from oracle import ncf_oracle as O
from movierec.engine import NCFEngine
from test_user_fold_gpu import _weights, _mixed_batch, CONFIG_C

for group in (2, 4, 8):
    shape = O.NCFShape(*CONFIG_C)
    w = _weights(shape, 60 + group)
    B = 1024
    users, items, y = _mixed_batch(shape, B, group, 61 + group)
    res = {}
    for kern in ("wave", "wave1"):
        eng = NCFEngine(shape.num_users, shape.num_items, shape.layers, shape.gmf_dim, max_batch=B, fb_kernel=kern)
        eng.set_keras_weights(w)
        grads = eng.alloc_grads()
        probs = torch.empty(B, dtype=torch.float32, device="cuda")
        eng.forward_backward(users, items, y, group=group, k=2, inv_batch=1.0 / B, grads=grads, probs_out=probs)
        torch.cuda.synchronize()
        res[kern] = (grads[0].cpu().numpy(), grads[1].cpu().numpy(), probs.cpu().numpy())
    a, b = res["wave"], res["wave1"]
    print("group", group, "probs maxdiff", np.max(np.abs(a[2] - b[2])), "mlp maxdiff", np.max(np.abs(a[1] - b[1])), "scale", np.max(np.abs(b[1])))
    d = np.abs(a[0] - b[0])
    scale = np.max(np.abs(b[0]))
    bad = np.argwhere(d > 1e-5 * scale)
    rows = sorted(set(int(r) for r, c in bad))
    cols = sorted(set(int(c) for r, c in bad))
    print("  emb bad rows", len(rows), rows[:20], "cols", cols[:10], "...", cols[-5:] if cols else None)
    for r in rows[:5]:
        if r < shape.num_users:
            idx = np.nonzero(users == r)[0]
            info = [(int(i), int(i % group), int(users[i - i % group])) for i in idx]
            print("   user", r, "samples (i, pos, head user):", info[:12])
        else:
            print("   item row", r)
