"""Debug: deferred-decay engine vs dense sweep, per step, printing the first differing rows."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movierecommender-tf-trt_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from oracle import ncf_oracle as O  # noqa: E402
from test_native_gpu import _weights, _batch, _engine  # noqa: E402

shape = O.NCFShape(200, 150, [128, 64, 32, 16], 64)
w = _weights(shape, 12)
dense = _engine(shape, w)
lazy = _engine(shape, w, lazy_adam=True)
for s in range(3):
    users, items, y = _batch(shape, 24, 4, 40 + s, dup_items=min(shape.num_items, 11) if s % 3 == 0 else None)
    rs_before = lazy.row_step.clone()
    dense.train_step(users, items, y, group=4, k=2)
    lazy.train_step(users, items, y, group=4, k=2)
    torch.cuda.synchronize()
    touched = set(users.tolist()) | set((items + 200).tolist())
    de, le = dense.emb.cpu().numpy(), lazy.emb.cpu().numpy()
    dm, lm = dense.emb_m.cpu().numpy(), lazy.emb_m.cpu().numpy()
    bad = [r for r in sorted(touched) if not np.array_equal(de[r], le[r])]
    badm = [r for r in sorted(touched) if not np.array_equal(dm[r], lm[r])]
    print("step", s, "touched", len(touched), "p-mismatch", len(bad), "m-mismatch", len(badm), flush=True)
    for r in bad[:3]:
        j = int(np.argmax(de[r] != le[r]))
        print("  row", r, "row_step before", int(rs_before[r]), "after", int(lazy.row_step[r]), "col", j,
              repr(de[r, j]), repr(le[r, j]), "m", repr(dm[r, j]), repr(lm[r, j]), flush=True)
