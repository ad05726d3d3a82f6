"""Diagnostic (GPU box): one counted-ahead step, then the scan ahead's outputs (the in-kernel
fill's inputs) read back and checked against numpy: cursors, cleared counts, per-block offsets,
totals, occupied-key numbering, heavy_n.  Runs no fill (the step counted ahead is not taken)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "movierecommender-tf-trt_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_index_in_kernel_gpu import _batch, _weights, LAYERS, GMF, GROUP  # noqa: E402
from oracle import ncf_oracle as O  # noqa: E402
from movierec import _native as N  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
U, I = 3000, 2000
K = U + I
e = NCFEngine(U, I, LAYERS, GMF, max_batch=B, lazy_adam=True)
e.set_keras_weights(_weights(O.NCFShape(U, I, LAYERS, GMF), 5))
b0, b1 = _batch(U, I, B, 40), _batch(U, I, B, 41)
e.train_step(*b0, group=GROUP, k=2, next_batch=(b1[0], b1[1]))
torch.cuda.synchronize()
off = (ctypes.c_int64 * 17)()
N.check(N.lib().ncf_debug_index_regions(ctypes.byref(e.shape), ctypes.c_int64(e.max_batch), off))
names = ["cnt", "cnt_ahead", "heavy_n", "err", "offs_local", "offs", "tot", "uloc", "utot", "nuniq", "touched",
         "touched_oc", "heavy", "list", "slist"]
o = dict(zip(names, list(off)[:15]))
nscan, list_cap = off[15], off[16]
print("regions", o, "nscan", nscan, "list_cap", list_cap, flush=True)
ws = e.ws.cpu().numpy()


def reg(name, count):
    return ws[o[name]:o[name] + 4 * count].view(np.int32).copy()


u = b1[0].cpu().numpy().astype(np.int64)
it = b1[1].cpu().numpy().astype(np.int64)
bad = 0
matched = False
for fold in (0, GROUP):
    keys = np.concatenate([u, U + it])
    if fold > 1:
        idx = np.arange(B)
        hd = idx - idx % fold
        keep = ~((idx != hd) & (u == u[hd]))
        keys = np.concatenate([u[keep], U + it])
    want = np.bincount(keys, minlength=K + 1).astype(np.int64)
    got = reg("cnt", K + 1)
    print("fold %d: cursor == counts: %s (sum got %d want %d)" % (fold, np.array_equal(got, want), got.sum(),
                                                                   want.sum()), flush=True)
    d = np.flatnonzero(got != want)
    print("  got min %d max %d nz %d; want nz %d; ahead sum %d; %d keys differ, first %s got %s want %s; "
          "users differ %d items differ %d" % (got.min(), got.max(), (got != 0).sum(), (want != 0).sum(),
                                               reg("cnt_ahead", K + 1).sum(), len(d), d[:6], got[d[:6]],
                                               want[d[:6]], (d < U).sum(), (d >= U).sum()), flush=True)
    if np.array_equal(got, want):
        matched = True
        blk = np.arange(K + 1) // 2048
        loc = np.zeros(K + 1, np.int64)
        uloc = np.zeros(K + 1, np.int64)
        tot, utot = [], []
        for b in range(nscan):
            m = blk == b
            c = want[m]
            loc[m] = np.cumsum(c) - c
            nz = (c > 0).astype(np.int64)
            uloc[m] = np.cumsum(nz) - nz
            tot.append(c.sum())
            utot.append(nz.sum())
        checks = {"offs_local": (reg("offs_local", K + 1), loc), "uloc": (reg("uloc", K + 1), uloc),
                  "tot": (reg("tot", nscan), np.array(tot)), "utot": (reg("utot", nscan), np.array(utot)),
                  "cnt_ahead": (reg("cnt_ahead", K + 1), np.zeros(K + 1)), "heavy_n": (reg("heavy_n", 1), [0])}
        for k, (g, w) in checks.items():
            ok = np.array_equal(np.asarray(g, np.int64), np.asarray(w, np.int64))
            bad += not ok
            print("  %-10s %s" % (k, "ok" if ok else "DIFFERS: got %s want %s" % (g[:8], np.asarray(w)[:8])))
            if not ok:
                d = np.flatnonzero(np.asarray(g, np.int64) != np.asarray(w, np.int64))
                print("    first diffs at", d[:10], np.asarray(g)[d[:10]], np.asarray(w)[d[:10]])
        pre = np.concatenate([[0], np.cumsum(tot)])[:-1]
        off_full = loc + pre[blk]
        print("  max list index %d (cap %d), unique %d" % (off_full[-1], list_cap, uloc[-1] + sum(utot[:-1])))
print("err flags 0x%x" % int(reg("err", 1)[0]))
print("SCAN BAD" if bad or not matched else "SCAN OK", flush=True)
sys.exit(1 if bad or not matched else 0)
