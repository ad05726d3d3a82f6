"""Diagnostic (GPU box): the in-kernel fill's row side at one counted step — the touched list,
(offset, count) per row and the heavy rows read back after the forward/backward and checked
against numpy; then the first step where the counted engine leaves the lazy one (bitwise)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "movierecommender-tf-trt_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_index_in_kernel_gpu import _batch, _weights, LAYERS, GMF, GROUP  # noqa: E402
from oracle import ncf_oracle as O  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 20480
U, I = 3000, 2000
w = _weights(O.NCFShape(U, I, LAYERS, GMF), 5)
eng = {}
for name, kw in (("lazy", dict(lazy_adam=True)), ("ahead", dict(lazy_adam=True))):
    e = NCFEngine(U, I, LAYERS, GMF, max_batch=B, **kw)
    e.set_keras_weights(w)
    eng[name] = e
batches = [_batch(U, I, B, 40 + s) for s in range(6)]
for s, (u, it, y) in enumerate(batches):
    nxt = (batches[s + 1][0], batches[s + 1][1]) if s + 1 < len(batches) else None
    eng["lazy"].train_step(u, it, y, group=GROUP, k=2)
    eng["ahead"].train_step(u, it, y, group=GROUP, k=2, next_batch=nxt)
    if s == 2:
        eng["ahead"].predict(u, it)
    torch.cuda.synchronize()
    a, l = eng["ahead"], eng["lazy"]
    # compare after flushing copies (flush changes nothing observable: dense state)
    a.flush(); l.flush()
    same = torch.equal(a.emb, l.emb) and torch.equal(a.mlp, l.mlp) and torch.equal(a.emb_m, l.emb_m)
    d = (a.emb - l.emb).abs()
    rows = torch.nonzero(d.amax(1) > 0).flatten()
    print("step %d: same %s, rows differing %d %s, max %g" % (s, same, rows.numel(), rows[:10].tolist(),
                                                             float(d.max())), flush=True)
    a._dirty = True; l._dirty = True
    if not same:
        break

# the last step's row side, read back: touched rows ascending with (offset, count) against numpy
a = eng["ahead"]
off = (ctypes.c_int64 * 17)()
from movierec import _native as N  # noqa: E402
N.check(N.lib().ncf_debug_index_regions(ctypes.byref(a.shape), ctypes.c_int64(a.max_batch), off))
names = ["cnt", "cnt_ahead", "heavy_n", "err", "offs_local", "offs", "tot", "uloc", "utot", "nuniq", "touched",
         "touched_oc", "heavy", "list", "slist"]
o = dict(zip(names, list(off)[:15]))
ws = a.ws.cpu().numpy()
reg = lambda k, c, dt=np.int32: ws[o[k]:o[k] + np.dtype(dt).itemsize * c].view(dt).copy()
u, it = batches[s][0].cpu().numpy().astype(np.int64), batches[s][1].cpu().numpy().astype(np.int64)
idx = np.arange(B)
hd = idx - idx % GROUP
keep = ~((idx != hd) & (u == u[hd]))
keys = np.concatenate([u[keep], U + it])
cnt = np.bincount(keys, minlength=U + I)
tk = np.flatnonzero(cnt)
nu = int(reg("nuniq", 1)[0])
got = reg("touched", nu)
toc = reg("touched_oc", 2 * nu).reshape(-1, 2)
print("nuniq %d want %d; touched equal %s" % (nu, len(tk), nu == len(tk) and np.array_equal(got, tk)))
if nu == len(tk):
    want_off = np.concatenate([[0], np.cumsum(cnt[tk])])[:-1]
    bad = np.flatnonzero((toc[:, 0] != want_off) | (toc[:, 1] != cnt[tk]))
    print("toc mismatches %d: first %s" % (len(bad), [(int(got[b]), toc[b].tolist(), int(want_off[b]), int(cnt[tk][b])) for b in bad[:6]]))
    for r in (4095, 4098, 4252):
        p = np.searchsorted(tk, r)
        print("row %d: in batch %s count %d toc %s row_step %d" % (r, p < len(tk) and tk[p] == r, cnt[r],
              toc[p].tolist() if p < len(tk) and tk[p] == r else None, int(a.row_step[r])))
    bad_pos = np.flatnonzero(got != tk)
    print("positions differing: %d, range %s; upre/utot %s %s" % (len(bad_pos), (int(bad_pos.min()), int(bad_pos.max())) if len(bad_pos) else None,
          np.cumsum(reg("utot", 3)).tolist(), reg("utot", 3).tolist()))
    al = lambda x: (x + 255) // 256 * 256
    tl_off = o["heavy"] + al((2 * B // 8 + 1) * 4)
    tocl_off = tl_off + al(3 * 2048 * 4)
    tl = ws[tl_off:tl_off + 3 * 2048 * 4].view(np.int32).reshape(3, 2048)
    tocl = ws[tocl_off:tocl_off + 3 * 2048 * 8].view(np.int32).reshape(3, 2048, 2)
    ut = reg("utot", 3)
    for b in range(3):
        kb = tk[(tk >= b * 2048) & (tk < (b + 1) * 2048)]
        ok = np.array_equal(tl[b, :len(kb)], kb)
        print("block %d: utot %d keys %d tl ok %s; counts ok %s" % (b, ut[b], len(kb), ok,
              np.array_equal(tocl[b, :len(kb), 1], cnt[kb])))
        if not ok:
            d = np.flatnonzero(tl[b, :len(kb)] != kb)
            print("   first tl diffs", d[:8].tolist(), tl[b, d[:8]].tolist(), kb[d[:8]].tolist())
    print("bad positions", bad_pos[:12].tolist(), got[bad_pos[:12]].tolist(), tk[bad_pos[:12]].tolist())
