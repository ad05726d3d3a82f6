"""Wall time per training step (config C) with the current library, for A/B checks of the
stream layout (run once with NCF_SIDE_STREAM=0, once without)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))
import torch  # noqa: E402

from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

B = 65536
eng = NCFEngine(138493, 27278, [128, 64, 32, 16], 64, max_batch=B)
eng.set_keras_weights(initial_weights(138493, 27278, [128, 64, 32, 16], 64, seed=0))
g = torch.Generator(device="cuda").manual_seed(1)
pool = []
for _ in range(4):
    u = torch.randint(0, 138493, (B // 4,), generator=g, device="cuda", dtype=torch.int32).repeat_interleave(4)
    it = torch.randint(0, 27278, (B,), generator=g, device="cuda", dtype=torch.int32)
    y = torch.tensor([0., 0., 0., 1.], device="cuda").repeat(B // 4)
    pool.append((u, it, y))
for i in range(10):
    eng.train_step(*pool[i % 4], group=4, k=3)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for i in range(50):
        eng.train_step(*pool[i % 4], group=4, k=3)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("side=%s step %.4f ms (host enqueue %.4f ms/step)" % (os.environ.get("NCF_SIDE_STREAM", "1"),
                                                               (t2 - t0) / 50 * 1e3, (t1 - t0) / 50 * 1e3))
# host cost split: python wrapper vs library call
import ctypes
from movierec import _native as N
u, it, y = pool[0]
h = eng.hyper
h.group, h.k, h.inv_batch = 4, 3, 1.0 / B
L = N.lib()
args = (ctypes.byref(eng.shape), ctypes.byref(eng.model_s), ctypes.byref(eng.optim_s), ctypes.byref(h), N.ptr(u),
        N.ptr(it), N.ptr(y), B, N.ptr(eng.stats), None, N.ptr(eng.ws), eng.ws_bytes, N.stream_handle())
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(50):
    L.ncf_train_step(*args)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("raw C call: step %.4f ms (host enqueue %.4f ms/step)" % ((t2 - t0) / 50 * 1e3, (t1 - t0) / 50 * 1e3))
