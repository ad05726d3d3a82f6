"""Host issue cost vs wall time of the single-table step (deferred decay, count-ahead), config C,
over K steps: is the step GPU-bound or host-bound?  Usage (GPU box): python tools/host_cost_single.py [K]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movierecommender-tf-trt_amd"), ROOT]

import torch  # noqa: E402

from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

U, I, LAYERS, G, B, g = 138493, 27278, [128, 64, 32, 16], 64, 65536, 4
K = int(sys.argv[1]) if len(sys.argv) > 1 else 500
eng = NCFEngine(U, I, LAYERS, G, max_batch=B, lazy_adam=True)
eng.set_keras_weights(initial_weights(U, I, LAYERS, G, seed=0))
gen = torch.Generator(device="cuda").manual_seed(1234)
pool = []
for _ in range(8):
    u = torch.randint(0, U, (B // g,), generator=gen, device="cuda", dtype=torch.int32).repeat_interleave(g)
    it = torch.randint(0, I, (B,), generator=gen, device="cuda", dtype=torch.int32)
    y = torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(B // g)
    pool.append((u.contiguous(), it.contiguous(), y.contiguous()))


def step(i):
    u, it, y = pool[i % 8]
    nu, ni, _ = pool[(i + 1) % 8]
    eng.train_step(u, it, y, group=g, k=3, inv_batch=1.0 / B, next_batch=(nu, ni))


for i in range(20):
    step(i)
eng.flush()
torch.cuda.synchronize()
marks = []
t0 = time.perf_counter()
for i in range(K):
    step(20 + i)
    if (i + 1) % 50 == 0:
        marks.append(time.perf_counter())
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("host issue %.1f us/step, wall %.1f us/step over %d steps" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6, K))
prev = t0
for m in marks:
    print("  host us/step per 50:", round((m - prev) / 50 * 1e6, 1))
    prev = m
for n in (50, 100, 200):
    torch.cuda.synchronize()
    a = time.perf_counter()
    for i in range(n):
        step(i)
    torch.cuda.synchronize()
    print("wall %d steps: %.1f us/step" % (n, (time.perf_counter() - a) / n * 1e6))
