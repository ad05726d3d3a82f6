"""Host issue cost of the single-table step at config B (4,095 samples, group 5, bf16 MLP): the
Python engine's share against the C library call's (GPU box).  Usage: python tools/host_cost_b.py"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movierecommender-tf-trt_amd"), ROOT]

import torch  # noqa: E402

from movierec import _native as N  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

U, I, LAYERS, G, B, g = 6040, 3706, [64, 32, 16, 8], 8, 4095, 5
eng = NCFEngine(U, I, LAYERS, G, max_batch=B, lazy_adam=True, precision="bf16")
eng.set_keras_weights(initial_weights(U, I, LAYERS, G, seed=0))
gen = torch.Generator(device="cuda").manual_seed(1234)
pool = []
for _ in range(8):
    u = torch.randint(0, U, (B // g,), generator=gen, device="cuda", dtype=torch.int32).repeat_interleave(g)
    it = torch.randint(0, I, (B,), generator=gen, device="cuda", dtype=torch.int32)
    y = torch.tensor([0.0] * (g - 1) + [1.0], device="cuda").repeat(B // g)
    pool.append((u.contiguous(), it.contiguous(), y.contiguous()))

lib = N.lib()
real = lib.ncf_train_step_ahead
acc = [0.0, 0]


def timed(*a):
    t = time.perf_counter()
    r = real(*a)
    acc[0] += time.perf_counter() - t
    acc[1] += 1
    return r


def step(i):
    u, it, y = pool[i % 8]
    nu, ni, _ = pool[(i + 1) % 8]
    eng.train_step(u, it, y, group=g, k=4, inv_batch=1.0 / B, next_batch=(nu, ni))


for i in range(30):
    step(i)
torch.cuda.synchronize()
K = 300
lib.ncf_train_step_ahead = timed
t0 = time.perf_counter()
for i in range(K):
    step(i)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("host issue %.1f us/step (library call %.1f us), wall %.1f us/step" %
      ((t1 - t0) / K * 1e6, acc[0] / max(acc[1], 1) * 1e6, (t2 - t0) / K * 1e6))
lib.ncf_train_step_ahead = real
pr = cProfile.Profile()
pr.enable()
for i in range(K):
    step(i)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
