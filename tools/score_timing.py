"""Time the all-item scorer at ml-20m scale (config E) on the GPU box."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))

import torch  # noqa: E402
from movierec import _native as N  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

U, I = int(os.environ.get("SU", 138493)), int(os.environ.get("SI", 27278))
layers, G = [128, 64, 32, 16], 64
eng = NCFEngine(U, I, layers, G, max_batch=1024)
eng.set_keras_weights(initial_weights(U, I, layers, G, seed=0))
users = torch.arange(U, dtype=torch.int32, device="cuda")
eng.score_topk(users[:4096], k=10)
torch.cuda.synchronize()
N.profile_enable([N.K_SCORE], 8)
t0 = time.perf_counter()
items, scores = eng.score_topk(users, k=10)
torch.cuda.synchronize()
wall = time.perf_counter() - t0
ms, n = N.profile_read(N.K_SCORE)
pairs = U * I
flops = pairs * 2 * (64 * 32 + 32 * 16 + 16 + 64)
print(json.dumps({"users": U, "items": I, "wall_ms": wall * 1e3, "kernel_ms": ms, "launches": n,
                  "pairs_per_s": pairs / (ms * 1e-3), "tflops": flops / (ms * 1e-3) / 1e12,
                  "first": items[0].tolist()}))
