"""Deferred-decay catch-up cost vs the debt it replays (GPU box).

Trains config C (bench.py's single-table path: fresh uniform batch per step, next batch counted
ahead) and, for each timed step, reads row_step before the step to measure the debt the
catch-up launch replays: rows of the batch that are stale, element-steps (debt x row width),
the longest debt.  Prints per-step catch-up ms next to those, and the replay rate.
Usage: python tools/catchup_probe.py [--steps 50] [--warmup 10]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "movierecommender-tf-trt_amd"), ROOT]

import torch  # noqa: E402

from movierec import _native as N  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--warmup", type=int, default=10)
a = ap.parse_args()
U, I, B, G = 138493, 27278, 65536, 4
eng = NCFEngine(U, I, [128, 64, 32, 16], 64, max_batch=B, lazy_adam=True)
eng.set_keras_weights(initial_weights(U, I, [128, 64, 32, 16], 64, seed=0))
gen = torch.Generator(device="cuda").manual_seed(1234)
pool = []
for _ in range(a.warmup + a.steps + 1):
    u = torch.randint(0, U, (B // G,), generator=gen, device="cuda", dtype=torch.int32).repeat_interleave(G)
    it = torch.randint(0, I, (B,), generator=gen, device="cuda", dtype=torch.int32)
    pool.append((u.contiguous(), it.contiguous(), torch.tensor([0.0] * (G - 1) + [1.0], device="cuda").repeat(B // G)))
for i in range(a.warmup):
    eng.train_step(*pool[i], group=G, k=3, next_batch=(pool[i + 1][0], pool[i + 1][1]))
eng.flush()
torch.cuda.synchronize()
rows = []
W = eng.row_width
for i in range(a.warmup, a.warmup + a.steps):
    u, it, y = pool[i]
    t = int(eng.step.item())
    touched = torch.cat([torch.unique(u.long()), U + torch.unique(it.long())])
    debt = (t - eng.row_step[touched].long()).clamp(min=0)
    N.profile_enable([N.K_CATCHUP, N.K_EMB_UPDATE, N.K_FWD_BWD], 4)
    eng.train_step(u, it, y, group=G, k=3, next_batch=(pool[i + 1][0], pool[i + 1][1]))
    torch.cuda.synchronize()
    ms_c, _ = N.profile_read(N.K_CATCHUP)
    ms_u, _ = N.profile_read(N.K_EMB_UPDATE)
    ms_f, _ = N.profile_read(N.K_FWD_BWD)
    N.profile_enable([], 0)
    rows.append(dict(step=i, catchup_ms=round(ms_c, 4), update_ms=round(ms_u, 4), fwd_bwd_ms=round(ms_f, 4),
                     stale_rows=int((debt > 0).sum()), elem_steps=int(debt.sum()) * W, max_debt=int(debt.max()),
                     mean_debt_stale=round(float(debt[debt > 0].float().mean()), 2) if (debt > 0).any() else 0))
for r in rows:
    print(json.dumps(r))
tail = rows[len(rows) // 2:]
es = sum(r["elem_steps"] for r in tail)
ms = sum(r["catchup_ms"] for r in tail)
print(json.dumps({"second_half_mean_catchup_ms": ms / len(tail), "elem_steps_per_step": es / len(tail),
                  "G_elem_steps_per_s": es / (ms * 1e-3) / 1e9}))
