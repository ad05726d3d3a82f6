"""Touched-row update launch with and without the next batch counted ahead (GPU box).

With next_batch the launch also counts the next batch's contributions and catches its stale rows
up (count blocks dispatched first); without it only the update (and dense-layer Adam) blocks
run and the catch-up replays go to the pre-forward launch.  Prints the average launch times.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))

import torch  # noqa: E402

from movierec import _native as N  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402


def run(ahead, B=65536, steps=30):
    eng = NCFEngine(138493, 27278, [128, 64, 32, 16], 64, max_batch=B, lazy_adam=True)
    eng.set_keras_weights(initial_weights(138493, 27278, [128, 64, 32, 16], 64, seed=0))
    g = torch.Generator(device="cuda").manual_seed(1)
    pool = []
    for _ in range(steps + 11):
        u = torch.randint(0, 138493, (B // 4,), generator=g, device="cuda", dtype=torch.int32).repeat_interleave(4)
        it = torch.randint(0, 27278, (B,), generator=g, device="cuda", dtype=torch.int32)
        pool.append((u.contiguous(), it))
    y = torch.tensor([0., 0., 0., 1.], device="cuda").repeat(B // 4)
    for i in range(10 + steps):
        if i == 10:
            torch.cuda.synchronize()
            N.profile_enable([N.K_EMB_UPDATE, N.K_CATCHUP, N.K_INDEX, N.K_FWD_BWD], 4 * steps)
        u, it = pool[i]
        eng.train_step(u, it, y, group=4, k=3, next_batch=pool[i + 1] if ahead else None)
    torch.cuda.synchronize()
    out = {}
    for name, k in (("update", N.K_EMB_UPDATE), ("catchup", N.K_CATCHUP), ("index", N.K_INDEX), ("fwd_bwd", N.K_FWD_BWD)):
        ms, cnt = N.profile_read(k)
        out[name + "_us"] = round(ms / max(cnt, 1) * 1e3, 2)
    N.profile_enable([], 0)
    return out


if __name__ == "__main__":
    # argv[1] (optional): "ahead" / "not_ahead" runs one mode only (a PMC pass per mode:
    # tools/pmc_update_roles.sh)
    modes = sys.argv[1:] or ["ahead", "not_ahead"]
    print(json.dumps({m: run(m == "ahead") for m in modes}))
