"""Phase timing of the sample-unit forward/backward kernel (profiling build).

Build:  python movierecommender-tf-trt_amd/csrc/build.py -D NCF_UNIT_TIMING \
            --out movierecommender-tf-trt_amd/movierec/_lib/var/utiming.so
Run:    NCF_LIB=<that .so> BATCH=65536 python tools/unit_timing.py   (GPU box)
Prints, per segment of the per-unit loop, the mean cycles of each wave over all workgroups
(first two units), from __builtin_readcyclecounter stamps.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movierecommender-tf-trt_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from movierec import _native as N  # noqa: E402
from movierec.engine import NCFEngine  # noqa: E402
from movierec.model import initial_weights  # noqa: E402

# stamps: 0 unit start, then before/after each barrier; 19 = dX done
SEG = [("gather", 0, 1), ("bar1", 1, 2), ("L1", 2, 3), ("bar2", 3, 4), ("L2", 4, 5), ("bar3", 5, 6),
       ("L3+out+G3", 6, 7), ("bar4", 7, 8), ("gmf_bwd+G2", 8, 13), ("bar5", 13, 14), ("G1", 14, 15),
       ("bar6", 15, 16), ("dX", 16, 19), ("dW+extras", 19, 17), ("bar7", 17, 18)]


def main():
    B = int(os.environ.get("BATCH", "65536"))
    eng = NCFEngine(138493, 27278, [128, 64, 32, 16], 64, max_batch=B, fb_kernel="unit")
    eng.set_keras_weights(initial_weights(138493, 27278, [128, 64, 32, 16], 64, seed=0))
    g = torch.Generator(device="cuda").manual_seed(1)
    u = torch.randint(0, 138493, (B // 4,), generator=g, device="cuda", dtype=torch.int32).repeat_interleave(4)
    it = torch.randint(0, 27278, (B,), generator=g, device="cuda", dtype=torch.int32)
    y = torch.tensor([0., 0., 0., 1.], device="cuda").repeat(B // 4)
    for _ in range(5):
        eng.train_step(u, it, y, group=4, k=3)
    N.profile_enable([N.K_FWD_BWD], 4)
    eng.train_step(u, it, y, group=4, k=3)
    torch.cuda.synchronize()
    ms, cnt = N.profile_read(N.K_FWD_BWD)
    fn = N.lib().ncf_debug_unit_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(256 * 2 * 4 * 20, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(256, 2, 4, 20).astype(np.int64)
    res = {"kernel_ms": ms / max(cnt, 1)}
    for w in range(4):
        res["wave%d" % w] = {name: round(float(np.mean(t[:, :, w, b] - t[:, :, w, a])), 1) for name, a, b in SEG}
    span = t[:, 1, 0, 18] - t[:, 0, 0, 0]
    res["two_units_cycles_mean"] = float(span.mean())
    U = int(os.environ.get("NCF_UNIT_SIZE", "64" if B >= 16384 else "32"))
    res["cycles_per_us_est"] = float(span.mean()) / 2 * (B // U / 256) / (ms / max(cnt, 1) * 1e3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
