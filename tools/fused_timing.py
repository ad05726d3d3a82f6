"""Phase timing of the fused forward/backward kernel (profiling build).

Build:  python movierecommender-tf-trt_amd/csrc/build.py -D NCF_FUSED_TIMING \
            --out movierecommender-tf-trt_amd/movierec/_lib/var/timing.so
Run:    NCF_LIB=<that .so> python tools/fused_timing.py   (GPU box)
Prints, per phase of the per-tile loop, the mean cycles of waves 0 and 3 over all
workgroups (first two tiles), from __builtin_readcyclecounter stamps.
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

PHASES = ["gather+gmf_fwd", "layer1", "layers2-3", "out+bce+metrics", "gmf_bwd", "g3+g2", "g1", "dX",
          "sync1", "dW", "bias", "sync2", "end_gmf_rows", "end_dx_chain", "end_dx_store"]
NP = len(PHASES)


def main():
    B = int(os.environ.get("BATCH", "65536"))
    eng = NCFEngine(138493, 27278, [128, 64, 32, 16], 64, max_batch=B)
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
    fn = N.lib().ncf_debug_fused_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(256 * 2 * 2 * 16, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(256, 2, 2, 16).astype(np.int64)
    res = {"kernel_ms": ms / max(cnt, 1)}
    for wi, wname in enumerate(["wave0", "wave3"]):
        d = np.diff(t[:, :, wi, :NP + 1], axis=-1).astype(np.float64)  # [wg, tile, NP]
        d[d < 0] = np.nan  # stamps a build does not record
        res[wname] = {PHASES[p]: round(float(np.nanmean(d[:, :, p])), 1) for p in range(NP)
                      if not np.isnan(d[:, :, p]).all()}
        res[wname]["tile_total"] = round(float((t[:, :, wi, 12] - t[:, :, wi, 0]).mean()), 1)
    span = (t[:, 1, 0, 12] - t[:, 0, 0, 0])
    res["two_tiles_cycles_mean"] = float(span.mean())
    res["cycles_per_us_est"] = float(span.mean()) / (ms / max(cnt, 1) * 1e3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
