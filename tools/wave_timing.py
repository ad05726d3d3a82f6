"""Phase timing of the wave-chain forward/backward kernel (profiling build).

Build:  python movierecommender-tf-trt_amd/csrc/build.py -D NCF_WAVE_TIMING \
            --out movierecommender-tf-trt_amd/movierec/_lib/var/wtiming.so
Run:    NCF_LIB=<that .so> BATCH=65536 python tools/wave_timing.py   (GPU box)
Prints the mean cycles of each segment of the per-unit loop over all waves (first two units),
the prologue and the epilogue, from __builtin_readcyclecounter stamps.
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

# stamps per unit: 0 start, 1 layer 1 done, 2 layers 2-3, 3 output + metrics, 4 G3 + GMF backward,
# 5 G2 + G1, 6 dX, 7 dW; per kernel: unit 0 slot 8 = prologue done, slot 9 = epilogue done
SEG = [("L1", 0, 1), ("L2+L3", 1, 2), ("output", 2, 3), ("G3+gmf_bwd", 3, 4), ("G2+G1", 4, 5), ("dX", 5, 6),
       ("dW", 6, 7)]


def spans(fn_name):
    """Per-wave span stamps (g_wave_s): entry / end on the 100 MHz realtime clock (aligned across
    CUs), prologue / units / epilogue in shader cycles."""
    fn = getattr(N.lib(), fn_name)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(256 * 4 * 16, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    s = buf.reshape(256, 4, 16).astype(np.int64)
    rt0, rt1 = s[:, :, 0], s[:, :, 13]
    units = s[:, :, 3:11]
    nu = int(np.sum(units[0, 0] > 0))
    out = {"entry_skew_us": round(float(rt0.max() - rt0.min()) / 100.0, 2),
           "end_skew_us": round(float(rt1.max() - rt1.min()) / 100.0, 2),
           "first_entry_to_last_end_us": round(float(rt1.max() - rt0.min()) / 100.0, 2),
           "wave_span_us_mean": round(float(np.mean(rt1 - rt0)) / 100.0, 2),
           "clock_ghz": round(float(np.mean((s[:, :, 12] - s[:, :, 1]) / np.maximum(rt1 - rt0, 1))) / 10.0, 3),
           "prologue_cyc": round(float(np.mean(s[:, :, 2] - s[:, :, 1])), 1),
           "to_first_unit_cyc": round(float(np.mean(s[:, :, 3] - s[:, :, 2])), 1),
           "units": nu}
    ends = [units[:, :, k + 1] if k + 1 < nu else s[:, :, 11] for k in range(nu)]
    out["unit_cyc"] = [round(float(np.mean(ends[k] - units[:, :, k])), 1) for k in range(nu)]
    out["epilogue_cyc"] = round(float(np.mean(s[:, :, 12] - s[:, :, 11])), 1)
    # where the end skew comes from: loop-end times (realtime clock, us after the first entry) by
    # XCD (workgroup i runs on XCD i % 8) and by wave slot, and their spread
    loop_end_rt = rt0 + (s[:, :, 11] - s[:, :, 1]) / np.maximum((s[:, :, 12] - s[:, :, 1]) / np.maximum(rt1 - rt0, 1), 1e-9)
    le = (loop_end_rt - rt0.min()) / 100.0
    out["loop_end_us_by_xcd"] = [round(float(le[x::8].mean()), 2) for x in range(8)]
    out["loop_end_us_by_wave"] = [round(float(le[:, w].mean()), 2) for w in range(4)]
    out["loop_end_us_pct"] = {q: round(float(np.percentile(le, q)), 2) for q in (0, 10, 50, 90, 100)}
    out["entry_us_by_xcd"] = [round(float(((rt0 - rt0.min()) / 100.0)[x::8].mean()), 2) for x in range(8)]
    out["epi_wait_first_barrier_cyc"] = round(float(np.mean(s[:, :, 14] - s[:, :, 11])), 1)
    out["epi_wg_loop_end_spread_cyc"] = round(float(np.mean(s[:, :, 11].max(axis=1) - s[:, :, 11].min(axis=1))), 1)
    out["epi_lds_sums_cyc"] = round(float(np.mean(s[:, :, 15] - s[:, :, 14])), 1)
    out["epi_slab_write_cyc"] = round(float(np.mean(s[:, :, 12] - s[:, :, 15])), 1)
    return out


def main():
    if os.environ.get("BATCHES"):
        res = {}
        for B in [int(b) for b in os.environ["BATCHES"].split(",")]:
            res[B] = run(B)
        print(json.dumps(res, indent=1))
        return
    print(json.dumps(run(int(os.environ.get("BATCH", "65536"))), indent=1))


def run(B):
    eng = NCFEngine(138493, 27278, [128, 64, 32, 16], 64, max_batch=B, fb_kernel="wave")
    eng.set_keras_weights(initial_weights(138493, 27278, [128, 64, 32, 16], 64, seed=0))
    g = torch.Generator(device="cuda").manual_seed(1)
    u = torch.randint(0, 138493, (B // 4,), generator=g, device="cuda", dtype=torch.int32).repeat_interleave(4)
    it = torch.randint(0, 27278, (B,), generator=g, device="cuda", dtype=torch.int32)
    y = torch.tensor([0., 0., 0., 1.], device="cuda").repeat(B // 4)
    # counted ahead (the bench's form: the index filled by the weight-gradient waves)
    for _ in range(5):
        eng.train_step(u, it, y, group=4, k=3, next_batch=(u, it))
    N.profile_enable([N.K_FWD_BWD], 4)
    eng.train_step(u, it, y, group=4, k=3, next_batch=(u, it))
    torch.cuda.synchronize()
    ms, cnt = N.profile_read(N.K_FWD_BWD)
    fn = N.lib().ncf_debug_wave_timing
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(256 * 4 * 2 * 10, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(256, 4, 2, 10).astype(np.int64)
    res = {"kernel_ms": ms / max(cnt, 1)}
    res["segments"] = {name: round(float(np.mean(t[:, :, :, b] - t[:, :, :, a])), 1) for name, a, b in SEG}
    res["unit_total"] = round(float(np.mean(t[:, :, :, 7] - t[:, :, :, 0])), 1)
    res["unit_to_unit"] = round(float(np.mean(t[:, :, 1, 0] - t[:, :, 0, 0])), 1)
    start = t[:, :, 0, 0].min(axis=1)
    res["prologue_to_first_unit"] = round(float(np.mean(t[:, :, 0, 0] - t[:, :, 0, 8])), 1)
    res["wg_span"] = round(float(np.mean(t[:, 0, 0, 9] - start)), 1)
    res["spans"] = spans("ncf_debug_wave_spans")
    return res


if __name__ == "__main__":
    main()
