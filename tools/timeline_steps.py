"""Step timeline of a bench run's kernel trace: the kernels of the last STEPS training steps
before the timed region ends, found by an anchor kernel that runs once per step (default: the
forward/backward), with start offset, duration and the idle gap before each (microseconds).
Usage: python tools/timeline_steps.py run_kernel_trace.csv [anchor_regex] [steps]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_fb_wave|k_fb_unit|k_fb_fused|k_lay_l1f|k_fb_generic")
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
idx = [i for i, r in enumerate(rows) if anchor.search(r["Kernel_Name"])]
# the timed region's steps: anchors before the evaluation (which uses forward-only kernels)
lo, hi = idx[-(steps + 1)], idx[-1]
sel = rows[lo:hi]
t0 = int(sel[0]["Start_Timestamp"])
prev_end = None
busy = 0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("ncf::", "")[:70]
    print("%9.1f %8.1f %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, name))
    prev_end = e if prev_end is None else max(prev_end, e)
span = (prev_end - t0) / 1e3
print("%d steps: span %.1f us (%.1f per step), busy %.1f us" % (steps, span, span / steps, busy / 1e3))
