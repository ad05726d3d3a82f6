"""Kernel timeline of one training step taken from the middle of a rocprofv3 kernel trace:
the kernels from the K-th launch of the forward/backward kernel up to the next one, with
durations and the idle gaps before each (microseconds).
Usage: python tools/step_window.py TRACE.csv [K] [fb-kernel-substring]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
fb = sys.argv[3] if len(sys.argv) > 3 else "k_fb_"
idx = [i for i, r in enumerate(rows) if fb in r["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
prev = None
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print("%8.1f %7.1f %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r["Kernel_Name"][:100]))
    prev = e if prev is None else max(prev, e)
print("step (fb start to next fb start): %.1f us" % ((int(rows[b]["Start_Timestamp"]) - t0) / 1e3))
