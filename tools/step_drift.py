"""Per-step duration along a run, from a rocprofv3 kernel trace (consecutive k_fb_fused starts),
and the mean duration of each kernel in the first and last fifth of the run.
Usage: python tools/step_drift.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if "k_fb_fused" in r["Kernel_Name"]]
d = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
n = len(d)
for k in range(0, n, max(1, n // 10)):
    seg = d[k:k + max(1, n // 10)]
    print("steps %4d-%4d: %.1f us/step" % (k, k + len(seg), sum(seg) / len(seg)))
t0, t1 = starts[0], starts[-1]
span = t1 - t0
for lo, hi, name in ((0.0, 0.2, "first fifth"), (0.8, 1.0, "last fifth")):
    acc = collections.defaultdict(list)
    for r in rows:
        s = int(r["Start_Timestamp"])
        if t0 + lo * span <= s < t0 + hi * span:
            acc[r["Kernel_Name"][:40]].append((int(r["End_Timestamp"]) - s) / 1e3)
    print(name, {k: round(sum(v) / len(v), 1) for k, v in acc.items() if len(v) > 5})
