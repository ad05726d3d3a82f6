"""Kernel timeline of bench.py's timed region from a rocprofv3 kernel trace: every kernel from the
pre-region flush (the first k_emb_flush) to the end-of-region flush (the last), with start offset,
duration and the idle gap before it (microseconds).
Usage: python tools/region_timeline.py TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
fl = [i for i, r in enumerate(rows) if "k_emb_flush" in r["Kernel_Name"]]
a, b = fl[-2], fl[-1]
t0 = int(rows[a]["End_Timestamp"])
prev = t0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%9.1f %7.1f %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, r["Kernel_Name"][:60]))
    prev = max(prev, e)
print("pre-region flush end -> end-of-region flush end: %.1f us" % ((prev - t0) / 1e3))
