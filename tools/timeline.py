"""Print the dispatch timeline of the last N kernels of a rocprofv3 kernel trace:
start offset, duration and the idle gap before each kernel (microseconds).
Usage: python tools/timeline.py gpurun_out/timeline/tl/run_kernel_trace.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = rows[-n:]
t0 = int(sel[0]["Start_Timestamp"])
prev_end = None
busy = 0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    print("%9.1f %8.1f %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r["Kernel_Name"][:90]))
    prev_end = e if prev_end is None else max(prev_end, e)
print("span %.1f us, busy %.1f us" % ((prev_end - t0) / 1e3, busy / 1e3))
