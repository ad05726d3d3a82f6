#!/bin/bash
# Kernel-trace stats of the user-partitioned step at an emulated world of 8 (GPU box, repo root).
R=$PWD
OUT=${1:-gpurun_out/trace_user}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --dp user --emulate-world 8 > $R/$OUT/trace.log 2>&1 || { tail -20 $R/$OUT/trace.log; exit 1; }
cd $R && python - $OUT <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_stats.csv")):
    if r["Name"].startswith(("ncf", "void ncf")):
        print("%-80s %5s %10.2f" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
