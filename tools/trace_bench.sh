#!/bin/bash
# kernel-trace stats of one default bench run (GPU box): per-kernel average microseconds
R=$PWD
OUT=${1:-gpurun_out/trace}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $R/$OUT/trace.log 2>&1 || exit 1
cd $R && python - <<PY
import csv
for r in csv.DictReader(open("$OUT/trace/run_kernel_stats.csv")):
    print("%-70s %5s %10.1f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
