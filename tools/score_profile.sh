#!/bin/bash
# Config E (all-item scoring) bench line + kernel-trace stats of the same command (GPU box)
R=$PWD
OUT=${1:-gpurun_out/score}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 > $OUT/bench_E.json 2> $OUT/bench_E.err || { tail -20 $OUT/bench_E.err; exit 1; }
cat $OUT/bench_E.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python $R/bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/trace.log 2>&1 || exit 1
cd $R && python - <<PY
import csv
for r in csv.DictReader(open("$OUT/trace/run_kernel_stats.csv")):
    print("%-60s %5s %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
