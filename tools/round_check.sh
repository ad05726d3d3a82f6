#!/bin/bash
# Full GPU-box check (run from the repo root): gpu tests, smoke, default bench line (with the
# CPU baseline), kernel-trace stats of the same bench command, and the FETCH/WRITE PMC passes.
# Usage: bash tools/round_check.sh OUTDIR
set -o pipefail
R=$PWD
OUT=${1:-gpurun_out/check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/gpu_profile.sh $OUT || exit 1
python - <<PY
import csv
for r in csv.DictReader(open("$OUT/trace/run_kernel_stats.csv")):
    print("%-60s %5s %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
cat $OUT/traffic/*.json
