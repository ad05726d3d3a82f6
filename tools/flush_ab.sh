#!/bin/bash
# Kernel-trace averages of the catch-up kernels (k_emb_catchup<true> is the bench's end-of-region
# flush) for each library given (GPU box, repo root).  Usage: bash tools/flush_ab.sh OUT lib...
R=$PWD; OUT=$1; shift
mkdir -p $OUT
for lib in "$@"; do
  tag=$(basename $lib .so)
  cd /tmp && export TMPDIR=/tmp
  NCF_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/$tag -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/$OUT/$tag.log 2>&1 || { tail -5 $R/$OUT/$tag.log; exit 1; }
  cd $R
  python - $OUT/$tag/run_kernel_stats.csv $tag <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "catchup" in r["Name"] or "row_step_fill" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
