#!/bin/bash
# A/B of two libraries in ONE GPU session at several bench configurations (clocks differ between
# boxes).  Usage: bash tools/exp_ab_batches.sh OUT libA libB   (BENCH_SETS: ";"-separated arg sets)
set -o pipefail
OUT=$1; A=$2; B=$3
mkdir -p $OUT
IFS=';' read -ra SETS <<< "${BENCH_SETS:---config C;--batch 8192;--config B}"
i=0
for args in "${SETS[@]}"; do
  for rep in 1 2; do
    for lib in $A $B; do
      tag=$(basename $lib .so)_s${i}_$rep
      timeout -k 10 120 env NCF_LIB=$lib python bench.py --steps 40 --warmup 5 --no-cpu-baseline $args > $OUT/$tag.json 2> $OUT/$tag.err || { tail -5 $OUT/$tag.err; exit 1; }
      python - $OUT/$tag.json "$tag $args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["roofline_emb_update"] if "roofline_emb_update" in d else d["roofline"]
print(sys.argv[2], round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", "update", e["avg_launch_ms"])
PY
    done
  done
  i=$((i+1))
done
