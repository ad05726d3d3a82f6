#!/bin/bash
# The other bench configurations after a change (GPU box): config A, D (layered, 11 GB table),
# E (all-item scoring), the on-device sampler (--e2e), the row-sharded layout at world 1.
set -o pipefail
OUT=${1:-gpurun_out/other}
mkdir -p $OUT
for c in "A:--config A" "D:--config D --steps 10 --warmup 2" "E:--config E --steps 3 --warmup 1" "e2e:--e2e" "sharded:--dp sharded --steps 10"; do
    name=${c%%:*}; args=${c#*:}
    timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { echo "$name failed"; tail -5 $OUT/bench_$name.err; exit 1; }
    python - $OUT/bench_$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("value"), d.get("unit"), d.get("ms_per_step"))
PY
done
