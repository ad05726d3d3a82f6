#!/bin/bash
# Every GPU test, smoke, then a default bench line (no CPU baseline) and the config B / 8192 lines.
# Usage: bash tools/exp_full_check.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/full}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 \
    || { tail -30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
for c in "C:" "B:--config B" "C8192:--batch 8192"; do
    name=${c%%:*}; args=${c#*:}
    timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { tail -20 $OUT/bench_$name.err; exit 1; }
done
python - $OUT <<'PY'
import json, sys
for f in ("C", "B", "C8192"):
    d = json.loads(open("%s/bench_%s.json" % (sys.argv[1], f)).read().strip().splitlines()[-1])
    fb = d["roofline"] if d["roofline"]["bound"] == "mfma" else d.get("roofline_fwd_bwd")
    print(f, round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", "fb", fb["avg_launch_ms"], fb["frac"],
          "index", d["index_build_ms"], "catchup", d["catchup_ms"])
PY
