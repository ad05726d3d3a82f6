# A/B of an environment knob on the default bench line, alternating runs.
# Usage: bash tools/exp_env_ab.sh OUT VAR "val1 val2" [rounds]
set -o pipefail
OUT=$1; VAR=$2; VALS=$3; R=${4:-2}
mkdir -p $OUT
for r in $(seq $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { tail -20 $OUT/bench_${v}_$r.err; exit 1; }
    python - $OUT/bench_${v}_$r.json "$VAR=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = {v["bound"]: v for k, v in d.items() if k.startswith("roofline")}
print("%-18s value %.1fM ms/step %.4f fwd_bwd %.4f emb %.4f catchup %s index %s" % (
    sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["mfma"]["avg_launch_ms"], r["hbm"]["avg_launch_ms"],
    d["catchup_ms"], d["index_build_ms"]))
PY
  done
done
