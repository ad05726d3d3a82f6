# GPU box: focused tests (TESTS=...), then bench lines (BENCHES="name:args;name:args").
# KEXPR: optional pytest -k expression.  Usage: TESTS="tests/x.py -k y" BENCHES="C:--steps 50;D:--config D --steps 50" bash tools/gpu_step.sh OUT
export TMPDIR=/tmp
O=${1:-gpurun_out/step}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS -m gpu ${KEXPR:+-k "$KEXPR"} > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -30; tail -60 $O/tests.log; exit 1; }
  grep -cE "PASSED" $O/tests.log; tail -1 $O/tests.log
fi
IFS=';' read -ra BS <<< "$BENCHES"
for b in "${BS[@]}"; do
  [ -z "$b" ] && continue
  name=${b%%:*}; args=${b#*:}
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name failed"; tail -20 $O/bench_$name.err; exit 1; }
  python - "$O/bench_$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {}); e = d.get("roofline_emb_update") or d.get("roofline_fwd_bwd") or {}
print(sys.argv[2], "%.1f M" % (d["value"] / 1e6), "%.4f ms/step" % d["ms_per_step"], "roof %s %.3f (%s ms)" % (r.get("kernel", "")[:30], r.get("frac") or 0, r.get("avg_launch_ms")),
      "other %.3f (%s ms)" % (e.get("frac") or 0, e.get("avg_launch_ms")), "idx", d.get("index_build_ms"), "cu", d.get("catchup_ms"), d.get("exchange", ""))
PY
done
