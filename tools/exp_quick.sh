# quick GPU check after a kernel change: the deferred-decay / count-ahead bitwise tests, the
# headline parity test, the catch-up probe and a default bench line.  Usage: bash tools/exp_quick.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/quick}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_headline_parity_gpu.py "tests/test_native_gpu.py::test_lazy_decay_bitwise_equals_dense_sweep" tests/test_native_gpu.py::test_count_ahead_equals_plain_steps tests/test_native_gpu.py::test_counted_ahead_ids_changed_in_place -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python tools/catchup_probe.py --steps 60 > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
tail -1 $OUT/probe.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = {v["bound"]: v for k, v in d.items() if k.startswith("roofline")}
print("value %.1fM ms/step %.4f fwd_bwd %.4f (frac %.3f) emb %.4f catchup %s index %s eval %s" % (
    d["value"] / 1e6, d["ms_per_step"], r["mfma"]["avg_launch_ms"], r["mfma"]["frac"], r["hbm"]["avg_launch_ms"],
    d["catchup_ms"], d["index_build_ms"], d["hr_at_10"].get("eval_ms")))
PY
