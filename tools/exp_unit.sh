# unit-kernel check: its tests, then the tile and unit kernels on config C (65536, 8192) and B.
# Usage: bash tools/exp_unit.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/unit}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_unit_kernel_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for args in "--config C" "--config C --batch 8192" "--config B"; do
  for k in tile unit; do
    tag=$(echo "$args $k" | tr ' ' '_' | tr -d '-')
    NCF_FB_KERNEL=$k timeout -k 10 300 python bench.py $args --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
    python - $OUT/bench_$tag.json "$args $k" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = {v["bound"]: v for k, v in d.items() if k.startswith("roofline")}
print("%-28s value %.1fM ms/step %.4f fwd_bwd %.4f (frac %.3f) emb %.4f kernel %s" % (
    sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["mfma"]["avg_launch_ms"], r["mfma"]["frac"],
    r["hbm"]["avg_launch_ms"], d["config"]["kernel_path"]))
PY
  done
done
