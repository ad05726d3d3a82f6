# every bench configuration and layout once (1 GPU): regression check of the non-default paths.
# Usage: bash tools/exp_configs.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/configs}
mkdir -p $OUT
for args in "--config A" "--config B" "--config B --precision fp32" "--config D --steps 10 --warmup 3" "--config E" \
            "--config C --dp user" "--config C --dp sharded" "--config C --dp replicated" "--config C --e2e"; do
  tag=$(echo "$args" | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py $args --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { echo "FAILED $args"; tail -20 $OUT/bench_$tag.err; exit 1; }
  python - $OUT/bench_$tag.json "$args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print("%-36s %s %.4g %s  ms/step %s  roofline %s frac %s  path %s" % (sys.argv[2], d["metric"][:30], d["value"], d["unit"],
      d.get("ms_per_step"), r.get("bound"), r.get("frac"), d.get("config", {}).get("kernel_path")))
PY
done
