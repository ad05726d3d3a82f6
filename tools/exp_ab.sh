# A/B of library variants (built with csrc/build.py -D ... --out movierec/_lib/var/<name>.so) on the
# default bench line; "default" = the in-tree library.  Usage: bash tools/exp_ab.sh OUT name...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
for v in "$@"; do
  if [ $v = default ]; then L=""; else L=movierecommender-tf-trt_amd/movierec/_lib/var/$v.so; fi
  NCF_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -20 $OUT/bench_$v.err; exit 1; }
  python - $OUT/bench_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = {v["bound"]: v for k, v in d.items() if k.startswith("roofline")}
print("%-10s value %.1fM ms/step %.4f fwd_bwd %.4f emb %.4f catchup %s index %s" % (
    sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["mfma"]["avg_launch_ms"], r["hbm"]["avg_launch_ms"],
    d["catchup_ms"], d["index_build_ms"]))
PY
done
