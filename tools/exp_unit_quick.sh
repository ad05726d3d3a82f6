# unit kernel quick loop: its tests, phase timing (timing build), C 65536 / 8192 bench lines
set -o pipefail
OUT=${1:-gpurun_out/uq}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_unit_kernel_gpu.py tests/test_user_fold_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for us in 2 1; do
NCF_UNIT_SCHED=$us NCF_LIB=movierecommender-tf-trt_amd/movierec/_lib/var/utiming.so BATCH=65536 timeout -k 10 200 python tools/unit_timing.py > $OUT/timing$us.json 2>&1 || { tail -20 $OUT/timing$us.json; exit 1; }
python - $OUT/timing$us.json $us <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read()[open(sys.argv[1]).read().index('{'):])
print("sched", sys.argv[2], 'kernel_ms', round(d['kernel_ms'], 4), 'two units', d['two_units_cycles_mean'])
for n in d['wave0']: print('%-12s' % n, ' '.join('%7.0f' % d['wave%d' % w][n] for w in range(4)))
PY
done
for args in "--config C" "--config C --batch 16384" "--config C --batch 8192" "--config B --precision fp32"; do
  for k in tile unit; do
    tag=$(echo "$args $k" | tr ' ' '_' | tr -d '-')
    NCF_FB_KERNEL=$k timeout -k 10 300 python bench.py $args --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python - $OUT/bench_$tag.json "$args $k" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = {v["bound"]: v for k, v in d.items() if k.startswith("roofline")}
print("%-28s value %.1fM ms/step %.4f fwd_bwd %.4f (frac %.3f) emb %.4f" % (
    sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["mfma"]["avg_launch_ms"], r["mfma"]["frac"], r["hbm"]["avg_launch_ms"]))
PY
  done
done
