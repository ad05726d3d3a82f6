# fused-kernel experiment on the GPU: fused-path tests, phase timing of the timing build, A/B
# against named variants.  Usage: bash tools/exp_fused.sh OUT variant...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_headline_parity_gpu.py tests/test_native_gpu.py -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
NCF_LIB=movierecommender-tf-trt_amd/movierec/_lib/var/timing.so timeout -k 10 120 python tools/fused_timing.py > $OUT/timing.json 2>&1 || exit 1
python - $OUT/timing.json <<'PY'
import json, sys
t = open(sys.argv[1]).read(); d = json.loads(t[t.index('{'):])
for w in ("wave0", "wave3"):
    print(w, round(d["kernel_ms"], 4), {k: int(v) for k, v in d[w].items() if v})
PY
bash tools/exp_ab.sh $OUT "$@"
