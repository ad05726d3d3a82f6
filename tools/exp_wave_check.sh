#!/bin/bash
# Wave/unit-kernel change check on the GPU box: the tests that run them (oracle parity incl.
# config C full size, unit/tile comparison, folding, bf16), span stamps at several batches, a
# default bench line, config B and 8192-sample lines.  Usage: bash tools/exp_wave_check.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/wcheck}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_unit_kernel_gpu.py \
    tests/test_user_fold_gpu.py tests/test_headline_parity_gpu.py tests/test_bf16_gpu.py > $OUT/tests.log 2>&1 \
    || { tail -30 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
bash tools/exp_span.sh $OUT || exit 1
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --config B > $OUT/bench_B.json 2> $OUT/bench_B.err \
    || { tail -20 $OUT/bench_B.err; exit 1; }
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --batch 8192 > $OUT/bench_8192.json 2> $OUT/bench_8192.err \
    || { tail -20 $OUT/bench_8192.err; exit 1; }
python - $OUT <<'PY'
import json, sys
for f in ("bench", "bench_B", "bench_8192"):
    d = json.loads(open("%s/%s.json" % (sys.argv[1], f)).read().strip().splitlines()[-1])
    fb = d["roofline"] if d["roofline"]["bound"] == "mfma" else d.get("roofline_fwd_bwd")
    print(f, round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", "fb", fb["avg_launch_ms"], fb["frac"])
PY
