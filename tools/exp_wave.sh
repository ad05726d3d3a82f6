#!/bin/bash
# Wave-chain kernel A/B on the GPU box: its GPU tests, then config C bench lines for the wave and
# unit kernels.  Usage: bash tools/exp_wave.sh OUT [pytest -k expr]
set -e
OUT=${1:-gpurun_out/wave}
mkdir -p $OUT
K=${2:-wave}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unit_kernel_gpu.py tests/test_user_fold_gpu.py -k "$K" > $OUT/tests.log 2>&1
timeout -k 10 120 env NCF_FB_KERNEL=wave python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_wave.json 2> $OUT/bench_wave.err
timeout -k 10 120 env NCF_FB_KERNEL=wave python bench.py --steps 30 --warmup 5 --no-cpu-baseline --batch 8192 > $OUT/bench_wave_8192.json 2> $OUT/bench_wave_8192.err
python - $OUT <<'PY'
import json, sys
for f in ("bench_wave", "bench_wave_8192"):
    d = json.loads(open("%s/%s.json" % (sys.argv[1], f)).read().strip().splitlines()[-1])
    fb = d["roofline"] if d["roofline"]["bound"] == "mfma" else d.get("roofline_fwd_bwd")
    print(f, round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", "fb", fb["avg_launch_ms"], fb["frac"])
PY
