#!/bin/bash
# Round-3 end evidence (second pass) on the GPU box (repo root): every GPU test, smoke, the default bench line
# with the CPU baseline, kernel-trace stats + FETCH/WRITE PMC traffic (tools/gpu_profile.sh), the
# MFMA-busy pass, the other configurations (A and B with their CPU baselines), the user layout.
# Usage: bash tools/final_r03.sh OUT
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=20 > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C", round(d["value"] / 1e6, 2), "M/s", d["ms_per_step"], "ms", d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"])
PY
bash tools/gpu_profile.sh $OUT || exit 1
bash tools/pmc_mfma.sh $OUT/pmc_mfma > $OUT/pmc_mfma.txt 2>&1 || { cat $OUT/pmc_mfma.txt; exit 1; }
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "$name failed"; tail -5 $OUT/bench_$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); c=d.get('cpu_baseline') or {}; print('$name', round(d['value']/1e6,3), 'M', d['unit'], d['ms_per_step'], 'ms; dominant', (d.get('roofline') or {}).get('avg_launch_ms'), (d.get('roofline') or {}).get('frac'), '; cpu', c.get('value'))"; }
run A --config A --steps 50
run B --config B --steps 50
run C_b8192 --no-cpu-baseline --batch 8192 --steps 200
run driver_form --gpus 1 --steps 20 --warmup 5
run D --no-cpu-baseline --config D --steps 50 --warmup 3
run E --no-cpu-baseline --config E --steps 3 --warmup 1
run e2e --no-cpu-baseline --e2e
run fit --no-cpu-baseline --fit-epochs
run user_w1 --no-cpu-baseline --dp user --steps 30 --warmup 5
run user_emul8_b65536 --no-cpu-baseline --dp user --emulate-world 8 --steps 30 --warmup 5
run user_emul8_b8192 --no-cpu-baseline --dp user --emulate-world 8 --batch 8192 --steps 30 --warmup 5
echo done
