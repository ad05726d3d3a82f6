# GPU box: every GPU test, smoke, the driver's bench command and config D. Usage: bash tools/gpu_check.sh OUT
export TMPDIR=/tmp
O=${1:-gpurun_out/check}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --config D --steps 50 --warmup 3 > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_D.json').read().strip().splitlines()[-1]); print('D', d['value']/1e6, d['ms_per_step'])"
