# round 3: flush back to the rows' joint one-step chains: deferred-decay / flush tests + the driver's command
export TMPDIR=/tmp
O=gpurun_out/r03f3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "lazy or deferred or decay or flush or catchup or stale or ahead or dp or user" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d$r.json 2> $O/d$r.err || { tail -5 $O/d$r.err; exit 1; }
python -c "import json; d=json.loads(open('$O/d$r.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'])"
done
