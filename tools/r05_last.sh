# GPU box: the whole GPU suite and smoke on the final code, then configs B and C at 8,192.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05_last}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in "B --config B" "C8k --batch 8192"; do set -- $c; n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" --steps 100 --warmup 20 > $O/bench_$n.json 2> $O/bench_$n.err || { echo "$n failed"; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,2), d['ms_per_step'])"
done
