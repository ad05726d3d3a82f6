# round 3: small-table index in one workgroup (fill + sort + residue + gate) — all GPU tests, then config B A/B
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { name=$1; sm=$2; shift 2; timeout -k 10 300 env NCF_INDEX_SMALL=$sm python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('%-14s %8.2f M/s %8.4f ms idx %s cu %s' % ('$name', d['value']/1e6, d['ms_per_step'], d.get('index_build_ms'), d.get('catchup_ms')))"; }
for r in 1 2; do
b B_small.$r 1 --config B --steps 200
b B_old.$r 0 --config B --steps 200
done
echo done
