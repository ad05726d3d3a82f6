# GPU box: one bench line per secondary configuration: B, C at 8,192, the emulated
# 8-rank user-partitioned step (8,192 and 65,536 per rank), D; with ALL=1 also E (the scorer) and A.
# Usage: [ALL=1] bash tools/configs.sh OUT
export TMPDIR=/tmp
O=${1:-gpurun_out/configs}; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-10s %8.1f M/s %8.4f ms/step  fb %s %s frac %s' % ('$name', d['value']/1e6, d['ms_per_step'], r['kernel'][:20], r.get('avg_launch_ms'), r['frac']))"; }
run B --config B --steps 100 --warmup 20 && run C8k --config C --batch 8192 --steps 100 --warmup 20 && run U8 --config C --dp user --emulate-world 8 --batch 8192 --steps 50 --warmup 10 && run U8b --config C --dp user --emulate-world 8 --steps 50 --warmup 10 && run D --config D --steps 30 --warmup 5 || exit 1
if [ -n "$ALL" ]; then
  run E --config E --steps 5 --warmup 2 && run A --config A --steps 50 --warmup 10 || exit 1
fi
if [ -n "$TRACE_B" ]; then
  bash tools/trace_var.sh $O/traceB "" --config B --steps 100 --warmup 20 > $O/traceB.log 2>&1 && head -14 $O/traceB.log
fi
