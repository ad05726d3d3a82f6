# GPU box: the other configs' bench lines with the final round-5 code (B, C at 8,192, D, E, A).
export TMPDIR=/tmp
O=${1:-gpurun_out/r05_cfgs}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "$n failed"; tail -5 $O/bench_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', round(d['value']/1e6,2), d['unit'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('frac'))"; }
run B --config B --steps 100 --warmup 20
run C8k --batch 8192 --steps 100 --warmup 20
run D --config D --steps 30 --warmup 5
run E --config E --steps 5 --warmup 2
run A --config A --steps 50 --warmup 10
run U8s --dp user --emulate-world 8 --batch 8192 --steps 100 --warmup 20
