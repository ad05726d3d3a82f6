# round 3: bench lines for config D (GMF product formed in k_lay_mid) and C at 8,192 (50 / 200 steps)
export TMPDIR=/tmp
O=gpurun_out/r03v2; mkdir -p $O
b() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %8.2f M/s %8.4f ms dom %.4f ms %.3f' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac']))"; }
b D --config D --steps 50 --warmup 3
b C8192_50 --batch 8192 --steps 50
b C8192_200 --batch 8192 --steps 200
b B_200 --config B --steps 200
