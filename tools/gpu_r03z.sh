# round 3: why the driver's 20-step form reads lower than 50 steps — warm-up length, step count, repeat
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
b() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('%-14s %8.2f M/s %8.4f ms fb %.4f upd %.4f' % ('$name', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_emb_update']['avg_launch_ms']))"; }
b s20w5.1 --steps 20 --warmup 5
b s20w30 --steps 20 --warmup 30
b s100w5 --steps 100 --warmup 5
b s20w5.2 --steps 20 --warmup 5
b s50w10 --steps 50 --warmup 10
b s20w5.3 --steps 20 --warmup 5
echo done
