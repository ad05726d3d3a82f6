# round 3: one launch group per sampled step in bench.py; replay step without v's "+ 0"
export TMPDIR=/tmp
O=gpurun_out/r03z4; mkdir -p $O
true
true
b() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; u=d.get('roofline_emb_update') or d.get('roofline_fwd_bwd'); print('%-10s %8.2f M/s %8.4f ms fb %.4f (%s) upd %.4f %s idx %s cu %s' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac'], u['avg_launch_ms'], u['timed_steps'][-20:], d['index_build_ms'], d['catchup_ms']))"; }
b s20.1 --gpus 1 --steps 20 --warmup 5
b s20.2 --gpus 1 --steps 20 --warmup 5
b s50 --steps 50
b s20.3 --gpus 1 --steps 20 --warmup 5
b C8192 --batch 8192 --steps 200
echo done
