# round 3: the driver's own bench command (20 steps, 5 warm-up) twice, and one run with the CPU baseline's full protocol
export TMPDIR=/tmp
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_form.1.json 2> $O/driver_form.1.err || { tail -5 $O/driver_form.1.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_form.2.json 2> $O/driver_form.2.err || { tail -5 $O/driver_form.2.err; exit 1; }
timeout -k 10 600 python bench.py --cpu-protocol full > $O/cpu_full.json 2> $O/cpu_full.err || { tail -5 $O/cpu_full.err; exit 1; }
for f in $O/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d.get('cpu_baseline') or {}; print('$f', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac'], c.get('value'), c.get('sample'))"; done
