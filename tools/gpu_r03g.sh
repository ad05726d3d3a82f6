# round 3 baseline measurements at the re-entry state: kernel trace + PMC traffic of the default
# bench, MFMA busy, the user layout (world 1, emulated world 8 at 65,536 and 8,192 per rank), other
# configs, small batches, the trainer-style epoch bench
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O
bash tools/gpu_profile.sh $O || exit 1
bash tools/pmc_mfma.sh $O/pmc_mfma > $O/pmc_mfma.txt 2>&1 || { cat $O/pmc_mfma.txt; exit 1; }
run() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { echo "$name failed"; tail -5 $O/bench_$name.err; exit 1; }; python -c "
import json,sys; d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1]); print('$name', round(d.get('value')/1e6,2), 'M', d.get('unit'), d.get('ms_per_step'), 'ms', (d.get('roofline') or {}).get('avg_launch_ms'), (d.get('roofline') or {}).get('frac'))"; }
run user_w1 --dp user --steps 30 --warmup 5
run user_emul8_b65536 --dp user --emulate-world 8 --steps 30 --warmup 5
run user_emul8_b8192 --dp user --emulate-world 8 --batch 8192 --steps 30 --warmup 5
run C_b8192 --batch 8192 --steps 50
run B --config B --steps 50
run A --config A --steps 50
run D --config D --steps 10 --warmup 2
run E --config E --steps 3 --warmup 1
run e2e --e2e
run fit --fit-epochs
echo done
