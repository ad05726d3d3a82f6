# round 3: host issue time of the timed region (bench.py's stderr diagnostic)
export TMPDIR=/tmp
O=gpurun_out/r03z2; mkdir -p $O
for a in "--steps 20 --warmup 5" "--steps 100 --warmup 5" "--steps 20 --warmup 5 --no-kernel-timing" "--steps 20 --warmup 5"; do
timeout -k 10 300 python bench.py --no-cpu-baseline $a > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
echo "$a: $(grep 'host issue' $O/b.err) $(python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
done
