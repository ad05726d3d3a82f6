export TMPDIR=/tmp
O=gpurun_out/r04_k; mkdir -p $O
for i in 1 2; do
 for which in r03 r04; do
  if [ $which = r03 ]; then B="python _ab_r03/bench.py"; else B="python bench.py"; fi
  timeout -k 10 200 $B --no-cpu-baseline --config B --steps 50 > $O/B_${which}_$i.json 2> $O/B_${which}_$i.err || exit 1
  python -c "import json; d=json.loads(open('$O/B_${which}_$i.json').read().strip().splitlines()[-1]); print('$which', $i, d['ms_per_step'], d['roofline']['avg_launch_ms'])"; grep host $O/B_${which}_$i.err
 done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --config B --steps 50 --no-kernel-timing > $O/B_nokt.json 2> $O/B_nokt.err && grep host $O/B_nokt.err
