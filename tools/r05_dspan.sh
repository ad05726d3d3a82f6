# GPU box: config D row-locality diagnostic (bench --id-span): the touched-row update and the
# forward/backward at user-id spans 1, 0.1 and 0.02 of the 10 M users (the TLB question).
export TMPDIR=/tmp
O=${1:-gpurun_out/r05_dspan}; mkdir -p $O
for sp in 1.0 0.1 0.02 1.0; do
  timeout -k 10 400 python bench.py --config D --steps 30 --warmup 5 --no-cpu-baseline --id-span $sp > $O/D_$sp.json 2> $O/D_$sp.err || { echo "span $sp failed"; tail -5 $O/D_$sp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/D_$sp.json').read().strip().splitlines()[-1]); r=d['roofline']; u=d.get('roofline_emb_update') or d.get('roofline_fwd_bwd') or {}; print('span $sp', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', r.get('kernel','')[:30], r.get('avg_launch_ms'), u.get('kernel','')[:30], u.get('avg_launch_ms'), u.get('replayed_rows_per_step'), u.get('gradient_rows_per_step'))"
done
