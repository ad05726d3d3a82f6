# GPU box: bench lines of the default library and of variants (NCF_LIB), printing the step and the
# forward/backward and touched-row update launch times.  Usage: VARS="a.so b.so" ARGS=... bash tools/r05_var.sh OUT
export TMPDIR=/tmp
O=${1:-gpurun_out/var}; mkdir -p $O
for i in $(seq 1 ${REPS:-1}); do
for v in base $VARS; do
  if [ $v = base ]; then unset NCF_LIB; else export NCF_LIB=$PWD/movierecommender-tf-trt_amd/movierec/_lib/var/$v; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline ${ARGS:---steps 50} > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v failed"; tail -5 $O/${v}_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; u=d.get('roofline_emb_update') or {}; print('%-10s %6.1f M %.4f ms fb %.4f upd %s' % ('$v', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], u.get('avg_launch_ms')))"
done
done
unset NCF_LIB
