# GPU box: config E scorer with library variants (VARS="name ..." = movierec/_lib/var/<name>.so)
# beside the in-tree library.  Usage: VARS="a b" bash tools/ab_score.sh OUT
O=${1:-gpurun_out/abs}; mkdir -p $O
export TMPDIR=/tmp
for v in base $VARS; do
  if [ "$v" = base ]; then unset NCF_LIB; else export NCF_LIB=$PWD/movierecommender-tf-trt_amd/movierec/_lib/var/$v.so; fi
  timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['frac'])"
done
