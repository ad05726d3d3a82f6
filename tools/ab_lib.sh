# GPU box: same-session A/B of the default library against a variant (NCF_LIB), bench lines
# alternating.  Usage: VAR=movierec/_lib/var/x.so ARGS="--steps 50" REPS=2 bash tools/ab_lib.sh OUT
export TMPDIR=/tmp
O=${1:-gpurun_out/ab}; mkdir -p $O
V=$PWD/movierecommender-tf-trt_amd/$VAR
for i in $(seq 1 ${REPS:-2}); do
  for which in base var; do
    if [ $which = var ]; then export NCF_LIB=$V; else unset NCF_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > $O/${which}_$i.json 2> $O/${which}_$i.err || { echo "$which $i failed"; tail -5 $O/${which}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/${which}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$which', $i, round(d['value']/1e6,1), d['ms_per_step'], r['kernel'][:24], r['avg_launch_ms'], r['frac'])"
  done
done
unset NCF_LIB
