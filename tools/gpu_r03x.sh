# round 3: zero-gradient replays U steps at a time (replay2) vs the one-step loop (NCF_REPLAY_UNROLL=1 / 2)
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "lazy or deferred or decay or flush or catchup or stale or ahead" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { name=$1; lib=$2; shift 2; timeout -k 10 300 env NCF_LIB=$lib python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d.get('roofline_emb_update') or d['roofline']; print('%-16s %8.2f M/s %8.4f ms upd %.4f ms' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms']))"; }
for rep in 1 2; do
for v in main u1 u2; do
lib=$L/libmovierec_ncf.so; [ $v = main ] || lib=$L/var/$v.so
b C_$v.$rep $lib --steps 50
b C8192_$v.$rep $lib --batch 8192 --steps 200
b B_$v.$rep $lib --config B --steps 200
done
done
echo done
