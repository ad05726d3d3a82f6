# round 3: scorer with the per-user ballot branch removed (logits always parked) vs the branchy loop
export TMPDIR=/tmp
O=gpurun_out/r03e2; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_score_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { name=$1; lib=$2; shift 2; timeout -k 10 300 env NCF_LIB=$lib python bench.py --no-cpu-baseline --config E --steps 3 --warmup 1 "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %8.2f G pairs/s %8.3f ms kernel %.3f ms %.3f' % ('$name', d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], r['frac']))"; }
for rep in 1 2; do
b free.$rep $L/libmovierec_ncf.so
b branchy.$rep $L/var/branchy.so
done
echo done
