# round 3: scorer variants — partial unroll (u8), branch-free user loop (nb), both (u8nb): tests + E
export TMPDIR=/tmp
O=gpurun_out/r03m; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
for v in sc_u8 sc_nb sc_u8nb; do
NCF_LIB=$L/var/$v.so timeout -k 10 300 python -u -m pytest tests/test_score_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1
echo "$v tests rc=$?: $(tail -1 $O/tests_$v.log)"
NCF_LIB=$L/var/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --config E --steps 3 --warmup 1 > $O/E_$v.json 2> $O/E_$v.err || { tail -3 $O/E_$v.err; continue; }
python -c "
import json; d=json.loads(open('$O/E_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['ms_per_step'], r['avg_launch_ms'] if 'avg_launch_ms' in r else '', r['frac'])"
done
echo done
