# round 3: stats + step bump folded into the fused row/dense update launch (last workgroup to finish)
export TMPDIR=/tmp
O=gpurun_out/r03s2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "apply_update or user or dp or replicated or fit or stats or metrics" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('%-22s %8.2f M/s %8.4f ms' % ('$name', d['value']/1e6, d['ms_per_step']))"; }
for r in 1 2; do
b user_emul8_b65536.$r --dp user --emulate-world 8 --steps 30 --warmup 5
b user_emul8_b8192.$r --dp user --emulate-world 8 --batch 8192 --steps 30 --warmup 5
b user_w1.$r --dp user --steps 30 --warmup 5
done
echo done
