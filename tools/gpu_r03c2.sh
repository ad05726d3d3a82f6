# round 3: count (+ catch-up ahead) blocks' contributions per pass: 8 below 32,768 contributions (ps8),
# 32 at >= 65,536 (pm32) vs main (16 / 64)
export TMPDIR=/tmp
O=gpurun_out/r03c2; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
b() { name=$1; lib=$2; shift 2; timeout -k 10 300 env NCF_LIB=$lib python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); u=d.get('roofline_emb_update') or d['roofline']; print('%-16s %8.2f M/s %8.4f ms upd %.4f' % ('$name', d['value']/1e6, d['ms_per_step'], u['avg_launch_ms']))"; }
for rep in 1 2; do
b C8192_main.$rep $L/libmovierec_ncf.so --batch 8192 --steps 200
b C8192_ps8.$rep $L/var/ps8.so --batch 8192 --steps 200
b B_main.$rep $L/libmovierec_ncf.so --config B --steps 200
b B_ps8.$rep $L/var/ps8.so --config B --steps 200
b C_main.$rep $L/libmovierec_ncf.so --steps 50
b C_pm32.$rep $L/var/pm32.so --steps 50
done
echo done
