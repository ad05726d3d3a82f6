# round 3: A/B of the stats tail in the fused row/dense update launch (main) vs its own launch (notail)
export TMPDIR=/tmp
O=gpurun_out/r03s3; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
b() { name=$1; lib=$2; shift 2; timeout -k 10 300 env NCF_LIB=$lib python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('%-22s %8.2f M/s %8.4f ms' % ('$name', d['value']/1e6, d['ms_per_step']))"; }
for r in 1 2; do
for v in main notail; do
lib=$L/libmovierec_ncf.so; [ $v = main ] || lib=$L/var/$v.so
b e8_65536_$v.$r $lib --dp user --emulate-world 8 --steps 30 --warmup 5
b e8_8192_$v.$r $lib --dp user --emulate-world 8 --batch 8192 --steps 30 --warmup 5
done
done
echo done
