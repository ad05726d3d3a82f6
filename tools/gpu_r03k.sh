# round 3: split wave kernel, late contraction (the weight-gradient wave works beside the chain's
# sections past layer 1) vs early; phase stamps; unit/native tests
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
timeout -k 10 600 python -u -m pytest tests/test_unit_kernel_gpu.py tests/test_user_fold_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -30; exit 1; }
NCF_LIB=$L/var/wtiming.so timeout -k 10 120 python tools/wave_timing.py > $O/wtiming_late.json 2> $O/wtiming_late.err || { tail -5 $O/wtiming_late.err; exit 1; }
python -c "
import json; d=json.load(open('$O/wtiming_late.json')); print('late', d['kernel_ms'], d['segments'], d['unit_total'], d['unit_to_unit'], d['spans']['unit_cyc'])"
b() { name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-22s %8.2f M/s %8.4f ms  fb %.4f ms frac %.3f' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac']))"; }
for rep in 1 2; do
b late.$rep python bench.py --no-cpu-baseline --steps 40
b early.$rep NCF_LIB=$L/var/early.so python bench.py --no-cpu-baseline --steps 40
b onewave.$rep NCF_WAVE_SPLIT=0 python bench.py --no-cpu-baseline --steps 40
done
echo done
