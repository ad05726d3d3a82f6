# round 3: split wave kernel diagnosis — phase stamps split vs one-wave; A/B of priority, of the
# weight-gradient waves' work and of the per-unit barrier
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
L=movierecommender-tf-trt_amd/movierec/_lib
for sp in 1 0; do
NCF_WAVE_SPLIT=$sp NCF_LIB=$L/var/wtiming.so timeout -k 10 120 python tools/wave_timing.py > $O/wtiming_split$sp.json 2> $O/wtiming_split$sp.err || { tail -5 $O/wtiming_split$sp.err; exit 1; }
python -c "
import json; d=json.load(open('$O/wtiming_split$sp.json')); print('split=$sp', d['kernel_ms'], d['segments'], d['unit_total'], d['unit_to_unit'], d['spans']['unit_cyc'], d['spans']['prologue_cyc'], d['spans']['epilogue_cyc'])"
done
b() { name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-22s %8.2f M/s %8.4f ms  fb %.4f ms frac %.3f' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac']))"; }
for rep in 1 2; do
b main.$rep python bench.py --no-cpu-baseline --steps 40
b onewave.$rep NCF_WAVE_SPLIT=0 python bench.py --no-cpu-baseline --steps 40
b prio0.$rep NCF_LIB=$L/var/prio0.so python bench.py --no-cpu-baseline --steps 40
b nodw.$rep NCF_LIB=$L/var/nodw.so python bench.py --no-cpu-baseline --steps 40
b nosync.$rep NCF_LIB=$L/var/nosync.so python bench.py --no-cpu-baseline --steps 40
done
echo done
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_unit_kernel_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -30; [ $rc -eq 1 ] || exit 1; }
for rep in 1 2; do
b B.$rep python bench.py --no-cpu-baseline --config B --steps 50
b C8192.$rep python bench.py --no-cpu-baseline --batch 8192 --steps 50
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_B -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --config B > $GRAFT_REPO_ROOT/$O/tl_B.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_D -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --config D > $GRAFT_REPO_ROOT/$O/tl_D.log 2>&1 || exit 1
echo done2
