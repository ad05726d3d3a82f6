# round 3: config D layers 2.. fused into one hand-written MFMA kernel (ncf_laymid.hip) — tests, A/B
export TMPDIR=/tmp
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py tests/test_config_d_gpu.py tests/test_distributed.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -40; exit 1; }
b() { name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-16s %8.2f M/s %8.4f ms  fb %.4f ms frac %.3f eval %s' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['hr_at_10']['eval_ms']))"; }
for rep in 1 2; do
b D_mid.$rep python bench.py --no-cpu-baseline --config D --steps 30 --warmup 3
b D_blas.$rep NCF_LAYMID_MFMA=0 python bench.py --no-cpu-baseline --config D --steps 30 --warmup 3
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_D -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --config D > $GRAFT_REPO_ROOT/$O/tl_D.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/step_window.py $O/tl_D/run_kernel_trace.csv 3 k_lay_l1f | cut -c1-110
echo done
