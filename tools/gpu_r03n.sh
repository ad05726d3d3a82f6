# round 3: index fill for large key spaces (k_prefix + k_fill_big) — config D tests, sharded D,
# config D bench at 50 steps, native tests
export TMPDIR=/tmp
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_config_d_gpu.py tests/test_distributed.py tests/test_native_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --config D --steps 50 --warmup 3 > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_D.json').read().strip().splitlines()[-1]); print('D', d['value']/1e6, d['ms_per_step'], d['index_build_ms'], d['catchup_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_D -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --config D > $GRAFT_REPO_ROOT/$O/tl_D.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/step_window.py $O/tl_D/run_kernel_trace.csv 3 k_lay_gather4 | cut -c1-110
echo done
