# round 3: split wave kernel (chain waves + weight-gradient waves) — tests, same-session A/B
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_unit_kernel_gpu.py tests/test_user_fold_gpu.py tests/test_headline_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/tests.log | head -20; exit 1; }
for rep in 1 2; do
for sp in 0 1; do
NCF_WAVE_SPLIT=$sp timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > $O/bench_split$sp.$rep.json 2> $O/bench_split$sp.$rep.err || { tail -5 $O/bench_split$sp.$rep.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_split$sp.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('split=$sp', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms', r['avg_launch_ms'], r['frac'])"
done
done
cd /tmp
NCF_WAVE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit 1
grep -E "k_fb_wave|k_emb_adam" $GRAFT_REPO_ROOT/$O/trace/run_kernel_stats.csv | cut -c1-60,200-
