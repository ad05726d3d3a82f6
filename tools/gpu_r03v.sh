# round 3: config D without the GMF product pass (k_lay_mid forms it from the rows); C at 8,192 re-check
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_config_d_gpu.py tests/test_native_gpu.py -k "layered or config_d or large_key" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %8.2f M/s %8.4f ms dom %.4f ms %.3f' % ('$name', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac']))"; }
b D --config D --steps 50 --warmup 3
b C8192.1 --batch 8192 --steps 50
b C8192.2 --batch 8192 --steps 200
b C.1 --steps 50
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/tr8192 -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --batch 8192 --steps 20 > $GRAFT_REPO_ROOT/$O/tr8192.log 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trD -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --config D --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/trD.log 2>&1 || exit 1
echo done
