# round 3: split wave kernel, index fill + sort beside the forward/backward, branch-free scorer
# loop — every GPU test, then same-session A/Bs
export TMPDIR=/tmp
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -30; [ $rc -eq 1 ] || exit 1; }
b() { name=$1; shift; timeout -k 10 300 env "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-28s %8.2f M/s %8.4f ms  dom %s %.4f ms frac %.3f' % ('$name', d['value']/1e6, d['ms_per_step'], r.get('kernel','')[:20], r['avg_launch_ms'], r['frac']))"; }
for rep in 1 2; do
b C_split1_beside1.$rep NCF_WAVE_SPLIT=1 NCF_INDEX_BESIDE=1 python bench.py --no-cpu-baseline --steps 50
b C_split0_beside1.$rep NCF_WAVE_SPLIT=0 NCF_INDEX_BESIDE=1 python bench.py --no-cpu-baseline --steps 50
b C_split1_beside0.$rep NCF_WAVE_SPLIT=1 NCF_INDEX_BESIDE=0 python bench.py --no-cpu-baseline --steps 50
b B_beside1.$rep NCF_INDEX_BESIDE=1 python bench.py --no-cpu-baseline --config B --steps 50
b B_beside0.$rep NCF_INDEX_BESIDE=0 python bench.py --no-cpu-baseline --config B --steps 50
b C8192_beside1.$rep NCF_INDEX_BESIDE=1 python bench.py --no-cpu-baseline --batch 8192 --steps 50
b C8192_beside0.$rep NCF_INDEX_BESIDE=0 python bench.py --no-cpu-baseline --batch 8192 --steps 50
done
b E python bench.py --no-cpu-baseline --config E --steps 3 --warmup 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit 1
grep -E "k_fb_wave|k_emb_adam|k_fill|k_emb_catchup|k_stats" $GRAFT_REPO_ROOT/$O/trace/run_kernel_stats.csv | cut -c1-50,180-
for cfg in "B --config B" "C8192 --batch 8192"; do set -- $cfg; n=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_$n -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/$O/tl_$n.log 2>&1 || exit 1
done
echo done
