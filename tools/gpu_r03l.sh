# round 3: user-partitioned step timelines (emulated world 8, 65,536 and 8,192 per rank) and the
# single-table step at the new kernel state; config D at 50 steps
export TMPDIR=/tmp
O=gpurun_out/r03l; mkdir -p $O
cd /tmp
for v in 65536 8192; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_user_$v -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --no-cpu-baseline --dp user --emulate-world 8 --batch $v > $GRAFT_REPO_ROOT/$O/tl_user_$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/tl_user_$v.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tl_C -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/tl_C.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline --config D --steps 50 --warmup 3 > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 1; }
tail -c 300 $O/bench_D.json
echo done
