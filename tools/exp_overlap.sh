# index-build overlap check (GPU box): tests, bench with/without the side stream, kernel trace
OUT=gpurun_out/r19; mkdir -p $OUT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/t.log 2>&1; tail -2 $OUT/t.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_main.json 2>/dev/null || exit 1
NCF_SIDE_STREAM=0 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_noside.json 2>/dev/null || exit 1
python tools/summarize_exp.py $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
