# tests + bench + kernel-trace stats of the same bench command (GPU box)
OUT=${1:-gpurun_out/bp}; mkdir -p $OUT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/t.log 2>&1; tail -2 $OUT/t.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_main.json 2>/dev/null || exit 1
python tools/summarize_exp.py $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/trace_bench.json 2>/dev/null
cd $GRAFT_REPO_ROOT && python - <<PY
import csv
for r in csv.DictReader(open("$OUT/trace/run_kernel_stats.csv")):
    print("%-60s %5s %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
