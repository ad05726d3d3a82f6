# GPU box: in-kernel index tests (the unsorted update path), update-pipeline A/B at C, C 8,192, B,
# and a kernel trace of the default bench.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_index_in_kernel_gpu.py tests/test_native_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARS="pipe0.so p2b6.so" REPS=3 bash tools/r05_var.sh $O/C || exit 1
VARS="pipe0.so p2b6.so" REPS=2 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C8k || exit 1
VARS="pipe0.so" REPS=2 ARGS="--config B --steps 100 --warmup 20" bash tools/r05_var.sh $O/B || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/trace_bench.json 2> $GRAFT_REPO_ROOT/$O/trace_bench.err || exit 1
cd $GRAFT_REPO_ROOT && python - <<PY
import csv
for r in csv.DictReader(open("$O/trace/run_kernel_stats.csv")):
    if r["Name"].startswith(("void rocprim", "void at::", "__amd")): continue
    print("%-70s %5s %10.1f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
