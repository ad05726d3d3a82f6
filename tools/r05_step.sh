# GPU box, round 5: the in-kernel index tests first, then the whole GPU suite, then a same-session
# A/B of the default library against a variant and a kernel trace of the default bench.
# Usage: VAR=movierec/_lib/var/x.so bash tools/r05_step.sh OUT   (SKIP_SUITE=1: new tests only)
export TMPDIR=/tmp
O=${1:-gpurun_out/r05}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_index_in_kernel_gpu.py -m gpu > $O/tests_new.log 2>&1 || { tail -60 $O/tests_new.log; exit 1; }
tail -1 $O/tests_new.log
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests_all.log 2>&1 || { tail -60 $O/tests_all.log; exit 1; }
  tail -1 $O/tests_all.log
fi
if [ -n "$VAR" ]; then
  VAR=$VAR ARGS="${ARGS:---steps 50}" REPS=${REPS:-2} bash tools/ab_lib.sh $O/ab || exit 1
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/trace_bench.json 2> $GRAFT_REPO_ROOT/$O/trace_bench.err || exit 1
cd $GRAFT_REPO_ROOT && python - <<PY
import csv
for r in csv.DictReader(open("$O/trace/run_kernel_stats.csv")):
    if r["Name"].startswith(("void rocprim", "void at::", "__amd")): continue
    print("%-70s %5s %10.1f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
