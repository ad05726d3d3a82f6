# GPU box: kernel-trace averages of the default bench under a variant library (NCF_LIB).
# Usage: bash tools/trace_var.sh OUT movierec/_lib/var/x.so [bench args]
export TMPDIR=/tmp
O=$1; shift
V=$1; shift
mkdir -p $O
[ -n "$V" ] && export NCF_LIB=$GRAFT_REPO_ROOT/movierecommender-tf-trt_amd/$V
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/$O/trace_bench.json 2> $GRAFT_REPO_ROOT/$O/trace_bench.err || exit 1
cd $GRAFT_REPO_ROOT && python - <<PY
import csv
for r in csv.DictReader(open("$O/trace/run_kernel_stats.csv")):
    if r["Name"].startswith(("void rocprim", "void at::", "__amd")): continue
    print("%-70s %5s %10.1f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
