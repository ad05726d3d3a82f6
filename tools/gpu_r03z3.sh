# round 3: kernel timeline of the driver's 20-step timed region
export TMPDIR=/tmp
O=gpurun_out/r03z3; mkdir -p $O
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tr -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/$O/tr.log 2>&1) || { tail -5 $O/tr.log; exit 1; }
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
python tools/region_timeline.py $f > $O/region.txt && rm -rf $O/tr && tail -40 $O/region.txt && head -30 $O/region.txt
