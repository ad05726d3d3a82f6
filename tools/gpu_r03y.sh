# round 3: kernel traces of C at 8,192 (200 steps) and config B (200 steps) after the replay change
export TMPDIR=/tmp
O=gpurun_out/r03y; mkdir -p $O
R=$GRAFT_REPO_ROOT
tr() { name=$1; k=$2; shift 2; (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/tr_$name -o run -- python $R/bench.py --no-cpu-baseline "$@" > $R/$O/tr_$name.log 2>&1) || { tail -5 $O/tr_$name.log; exit 1; }
  f=$(find $O/tr_$name -name 'run_kernel_trace.csv' | head -1); s=$(find $O/tr_$name -name 'run_kernel_stats.csv' | head -1)
  python tools/step_window.py $f $k > $O/tl_$name.txt && cp $s $O/stats_$name.csv && rm -rf $O/tr_$name && cat $O/tl_$name.txt; }
tr C8192 180 --batch 8192 --steps 200
tr B 180 --config B --steps 200
echo done
