# round 3: config D step timeline (kernel trace, one step window)
export TMPDIR=/tmp
O=gpurun_out/r03d2; mkdir -p $O
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/tr -o run -- python $R/bench.py --no-cpu-baseline --config D --steps 10 --warmup 2 > $R/$O/tr.log 2>&1) || { tail -5 $O/tr.log; exit 1; }
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1); s=$(find $O/tr -name 'run_kernel_stats.csv' | head -1)
python tools/step_window.py $f 6 k_lay_l1f > $O/tl_D.txt && cp $s $O/stats_D.csv && rm -rf $O/tr && cat $O/tl_D.txt
