# GPU box: write-through (sc1) stores A/B — forward/backward gradient rows (wt_gs), touched-row
# update p/m/v (wt_upd), both — at C, C 8,192 and B.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s4}; mkdir -p $O
VARS="wt_upd.so wt_mv.so" REPS=4 bash tools/r05_var.sh $O/C || exit 1
VARS="wt_upd.so wt_mv.so" REPS=2 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C8k || exit 1
VARS="wt_upd.so wt_mv.so" REPS=2 ARGS="--config B --steps 100 --warmup 20" bash tools/r05_var.sh $O/B || exit 1
