# GPU box: same-session A/B of the default library against a variant at configs C, C at 8,192 and B.
# Usage: VAR=movierec/_lib/var/x.so bash tools/ab3.sh OUT
O=${1:-gpurun_out/ab3}; mkdir -p $O
VAR=$VAR REPS=2 ARGS="--steps 50" bash tools/ab_lib.sh $O/C || exit 1
VAR=$VAR REPS=2 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/ab_lib.sh $O/C8k || exit 1
VAR=$VAR REPS=2 ARGS="--config B --steps 100 --warmup 20" bash tools/ab_lib.sh $O/B || exit 1
