# GPU box: count-block contributions per pass below 32,768 contributions (NCF_COUNT_PER_SMALL) at C
# 8,192 and B.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s11}; mkdir -p $O
VARS="cps32.so cps64.so" REPS=4 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C8k || exit 1
VARS="cps32.so cps64.so" REPS=3 ARGS="--config B --steps 100 --warmup 20" bash tools/r05_var.sh $O/B || exit 1
