# GPU box: C at 8,192 tunables — unit-launch fill workgroup cap and count-block contributions per pass.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s10}; mkdir -p $O
VARS="fb384.so fb512.so cps8.so cps32.so" REPS=3 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C8k || exit 1
