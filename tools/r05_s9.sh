# GPU box: count (+ catch-up ahead) blocks of the touched-row update at priority 1 (NCF_COUNT_PRIO)
# — A/B at C and C 8,192.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s9}; mkdir -p $O
VARS="cprio.so pkeep.so" REPS=4 bash tools/r05_var.sh $O/C || exit 1
VARS="cprio.so pkeep.so" REPS=3 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C8k || exit 1
