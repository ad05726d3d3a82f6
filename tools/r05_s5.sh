# GPU box: write-through touched-row stores (st_row, batches >= 8,192) — tests, then A/B against the
# previous commit (var/head.so) at C, C 8,192 and B.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_index_in_kernel_gpu.py tests/test_native_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARS="head.so" REPS=4 bash tools/r05_var.sh $O/C || exit 1
VARS="head.so" REPS=3 ARGS="--batch 8192 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C8k || exit 1
VARS="head.so" REPS=3 ARGS="--config B --steps 100 --warmup 20" bash tools/r05_var.sh $O/B || exit 1
