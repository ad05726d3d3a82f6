export TMPDIR=/tmp
O=gpurun_out/r05s1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_index_in_kernel_gpu.py tests/test_native_gpu.py tests/test_fit_parity_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VAR=movierec/_lib/var/head.so REPS=3 ARGS="--steps 50" bash tools/ab_lib.sh $O/C || exit 1
VAR=movierec/_lib/var/head.so REPS=2 ARGS="--config B --steps 100 --warmup 20" bash tools/ab_lib.sh $O/B || exit 1
VARS="norep.so noupd.so fill2.so" REPS=2 bash tools/r05_var.sh $O/diag || exit 1
