# GPU box: chain waves at priority 1 from phase 0 (NCF_PRIO_P0) — index tests, A/B at C and 16,384.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s6}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_index_in_kernel_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARS="noprio.so" REPS=4 bash tools/r05_var.sh $O/C || exit 1
VARS="noprio.so" REPS=2 ARGS="--batch 16384 --steps 100 --warmup 20" bash tools/r05_var.sh $O/C16k || exit 1
