# GPU box: the GPU tests that run the count / catch-up-ahead path at small batches, after the
# count-per-pass change.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s12}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_index_in_kernel_gpu.py tests/test_native_gpu.py tests/test_fit_parity_gpu.py tests/test_user_fold_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
