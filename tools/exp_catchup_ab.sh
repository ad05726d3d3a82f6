set -o pipefail
mkdir -p gpurun_out/cu
timeout -k 10 300 python -u -m pytest tests/test_headline_parity_gpu.py::test_deferred_decay_long_gaps_bitwise "tests/test_native_gpu.py::test_lazy_decay_bitwise_equals_dense_sweep" tests/test_native_gpu.py::test_count_ahead_equals_plain_steps -q --timeout 200 --timeout-method thread > gpurun_out/cu/tests.log 2>&1 || { tail -30 gpurun_out/cu/tests.log; exit 1; }
tail -2 gpurun_out/cu/tests.log
for v in default cu8192 cu4096 cu_f4; do
  if [ $v = default ]; then L=""; else L=movierecommender-tf-trt_amd/movierec/_lib/var/$v.so; fi
  NCF_LIB=$L timeout -k 10 200 python tools/catchup_probe.py --steps 60 > gpurun_out/cu/probe_$v.log 2>&1 || exit 1
  echo $v $(tail -1 gpurun_out/cu/probe_$v.log)
done
