set -o pipefail
mkdir -p gpurun_out/pf
timeout -k 10 300 python -u -m pytest tests/test_headline_parity_gpu.py tests/test_native_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pf/tests.log 2>&1 || { tail -30 gpurun_out/pf/tests.log; exit 1; }
tail -1 gpurun_out/pf/tests.log
for v in timing timing_nopf; do NCF_LIB=movierecommender-tf-trt_amd/movierec/_lib/var/$v.so timeout -k 10 120 python tools/fused_timing.py > gpurun_out/pf/$v.json 2>&1 || exit 1; done
bash tools/exp_ab.sh gpurun_out/pf default nopf default nopf
