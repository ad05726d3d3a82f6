export TMPDIR=/tmp
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_distributed.py tests/test_fit_dp_gpu.py tests/test_config_d_gpu.py tests/test_headline_parity_gpu.py tests/test_native_gpu.py tests/test_score_gpu.py -m gpu -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1; tail -3 $O/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_C.json 2> $O/bench_C.err; tail -c 300 $O/bench_C.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dp user --emulate-world 8 > $O/bench_user_emul8.json 2> $O/bench_user_emul8.err; tail -c 200 $O/bench_user_emul8.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dp user --emulate-world 8 --batch 8192 > $O/bench_user_emul8_b8192.json 2> $O/bench_user_emul8_b8192.err; tail -c 200 $O/bench_user_emul8_b8192.json
timeout -k 10 300 python bench.py --steps 3 --fit-epochs > $O/bench_fit.json 2> $O/bench_fit.err; tail -c 300 $O/bench_fit.json
