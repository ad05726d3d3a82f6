# round 3: build-ahead native user step, layered forward for predict/evaluate, count-claimed
# catch-up ahead — tests + benches
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_fit_dp_gpu.py tests/test_headline_parity_gpu.py tests/test_native_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { rc=$?; tail -3 $O/gputest.log; [ $rc -eq 1 ] || exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_C.json 2> $O/bench_C.err || exit 1
for v in 65536 8192; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dp user --emulate-world 8 --batch $v > $O/bench_user_emul8_b$v.json 2> $O/bench_user_emul8_b$v.err || { tail -5 $O/bench_user_emul8_b$v.err; exit 1; }
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dp user > $O/bench_user_w1.json 2> $O/bench_user_w1.err || exit 1
timeout -k 10 300 python bench.py --config D --steps 40 --warmup 3 > $O/bench_D.json 2> $O/bench_D.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tl_user_65536 -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --dp user --emulate-world 8 > $R/$O/tl_user_65536.log 2>&1 || { tail -5 $R/$O/tl_user_65536.log; exit 1; }
echo done
