# round 3: parity re-checks + step timelines of the user layout (GPU box, repo root)
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_config_d_gpu.py tests/test_headline_parity_gpu.py tests/test_sampler_gpu.py tests/test_fit_dp_gpu.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gputest.log 2>&1; tail -3 $O/gputest.log
timeout -k 10 300 python bench.py --steps 3 --fit-epochs > $O/bench_fit.json 2> $O/bench_fit.err; tail -c 300 $O/bench_fit.json
cd /tmp
for v in "65536" "8192"; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tl_user_$v -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --dp user --emulate-world 8 --batch $v > $R/$O/tl_user_$v.log 2>&1 || { tail -5 $R/$O/tl_user_$v.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tl_single -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/tl_single.log 2>&1 || { tail -5 $R/$O/tl_single.log; exit 1; }
echo done
