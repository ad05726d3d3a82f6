# round 3: native RCCL user-partitioned step — tests, emulated per-rank benches, timelines
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_headline_parity_gpu.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/gputest.log 2>&1; tail -3 $O/gputest.log
for v in 65536 8192; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dp user --emulate-world 8 --batch $v > $O/bench_user_emul8_b$v.json 2> $O/bench_user_emul8_b$v.err || { tail -5 $O/bench_user_emul8_b$v.err; exit 1; }
tail -c 150 $O/bench_user_emul8_b$v.json
done
cd /tmp
for v in 65536 8192; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tl_user_$v -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --dp user --emulate-world 8 --batch $v > $R/$O/tl_user_$v.log 2>&1 || { tail -5 $R/$O/tl_user_$v.log; exit 1; }
done
echo done
