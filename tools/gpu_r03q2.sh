# round 3: list sort over the touched rows only above 1 M keys (config D)
export TMPDIR=/tmp
O=gpurun_out/r03q2; mkdir -p $O
R=$GRAFT_REPO_ROOT
NCF_LIB=$R/movierecommender-tf-trt_amd/movierec/_lib/var/listed.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { name=$1; shift; NCF_LIB=$R/movierecommender-tf-trt_amd/movierec/_lib/var/listed.so timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('%-10s %8.2f M/s %8.4f ms idx %s cu %s' % ('$name', d['value']/1e6, d['ms_per_step'], d.get('index_build_ms'), d.get('catchup_ms')))"; }
b D --config D --steps 50 --warmup 3
b C --steps 50
(cd /tmp && NCF_LIB=$R/movierecommender-tf-trt_amd/movierec/_lib/var/listed.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tr -o run -- python $R/bench.py --no-cpu-baseline --config D --steps 10 --warmup 2 > $R/$O/tr.log 2>&1) || { tail -5 $O/tr.log; exit 1; }
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -1)
python tools/step_window.py $f 6 k_lay_l1f > $O/tl_D.txt && rm -rf $O/tr && cat $O/tl_D.txt
