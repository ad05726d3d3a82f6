#!/bin/bash
# GPU box: config E scorer profile: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE passes
# (separate runs, MI355X_MICROARCH.md) -> OUT/traffic/E_b138493_all-items_k_score_topk.json
# (copy it to profiles/traffic/ for bench.py).  Usage: bash tools/gpu_profile_e.sh OUT
set -e
R=$PWD
OUT=${1:-gpurun_out/prof_e}
mkdir -p $OUT/traffic
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python $R/bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_score_topk" --output-format csv -d $R/$OUT/fetch -o run -- python $R/bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_score_topk" --output-format csv -d $R/$OUT/write -o run -- python $R/bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/write.log 2>&1
cd $R
python tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv k_score_topk $OUT/traffic/E_b138493_all-items_k_score_topk.json E 138493 all-items
