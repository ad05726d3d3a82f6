#!/bin/bash
# One GPU session: kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes (separate, per
# MI355X_MICROARCH.md), traffic JSON for bench.py (copy $OUT/traffic/*.json to profiles/traffic/).
# Run from the repo root on the GPU box.  Usage: bash tools/gpu_profile.sh OUT [extra bench args]
# (the traffic files are keyed as config C, batch 65536, single layout: the default bench run)
set -e
R=$PWD
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT/traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/$OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_emb_update|k_emb_adam_touched|k_fb_fused|k_fb_unit|k_fb_wave" --output-format csv -d $R/$OUT/fetch -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_emb_update|k_emb_adam_touched|k_fb_fused|k_fb_unit|k_fb_wave" --output-format csv -d $R/$OUT/write -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/write.log 2>&1
cd $R
python tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv k_emb_adam_touched $OUT/traffic/C_b65536_single-ahead_k_emb_adam_touched.json C 65536 single-ahead
python tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv k_fb_wave $OUT/traffic/C_b65536_single_k_fb_wave.json
