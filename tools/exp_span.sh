#!/bin/bash
# Wave-kernel span stamps at several batch sizes (timing build), then a default bench line.
# Usage: bash tools/exp_span.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/span}
mkdir -p $OUT
timeout -k 10 180 env NCF_LIB=movierecommender-tf-trt_amd/movierec/_lib/var/wtiming.so \
    BATCHES=${BATCHES:-16384,32768,65536,131072} python tools/wave_timing.py > $OUT/spans.json 2> $OUT/spans.err \
    || { tail -20 $OUT/spans.err; exit 1; }
cat $OUT/spans.json
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
