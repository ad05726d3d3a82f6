#!/bin/bash
# Per-dispatch kernel trace (timestamps) of one bench run, for step-timeline analysis
# (tools/timeline.py).  Usage: bash tools/timeline.sh OUTDIR [bench args...]
R=$PWD
OUT=${1:-gpurun_out/timeline}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/tl -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $R/$OUT/tl.log 2>&1 || { tail -20 $R/$OUT/tl.log; exit 1; }
tail -1 $R/$OUT/tl.log
