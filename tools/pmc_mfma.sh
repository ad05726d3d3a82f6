#!/bin/bash
# MFMA utilisation of the MFMA forward/backward (GPU box, repo root): one PMC pass with
# SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE on k_fb_unit / k_fb_wave / k_fb_fused (its own
# run, no trace domains), then tools/pmc_mfma.py.  Usage: bash tools/pmc_mfma.sh OUTDIR [bench args]
R=$PWD
OUT=${1:-gpurun_out/pmc_mfma}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_fb_unit|k_fb_wave|k_fb_fused" --output-format csv -d $R/$OUT/pmc -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $R/$OUT/pmc.log 2>&1 || { tail -5 $R/$OUT/pmc.log; exit 1; }
cd $R && python tools/pmc_mfma.py $OUT/pmc/run_counter_collection.csv
