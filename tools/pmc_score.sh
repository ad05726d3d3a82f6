# GPU box: two PMC passes over the config E scorer (bench.py --config E, 2 steps).  Usage: bash tools/pmc_score.sh OUT
O=${1:-gpurun_out/pmc_score}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $A -d $O/a -o pmc --output-format csv -- python bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline > $O/a.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc $B -d $O/b -o pmc --output-format csv -- python bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline > $O/b.log 2>&1
