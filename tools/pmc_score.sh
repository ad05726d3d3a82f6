cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/scpmc
SU=20000 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU --kernel-include-regex k_score_topk --output-format csv -d $R/gpurun_out/scpmc/p1 -o run -- python3 $R/tools/score_timing.py > $R/gpurun_out/scpmc/p1.log 2>&1
SU=20000 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT --kernel-include-regex k_score_topk --output-format csv -d $R/gpurun_out/scpmc/p2 -o run -- python3 $R/tools/score_timing.py > $R/gpurun_out/scpmc/p2.log 2>&1
cd $R && python3 - <<'PY'
import csv,glob
for p in ["p1","p2"]:
    for f in glob.glob("gpurun_out/scpmc/%s/*counter_collection.csv"%p):
        rows=list(csv.DictReader(open(f)))
        agg={}
        for r in rows:
            agg.setdefault(r["Counter_Name"],[]).append(float(r["Counter_Value"]))
        for k,v in agg.items(): print(p,k,len(v),v[-1])
PY
