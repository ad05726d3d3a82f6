# round 3: config E scorer counters (two PMC passes of their own: SQ instruction mix, then wait/busy states)
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
R=$GRAFT_REPO_ROOT
p() { name=$1; shift; (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_score_topk" --output-format csv -d $R/$O/$name -o run -- python $R/bench.py --no-cpu-baseline --config E --steps 1 --warmup 1 > $R/$O/$name.log 2>&1) || { tail -5 $O/$name.log; exit 1; }
  f=$(find $O/$name -name 'run_counter_collection.csv' | head -1); python - $f <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc): print("%-32s %16.0f  (%d rows)" % (k, acc[k], n[k]))
PY
}
p pa SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
p pb SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_COUNT
echo done
