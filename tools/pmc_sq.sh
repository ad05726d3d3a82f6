# Where the forward/backward kernel's waves spend their cycles (GPU box, repo root): one PMC pass
# of SQ wave-state counters on k_fb_wave (its own run, no trace domains).  Usage: bash tools/pmc_sq.sh OUT
R=$PWD
OUT=${1:-gpurun_out/pmc_sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS --kernel-include-regex "k_fb_wave" --output-format csv -d $R/$OUT/pmc -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/pmc.log 2>&1 || { tail -5 $R/$OUT/pmc.log; exit 1; }
cd $R && python - $OUT/pmc/run_counter_collection.csv <<'PY'
import collections, csv, json, sys
per = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_fb_wave" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
keys = sorted(next(iter(per.values())))
avg = {k: sum(d[k] for d in per.values()) / len(per) for k in keys}
wc = avg["SQ_WAVE_CYCLES"]
print(json.dumps({k: (round(v / wc, 4) if k != "SQ_WAVE_CYCLES" and k != "SQ_INSTS_LDS" else v) for k, v in avg.items()}, indent=1))
PY
