# GPU box: HBM-side traffic of the touched-row update launch (k_emb_adam_touched) at config C,
# with the next batch counted and its stale rows caught up ahead (the bench's form) and without
# (update + dense-layer Adam blocks only): separate FETCH_SIZE / WRITE_SIZE passes per mode, plus
# an L2 hit-rate pass.  Usage: bash tools/pmc_update_roles.sh OUT
R=$PWD
OUT=${1:-gpurun_out/pmc_roles}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for mode in ahead not_ahead; do
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_emb_adam_touched" --output-format csv \
      -d $R/$OUT/${mode}_$tag -o run -- python $R/tools/update_split.py $mode > $R/$OUT/${mode}_$tag.log 2>&1 || { echo "pass $mode $tag failed"; tail -5 $R/$OUT/${mode}_$tag.log; exit 1; }
  done
done
cd $R
python - $OUT <<'PY'
import csv, json, sys, glob
out = sys.argv[1]
res = {}
for mode in ("ahead", "not_ahead"):
    r = {}
    for tag, names in (("FETCH_SIZE", ["FETCH_SIZE"]), ("WRITE_SIZE", ["WRITE_SIZE"]), ("TCC_HIT_sum", ["TCC_HIT_sum", "TCC_MISS_sum"])):
        f = glob.glob("%s/%s_%s/**/run_counter_collection.csv" % (out, mode, tag), recursive=True)
        rows = list(csv.DictReader(open(f[0])))
        for n in names:
            v = [float(x["Counter_Value"]) for x in rows if x["Counter_Name"] == n]
            v = v[10:] if len(v) > 12 else v          # past the 10 warm-up steps
            r[n] = sum(v) / len(v)
    r["fetch_bytes_x2"] = 2 * r["FETCH_SIZE"] * 1024
    r["write_bytes"] = r["WRITE_SIZE"] * 1024
    r["l2_hit_rate"] = r["TCC_HIT_sum"] / (r["TCC_HIT_sum"] + r["TCC_MISS_sum"])
    res[mode] = r
json.dump(res, open(out + "/roles.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
