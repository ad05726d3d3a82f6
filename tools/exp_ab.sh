#!/bin/bash
# A/B of forward/backward kernel variants in ONE GPU session (clocks differ between boxes):
# config C bench lines alternating the libraries given.  Usage: bash tools/exp_ab.sh OUT lib1 lib2 ...
# (env for every run: NCF_FB_KERNEL, default wave)
set -e
OUT=$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)_$rep
    timeout -k 10 120 env NCF_LIB=$lib NCF_FB_KERNEL=${NCF_FB_KERNEL:-wave} python bench.py --steps 40 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > $OUT/$tag.json 2> $OUT/$tag.err
  done
done
python - $OUT "$@" <<'PY'
import json, os, sys
out = sys.argv[1]
for lib in sys.argv[2:]:
    for rep in (1, 2):
        tag = os.path.basename(lib)[:-3] + "_%d" % rep
        d = json.loads(open("%s/%s.json" % (out, tag)).read().strip().splitlines()[-1])
        fb = d["roofline"] if d["roofline"]["bound"] == "mfma" else d.get("roofline_fwd_bwd")
        print(tag, round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", "fb", fb["avg_launch_ms"], fb["frac"])
PY
