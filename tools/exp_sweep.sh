#!/bin/bash
# Unit vs wave forward/backward kernel over batch sizes (config C) and config B fp32, one session.
# Usage: bash tools/exp_sweep.sh OUT
set -e
OUT=${1:-gpurun_out/sweep}
mkdir -p $OUT
for b in 8192 16384 32768 65536 131072; do
  for k in unit wave; do
    timeout -k 10 120 env NCF_FB_KERNEL=$k python bench.py --steps 30 --warmup 5 --no-cpu-baseline --batch $b > $OUT/C_${b}_$k.json 2> $OUT/C_${b}_$k.err
  done
done
for k in unit wave; do
  timeout -k 10 120 env NCF_FB_KERNEL=$k python bench.py --config B --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/B_$k.json 2> $OUT/B_$k.err
done
python - $OUT <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    fb = d["roofline"] if d["roofline"]["bound"] == "mfma" else d.get("roofline_fwd_bwd")
    print(os.path.basename(f)[:-5], round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", "fb", fb["avg_launch_ms"], fb["frac"])
PY
