# GPU box: same-session A/B of library variants on the touched-row update launch (config C, 50
# steps): VARS="name ..." (movierec/_lib/var/<name>.so), REPS.  Usage: bash tools/ab_update.sh OUT
O=${1:-gpurun_out/abu}; mkdir -p $O
for v in $VARS; do
  VAR=movierec/_lib/var/$v.so ARGS="--steps 50" REPS=${REPS:-2} bash tools/ab_lib.sh $O/$v > /dev/null || exit 1
  for f in $O/$v/*.json; do
    python - "$f" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; e = d.get("roofline_emb_update") or d.get("roofline_fwd_bwd") or {}
up = r if "embedding" in r["kernel"] else e
fb = r if "forward" in r["kernel"] else e
print(sys.argv[2], sys.argv[1].split("/")[-1], d["ms_per_step"], "fb", fb["avg_launch_ms"], "upd", up["avg_launch_ms"])
PY
  done
done
