#!/bin/bash
# Round-end evidence on the GPU box: tools/round_check.sh (GPU tests, smoke, default bench line
# with the CPU baseline, kernel-trace stats, FETCH/WRITE PMC traffic), the MFMA-busy PMC pass,
# the user-partitioned layout at world 1 (RCCL communicator of one rank) and its per-rank compute
# at an emulated world of 8.  Usage: bash tools/final_check.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/final}
bash tools/round_check.sh $OUT || exit 1
bash tools/pmc_mfma.sh $OUT/pmc_mfma > $OUT/pmc_mfma.txt 2>&1 || { cat $OUT/pmc_mfma.txt; exit 1; }
cat $OUT/pmc_mfma.txt
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dp user > $OUT/bench_user_world1.json 2> $OUT/bench_user_world1.err \
    || { tail -20 $OUT/bench_user_world1.err; exit 1; }
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dp user --emulate-world 8 > $OUT/bench_user_emul8.json 2> $OUT/bench_user_emul8.err \
    || { tail -20 $OUT/bench_user_emul8.err; exit 1; }
python - $OUT <<'PY'
import json, sys
for f in ("bench_user_world1", "bench_user_emul8"):
    d = json.loads(open("%s/%s.json" % (sys.argv[1], f)).read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms/step", d.get("exchange"))
PY
