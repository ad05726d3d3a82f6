#!/bin/bash
# Wave-kernel change check on the GPU box: the tests that run it (oracle parity incl. config C
# full size, unit/tile comparison, folding), span stamps at several batches, a default bench line.
# Usage: bash tools/exp_wave_check.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/wcheck}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_unit_kernel_gpu.py \
    tests/test_user_fold_gpu.py tests/test_headline_parity_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
bash tools/exp_span.sh $OUT
