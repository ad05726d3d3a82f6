# GPU box: scorer output-MFMA deferral (NCF_SCORE_OUT_DEFER) — score tests, then A/B twice.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05e1}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_score_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARS="nodefer" bash tools/ab_score.sh $O/a || exit 1
VARS="nodefer" bash tools/ab_score.sh $O/b || exit 1
