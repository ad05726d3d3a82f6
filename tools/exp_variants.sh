# Usage: bash tools/exp_variants.sh OUTDIR "name1 name2 ..." "tname1 ..."  (GPU box)
# bench for the main library and each movierec/_lib/var/<name>.so; fused-kernel phase timing
# for each var/<tname>.so (timing builds)
OUT=$1; V=$GRAFT_REPO_ROOT/movierecommender-tf-trt_amd/movierec/_lib/var
mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_main.json 2>/dev/null || exit 1
for n in $2; do
  NCF_LIB=$V/$n.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_$n.json 2>/dev/null || exit 1
done
for n in $3; do
  NCF_LIB=$V/$n.so timeout -k 10 120 python tools/fused_timing.py 2>/dev/null | grep -v amdgpu.ids > $OUT/timing_$n.json || exit 1
done
python tools/summarize_exp.py $OUT
