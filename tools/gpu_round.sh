# GPU box, round evidence: every GPU test, smoke, the driver's bench command, config lines (B, C at
# 8,192, D, D row-sharded emulated world 8, user layout emulated world 8, E), kernel-trace stats
# and PMC traffic (C, D).  Usage: bash tools/gpu_round.sh OUT
export TMPDIR=/tmp
O=${1:-gpurun_out/round}; mkdir -p $O
bash tools/gpu_check.sh $O || exit 1
TESTS= BENCHES="B:--config B --steps 50;C8192:--batch 8192 --steps 200;Ds8:--config D --dp sharded --emulate-world 8 --steps 50 --warmup 3;U8:--dp user --emulate-world 8 --steps 50;U8s:--dp user --emulate-world 8 --global-batch 8192 --steps 100;E:--config E --steps 3 --warmup 1" bash tools/gpu_step.sh $O || exit 1
bash tools/gpu_profile.sh $O/prof || exit 1
cd /tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O/profD
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/profD/trace -o run -- python $R/bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline > $R/$O/profD/trace.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_emb_adam_touched|k_lay_l1f|k_lay_l1b|k_lay_mid|k_lay_dw1" --output-format csv -d $R/$O/profD/$c -o run -- python $R/bench.py --config D --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/profD/$c.log 2>&1 || exit 1
done
cd $R
python tools/pmc_traffic.py $O/profD/FETCH_SIZE/run_counter_collection.csv $O/profD/WRITE_SIZE/run_counter_collection.csv k_emb_adam_touched $O/prof/traffic/D_b65536_single-ahead_k_emb_adam_touched.json D 65536 single-ahead
