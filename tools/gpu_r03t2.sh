# round 3: FETCH_SIZE / WRITE_SIZE passes (each its own run) for configs A, B, C at 8,192 and D, so
# their bench lines carry measured traffic (profiles/traffic/<config>_b<batch>_single_<kernel>.json)
export TMPDIR=/tmp
O=gpurun_out/r03t2; mkdir -p $O/traffic
R=$GRAFT_REPO_ROOT
RX="k_emb_adam_touched|k_fb_unit|k_fb_wave|k_fb_fused"
pp() { tag=$1; cfg=$2; batch=$3; shift 3
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$RX" --output-format csv -d $R/$O/${tag}_$c -o run -- python $R/bench.py --no-cpu-baseline "$@" > $R/$O/${tag}_$c.log 2>&1) || { tail -5 $O/${tag}_$c.log; exit 1; }
  done
  f=$(find $O/${tag}_FETCH_SIZE -name 'run_counter_collection.csv' | head -1); w=$(find $O/${tag}_WRITE_SIZE -name 'run_counter_collection.csv' | head -1)
  for k in $KERNELS; do python tools/pmc_traffic.py $f $w $k $O/traffic/${cfg}_b${batch}_single_$k.json $cfg $batch single || exit 1; done
  rm -rf $O/${tag}_FETCH_SIZE $O/${tag}_WRITE_SIZE
}
KERNELS="k_emb_adam_touched k_fb_unit" pp C8192 C 8192 --batch 8192 --steps 5 --warmup 2
KERNELS="k_emb_adam_touched k_fb_unit" pp B B 4095 --config B --steps 5 --warmup 2
KERNELS="k_emb_adam_touched" pp D D 65536 --config D --steps 3 --warmup 1
ls $O/traffic
