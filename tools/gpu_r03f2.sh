# round 3: end-of-region flush with the replay 4 steps at a time (main), 1 (fu1), 2 (fu2), 4 at 2 waves/SIMD (fu4w2)
export TMPDIR=/tmp
O=gpurun_out/r03f2; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=movierecommender-tf-trt_amd/movierec/_lib
for rep in 1 2; do
for v in main fu1 fu2 fu4w2; do
lib=$R/$L/libmovierec_ncf.so; [ $v = main ] || lib=$R/$L/var/$v.so
(cd /tmp && NCF_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tr_$v -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/$O/tr_$v.log 2>&1) || { tail -5 $O/tr_$v.log; exit 1; }
f=$(find $O/tr_$v -name 'run_kernel_trace.csv' | head -1)
python - $f $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_emb_flush" in r["Kernel_Name"]]
print(sys.argv[2], ["%.1f" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows])
PY
rm -rf $O/tr_$v
done
done
echo done
