#!/bin/bash
# run bench for each library variant; prints one line per variant
R=$PWD
for v in base nosb ch16 nosb_ch16; do
  if [ "$v" = base ]; then L=""; else L=$R/movierecommender-tf-trt_amd/movierec/_lib/var/$v.so; fi
  NCF_LIB=$L timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/var_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('$v', d['value'], d['ms_per_step'])"
done
