mkdir -p gpurun_out/r10
V=$GRAFT_REPO_ROOT/movierecommender-tf-trt_amd/movierec/_lib/var
NCF_LIB=$V/timing_nt.so timeout -k 10 120 python tools/fused_timing.py > gpurun_out/r10/timing_nt.json 2>&1 &&
NCF_LIB=$V/timing_st.so timeout -k 10 120 python tools/fused_timing.py > gpurun_out/r10/timing_st.json 2>&1 &&
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r10/bench_nt.json 2>/dev/null &&
NCF_LIB=$V/st.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r10/bench_st.json 2>/dev/null
python - <<'PY'
import json
for v in ["nt","st"]:
    t=json.load(open("gpurun_out/r10/timing_%s.json"%v))
    print(v, "kernel_ms", round(t["kernel_ms"],4), {k:round(x) for k,x in t["wave0"].items()})
    b=json.loads(open("gpurun_out/r10/bench_%s.json"%v).read().strip().splitlines()[-1])
    print(v, "step_ms", b["ms_per_step"], "emb_ms", b["roofline"]["avg_launch_ms"], "fb_ms", b["roofline_fwd_bwd"]["avg_launch_ms"], "idx", b["index_build_ms"])
PY
