"""Summarize tools/exp_variants.sh output: one line per bench / timing file."""
import glob
import json
import os
import sys

out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "bench_*.json"))):
    try:
        b = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        print(os.path.basename(f), "unreadable")
        continue
    print("%-22s step %.4f ms  value %.1fM  emb %.4f  fb %.4f  idx %.4f" % (
        os.path.basename(f), b["ms_per_step"], b["value"] / 1e6, b["roofline"]["avg_launch_ms"],
        b["roofline_fwd_bwd"]["avg_launch_ms"], b["index_build_ms"]))
for f in sorted(glob.glob(os.path.join(out, "timing_*.json"))):
    try:
        t = json.load(open(f))
    except ValueError:
        print(os.path.basename(f), "unreadable")
        continue
    print("%-22s kernel %.4f ms" % (os.path.basename(f), t["kernel_ms"]))
    for w in ("wave0", "wave3"):
        print("   ", w, " ".join("%s=%d" % (k, v) for k, v in t[w].items()))
