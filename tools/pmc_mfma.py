"""MFMA busy fraction of the MFMA forward/backward (k_fb_unit / k_fb_wave: v_mfma_f32_16x16x4_f32,
32 busy cycles each; k_fb_fused: v_mfma_f32_32x32x2_f32, 64) from one rocprofv3 PMC pass
(tools/pmc_mfma.sh).  SQ_VALU_MFMA_BUSY_CYCLES counts MFMA busy cycles summed over the SIMDs;
GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the kernel's clock
cycles are GRBM_GUI_ACTIVE / 8 (MI355X_MICROARCH.md).  busy fraction = MFMA_BUSY /
(1024 SIMDs x kernel cycles); the effective clock = kernel cycles / duration."""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = collections.defaultdict(dict)
dur = {}
for r in rows:
    kname = next((k for k in ("k_fb_unit", "k_fb_wave", "k_fb_fused") if k in r["Kernel_Name"]), None)
    if kname is None:
        continue
    d = r["Dispatch_Id"]
    per[d][r["Counter_Name"]] = float(r["Counter_Value"])
    dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
out = []
for d, c in per.items():
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    out.append({"mfma_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc),
                "mfma_count_est": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (64.0 if kname == "k_fb_fused" else 32.0),
                "clock_GHz": cyc / dur[d] / 1e9, "dur_us": dur[d] * 1e6})
res = {k: sum(o[k] for o in out) / len(out) for k in out[0]}
res["dispatches"] = len(out)
res["kernel"] = kname
print(json.dumps(res, indent=1))
