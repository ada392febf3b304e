"""Summarise tools/pmc_fwd_sq.sh: per-dispatch means of every counter over the dual-forward dispatches
(agent_q_fwd_h3_kernel, grid 262144), plus derived fractions. Usage: python tools/pmc_fwd_sum.py <dir>
[<kernel-name substring> <label>] (tools/pmc_roll_sq.sh: rollout_step_kernel)"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
KN = sys.argv[2] if len(sys.argv) > 2 else "agent_q_fwd_h3_kernel"
LABEL = sys.argv[3] if len(sys.argv) > 3 else "agent_q_fwd_h3_kernel<64,64,64,1> dual (grid 262144 = 256 blocks x 1024)"
acc = {}
dur = []
for path in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = {}                                # (counter, dispatch) -> sum over the counter's instances
    for r in csv.DictReader(open(path)):
        if KN not in r["Kernel_Name"] or int(r["Grid_Size"]) != 262144:
            continue
        key = (r["Counter_Name"], path, r["Dispatch_Id"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (name, _, _), v in per.items():
        acc.setdefault(name, []).append(v)
for path in glob.glob(os.path.join(d, "p*", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        if KN in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 262144:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
mean = {k: sum(v) / len(v) for k, v in acc.items()}
out = {"kernel": LABEL,
       "dispatches": {k: len(v) for k, v in acc.items()}, "mean_per_dispatch": mean}
if dur:
    out["mean_us_traced"] = sum(dur) / len(dur)
w = mean.get("SQ_WAVES")
if w:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        if k in mean:
            out[k + "_per_wave"] = mean[k] / w
g = mean.get("GRBM_GUI_ACTIVE")
if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
    simd_cycles = g / 8 * 1024          # GRBM_GUI_ACTIVE sums the 8 XCDs; 256 CUs x 4 SIMDs
    out["mfma_busy_frac_of_simd_cycles"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
    out["effective_clock_ghz"] = g / 8 / (out["mean_us_traced"] * 1e3) if dur else None
wc = mean.get("SQ_WAVE_CYCLES")
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA",
              "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
        if k in mean:
            out[k + "_frac_of_wave_cycles"] = mean[k] / wc
print(json.dumps(out, indent=1))
