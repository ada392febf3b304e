"""Summarise an SQ / GRBM counter run (tools/pmc_roll_sq.sh and friends): per-dispatch means of every counter over
the dispatches of one kernel, plus derived fractions. Usage:
    python tools/pmc_fwd_sum.py <dir> [<kernel-name substring> <label> [<grid size>]]

Normalisation (verdict r04 item 7): a counter run is several `rocprofv3 --pmc` passes, each with its own kernel
trace; GRBM_GUI_ACTIVE and the kernel duration are matched PER DISPATCH WITHIN ONE PASS (same Dispatch_Id in that
pass's counter_collection.csv and kernel_trace.csv), never a counter of one pass against a duration of another.
From the matched pairs: effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration. MFMA busy is reported against
SIMD-cycles = (duration x clock) x 1024 SIMDs with clock = min(effective clock, 2.4 GHz) — the GRBM window can
include counter start / stop around the dispatch (an effective clock above the 2.4 GHz peak engine clock shows
it), so the kernel's own duration at the peak clock is the cap (a lower bound on the busy fraction is the same
ratio at 2.4 GHz, an upper bound at the effective clock if that is lower)."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
KN = sys.argv[2] if len(sys.argv) > 2 else "agent_q_fwd_h3_kernel"
LABEL = sys.argv[3] if len(sys.argv) > 3 else KN
GRID = int(sys.argv[4]) if len(sys.argv) > 4 else 262144
PEAK_GHZ, SIMDS, XCDS = 2.4, 1024, 8

acc, clocks, durs = {}, [], []
busy_cycles = {}      # counter -> list of (value, simd-cycles of the same dispatch)
for pdir in sorted(glob.glob(os.path.join(d, "p*"))):
    if not os.path.isdir(pdir):
        continue
    dur = {}
    for path in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if KN in r["Kernel_Name"] and int(r["Grid_Size_X"]) == GRID:
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = {}                                # (counter, dispatch) -> sum over the counter's instances
    for path in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if KN not in r["Kernel_Name"] or int(r["Grid_Size"]) != GRID:
                continue
            key = (r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (name, did), v in per.items():
        acc.setdefault(name, []).append(v)
    for (name, did), v in per.items():
        if name != "GRBM_GUI_ACTIVE" or did not in dur:
            continue
        t = dur[did]
        clk = v / XCDS / t / 1e9
        clocks.append(clk)
        durs.append(t)
        cyc = t * min(clk, PEAK_GHZ) * 1e9 * SIMDS
        for (n2, d2), v2 in per.items():
            if d2 == did and n2 in ("SQ_VALU_MFMA_BUSY_CYCLES",):
                busy_cycles.setdefault(n2, []).append((v2, cyc, t * PEAK_GHZ * 1e9 * SIMDS))
mean = {k: sum(v) / len(v) for k, v in acc.items()}
out = {"kernel": LABEL, "dispatches": {k: len(v) for k, v in acc.items()}, "mean_per_dispatch": mean}
if durs:
    out["mean_us_traced_matched"] = 1e6 * sum(durs) / len(durs)
    out["effective_clock_ghz"] = sum(clocks) / len(clocks)
    out["effective_clock_ghz_max"] = max(clocks)
    out["clock_normalisation"] = ("per dispatch within one pass: GRBM_GUI_ACTIVE / 8 / duration; SIMD-cycles = "
                                  "duration x min(that clock, 2.4 GHz) x 1024")
for k, v in busy_cycles.items():
    out["mfma_busy_frac_of_simd_cycles"] = sum(a for a, _, _ in v) / sum(c for _, c, _ in v)
    out["mfma_busy_frac_at_peak_clock"] = sum(a for a, _, _ in v) / sum(p for _, _, p in v)
w = mean.get("SQ_WAVES")
if w:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
              "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
        if k in mean:
            out[k + "_per_wave"] = mean[k] / w
wc = mean.get("SQ_WAVE_CYCLES")
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA",
              "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
        if k in mean:
            out[k + "_frac_of_wave_cycles"] = mean[k] / wc
print(json.dumps(out, indent=1))
