"""Summarise an SQ / GRBM counter run (tools/pmc_chunk.sh and friends): per-dispatch means of every counter over
the dispatches of one kernel, plus derived fractions. Usage:
    python tools/pmc_fwd_sum.py <dir> [<kernel-name substring> <label> [<grid size>]]   (grid size 0: any grid)

Clock normalisation (verdict r05 item 5): a counter run is several `rocprofv3 --pmc` passes, each with its own kernel
trace; counters and the kernel duration are matched PER DISPATCH WITHIN ONE PASS (same Dispatch_Id in that pass's
counter_collection.csv and kernel_trace.csv). The clock of a dispatch is SQ_BUSY_CYCLES / 32 shader engines /
duration (SQ_BUSY_CYCLES counts engine cycles per SE, summed over the 8 XCDs x 4 SEs): it agrees with the in-kernel
s_memtime clock of the chunk kernel's debug build (tools/chunk_trace.py) and stays below the 2.4 GHz peak, where
GRBM_GUI_ACTIVE / 8 / duration reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS) — that
quotient is kept only as a diagnostic, never capped or used. MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (duration x
SQ clock x 1024 SIMDs), both from the same dispatch of the same pass."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
KN = sys.argv[2] if len(sys.argv) > 2 else "agent_q_fwd_h3_kernel"
LABEL = sys.argv[3] if len(sys.argv) > 3 else KN
GRID = int(sys.argv[4]) if len(sys.argv) > 4 else 262144
PEAK_GHZ, SIMDS, XCDS, SES = 2.4, 1024, 8, 32

acc, clocks, grbm_clocks, durs = {}, [], [], []
busy_cycles = {}      # counter -> list of (value, simd-cycles of the same dispatch)
for pdir in sorted(glob.glob(os.path.join(d, "p*"))):
    if not os.path.isdir(pdir):
        continue
    dur = {}
    for path in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if KN in r["Kernel_Name"] and (GRID == 0 or int(r["Grid_Size_X"]) == GRID):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = {}                                # (counter, dispatch) -> sum over the counter's instances
    for path in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if KN not in r["Kernel_Name"] or (GRID != 0 and int(r["Grid_Size"]) != GRID):
                continue
            key = (r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (name, did), v in per.items():
        acc.setdefault(name, []).append(v)
    for (name, did), v in per.items():
        if did not in dur:
            continue
        t = dur[did]
        if name == "GRBM_GUI_ACTIVE":
            grbm_clocks.append(v / XCDS / t / 1e9)
        if name != "SQ_BUSY_CYCLES":
            continue
        clk = v / SES / t / 1e9
        clocks.append(clk)
        durs.append(t)
        cyc = t * clk * 1e9 * SIMDS
        for (n2, d2), v2 in per.items():
            if d2 == did and n2 in ("SQ_VALU_MFMA_BUSY_CYCLES",):
                busy_cycles.setdefault(n2, []).append((v2, cyc, t * PEAK_GHZ * 1e9 * SIMDS))
mean = {k: sum(v) / len(v) for k, v in acc.items()}
out = {"kernel": LABEL, "dispatches": {k: len(v) for k, v in acc.items()}, "mean_per_dispatch": mean}
if durs:
    out["mean_us_traced_matched"] = 1e6 * sum(durs) / len(durs)
    out["effective_clock_ghz"] = sum(clocks) / len(clocks)
    out["effective_clock_ghz_min"] = min(clocks)
    out["effective_clock_ghz_max"] = max(clocks)
    out["clock_normalisation"] = ("per dispatch within one pass: SQ_BUSY_CYCLES / 32 SEs / duration; SIMD-cycles = "
                                  "duration x that clock x 1024")
if grbm_clocks:
    out["grbm_gui_active_clock_ghz_diagnostic"] = {"mean": sum(grbm_clocks) / len(grbm_clocks), "max": max(grbm_clocks),
                                                   "note": "GRBM_GUI_ACTIVE / 8 / duration: reads high on short "
                                                           "dispatches; not used"}
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
