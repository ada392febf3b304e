"""Summarise tools/pmc_mappo.sh: mean per-dispatch HBM bytes of every mappo kernel (FETCH_SIZE doubled
per the gfx950 correction of MI355X_MICROARCH.md's HBM section, WRITE_SIZE as is) and the SQ counters
of the fused gradient kernel. usage: python tools/pmc_mappo_sum.py <outdir>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counters):
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] in counters:
                per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": len(next(iter(cs.values())))}
            for k, cs in agg.items()}


def main():
    o = sys.argv[1]
    fe, wr = load(os.path.join(o, "fetch"), {"FETCH_SIZE"}), load(os.path.join(o, "write"), {"WRITE_SIZE"})
    sq = load(os.path.join(o, "sq"), {"SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
                                     "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_WAIT_INST_ANY"})
    res = {"command": "tools/mb_mappo.py --episodes 1 --epochs 2 (cfg3: 4096 envs x 8 agents, T=100, L=5)",
           "units": "bytes per dispatch; fetch = 2 x FETCH_SIZE(KB) x 1024 (gfx950 correction), write = WRITE_SIZE x 1024",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        if "mappo" not in k:
            continue
        f = fe.get(k, {}).get("FETCH_SIZE", 0.0) * 2 * 1024
        w = wr.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        res["kernels"][k] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w,
                             "dispatches": fe.get(k, {}).get("dispatches", 0)}
    for k, cs in sq.items():
        for name in ("mappo_grad_kernel", "mappo_grad_gru_kernel", "mappo_grad_mlp_kernel"):
            if name in k:   # round 4: the pass is split in a recurrent and a row-parallel MLP kernel
                res["sq_" + name] = cs
    json.dump(res, open(os.path.join(o, "pmc_mappo.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
