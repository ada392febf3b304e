"""HBM traffic per dispatch of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <grid_size> <alg_bytes> <out.json> <cmd>
FETCH_SIZE / WRITE_SIZE are in KB per dispatch (summed over the XCD instances); on gfx950
FETCH_SIZE reports 1/2 of a wide coalesced stream (MI355X_MICROARCH.md, HBM section), so it
is doubled; WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter, kern, grid):
    vals = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter and r.get("Grid_Size", "") == str(grid):
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, kern, grid, alg, out, cmd = sys.argv[1:8]
    fe = per_dispatch(fdir, "FETCH_SIZE", kern, grid)
    wr = per_dispatch(wdir, "WRITE_SIZE", kern, grid)
    fkb, wkb = sum(fe) / len(fe), sum(wr) / len(wr)
    res = {"command": cmd, "kernel": kern, "grid_size": int(grid),
           "units": "KB per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE)",
           "fetch_size_kb_mean": fkb, "fetch_size_dispatches": len(fe),
           "write_size_kb_mean": wkb, "write_size_dispatches": len(wr),
           "traffic_bytes_corrected": (2 * fkb + wkb) * 1024,
           "correction": "gfx950: FETCH_SIZE reports 1/2 of a wide coalesced stream (MI355X_MICROARCH.md HBM "
                         "section) -> doubled; WRITE_SIZE as is",
           "algorithmic_bytes": int(alg)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
