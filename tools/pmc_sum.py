"""Average rocprofv3 --pmc counters per (kernel, grid size) from counter_collection.csv files.

usage: python tools/pmc_sum.py <dir> [kernel-substring]   (searches <dir> recursively)
"""
import collections
import csv
import glob
import os
import sys


def main(d, filt=""):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if filt not in name:
                continue
            key = (name[:80], r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
            acc[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for key, m in acc.items():
        per = collections.defaultdict(list)
        for (disp, cname), vals in m.items():
            per[cname].append(sum(vals))  # sum over dimensions (XCD/SE instances) of one dispatch
        print(key)
        for cname in sorted(per):
            v = per[cname]
            print(f"   {cname:32s} n={len(v):4d} avg={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
