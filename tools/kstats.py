"""Print the top kernels of rocprofv3 *_kernel_stats.csv files (usage: kstats.py file... [top])."""
import csv
import sys

top = 16
files = [a for a in sys.argv[1:] if a.endswith(".csv")]
for a in sys.argv[1:]:
    if a.isdigit():
        top = int(a)
for f in files:
    print(f)
    rows = list(csv.DictReader(open(f)))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f'  {r["Name"][:72]:72s} calls {int(r["Calls"]):6d} avg_us {float(r["AverageNs"]) / 1e3:9.2f} '
              f'pct {float(r["Percentage"]):6.2f}')
