"""Summarise a rocprofv3 --kernel-trace --stats CSV directory (kernel stats + per-step timeline)."""
import csv
import sys


def main(d):
    import glob
    rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0])))
    for r in rows:
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6} avg_us={float(r['AverageNs'])/1e3:9.2f} "
              f"total_ms={float(r['TotalDurationNs'])/1e6:8.3f} pct={float(r['Percentage']):6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
