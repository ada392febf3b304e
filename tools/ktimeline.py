"""Timeline of the last dispatches in a rocprofv3 --kernel-trace csv directory: start offset and duration (us), queue
id, kernel, from the last dispatch of <first-kernel substring> on. usage: ktimeline.py <dir> <first-kernel> [max]"""
import csv
import glob
import sys

d, first = sys.argv[1], sys.argv[2]
mx = int(sys.argv[3]) if len(sys.argv) > 3 else 60
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
i0 = idx[-2] if len(idx) > 1 else idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + mx]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} {r.get('Queue_Id', r.get('Stream_Id', '?')):>3} {r['Kernel_Name'][:100]}")
