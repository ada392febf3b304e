#!/bin/bash
# kernel stats of the MAPPO train passes (cfg3: 4096 x 8, T 100, L 5): tools/mb_mappo.py under rocprofv3
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_mappo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mappo -- python3 tools/mb_mappo.py --episodes 1 --epochs 3 > gpurun_out/prof_mappo.log 2>&1 || { tail -5 gpurun_out/prof_mappo.log; exit 1; }
f=$(find gpurun_out/prof_mappo -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r[:12]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us avg', round(float(x['TotalDurationNs'])/1e6,2), 'ms')
"
