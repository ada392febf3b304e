#!/bin/bash
# Kernel stats of the cfg5 QMIX update (tools/mb_cfg5.py) -> gpurun_out/prof_cfg5/kernel_stats.txt
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_cfg5
mkdir -p $OUT
timeout -k 10 300 python3 tools/mb_cfg5.py 4096 5 > $OUT/mb.log 2>&1
cat $OUT/mb.log | grep B
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -- python3 tools/mb_cfg5.py 4096 5 > $OUT/stats.log 2>&1
python3 profiles/summarize.py $OUT/stats > $OUT/kernel_stats.txt
head -30 $OUT/kernel_stats.txt
