#!/bin/bash
# kernel stats of the QMIX learner update at the throughput batch (B = 4096, C = 10, GRU-64, Hm = 64)
export TMPDIR=/tmp
O=gpurun_out/pb4096
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 tools/mb_learner_big.py 4096 > $O/log.txt 2>&1
rc=$?
tail -1 $O/log.txt
python3 profiles/summarize.py $O/stats > $O/kernel_stats.txt
head -16 $O/kernel_stats.txt
exit $rc
