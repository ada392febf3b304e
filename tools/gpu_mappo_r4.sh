#!/bin/bash
# MAPPO gradient pass (split recurrent / MLP passes): parity tests, the cfg3 timing, kernel stats
export TMPDIR=/tmp
O=gpurun_out/mappo_r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mappo.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/mb_mappo.py --episodes 2 > $O/mb.log 2>&1 && tail -1 $O/mb.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 -u tools/mb_mappo.py --episodes 1 > $O/mb_prof.log 2>&1
python3 profiles/summarize.py $O/stats > $O/kernel_stats.txt 2>&1; head -12 $O/kernel_stats.txt
exit $rc
