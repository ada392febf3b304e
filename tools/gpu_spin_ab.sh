#!/bin/bash
# blocking vs spinning synchronize on the region probe (20-step regions), interleaved twice
export TMPDIR=/tmp
O=gpurun_out/spin_ab
mkdir -p $O
for r in 1 2; do
  for sp in 0 1; do
    MB_SPIN=$sp MB_MODES=region MB_R=30 timeout -k 10 200 python3 -u tools/region_probe.py > $O/spin${sp}_$r.jsonl 2>/dev/null || exit 1
    python3 -c "
import json,sys
d=json.loads(open('$O/spin${sp}_$r.jsonl').readline()); ms=sorted(x['ms'] for x in d['regions'])
print('spin=$sp run $r median_ms_per_step', round(ms[len(ms)//2]/20,5), 'min', round(ms[0]/20,5))"
  done
done
