#!/bin/bash
# Region fixed-cost probe: host timings per 20-step region for the chunk / single-step
# replays and for one captured region graph, plus a kernel trace of the same run for the gaps.
export TMPDIR=/tmp
OUT=gpurun_out/region
mkdir -p $OUT
MB_MODES=steps,region timeout -k 10 240 python3 -u tools/region_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err && \
MB_MODES=steps,region timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -- \
  python3 -u tools/region_probe.py > $OUT/probe_traced.jsonl 2> $OUT/probe_traced.err
rc=$?
cut -c1-200 $OUT/probe.jsonl
exit $rc
