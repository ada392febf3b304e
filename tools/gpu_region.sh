#!/bin/bash
# Region fixed-cost probe: host timings per 20-step region for the chunk / single-step
# replays and for one captured region graph, blocking vs spinning synchronize, plus a kernel trace.
export TMPDIR=/tmp
OUT=gpurun_out/region
mkdir -p $OUT
MB_MODES=steps,region timeout -k 10 240 python3 -u tools/region_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err && \
MB_SPIN=1 MB_MODES=region timeout -k 10 240 python3 -u tools/region_probe.py > $OUT/probe_spin.jsonl 2> $OUT/probe_spin.err && \
MB_SPIN=1 MB_MODES=region timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_spin -- \
  python3 -u tools/region_probe.py > $OUT/probe_spin_traced.jsonl 2> $OUT/probe_spin_traced.err
rc=$?
cut -c1-120 $OUT/probe.jsonl $OUT/probe_spin.jsonl
exit $rc
