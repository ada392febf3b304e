#!/bin/bash
# Fixed cost of a 20-step timed region on the fused engine: host stamps per region (region_probe) + a kernel trace
# of the same run, to place t0 -> first kernel and last kernel -> synchronize return.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/region4}
mkdir -p $OUT
MB_MODES=region timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -- \
  python3 -u tools/region_probe.py > $OUT/probe_traced.jsonl 2> $OUT/probe_traced.err
rc=$?; cut -c1-200 $OUT/probe_traced.jsonl; exit $rc
