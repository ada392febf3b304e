#!/bin/bash
# Full GPU test suite (verbose log under gpurun_out/, no -x) then smoke; both bounded.
mkdir -p gpurun_out
timeout -k 10 ${1:-600} python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_all.log | tail -30
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; }
fi
exit $rc
