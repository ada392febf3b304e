#!/bin/bash
# round-3 check: PER / learner / headline parity tests, then PER insert + cfg5 update microbenchmarks,
# the headline-only bench and the cfg5 kernel profile
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "${PYTEST_K:-per_ or cfg5 or learner or headline}" > gpurun_out/r3a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/mb_per.py | tee gpurun_out/r3a_mbper.log || exit 1
bash tools/gpu_quick_bench.sh || exit 1
bash tools/prof_cfg5.sh
