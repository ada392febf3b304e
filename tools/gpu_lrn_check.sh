#!/bin/bash
# learner parity tests + the three learner timings (B=32 at the bench's PER shape, cfg5, B=4096)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "${PYTEST_K:-cfg5 or learner or chunk_sequence or b4096 or pre_h3 or adapter or train}" > gpurun_out/lrn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lrn_tests.log; [ $rc -eq 0 ] || exit $rc
MB_E=4096 MB_CAP=65536 timeout -k 10 200 python3 tools/mb_learner.py || exit 1
timeout -k 10 300 python3 tools/mb_cfg5.py 4096 5 || exit 1
timeout -k 10 300 python3 tools/mb_learner_big.py 2>&1 | tail -1
