#!/bin/bash
# round-6 check: the chunk / checkpoint / headline / trainer tests (args: pytest selectors), then the quick headline bench
mkdir -p gpurun_out
sel=${@:-tests/test_gpu_chunk.py tests/test_gpu_checkpoint.py tests/test_gpu_headline.py tests/test_gpu_train.py}
timeout -k 10 600 python -u -m pytest $sel -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/g1.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" gpurun_out/g1.log | tail -60
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_quick_bench.sh --steps 20 --warmup 5
