mkdir -p gpurun_out/hl
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -k "eviction" > gpurun_out/hl/t.log 2>&1
rc=$?; tail -3 gpurun_out/hl/t.log; grep "^E  \|FAILED" gpurun_out/hl/t.log | head -8; exit $rc
