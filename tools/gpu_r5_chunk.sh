# chunk-persistent rollout: parity tests first (bounded), then the A/B microbenchmark
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_chunk.py tests/test_gpu_fused_step.py tests/test_gpu_mappo.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/chunk_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/chunk_tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mb_chunk.py > gpurun_out/mb_chunk.json 2> gpurun_out/mb_chunk.err
rc=$?
cat gpurun_out/mb_chunk.json; tail -3 gpurun_out/mb_chunk.err

timeout -k 10 120 python -u tools/mb_mappo_roll.py > gpurun_out/mb_mappo_roll.json 2>&1; cat gpurun_out/mb_mappo_roll.json | tail -2
