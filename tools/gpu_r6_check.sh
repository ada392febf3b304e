mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_chunk.py::test_chunk_handoff_timeout_is_reported_and_grid_drains tests/test_gpu_checkpoint.py "tests/test_gpu_learner.py::test_multi_sample_blocks_bit_identical" tests/test_gpu_headline.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/g1.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" gpurun_out/g1.log | tail -40
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_quick_bench.sh --steps 20 --warmup 5
