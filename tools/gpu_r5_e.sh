mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunk.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/chunk_t.log 2>&1
rc=$?; tail -3 gpurun_out/chunk_t.log; grep "^E  " gpurun_out/chunk_t.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mb_chunk.py > gpurun_out/mb_chunk.json 2> gpurun_out/mb_chunk.err || { tail -5 gpurun_out/mb_chunk.err; exit 1; }
cat gpurun_out/mb_chunk.json
timeout -k 10 200 python -u tools/chunk_trace.py > gpurun_out/ctrace.txt 2>&1; grep -v "^{" gpurun_out/ctrace.txt | head -24
