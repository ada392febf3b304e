mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mappo.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "full_train_15 or cfg3_full_size" > gpurun_out/mappo_t.log 2>&1
grep -E "PASSED|FAILED|^E " gpurun_out/mappo_t.log | tail -8
timeout -k 10 300 python -u tools/mb_chunk.py > gpurun_out/mb_chunk.json 2> gpurun_out/mb_chunk.err || { tail -5 gpurun_out/mb_chunk.err; exit 1; }
cat gpurun_out/mb_chunk.json
timeout -k 10 120 python -u tools/mb_mappo_roll.py > gpurun_out/mb_mappo_roll.json 2>&1; tail -2 gpurun_out/mb_mappo_roll.json
