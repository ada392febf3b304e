mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_eval.py -x -q --timeout 120 --timeout-method thread > gpurun_out/env_tests.log 2>&1 || { tail -30 gpurun_out/env_tests.log; exit 1; }
tail -2 gpurun_out/env_tests.log
for v in new old new old; do
  if [ $v = old ]; then export MM_LIB=$PWD/mini-marl_amd/lib_ab/libminimarl_old.so; else unset MM_LIB; fi
  MB_CUR=0 timeout -k 10 60 python tools/mb_env.py > gpurun_out/mbe_$v.log 2>&1 || exit 1; echo "$v $(tail -1 gpurun_out/mbe_$v.log)"
done
