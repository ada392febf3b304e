# fp16x3 forward: packed-f32 gates (default build) vs scalar gates (lib_ab/libminimarl_nopk.so)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pk_tests.log 2>&1 || { tail -30 gpurun_out/pk_tests.log; exit 1; }
tail -2 gpurun_out/pk_tests.log
for v in pk nopk pk nopk; do
  if [ $v = nopk ]; then export MM_LIB=$PWD/mini-marl_amd/lib_ab/libminimarl_nopk.so; else unset MM_LIB; fi
  timeout -k 10 60 python tools/mb_fwd.py > gpurun_out/mbpk_$v.log 2>&1 || exit 1; echo "$v $(tail -1 gpurun_out/mbpk_$v.log)"
done
