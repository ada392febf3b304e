# pack / range-guard tests + rollout + learner tests, then the learner microbench at the bench's PER shape
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_learner.py tests/test_gpu_headline.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 || { tail -30 gpurun_out/pack_tests.log; exit 1; }
tail -2 gpurun_out/pack_tests.log
for f in 1 1 1; do MB_FUSED=$f MB_E=4096 MB_CAP=65536 timeout -k 10 120 python tools/mb_learner.py > gpurun_out/mbl_$f.log 2>&1 || { tail -5 gpurun_out/mbl_$f.log; exit 1; }; tail -1 gpurun_out/mbl_$f.log; done
