# learner changes: learner / checkpoint / train / adapter / eval tests, update time (1 and 10 updates per graph
# launch), kernel timeline
mkdir -p gpurun_out/lrn
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_checkpoint.py tests/test_gpu_train.py tests/test_gpu_adapters.py tests/test_gpu_eval.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lrn/t.log 2>&1
rc=$?; tail -3 gpurun_out/lrn/t.log; grep "^E  \|FAILED" gpurun_out/lrn/t.log | head -8; [ $rc -eq 0 ] || exit $rc
for k in 1 10 1 10; do
  MB_K=$k MB_E=4096 MB_CAP=65536 timeout -k 10 200 python -u tools/mb_learner.py 2> gpurun_out/lrn/mb.err || { tail -5 gpurun_out/lrn/mb.err; exit 1; }
done
MB_K=1 MB_E=4096 MB_CAP=65536 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lrn/kt5 -- python3 tools/mb_learner.py > gpurun_out/lrn/kt5.log 2>&1 || { tail -5 gpurun_out/lrn/kt5.log; exit 1; }
python3 tools/ktimeline.py gpurun_out/lrn/kt5 per_sample_kernel 16
